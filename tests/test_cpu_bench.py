"""bench.py's host-side contract pieces, on CPU: the synthetic workload (BASELINE configs[1] shapes, seeded,
masks in the reference's convention), the parallel-layout label (a rank count above the distinct devices is a
rehearsal, never an N-GPU line), and the roofline's traffic lookup (the newest committed PMC summary that
holds the kernel, a per-launch byte count, its source path)."""
import json
import os

import pytest
import torch

import bench


def test_synth_inputs_shapes_seeded():
    gt, mask = bench.synth_inputs(3, 64, seed=11, device=torch.device("cpu"))
    assert gt.shape == (3, 3, 64, 64) and mask.shape[0] == 3 and mask.shape[-2:] == (64, 64)
    assert gt.dtype == torch.float32 and float(gt.abs().max()) <= 1.0
    assert set(torch.unique(mask).tolist()) <= {0.0, 1.0} and 0 < float(mask.mean()) < 1
    gt2, mask2 = bench.synth_inputs(3, 64, seed=11, device=torch.device("cpu"))
    assert torch.equal(gt, gt2) and torch.equal(mask, mask2)
    gt3, _ = bench.synth_inputs(3, 64, seed=12, device=torch.device("cpu"))
    assert not torch.equal(gt, gt3)


def test_parallelism_note_labels_rehearsals():
    assert bench.parallelism_note(1, 1) == "dp1 (one GPU)"
    # (a world size > 1 needs an initialised process group for the backend name: covered by the gloo tests)


def test_pmc_traffic_picks_newest_summary(tmp_path, monkeypatch):
    for tag, nbytes in (("r01x", 1.0e9), ("r02x", 6.0e8)):
        d = tmp_path / "profiles" / tag
        d.mkdir(parents=True)
        (d / "pmc_summary.json").write_text(json.dumps(
            {"tag": tag, "kernels": {"conv_x3_kernel<0,false,32,3>": {"hbm_bytes_per_launch": nbytes,
                                                                      "mfma_busy_frac": 0.7}}}))
    (tmp_path / "profiles" / "r03x").mkdir()
    (tmp_path / "profiles" / "r03x" / "pmc_summary.json").write_text("{not json")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got = bench.pmc_traffic("conv_x3_kernel<0,false,32,3>")
    assert got["traffic"] == pytest.approx(6.0e8)
    assert got["mfma_busy"] == pytest.approx(0.7)
    assert got["traffic_source"] == os.path.join("profiles", "r02x", "pmc_summary.json")
    assert bench.pmc_traffic("no_such_kernel") == {"traffic": None}


def test_committed_pmc_summary_has_the_dominant_kernel():
    got = bench.pmc_traffic("conv_x3_kernel<0,false,32,3>")
    assert got["traffic"] and got["traffic"] > 1e8
