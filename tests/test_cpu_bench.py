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


def test_parity_mode_requests_batch_invariant():
    """`--noise parity` builds the model with the batch-invariant conv geometry: a
    rank's shard is then bit-equal to the same images in any other batch, so the line is
    GPU-count-independent; the default throughput mode keeps the fastest geometry."""
    ap = bench.build_parser()
    assert bench.model_options(ap.parse_args(["--noise", "parity"])) == {"batch_invariant": 1}
    assert bench.model_options(ap.parse_args(["--noise", "parity", "--workload", "c4"])) == {"batch_invariant": 1}
    assert bench.model_options(ap.parse_args([])) == {}


def test_device_key_keeps_pci_ids_beside_uuid():
    """Two devices whose ROCm build reports the same (e.g. all-zero) UUID still count as two."""
    from types import SimpleNamespace
    a = SimpleNamespace(uuid="00000000-0000-0000-0000-000000000000", pci_domain_id=0, pci_bus_id=0x15, pci_device_id=0)
    b = SimpleNamespace(uuid="00000000-0000-0000-0000-000000000000", pci_domain_id=0, pci_bus_id=0x75, pci_device_id=0)
    assert bench.device_key("n0", a) != bench.device_key("n0", b)
    assert bench.device_key("n0", a) == bench.device_key("n0", SimpleNamespace(**vars(a)))
    assert bench.device_key("n0", a) != bench.device_key("n1", a)


def test_script_ddim_pass_is_the_reference_loop():
    """bench's drop-in workload restates the reference script's loop (code/test_inp_ddim_100.py:470-576 +
    the final blend :692-696) around model(): on CPU with a stand-in model it equals the oracle's
    restatement of the same script (tests/golden pins that oracle bit-exact to the reference) bit for bit."""
    from oracle import ref_diffusion
    tb = ref_diffusion.Tables(ref_diffusion.get_named_beta_schedule("cosine", 1000))

    def stub_unet(x, t, masked, m):  # deterministic, depends on every input
        s = (t.to(torch.float32) / 1000.0).view(-1, 1, 1, 1)
        eps = 0.3 * x + 0.2 * masked - 0.1 * m + s
        return torch.cat([eps, 0.5 * eps], dim=1)

    class Stub:
        def __call__(self, x, t, masked_image=None, mask=None):
            return stub_unet(x, t, masked_image, mask)

    gt, mask = bench.synth_inputs(2, 32, seed=5, device="cpu")
    shape = (2, 3, 32, 32)
    torch.manual_seed(11)
    a = bench.script_ddim_pass(Stub(), tb.ac, shape, gt, mask, 10, 0.75, "cpu")
    torch.manual_seed(11)
    b = ref_diffusion.final_blend(ref_diffusion.script_ddim_loop(tb, ref_diffusion.model_fn_factory(stub_unet), shape,
                                                                 gt, mask, 10, clip=True, eta=0.75), gt, mask)
    assert torch.equal(a, b)


def test_fp32_accuracy_note_reads_newest_parity(tmp_path, monkeypatch):
    """The fp32_exact entry states its measured accuracy against the reference: the ratio of
    the mode's per-eval error vs fp64 to the reference's own, from the newest parity record that holds it."""
    for tag, g in (("r01x", 4e-7), ("r02x", 2e-7)):
        d = tmp_path / "profiles" / tag
        d.mkdir(parents=True)
        (d / "parity.json").write_text(json.dumps({"c1_eval0/fp32": {
            "gpu_vs_fp64": {"mean": g, "p999": 2 * g, "max": 4 * g},
            "reference_vs_fp64": {"mean": 1e-7, "p999": 2e-7, "max": 4e-7}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    note = bench.fp32_accuracy_note()
    assert note["per_eval_error_vs_reference_own"] == {"mean": 2.0, "p999": 2.0, "max": 2.0}
    assert note["source"].endswith("r02x/parity.json")
    assert "NOT fp32-class" in note["note"]


def test_headline_line_carries_a_training_leg():
    """BASELINE configs[4] on the driver's clock: the default N=1 bench run times 3xf16 training steps at B = 32
    (`train` in the JSON line) after the sampler's lines; the profiler passes of tools/gpu_round.sh switch it off."""
    import bench
    a = bench.build_parser().parse_args([])
    assert a.train_steps == 5 and a.train_batch == 32
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "gpu_round.sh")).read()
    assert src.count("--train-steps 0") == 2
