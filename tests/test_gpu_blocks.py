"""Block-level GPU checks, forward and backward, against the reference's own modules (code/nn.py):
ResBlock plain, 192->64 with the 1x1 skip, down, up; AttentionBlock at T = 16, 64, 256 — each in
isolation through the training ops (include/ifd_train.h, ifd.train.BlockTrainer). Fixtures:
tests/golden/make_golden_blocks.py (blocks.npz / blocks_meta.json, made by the reference).

Tolerances (fp32): y and dx within 1e-5 x max|ref| (max-abs), demb likewise, every parameter
gradient's norm within 1e-4 relative and its recorded values within 1e-4 of the tensor's max.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLDEN)

META = json.load(open(os.path.join(GOLDEN, "blocks_meta.json")))


@pytest.fixture(scope="module")
def blocks():
    return dict(np.load(os.path.join(GOLDEN, "blocks.npz")))


def _rel(a, b):
    return float((a.double().cpu() - b.double()).abs().max() / b.double().abs().max())


@pytest.mark.parametrize("name", sorted(META["cases"]))
def test_block_forward_backward(blocks, record, name):
    from make_golden_blocks import init_block, sample_idx
    from ifd.train import BlockTrainer
    rec = META["cases"][name]
    shapes = [(k, tuple(s)) for k, s in rec["params"]]
    bt = BlockTrainer(rec["kind"], rec["cin"], rec["cout"], emb_dim=META["emb_dim"], device=DEV)
    bt.load_state_dict(init_block(shapes, rec["seed"]))
    x = torch.from_numpy(blocks[f"{name}/x"])
    emb = torch.from_numpy(blocks[f"{name}/emb"]) if rec["kind"].startswith("res") else None
    with torch.no_grad():
        y = bt.forward_block(x.to(DEV), None if emb is None else emb.to(DEV))
        dx, demb = bt.backward_block(torch.from_numpy(blocks[f"{name}/dy"]).to(DEV))
    torch.cuda.synchronize()
    res = {"y": _rel(y, torch.from_numpy(blocks[f"{name}/y"])), "dx": _rel(dx, torch.from_numpy(blocks[f"{name}/dx"]))}
    if demb is not None:
        res["demb"] = _rel(demb, torch.from_numpy(blocks[f"{name}/demb"]))
    gworst = 0.0
    nworst = 0.0
    for k, shape in shapes:
        g = bt.g(k).flatten()
        gr = torch.from_numpy(blocks[f"{name}/g/{k}"]).double()
        gs = g[torch.from_numpy(sample_idx(g.numel())).to(DEV)].double().cpu()
        gworst = max(gworst, float((gs - gr).abs().max() / max(float(gr.abs().max()), 1e-30)))
        nworst = max(nworst, abs(float(g.double().norm()) - rec["gnorm"][k]) / max(rec["gnorm"][k], 1e-30))
    res.update(param_grad_rel=gworst, param_norm_rel=nworst)
    record(f"block/{name}", **res)
    assert res["y"] <= 1e-5 and res["dx"] <= 1e-5 and res.get("demb", 0.0) <= 1e-5, res
    assert gworst <= 1e-4 and nworst <= 1e-4, res
