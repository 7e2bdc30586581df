"""Per-block phase timing of one conv launch (development tool; needs an IFD_TRACE=1 build).

    make -C face-inpainting-diffusion-models_amd variant V=trace DEFS=-DIFD_TRACE=1
    python tools/conv_trace.py "r256 128+0->128 skip0 xf0" ["r256 128+128->128 skip0 xf0" ...]

For each layer-name substring: one warm UNet eval (B=16, full config), then one eval with the
trace armed; prints the phase breakdown (fill, main loop, epilogue), the per-CU concurrency and
the gaps between consecutive blocks on a CU.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("IFD_LIB_PATH", os.path.join(ROOT, "face-inpainting-diffusion-models_amd", "build_trace",
                                                   "libifd.so"))
sys.path.insert(0, os.path.join(ROOT, "face-inpainting-diffusion-models_amd"))
import torch  # noqa: E402
from ifd.manifest import make_state_dict  # noqa: E402
from ifd.model import DiffusionInpaintingModel  # noqa: E402
from ifd.topology import FULL  # noqa: E402

TICK_NS = 10.0  # s_memrealtime: 100 MHz


def analyze_stream(meta, a):
    """conv_stream records: s_memtime stamps of intervals 8..15 (see conv_stream.hip)."""
    a = a[a[:, 63] != 0]
    st = a[:, :64].reshape(len(a), 8, 8)[:, :, :7].astype(np.float64)  # [block, interval, slot]
    P0, P1, P2, P3, C0, C1, P6 = (st[:, :, i] for i in range(7))

    def q(v):
        v = np.asarray(v).ravel()
        return {"p10": round(float(np.percentile(v, 10))), "p50": round(float(np.median(v))),
                "p90": round(float(np.percentile(v, 90)))}
    return {"meta": meta, "blocks": int(len(a)), "units": "shader cycles",
            "interval (consumer start->start)": q(C0[:, 1:] - C0[:, :-1]),
            "consumer MFMA issue": q(C1 - C0), "consumer wait at barrier": q(C0[:, 1:] - C1[:, :-1]),
            "producer drain (old loads)": q(P6 - P0), "producer load issue after drain": q(P1 - P6), "producer store (incl. vmcnt waits)": q(P2 - P1),
            "producer epilogue": q(P3 - P2), "producer wait at barrier": q(P0[:, 1:] - P3[:, :-1]),
            "producer busy": q(P3 - P0)}


def analyze(fn):
    meta = json.load(open(fn + ".json"))
    a = np.fromfile(fn, dtype=np.uint64).reshape(-1, 64).astype(np.int64)
    if meta.get("stream"):
        return analyze_stream(meta, a)
    a = a[:, :8]
    live = a[:, 0] > 0
    a = a[live]
    t0 = a[:, 0].min()
    ts = (a[:, [0, 1, 2, 3, 4, 6]] - t0) * TICK_NS / 1e3  # us
    entry, cons_go, main_end, epi_end, prod_first, prod_end = ts.T
    hw = a[:, 5] & 0xFFFFFFFF
    xcc = a[:, 5] >> 32
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    cu_key = xcc * 1000 + se * 100 + sh * 16 + cu
    ghz = a[:, 7] / ((a[:, 3] - a[:, 0]) * TICK_NS)

    def q(v):
        return {"p10": round(float(np.percentile(v, 10)), 2), "p50": round(float(np.median(v)), 2),
                "p90": round(float(np.percentile(v, 90)), 2)}

    res = {"meta": meta, "blocks": int(len(a)), "kernel_us": round(float(epi_end.max()), 1),
           "shader_ghz": q(ghz),
           "fill_us (entry->consumer past 1st barrier)": q(cons_go - entry),
           "producer_first_chunk_us": q(prod_first - entry),
           "main_us": q(main_end - cons_go),
           "epilogue_us": q(epi_end - main_end),
           "block_us": q(epi_end - entry)}
    # per-CU timeline: concurrency and dispatch gaps
    gaps, conc = [], []
    for k in np.unique(cu_key):
        idx = np.where(cu_key == k)[0]
        order = idx[np.argsort(entry[idx])]
        st, en = entry[order], epi_end[order]
        for i in range(len(order)):
            conc.append(int(((st <= st[i]) & (en > st[i])).sum()))
        # gap: for each block start after the first wave, time since the latest earlier end
        for i in range(len(order)):
            prev_end = en[(en <= st[i])]
            if len(prev_end):
                gaps.append(st[i] - prev_end.max())
    res["cus"] = int(len(np.unique(cu_key)))
    res["blocks_per_cu_at_start"] = q(np.array(conc))
    res["dispatch_gap_us"] = q(np.array(gaps)) if gaps else None
    n_ch = meta["chunks"]
    res["us_per_chunk_main"] = round(float(np.median(main_end - cons_go)) / max(n_ch, 1), 3)
    return res


def main():
    layers = sys.argv[1:] or ["r256 128+0->128 skip0 xf0"]
    dev = torch.device("cuda:0")
    m = DiffusionInpaintingModel(FULL, device=dev)
    m.load_state_dict(make_state_dict(FULL, seed=1))
    B = 16
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, 3, 256, 256, device=dev, generator=g)
    mk = (torch.rand(B, 1, 256, 256, device=dev, generator=g) > 0.5).float()
    t = torch.full((B,), 500, device=dev)
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    with torch.no_grad():
        m(x, t, masked_image=x, mask=mk)
        torch.cuda.synchronize()
        allres = {}
        for i, lay in enumerate(layers):
            fn = os.path.join(out_dir, f"conv_trace_{i}.bin")
            os.environ["IFD_TRACE_MATCH"] = lay
            os.environ["IFD_TRACE_NTH"] = "0"
            os.environ["IFD_TRACE_FILE"] = fn
            m(x, t, masked_image=x, mask=mk)
            torch.cuda.synchronize()
            os.environ.pop("IFD_TRACE_MATCH")
            r = analyze(fn)
            allres[lay] = r
            print(json.dumps({lay: r}, indent=1), flush=True)
    json.dump(allres, open(os.path.join(out_dir, "conv_trace_summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
