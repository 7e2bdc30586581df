"""Collect one gpu_round.sh run into profiles/<tag>/: bench line, rocprof kernel stats, PMC traffic
of the dominant kernel, and the rocprof-vs-live average-duration agreement check.
usage: python tools/summarize_round.py <tag>"""
import csv, json, os, shutil, sys
tag = sys.argv[1]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
g = os.path.join(root, "gpurun_out")
out = os.path.join(root, "profiles", tag)
os.makedirs(out, exist_ok=True)
bench = json.load(open(os.path.join(g, f"bench_{tag}.json")))
shutil.copy(os.path.join(g, f"bench_{tag}.json"), os.path.join(out, "bench.json"))
shutil.copy(os.path.join(g, f"prof_{tag}", "trace_kernel_stats.csv"), os.path.join(out, "rocprof_kernel_stats.csv"))
rf = bench["roofline"]
dom = rf["kernel"]  # e.g. conv_stream2_kernel<0> or conv_kernel<256,64,4,1,9,0>
kname, args = dom[:-1].split("<", 1)
# rocprof names: "void ifd::conv_kernel<256, 64, 4, 1, 9, 0, 4, true>(ifd::ConvParams)" (extra args
# possible), "void ifd::(anonymous namespace)::conv_stream2_kernel<0>(ifd::ConvParams)"
pref = kname + "<" + ", ".join(args.split(","))
rows = [r for r in csv.DictReader(open(os.path.join(out, "rocprof_kernel_stats.csv"))) if pref in r["Name"]]
calls = sum(int(r["Calls"]) for r in rows)
tot_ns = sum(float(r["TotalDurationNs"]) for r in rows)
rocprof_avg_ms = tot_ns / calls / 1e6
def pmc(path):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if pref in r["Kernel_Name"]]
    return sum(v) / len(v), len(v)
fk, nf = pmc(os.path.join(g, f"pmc_fetch_{tag}", "pmc_counter_collection.csv"))
wk, nw = pmc(os.path.join(g, f"pmc_write_{tag}", "pmc_counter_collection.csv"))
summary = {
    "dominant_kernel": dom,
    "live_avg_launch_ms (bench.py hipEvents)": rf["avg_launch_ms"],
    "rocprof_avg_launch_ms (kernel-trace --stats)": rocprof_avg_ms,
    "rocprof_vs_live_rel_diff": rocprof_avg_ms / rf["avg_launch_ms"] - 1,
    "achieved_tflops": rf["achieved"], "peak_tflops": rf["peak"], "frac": rf["frac"],
    "algorithmic_bytes_per_launch": rf.get("algorithmic_bytes_per_launch"),
    "pmc": {"dispatches": nf, "FETCH_SIZE_KiB_avg": fk, "WRITE_SIZE_KiB_avg": wk,
            "hbm_bytes_per_launch_corrected": (2 * fk + wk) * 1024,
            "correction": "FETCH_SIZE x2 (gfx950 reports half of 16-B streaming reads); WRITE_SIZE raw (4-B epilogue stores: uncalibrated)",
            "note": "PMC passes ran --ddim-steps 10 (11 evals): same per-eval layer mix, so per-launch averages are comparable"},
}
json.dump(summary, open(os.path.join(out, "roofline_summary.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
