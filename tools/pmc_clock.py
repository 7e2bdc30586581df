"""Per-layer clock / MFMA-busy comparison of two counter passes over the same workload (development helper).
usage: python tools/pmc_clock.py DIR_A DIR_B   (rocprofv3 --pmc dirs holding *counter_collection.csv with
GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES, SQ_VALU_MFMA_BUSY_CYCLES; the same sequence of conv_x3 dispatches in both)
Per dispatch: duration, effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration, MFMA busy = MFMA busy cycles /
(GUI / 8 x 1024 SIMDs); dispatches are matched by position (the eval repeats the same layer sequence)."""
import csv, glob, os, sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    disp = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        disp[k]["name"] = r["Kernel_Name"].split("<", 1)[1].split(">")[0] if "<" in r["Kernel_Name"] else r["Kernel_Name"]
        disp[k]["grid"] = int(r["Grid_Size"])
        disp[k]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        disp[k][r["Counter_Name"]] = float(r["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def stats(ds):
    gui = sum(d["GRBM_GUI_ACTIVE"] for d in ds) / 8
    dur = sum(d["dur"] for d in ds)
    mf = sum(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for d in ds)
    return dur * 1e3 / len(ds), gui / dur / 1e9, mf / (gui * 1024), gui / len(ds)


a, b = load(sys.argv[1]), load(sys.argv[2])
n = min(len(a), len(b))
groups = defaultdict(lambda: ([], []))
for i in range(n):
    if a[i]["name"] != b[i]["name"]:
        continue
    key = (a[i]["name"], a[i]["grid"], round(a[i]["dur"] * 1e5))  # layer signature (kernel, grid, ~duration)
    groups[(a[i]["name"], a[i]["grid"], i % 1000)]  # placeholder to keep order
tot = defaultdict(lambda: ([], []))
for i in range(n):
    if a[i]["name"] == b[i]["name"]:
        tot[(a[i]["name"], round(a[i]["dur"] * 1e4))][0].append(a[i])
        tot[(a[i]["name"], round(a[i]["dur"] * 1e4))][1].append(b[i])
print(f"{'kernel':22s} {'~ms':>5s} {'n':>4s} | {'ms A':>7s} {'GHz A':>6s} {'busy A':>6s} {'Mcyc A':>7s} | {'ms B':>7s} {'GHz B':>6s} {'busy B':>6s} {'Mcyc B':>7s}")
for (name, d), (da, db) in sorted(tot.items(), key=lambda kv: -sum(x["dur"] for x in kv[1][0])):
    if len(da) < 2:
        continue
    sa, sb = stats(da), stats(db)
    print(f"{name:22s} {d / 10:5.2f} {len(da):4d} | {sa[0]:7.4f} {sa[1]:6.3f} {sa[2]:6.3f} {sa[3] / 1e6:7.3f} | "
          f"{sb[0]:7.4f} {sb[1]:6.3f} {sb[2]:6.3f} {sb[3] / 1e6:7.3f}")
