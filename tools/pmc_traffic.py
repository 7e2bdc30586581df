"""Per-launch HBM traffic of a kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE / WRITE_SIZE are in KiB. gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports
half the bytes of 16-B-per-lane streaming reads -> x2; WRITE_SIZE is exact for 16-B stores (our
epilogue stores are 4-B per lane: reported raw, flagged as uncalibrated).
usage: python tools/pmc_traffic.py <fetch_csv> <write_csv> <kernel-substring>
"""
import csv, json, sys
fetch_csv, write_csv, pat = sys.argv[1:4]
def avg(path):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
    return sum(v) / len(v), len(v)
f, nf = avg(fetch_csv)
w, nw = avg(write_csv)
out = {"kernel_pattern": pat, "dispatches": nf, "fetch_kib_raw": f, "write_kib_raw": w,
       "hbm_bytes_per_launch_corrected": (2 * f + w) * 1024, "hbm_bytes_per_launch_raw": (f + w) * 1024,
       "correction": "FETCH x2 (gfx950 16-B streaming reads); WRITE raw"}
print(json.dumps(out))
