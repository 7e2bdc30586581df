"""Per-kernel PMC summary of one measurement session (tools/gpu_round.sh): HBM traffic and MFMA use.

Inputs (rocprofv3 --pmc CSVs, one pass each, same bench command):
  pmc1: FETCH_SIZE   pmc2: WRITE_SIZE
  pmc3: SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
  cal_FETCH_SIZE / cal_WRITE_SIZE: tools/micro/pmc_cal (512 MiB of dword / dwordx4 / epilogue-pattern
  reads and writes) -> the correction factors actually measured on this box.
Corrections (MI355X_MICROARCH.md §HBM, re-measured by pmc_cal): HBM bytes = FETCH_SIZE x f_read +
WRITE_SIZE x f_write with f = true bytes / counter bytes of the calibration kernels.
MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 4 SIMDs x 256 CUs)
(GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy cycles over every SIMD). Effective clock per dispatch
= GRBM_GUI_ACTIVE / 8 / dispatch duration (MI355X_MICROARCH.md, DVFS give-back), median over launches.
usage: python tools/pmc_summary.py gpurun_out TAG [lib_sha16] > summary.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out_dir, tag = sys.argv[1], sys.argv[2]
CUS, SIMDS = 256, 4


def rows(pattern):
    fs = glob.glob(os.path.join(out_dir, pattern, "**", "*counter_collection.csv"), recursive=True)
    return [r for f in fs for r in csv.DictReader(open(f))]


def short(name):
    n = name.replace("void ifd::(anonymous namespace)::", "").replace("void ifd::", "")
    n = n.replace("(ifd::ConvParams)", "").replace(" ", "")
    return n.split("(")[0]


def per_kernel(rs):
    acc = defaultdict(lambda: defaultdict(list))
    for r in rs:
        acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("Start_Timestamp") and r.get("End_Timestamp"):
            # effective shader clock of the dispatch: GUI-active cycles (summed over the 8 XCDs) / 8 / duration
            ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            if ns > 0:
                acc[short(r["Kernel_Name"])]["_clock_ghz"].append(float(r["Counter_Value"]) / 8 / ns)
    return acc


cal_f = {short(r["Kernel_Name"]): float(r["Counter_Value"]) for r in rows(f"cal_FETCH_SIZE_{tag}")}
cal_w = {short(r["Kernel_Name"]): float(r["Counter_Value"]) for r in rows(f"cal_WRITE_SIZE_{tag}")}
true_kib = 512 * 1024
f_read = true_kib / cal_f["r_dwordx4"] if cal_f.get("r_dwordx4") else 2.0
f_read_dword = true_kib / cal_f["r_dword"] if cal_f.get("r_dword") else 2.0
f_write = true_kib / cal_w["w_epi"] if cal_w.get("w_epi") else 1.0

fetch = per_kernel(rows(f"pmc1_{tag}"))
write = per_kernel(rows(f"pmc2_{tag}"))
mf = per_kernel(rows(f"pmc3_{tag}"))
out = {"tag": tag, "calibration": {"fetch_factor_dwordx4": f_read, "fetch_factor_dword": f_read_dword,
                                   "write_factor_epilogue_pattern": f_write,
                                   "write_factor_dwordx4": true_kib / cal_w["w_dwordx4"] if cal_w.get("w_dwordx4") else None,
                                   "source": "tools/micro/pmc_cal.hip, 512 MiB per dispatch"},
       "kernels": {}}
if len(sys.argv) > 3:
    out["lib_sha16"] = sys.argv[3]
for k in sorted(set(fetch) | set(mf)):
    d = {}
    if k in fetch and k in write:
        fv = fetch[k]["FETCH_SIZE"]
        wv = write[k]["WRITE_SIZE"]
        d["launches"] = len(fv)
        d["hbm_bytes_per_launch"] = (sum(fv) / len(fv) * f_read + sum(wv) / len(wv) * f_write) * 1024
        d["fetch_bytes_per_launch"] = sum(fv) / len(fv) * f_read * 1024
        d["write_bytes_per_launch"] = sum(wv) / len(wv) * f_write * 1024
    if k in mf and mf[k].get("GRBM_GUI_ACTIVE"):
        busy = sum(mf[k]["SQ_VALU_MFMA_BUSY_CYCLES"])
        gui = sum(mf[k]["GRBM_GUI_ACTIVE"])
        d["mfma_busy_frac"] = busy / (gui / 8 * SIMDS * CUS)
        if mf[k].get("SQ_INSTS_VALU_MFMA_MOPS_F16"):
            d["mfma_mops_f16_per_launch"] = sum(mf[k]["SQ_INSTS_VALU_MFMA_MOPS_F16"]) / len(mf[k]["SQ_INSTS_VALU_MFMA_MOPS_F16"])
        d["sq_busy_frac"] = sum(mf[k]["SQ_BUSY_CYCLES"]) / (gui / 8 * CUS) if mf[k].get("SQ_BUSY_CYCLES") else None
        d["gui_active_cycles_per_launch"] = gui / 8 / len(mf[k]["GRBM_GUI_ACTIVE"])
        if mf[k].get("_clock_ghz"):
            ck = sorted(mf[k]["_clock_ghz"])
            d["eff_clock_ghz_median"] = ck[len(ck) // 2]
            # MFMA busy x clock / 2.4 GHz nominal = the fraction of the nominal dense peak the launch reached
            d["busy_x_clock_over_nominal"] = d["mfma_busy_frac"] * ck[len(ck) // 2] / 2.4
    out["kernels"][k] = d
print(json.dumps(out, indent=1))
