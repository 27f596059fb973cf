"""MFMA-busy / wait / traffic table of our GEMM dispatches from tools/gemm_pmc.sh (or fp8_pmc.sh) counter passes.
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs) (as profiles/r03_gemm_pmc_epilogue.txt);
wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES; LDS-wait = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES; read = 2 x FETCH_SIZE KiB.
Usage: pmc_table.py DIR_PASS1 [DIR_PASS2 ...] -- dispatches are matched across passes by order of our kernels."""
import csv, glob, os, sys
from collections import OrderedDict

OURS = ("gemm_pp_kernel", "gemm_w4p", "gemm_fp8_kernel", "gemm_w4p8", "gemm256", "gemm_bf16")


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    by = OrderedDict()
    for r in csv.DictReader(open(f)):
        if not any(k in r["Kernel_Name"] for k in OURS):
            continue
        e = by.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "c": {}})
        e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(by.values())


passes = [load(d) for d in sys.argv[1:]]
n = min(len(p) for p in passes)
for i in range(n):
    c = {}
    for p in passes:
        c.update(p[i]["c"])
    e = passes[0][i]
    name = e["name"].replace("(anonymous namespace)::", "")[:60]
    parts = [f"{i:3d} {name:60s} grid {e['grid']:8d}"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        parts.append(f"MFMA busy {100 * c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 1024):5.1f}%")
        parts.append(f"wait {100 * c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:5.1f}%")
    if "SQ_WAIT_INST_LDS" in c and "SQ_WAVE_CYCLES" in c:
        parts.append(f"LDS-wait {100 * c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:4.1f}%")
    if "SQ_LDS_BANK_CONFLICT" in c:
        parts.append(f"LDS conflicts {int(c['SQ_LDS_BANK_CONFLICT'])}")
    if "FETCH_SIZE" in c:
        parts.append(f"read {2 * c['FETCH_SIZE'] * 1024 / 1e9:6.3f} GB")
    if "WRITE_SIZE" in c:
        parts.append(f"write {c['WRITE_SIZE'] * 1024 / 1e9:6.3f} GB")
    print("  ".join(parts))
