"""Summarise tools/attn_pmc.sh's three passes: per attention kernel and grid (one line per
distinct launch shape), mean over its launches of MFMA busy %, LDS-wait %, bank-conflict share,
and HBM bytes (FETCH_SIZE x2, WRITE_SIZE) with the effective clock.
Usage: attn_pmc_summary.py DIR_PREFIX (e.g. gpurun_out/r02_attn)"""
import csv, glob, os, sys
from collections import defaultdict

pre = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for i in (1, 2, 3):
    f = glob.glob(os.path.join(f"{pre}_p{i}", "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(float)
    meta = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = k[k.find("attn"):]
        k = k[:k.find("(")] if "(" in k else k[:40]
        key = (k, int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"])))
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        meta[r["Dispatch_Id"]] = (key, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    for (d, c), v in per.items():
        acc[meta[d][0]][c].append(v)
        if c in ("FETCH_SIZE", "SQ_BUSY_CYCLES"):
            acc[meta[d][0]]["dur"].append(meta[d][1])
print(f"{'kernel':28s} {'WGs':>6s} {'ms':>7s} {'GHz':>5s} {'MFMA%':>6s} {'LDSwait%':>8s} {'conf%':>6s} {'read GB':>8s} {'write GB':>8s} {'GB/s':>7s}")
for (k, g), c in sorted(acc.items()):
    m = lambda n: sum(c[n]) / len(c[n]) if c.get(n) else float("nan")
    dur = m("dur")
    clk = m("GRBM_GUI_ACTIVE") / 8 / dur / 1e9
    mf = m("SQ_VALU_MFMA_BUSY_CYCLES") / (m("GRBM_GUI_ACTIVE") / 8 * 1024) * 100
    lw = m("SQ_WAIT_INST_LDS") / m("SQ_WAVE_CYCLES") * 100
    cf = m("SQ_LDS_BANK_CONFLICT") / max(1.0, m("SQ_LDS_IDX_ACTIVE")) * 100
    rd, wr = 2 * 1024 * m("FETCH_SIZE") / 1e9, 1024 * m("WRITE_SIZE") / 1e9
    print(f"{k:28s} {g:6d} {dur * 1e3:7.3f} {clk:5.2f} {mf:6.1f} {lw:8.1f} {cf:6.1f} {rd:8.3f} {wr:8.3f} {(rd + wr) / dur:7.0f}")
