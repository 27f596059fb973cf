"""Cross-check bench.py's live roofline timing against a rocprofv3 kernel trace of the same
command: mean duration of each GEMM family's launches on the caller's stream (the stream the
vision attention kernel runs on; the text tower has its own).  Usage: roofline_check.py TRACE.csv"""
import csv, sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
main = None
for r in rows:
    if "attn_fwd_pf<14" in r["Kernel_Name"]:
        main = r["Stream_Id"]
        break
# r03: the persistent 4-wave kernel carries the weight gradients and the K >= 1536 forward/dgrad
# products (plus fc2's input gradient), demangled or mangled names
FAMILIES = {"gemm256_wgrad": ("gemm256_kernel<false, false, float, 0,", "gemm256_kernelILb0ELb0EfLi0E",
                              "gemm_w4p_kernel<false, false, float", "gemm_w4p_kernelILb0ELb0Ef"),
            "gemm256_fwd_dgrad": ("gemm_pp_kernel", "gemm_w4p_kernel<true", "gemm_w4p_kernelILb1")}
for fam, pats in FAMILIES.items():
    dur = defaultdict(list)
    for r in rows:
        if any(p in r["Kernel_Name"] for p in pats):
            dur[r["Stream_Id"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for sid, d in dur.items():
        tag = "caller's stream (timed live)" if sid == main else "side stream"
        print(f"{fam} stream {sid} [{tag}]: {len(d)} launches, mean {sum(d) / len(d):.4f} ms")
