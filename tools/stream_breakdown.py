"""Per-stream time breakdown of a bench.py rocprofv3 --kernel-trace: for the caller's stream (the
one the vision attention runs on) and the side stream, kernel time per step by family, and the
caller stream's busy fraction.  Usage: stream_breakdown.py kernel_trace.csv STEPS"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
main = next(r["Stream_Id"] for r in rows if re.search(r"attn_fwd_(pf|x3)(<|ILi)14", r["Kernel_Name"]))
FAM = [("gemm fwd/dgrad 8-wave", r"gemm_pp_kernel"), ("gemm 4-wave persistent (fwd/dgrad)", r"gemm_w4p_kernel(ILb1|<true)"),
       ("gemm 4-wave persistent (wgrad)", r"gemm_w4p_kernel(ILb0|<false)"), ("gemm wgrad 8-wave", r"gemm256_kernel"),
       ("split-K reduce", r"splitk_reduce"), ("bf16x3 split", r"split3"), ("attention fwd", r"attn_fwd"), ("attention bwd", r"attn_bwd"),
       ("layernorm fwd", r"ln_fwd"), ("layernorm bwd", r"ln_bwd"), ("LN affine-grad reduce", r"reduce_partials"),
       ("adamw / norm", r"adamw|sumsq|grad_norm"), ("embeddings / im2col / pooling", r"im2col|text_embed|id_|period_sum|pool|scatter|gather"),
       ("contrastive", r"ce_|l2norm|gemm_f32|sum2"), ("torch / copies", r"at::native|rocclr")]
for sid in sorted({r["Stream_Id"] for r in rows}):
    rs = [r for r in rows if r["Stream_Id"] == sid]
    if len(rs) < 20:
        continue
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in rs:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        f = next((n for n, p in FAM if re.search(p, r["Kernel_Name"])), "other: " + r["Kernel_Name"][:40])
        tot[f] += d
        cnt[f] += 1
    t0 = min(int(r["Start_Timestamp"]) for r in rs)
    t1 = max(int(r["End_Timestamp"]) for r in rs)
    busy = sum(tot.values())
    tag = "caller (vision)" if sid == main else "side"
    print(f"== stream {sid} [{tag}]: {busy / steps:.1f} ms kernel time per step, span {(t1 - t0) / 1e6 / steps:.1f} ms/step")
    for f, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"  {v / steps:8.2f} ms/step  {cnt[f] / steps:6.1f} launches  {f}")
