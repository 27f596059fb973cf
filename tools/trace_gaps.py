"""Where the step's wall time goes, from a rocprofv3 --kernel-trace of bench.py: per step (steps
delimited by the fused AdamW launch), the GPU-busy union over all streams, the time both
streams run kernels at once, and the idle gaps (no kernel on any stream) with the kernels on
either side of the largest ones (host stalls, launch latency, syncs).
Usage: trace_gaps.py KERNEL_TRACE.csv [top_gaps]"""
import csv, sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return n[:70]


rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows))
ends = [e for s, e, sid, n in ev if "adamw_kernel" in n]
if len(ends) < 2:
    sys.exit("need at least two AdamW launches (steps) in the trace")
for a, b in zip(ends[:-1], ends[1:]):
    win = [(max(s, a), min(e, b), sid, n) for s, e, sid, n in ev if e > a and s < b]
    busy, cur_s, cur_e, cur_n = 0, None, None, None
    gaps = []
    for s, e, sid, n in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, cur_n, n))
            cur_s, cur_e, cur_n = s, e, n
        elif e > cur_e:
            cur_e, cur_n = e, n
    busy += cur_e - cur_s
    span = b - a
    per = defaultdict(int)
    for s, e, sid, n in win:
        per[sid] += e - s
    # time with >= 2 kernels running (sweep)
    pts = sorted([(s, 1) for s, e, _, _ in win] + [(e, -1) for s, e, _, _ in win])
    level, t0, both = 0, a, 0
    for t, d in pts:
        if level >= 2:
            both += t - t0
        level += d
        t0 = t
    idle = span - busy
    print(f"step {a / 1e6:.1f}..{b / 1e6:.1f} ms: span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f}, idle {idle / 1e6:.2f} "
          f"({100 * idle / span:.1f} %), >=2 kernels {both / 1e6:.2f} ms, kernel-time per stream "
          + ", ".join(f"{k}: {v / 1e6:.1f}" for k, v in sorted(per.items())))
    big = sorted(gaps, reverse=True)[:top]
    hist = defaultdict(lambda: [0, 0])
    for g, _, _ in gaps:
        k = "<5us" if g < 5e3 else "5-20us" if g < 2e4 else "20-100us" if g < 1e5 else ">=100us"
        hist[k][0] += 1
        hist[k][1] += g
    print("   gaps: " + ", ".join(f"{k} n={v[0]} sum={v[1] / 1e6:.2f} ms" for k, v in sorted(hist.items())))
    for g, p, n in big:
        print(f"   gap {g / 1e3:8.1f} us  after {short(p or '?')}  before {short(n)}")
