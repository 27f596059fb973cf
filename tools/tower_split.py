"""Per-tower split of the 4-wave weight-gradient GEMM launches in a serial-tower trace (CLIPMI_OVERLAP=0, one
stream): the vision tower's launches (R = B * 197 tokens, D = 768; as many per step as the overlapped trace's
vision stream has) are the longest ones, the text tower's (R = B * 77, D = 512) the rest; compared with the
overlapped trace's per-stream totals.  Usage: tower_split.py SERIAL.csv OVERLAP.csv STEPS"""
import csv
import sys


def wgrad(f):
    rows = list(csv.DictReader(open(f)))
    return [(r["Stream_Id"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows
            if "gemm_w4p_kernel<false, false" in r["Kernel_Name"]]


steps = float(sys.argv[3])
ser = sorted((d for _, d in wgrad(sys.argv[1])), reverse=True)
ov = wgrad(sys.argv[2])
nvis = sum(1 for s_, _ in ov if s_ == "0")  # stream 0 = the caller's (vision) stream
vis, txt = ser[:nvis], ser[nvis:]
print(f"serial towers ({sys.argv[1]}): vision wgrad {len(vis) / steps:.0f} launches/step, {sum(vis) / steps / 1e3:.2f} ms/step "
      f"(mean {sum(vis) / max(1, len(vis)):.0f} us); text {len(txt) / steps:.0f}/step, {sum(txt) / steps / 1e3:.2f} ms/step")
for sid in sorted({s for s, _ in ov}):
    v = [d for s, d in ov if s == sid]
    print(f"overlapped ({sys.argv[2]}) stream {sid}: {len(v) / steps:.0f} launches/step, {sum(v) / steps / 1e3:.2f} ms/step "
          f"(mean {sum(v) / len(v):.0f} us)")
