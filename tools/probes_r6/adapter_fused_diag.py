"""Phase timing of the fused adapter forward (CLIPMI_ADAPTER_FUSED_DIAG bits: 1 no down MFMA loop, 2 no up loop,
4 no LayerNorm; outputs then wrong -- timing only), R = 1024, D = 768, A = 256."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "vlm-clip_amd"))
import torch
from clipmi import kernels as K, towers as T
from clipmi._lib import BF16
s = K.stream()
R, D, A = 1024, 768, 256
mk = lambda *sh: (torch.randn(*sh, device="cuda") * 0.05).to(torch.bfloat16)
ws = [mk(A, D), mk(A), mk(D, A), mk(D), mk(D) + 1, mk(D)]
x = mk(R, D)
y, z = (torch.empty(R, D, dtype=torch.bfloat16, device="cuda") for _ in range(2))
pre, act = (torch.empty(R, A, dtype=torch.bfloat16, device="cuda") for _ in range(2))
st = torch.empty(2, R, device="cuda")
f = lambda: T.call("clipmi_adapter_fwd", s, BF16, R, D, A, x.data_ptr(), D, *(w.data_ptr() for w in ws), 1e-5, 1,
                   y.data_ptr(), D, pre.data_ptr(), act.data_ptr(), z.data_ptr(), st[0].data_ptr(), st[1].data_ptr())
for d in (0, 1, 2, 4, 7, 0):
    os.environ["CLIPMI_ADAPTER_FUSED_DIAG"] = str(d)
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        f()
    e1.record()
    torch.cuda.synchronize()
    print(f"diag {d}: {e0.elapsed_time(e1) / 200 * 1e3:6.1f} us", flush=True)
