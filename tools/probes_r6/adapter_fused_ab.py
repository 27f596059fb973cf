"""clipmi_adapter_fwd (bf16, with the LayerNorm): the fused one-kernel forward (adapter_fused.hip) vs the launch
sequence (CLIPMI_ADAPTER_FUSED=0), alternating in one process, at the pooled-row sizes (R = per-GPU batch)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "vlm-clip_amd"))
import torch
from clipmi import kernels as K, towers as T
from clipmi._lib import BF16


def timed(f, n=200):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


s = K.stream()
for R in (256, 1024, 4096):
    for D in (512, 768, 1024):
        A = 256
        mk = lambda *sh: (torch.randn(*sh, device="cuda") * 0.05).to(torch.bfloat16)
        ws = [mk(A, D), mk(A), mk(D, A), mk(D), mk(D) + 1, mk(D)]
        x = mk(R, D)
        y, z = (torch.empty(R, D, dtype=torch.bfloat16, device="cuda") for _ in range(2))
        pre, act = (torch.empty(R, A, dtype=torch.bfloat16, device="cuda") for _ in range(2))
        st = torch.empty(2, R, device="cuda")
        f = lambda: T.call("clipmi_adapter_fwd", s, BF16, R, D, A, x.data_ptr(), D, *(w.data_ptr() for w in ws), 1e-5,
                           1, y.data_ptr(), D, pre.data_ptr(), act.data_ptr(), z.data_ptr(), st[0].data_ptr(),
                           st[1].data_ptr())
        res = {}
        for rep in range(2):
            for fz in ("1", "0"):
                os.environ["CLIPMI_ADAPTER_FUSED"] = fz
                res.setdefault(fz, []).append(timed(f))
        print(f"R={R:5d} D={D:5d} A={A}: fused {min(res['1']):6.1f} us   sequence {min(res['0']):6.1f} us", flush=True)
