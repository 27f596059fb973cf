"""Pooled-row adapter forward + backward (GPU): the fused clipmi_adapter_fwd / _bwd against the
GEMM path AdapterFn takes on full hidden states, at the bench configs' per-GPU rows.
  python tools/adapter_bench.py [R ...]     (default 1024; D 512 / 768 / 1024, A 256, bf16)"""
import os
import sys
import types

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch  # noqa: E402

from clipmi import synth, towers as T  # noqa: E402
from clipmi.modules import AdapterParams  # noqa: E402


def timed(f, n=50):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for R in [int(a) for a in sys.argv[1:]] or [1024]:
    for D in (512, 768, 1024):
        mod = AdapterParams(D, 256, "cuda", ln=True, shadow=True)
        mod.load_numpy(synth.adapter_state_dict(D, 256, 7, "text_adapter"))
        rt = types.SimpleNamespace(dtype=torch.bfloat16)
        anchor = next(iter(mod.parameters()))
        x = torch.randn(R, 1, D, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
        gy = torch.randn(R, 1, D, device="cuda", dtype=torch.bfloat16)
        res = {}
        for name, cap in (("fused", 4096), ("gemm", 0)):
            T.AdapterFn.FUSED_MAX_ROWS = cap
            fwd = lambda: T.AdapterFn.apply(x.detach(), anchor, rt, mod, False)
            def fb():
                y = T.AdapterFn.apply(x, anchor, rt, mod, True)
                y.backward(gy)
            res[name] = (timed(fwd), timed(fb))
        print(f"R={R} D={D} A=256: fused fwd {res['fused'][0]:6.1f} us fwd+bwd {res['fused'][1]:6.1f} us | "
              f"gemm path fwd {res['gemm'][0]:6.1f} us fwd+bwd {res['gemm'][1]:6.1f} us", flush=True)
