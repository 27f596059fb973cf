"""AdamW kernel throughput (GPU): the 4-per-lane path (16-B-aligned arenas) vs the scalar path
(4-B offset), n = the ViT-B/16 full-fine-tune arena size; bytes = 28 B/param + 2 B shadow."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch
from clipmi import kernels as K, towers as T

n = 149_620_737
bufs = [torch.rand(n + 4, device="cuda") for _ in range(4)]
sh = torch.empty(n + 4, dtype=torch.bfloat16, device="cuda")
s = K.stream()
for rep in range(3):
    for off in (0, 1):
        p, g, m, v = (b[off:off + n] for b in bufs)
        f = lambda: T.call("clipmi_adamw", s, p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
                           sh[off:].data_ptr(), n, 1e-5, 0.9, 0.999, 1e-8, 0.01, 3, None)
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(f"adamw {'vec4' if off == 0 else 'scalar'}: {ms * 1e3:8.1f} us {n * 30 / ms / 1e6:7.0f} GB/s", flush=True)
