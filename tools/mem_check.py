"""Diagnostic: peak memory per training step must not grow (graph leak check)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from clipmi import CLIPWithAdapters, config as C
from clipmi.trainer import FusedAdamW
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
m = CLIPWithAdapters("B/16", use_text_adapter=False, use_vision_adapter=False, use_shared_adapters=False,
                     freeze_clip=False, device="cuda", fast_init=True)
opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=5e-5, arenas=m.arenas())
b = bench.synthetic_batch(C.resolve("B/16"), B, 0, torch.device("cuda"))
for i in range(4):
    out = m(**b); loss = out["loss"]; opt.zero_grad(); loss.backward(); opt.clip_grad_norm(1.0); opt.step()
    torch.cuda.synchronize()
    print(i, "alloc GB", torch.cuda.memory_allocated() / 1e9, "peak GB", torch.cuda.max_memory_allocated() / 1e9, flush=True)
