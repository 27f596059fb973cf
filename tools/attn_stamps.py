"""Where an item of the prefetching attention backward (attn_bwd_pf) spends its cycles (GPU; diagnostic build).

  make -C vlm-clip_amd alt NAME=attst EXTRA=-DCLIPMI_ATTN_STAMPS
  CLIPMI_LIB=vlm-clip_amd/clipmi/alt/libclipmi_attst.so python tools/attn_stamps.py [NW ...]
NW: CLIPMI_ATTN_BWD_NW values to compare (default 8 4), ViT-B/16 shape (B 1024, N 197, 12 heads).
Phases (medians over workgroups, waves and items >= 1, shader cycles):
  wait    0 -> 1  vmcnt(0) + barrier: Q / dO / O images of the item landed
  delta   1 -> 2  delta = rowsum(dO o O) + barrier + K / V DMA issue
  phaseA  2 -> 3  dK, dV
  waitkv  3 -> 4  vmcnt(0) + barrier: K / V images landed, every wave's phase A done
  prep    4 -> 5  next item's K / V fragments and meta loads, Q / dO fragments, barrier, Q / dO / O DMA issue
  phaseB  5 -> 6  dQ
  gap     6 -> next 0"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch  # noqa: E402

from clipmi import _lib, towers as T, kernels as K  # noqa: E402

_lib.declare("clipmi_gemm_stamps", [ctypes.c_void_p])
L = _lib.lib()
B, N, H = 1024, 197, 12
D = H * 64
qkv = torch.randn(B * N, 3 * D, device="cuda").to(torch.bfloat16)
o = torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda")
lse = torch.empty(B * H * N, device="cuda")
do = torch.randn(B * N, D, device="cuda").to(torch.bfloat16)
dqkv = torch.empty_like(qkv)
s = K.stream()
buf = torch.zeros(256 * 16 * 16 * 8, dtype=torch.int64, device="cuda")
w = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for _ in range(100):  # clock warm-up
    w @ w
del w
T.call("clipmi_attention_fwd", s, 1, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), None, 0, B, H, N, D)
names = ["wait", "delta", "phaseA", "waitkv", "prep", "phaseB"]
for nw in sys.argv[1:] or ["8", "4"]:
    os.environ["CLIPMI_ATTN_BWD_NW"] = nw
    bwd = lambda: T.call("clipmi_attention_bwd", s, 1, qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), do.data_ptr(),
                         dqkv.data_ptr(), None, 0, B, H, N, D)
    for _ in range(3):
        bwd()
    buf.zero_()
    L.clipmi_gemm_stamps(ctypes.c_void_p(buf.data_ptr()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    bwd()
    e1.record()
    torch.cuda.synchronize()
    L.clipmi_gemm_stamps(ctypes.c_void_p(0))
    st = buf.view(256, 16, 16, 8).cpu().numpy().astype(np.float64)
    nwv = int(nw) if nw in ("4", "16") else 8
    st = st[:, :nwv]
    valid = st[..., 6] > 0
    sel = valid.copy()
    sel[:, :, 0] = False
    q = lambda x: f"med {np.median(x):7.0f} p10 {np.percentile(x, 10):7.0f} p90 {np.percentile(x, 90):7.0f}"
    print(f"NW={nw}: {e0.elapsed_time(e1) * 1e3:.0f} us (stamped), items/WG ~{int(valid[0, 0].sum())}")
    for i, nm in enumerate(names):
        print(f"  {nm:7s} {q((st[..., i + 1] - st[..., i])[sel])}")
    gap = st[:, :, 1:, 0] - st[:, :, :-1, 6]
    gv = valid[:, :, 1:] & valid[:, :, :-1]
    print(f"  gap     {q(gap[gv])}")
    print(f"  item    {q((st[:, :, 1:, 0] - st[:, :, :-1, 0])[gv])}", flush=True)
