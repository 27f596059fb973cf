"""Where an item of the persistent 4-wave GEMM spends its cycles (GPU; diagnostic build).

Needs the stamped library: make -C vlm-clip_amd alt NAME=w4pst EXTRA=-DCLIPMI_W4P_STAMPS, then
  CLIPMI_LIB=vlm-clip_amd/clipmi/alt/libclipmi_w4pst.so python tools/w4p_stamps.py qkv_fwd [fc1_fwd_dact ...]
Per workgroup < 256, wave and item < 20 the kernel stamps s_memtime at the item's top (0), after its
start sync (1), after its main loop (2), after the next item's prologue DMAs (3) and after its
epilogue (4).  Printed in shader cycles (medians over workgroups, waves and items >= 1):
  sync      0 -> 1  (waiting for the prologue stages and the other waves)
  loop      1 -> 2  (all k-steps)
  prologue  2 -> 3  (issuing the next item's first two stages)
  epilogue  3 -> 4
  gap       4 -> next 0
and the in-kernel clock (s_memtime / s_memrealtime over the kernel)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch  # noqa: E402

from clipmi import _lib, kernels as K  # noqa: E402

R = 1024 * 197
SH = {"qkv_fwd": (R, 2304, 768, True, _lib.EPI_BIAS), "out_fwd": (R, 768, 768, True, _lib.EPI_BIAS | _lib.EPI_RESID),
      "fc2_fwd": (R, 768, 3072, True, _lib.EPI_BIAS | _lib.EPI_RESID),
      "fc1_fwd_dact": (R, 3072, 768, True, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_DACT),
      "fc1_fwd_bias": (R, 3072, 768, True, _lib.EPI_BIAS),
      "fc2_dgrad_ma": (R, 3072, 768, False, _lib.EPI_MUL_AUX), "fc1_dgrad": (R, 768, 3072, False, 0),
      "out_dgrad": (R, 768, 768, False, 0), "qkv_k64": (R, 2304, 64, True, _lib.EPI_BIAS),
      "qkv_noepi": (R, 2304, 768, True, 0)}
VAR = int(os.environ.get("W4P_VAR", "28"))
# diagnostic: a shape name suffixed ":a", ":b" or ":ab" runs with lda / ldb = 0 (every row of that
# operand aliases one 128-B line: its DMAs hit the CU's own cache), to separate the memory side of
# the main loop from the LDS-DMA / issue side.  Results are then meaningless, times are not.
_lib.declare("clipmi_gemm_stamps", [ctypes.c_void_p])
L = _lib.lib()
buf = torch.zeros(256 * 4 * 128, dtype=torch.int64, device="cuda")
w = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for _ in range(100):  # clock warm-up
    w @ w
torch.cuda.synchronize()
del w
for arg in sys.argv[1:] or ["qkv_fwd"]:
    name, _, alias = arg.partition(":")
    M, N, Kd, bkm, flags = SH[name]
    A = (torch.rand(M * Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N * Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(N, device="cuda").to(torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    res = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    kw = dict(bias=bias, residual=res, ldr=N, aux=aux, ldaux=N, flags=flags)
    lda = 0 if "a" in alias else Kd
    ldb = 0 if "b" in alias else (Kd if bkm else N)
    f = lambda: K.gemm(M, N, Kd, A, lda, True, B, ldb, bkm, C, N, small_tile=VAR, **kw)
    for _ in range(5):
        f()
    buf.zero_()
    L.clipmi_gemm_stamps(ctypes.c_void_p(buf.data_ptr()))
    f()
    torch.cuda.synchronize()
    L.clipmi_gemm_stamps(ctypes.c_void_p(0))
    s = buf.view(256, 4, 128).cpu().numpy().astype(np.float64)
    it = s[:, :, :120].reshape(256, 4, 20, 6)
    valid = it[:, :, :, 4] > 0
    n_it = int(valid[0, 0].sum())
    ph = {"sync": it[..., 1] - it[..., 0], "loop": it[..., 2] - it[..., 1], "prologue": it[..., 3] - it[..., 2],
          "epilogue": it[..., 4] - it[..., 3]}
    gap = it[:, :, 1:, 0] - it[:, :, :-1, 4]
    gvalid = valid[:, :, 1:] & valid[:, :, :-1]
    ok = s[:, :, 127] > s[:, :, 126]
    clk = ((s[:, :, 124] - s[:, :, 125]) / np.maximum(1, (s[:, :, 127] - s[:, :, 126]) * 10.0))[ok]  # GHz (100 MHz)
    q = lambda x: f"med {np.median(x):7.0f} p10 {np.percentile(x, 10):7.0f} p90 {np.percentile(x, 90):7.0f}"
    steps = (Kd + 63) // 64
    print(f"{arg} var {VAR}: M={M} N={N} K={Kd} steps={steps} items/WG~{n_it} clock {np.median(clk):.2f} GHz")
    sel = valid.copy()
    sel[:, :, 0] = False  # item 0 waits for the kernel-start prologue
    for k, x in ph.items():
        extra = f"  per step {np.median(x[sel]) / steps:6.0f}" if k == "loop" else ""
        print(f"  {k:9s} {q(x[sel])}{extra}")
    print(f"  gap       {q(gap[gvalid])}")
    tot = np.median((it[..., 4] - it[..., 0])[sel]) + np.median(gap[gvalid])
    print(f"  item total ~{tot:7.0f} cycles; ideal MFMA {steps * 2048}", flush=True)
    del A, B, C, aux, res
    torch.cuda.empty_cache()
