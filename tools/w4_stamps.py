"""Where a 4-wave GEMM k-step spends its cycles (GPU; diagnostic build variant 22 of gemm4.hip).

Runs one CLIP shape with in-kernel s_memtime stamps (workgroups < 512, every wave) and prints,
in shader cycles: prologue (kernel start -> main loop), per k-step compute (barrier exit ->
next barrier entry: half-step 1 + half-step 0 = 128 MFMAs, ideal 2048), per-step barrier wait
(entry -> exit: the vmcnt wait for the next stage's DMAs + the wait for the other waves),
epilogue (main loop end -> kernel end) and the in-kernel clock (s_memtime / s_memrealtime).
  python tools/w4_stamps.py fc1_dgrad [qkv_fwd ...]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import ctypes
import torch
from clipmi import kernels as K, _lib

R = 1024 * 197
SH = {"fc1_fwd": (R, 3072, 768, True, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_PRE),
      "fc2_fwd": (R, 768, 3072, True, _lib.EPI_BIAS | _lib.EPI_RESID),
      "qkv_fwd": (R, 2304, 768, True, _lib.EPI_BIAS), "out_fwd": (R, 768, 768, True, _lib.EPI_BIAS | _lib.EPI_RESID),
      "fc2_dgrad": (R, 3072, 768, False, _lib.EPI_DQGELU), "fc1_dgrad": (R, 768, 3072, False, 0),
      "sq8k": (8192, 8192, 8192, True, 0),
      # few-tile shapes (~60 workgroups = ~60 storing CUs): the epilogue's per-CU rate when the chip's
      # write bandwidth is not shared by all 256 CUs
      "qkv_fwd_60": (7 * 256, 2304, 768, True, _lib.EPI_BIAS),
      "fc1_fwd_60": (5 * 256, 3072, 768, True, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_PRE),
      # fc1's epilogue without the pre-activation store / without the gelu as well
      "fc1_fwd_nopre": (R, 3072, 768, True, _lib.EPI_BIAS | _lib.EPI_QGELU),
      "fc1_fwd_bias": (R, 3072, 768, True, _lib.EPI_BIAS),
      "fc2_dgrad": (R, 3072, 768, False, _lib.EPI_DQGELU), "fc2_dgrad_plain": (R, 3072, 768, False, 0),
      "fc1_fwd_dact": (R, 3072, 768, True, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_DACT),
      "fc2_dgrad_ma": (R, 3072, 768, False, _lib.EPI_MUL_AUX)}
_lib.declare("clipmi_gemm_stamps", [ctypes.c_void_p])
L = _lib.lib()
buf = torch.zeros(512 * 4 * 128, dtype=torch.int64, device="cuda")
for name in sys.argv[1:] or ["fc1_dgrad"]:
    M, N, Kd, bkm, flags = SH[name]
    A = (torch.rand(M * Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N * Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(N, device="cuda").to(torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    res = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    kw = dict(bias=bias, residual=res, ldr=N, aux=aux, ldaux=N, flags=flags)
    f = lambda v: K.gemm(M, N, Kd, A, Kd, True, B, Kd if bkm else N, bkm, C, N, small_tile=v, **kw)
    for _ in range(3):
        f(20)
    vs = ((22, "production"), (23, "no main-loop DMAs"), (24, "no fragment reads"), (25, "MFMAs only"))
    if os.environ.get("W4_ST_PROD_ONLY"):
        vs = vs[:1]
    for var, what in vs:
        L.clipmi_gemm_stamps(ctypes.c_void_p(buf.data_ptr()))
        f(var)
        torch.cuda.synchronize()
        L.clipmi_gemm_stamps(ctypes.c_void_p(0))
        s = buf.view(512, 4, 128).cpu().numpy().astype(np.float64)
        ns = min(58, (Kd + 63) // 64)
        nblk = min(512, ((M + 255) // 256) * ((N + 255) // 256))
        s = s[:nblk]
        pro = s[:, :, 1] - s[:, :, 0]
        epi = s[:, :, 3] - s[:, :, 2]
        loop = s[:, :, 2] - s[:, :, 1]
        clk = (s[:, :, 3] - s[:, :, 0]) / np.maximum(1, s[:, :, 127] - s[:, :, 126]) * 0.1  # GHz
        wait = s[:, :, 5:4 + 2 * ns:2] - s[:, :, 4:4 + 2 * ns:2]          # barrier entry -> exit
        comp = s[:, :, 4 + 2:4 + 2 * ns:2] - s[:, :, 5:4 + 2 * ns - 2:2]  # exit(s) -> entry(s+1)
        q = lambda x: f"med {np.median(x):7.0f} p10 {np.percentile(x, 10):7.0f} p90 {np.percentile(x, 90):7.0f}"
        print(f"{name} [{what}]: M={M} N={N} K={Kd} steps={ns} blocks={nblk} clock {np.median(clk):.2f} GHz")
        print(f"  prologue  {q(pro)}")
        print(f"  step comp {q(comp)}   (128 MFMAs: 2048 ideal)")
        print(f"  step wait {q(wait)}")
        print(f"  loop      {q(loop)}  per step {np.median(loop) / ((Kd + 63) // 64):.0f}")
        print(f"  epilogue  {q(epi)}", flush=True)
    del A, B, C, aux, res
    torch.cuda.empty_cache()
