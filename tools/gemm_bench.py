"""Per-shape GEMM throughput of libclipmi on the ViT-B/16 B=1024 training shapes (GPU)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch
from clipmi import kernels as K, _lib

R = 1024 * 197
SHAPES = [  # name, M, N, K, a_kmajor, b_kmajor, out dtype, flags, split
    ("fc1_fwd", R, 3072, 768, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_QGELU | _lib.EPI_STORE_PRE, 1),
    ("fc2_fwd", R, 768, 3072, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    ("qkv_fwd", R, 2304, 768, True, True, torch.bfloat16, _lib.EPI_BIAS, 1),
    ("out_fwd", R, 768, 768, True, True, torch.bfloat16, _lib.EPI_BIAS | _lib.EPI_RESID, 1),
    ("fc2_dgrad", R, 3072, 768, True, False, torch.bfloat16, _lib.EPI_DQGELU, 1),
    ("fc1_dgrad", R, 768, 3072, True, False, torch.bfloat16, 0, 1),
    ("qkv_dgrad", R, 768, 2304, True, False, torch.bfloat16, 0, 1),
    ("fc1_wgrad", 3072, 768, R, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("fc2_wgrad", 768, 3072, R, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("qkv_wgrad", 2304, 768, R, False, False, torch.float32, _lib.EPI_BETA, 2),
    ("out_wgrad", 768, 768, R, False, False, torch.float32, _lib.EPI_BETA, 8),
    # reference points (not on the CLIP path): square, operands resident in MALL
    ("sq4k", 4096, 4096, 4096, True, True, torch.bfloat16, 0, 1),
    ("sq8k", 8192, 8192, 8192, True, True, torch.bfloat16, 0, 1),
    ("fc2_fwd_l2", 16384, 768, 3072, True, True, torch.bfloat16, 0, 1),
]
VARIANTS = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0,1").split(",")]
only = sys.argv[1:] if len(sys.argv) > 1 else None
torch.manual_seed(0)
for name, M, N, Kd, akm, bkm, odt, flags, split in SHAPES:
    if (only and name not in only) or (not only and name in ("sq4k", "sq8k", "fc2_fwd_l2")):
        continue
    A = torch.randn(M * Kd, device="cuda").to(torch.bfloat16)
    B = torch.randn(N * Kd, device="cuda").to(torch.bfloat16)
    lda = Kd if akm else M
    ldb = Kd if bkm else N
    C = torch.zeros(M, N, device="cuda", dtype=odt)
    bias = torch.randn(N, device="cuda").to(torch.bfloat16)
    aux = torch.randn(M, N, device="cuda").to(odt) if flags & (_lib.EPI_DQGELU | _lib.EPI_STORE_PRE) else None
    res = torch.randn(M, N, device="cuda").to(odt) if flags & _lib.EPI_RESID else None
    if split == 2:  # engine's choice for 256 tiles
        tiles = ((M + 255) // 256) * ((N + 255) // 256)
        split = max(1, min(32, 512 // tiles))
    ws = torch.empty(split * M * N, device="cuda") if split > 1 else None
    bg = torch.zeros(M, device="cuda") if odt == torch.float32 else None
    kw = dict(bias=bias if flags & _lib.EPI_BIAS else None, residual=res, ldr=N, aux=aux, ldaux=N, flags=flags,
              split_k=split, workspace=ws, bias_grad=bg)
    if os.environ.get("GEMM_TORCH"):  # hipBLASLt via torch.matmul, plain product, for comparison
        a2 = A.view(M, Kd) if akm else A.view(Kd, M).t()
        b2 = B.view(N, Kd).t() if bkm else B.view(Kd, N)
        g = lambda: torch.matmul(a2, b2)
        for _ in range(3):
            g()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            g()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{name:10s} torch M={M} N={N} K={Kd}: {ms * 1e3:8.1f} us {2 * M * N * Kd / ms / 1e9:7.1f} TF/s", flush=True)
    for small in VARIANTS:  # 0 = production schedule, 1 = 128 tile, 2 = up-front DMA issue
        if small == 1 and bg is not None:
            kw2 = dict(kw, bias_grad=None)
        else:
            kw2 = kw
        f = lambda: K.gemm(M, N, Kd, A, lda, akm, B, ldb, bkm, C, N, small_tile=small, **kw2)
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        n = 10
        for _ in range(n):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        print(f"{name:10s} v{small} M={M} N={N} K={Kd} split={split}: {ms * 1e3:8.1f} us "
              f"{2 * M * N * Kd / ms / 1e9:7.1f} TF/s", flush=True)
