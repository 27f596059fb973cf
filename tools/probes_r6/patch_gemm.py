"""Config 5's patch-embedding product (ViT-L/14@336, B = 4096: M = 4096 x 577 rows, N = 1024, K = 588 padded to
640, bf16, both operands k-major, no epilogue) against neighbouring shapes, to locate its slowness in the step."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "vlm-clip_amd"))
import torch
from clipmi import kernels as K


def timeit(f, n=5):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for M, N, Kd in ((4096 * 577, 1024, 640), (4096 * 577, 1024, 768), (4096 * 577, 1024, 1024), (1024 * 577, 1024, 640),
                 (1024 * 197, 768, 768)):
    A = (torch.randn(M, Kd, device="cuda") * 0.1).to(torch.bfloat16)
    W = (torch.randn(N, Kd, device="cuda") * 0.1).to(torch.bfloat16)
    C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    ms = timeit(lambda: K.gemm(M, N, Kd, A, Kd, True, W, Kd, True, C, N))
    mt = timeit(lambda: torch.matmul(A, W.t()))
    print(f"M={M:8d} N={N} K={Kd}: clipmi {ms * 1e3:8.1f} us ({2 * M * N * Kd / ms / 1e9:6.0f} TF/s)   "
          f"torch {mt * 1e3:8.1f} us", flush=True)
    del A, W, C
