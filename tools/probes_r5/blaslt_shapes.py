"""torch.matmul (hipBLASLt) on the CLIP GEMM shapes, for rocprofv3 --kernel-trace: which kernel the
vendor library picks (its name encodes the macro tile, MFMA shape, waves and prefetch depth) and its
resources (VGPR / LDS / workgroup size), beside our own GEMM on the same shapes."""
import torch
R = 1024 * 197
shapes = [("sq8k", 8192, 8192, 8192), ("qkv", R, 2304, 768), ("fc2", R, 768, 3072), ("fc1", R, 3072, 768),
          ("out", R, 768, 768)]
for name, M, N, K in shapes:
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    for _ in range(3):
        c = a @ b.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        c = a @ b.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{name} M={M} N={N} K={K}: {ms*1e3:.1f} us {2*M*N*K/ms/1e9:.1f} TF/s", flush=True)
    del a, b, c
