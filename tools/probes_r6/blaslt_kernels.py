"""Which hipBLASLt kernels torch.matmul picks for the square 8192^3 product and config 3's K = 768 / 3072 shapes
(bf16, the layouts the towers use), timed with CUDA events.  Run under rocprofv3 --kernel-trace to read each
kernel's name (macro tile, MFMA, wave grouping) and its VGPR / AGPR / LDS use from the trace CSV."""
import torch

dev = torch.device("cuda", 0)
shapes = {"sq8k": (8192, 8192, 8192), "qkv_fwd": (201728, 2304, 768), "fc1_dgrad": (201728, 768, 3072),
          "out_fwd": (201728, 768, 768)}
for name, (M, N, K) in shapes.items():
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ w.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        c = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{name:10s} M={M} N={N} K={K}: {ms * 1e3:8.1f} us  {2 * M * N * K / ms / 1e9:7.1f} TF/s", flush=True)
    del a, w, c
