"""MXFP8 tower GEMMs (BASELINE config 5) on ViT-L/14@336 shapes at B=512 (GPU): per shape the fp8
kernel's time and TF/s beside the bf16 production GEMM on the same shape, plus the producers that
write fp8 operands (quantiser, LayerNorm -> MXFP8).

    python tools/fp8_bench.py [B]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch  # noqa: E402
from clipmi import kernels as K, _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
R, D, F = B * 577, 1024, 4096
REPS = int(os.environ.get("FP8_REPS", "10"))
ONLY = os.environ.get("FP8_SHAPES", "").split(",") if os.environ.get("FP8_SHAPES") else None
# FP8_VARIANTS=0,40: the production dispatch (persistent 4-wave kernel where it applies) and the 8-wave kernel
VARIANTS = [int(v) for v in os.environ.get("FP8_VARIANTS", "0").split(",")]


def timeit(f, n=REPS):
    for _ in range(2):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def mx(r, c):
    return K.MX8(torch.empty(r, c, dtype=torch.uint8, device="cuda"), torch.empty(r, c // 32, dtype=torch.uint8,
                                                                                   device="cuda"))


torch.manual_seed(0)
_w = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for _ in range(100):  # clock warm-up
    _w @ _w
torch.cuda.synchronize()
del _w
if os.environ.get("FP8_KSWEEP"):  # time(K) = per-tile fixed cost + K/64 stages: split them (N = 3072, bias)
    for Kd in (128, 256, 512, 1024, 2048, 4096):
        x = (torch.randn(R, Kd, device="cuda") * 0.5).to(torch.bfloat16)
        w = (torch.randn(3 * D, Kd, device="cuda") * 0.02).to(torch.bfloat16)
        bias = torch.randn(3 * D, device="cuda").to(torch.bfloat16)
        A, Bq = K.quant_mxfp8(x), K.quant_mxfp8(w)
        C = torch.empty(R, 3 * D, device="cuda", dtype=torch.bfloat16)
        ms8 = timeit(lambda: K.gemm_fp8(R, 3 * D, Kd, A, Bq, C, 3 * D, bias=bias, flags=_lib.EPI_BIAS))
        msb = timeit(lambda: K.gemm(R, 3 * D, Kd, x, Kd, True, w, Kd, True, C, 3 * D, bias=bias, flags=_lib.EPI_BIAS))
        print(f"ksweep K={Kd:5d}: fp8 {ms8 * 1e3:8.1f} us  bf16 {msb * 1e3:8.1f} us", flush=True)
        del x, w, A, Bq, C
        torch.cuda.empty_cache()
    sys.exit(0)
QGB = _lib.EPI_BIAS | _lib.EPI_QGELU
for name, N, Kd, flags, q8o in (("qkv", 3 * D, D, _lib.EPI_BIAS, False),
                                ("out", D, D, _lib.EPI_BIAS | _lib.EPI_RESID, False),
                                ("fc1", F, D, QGB, False),
                                ("fc1_q8", F, D, QGB, True),
                                ("fc2", D, F, _lib.EPI_BIAS | _lib.EPI_RESID, False)):
    if ONLY and name not in ONLY:
        continue
    x = (torch.randn(R, Kd, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device="cuda") * 0.02).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda").to(torch.bfloat16)
    res = torch.randn(R, N, device="cuda").to(torch.bfloat16) if flags & _lib.EPI_RESID else None
    A, Bq = K.quant_mxfp8(x), K.quant_mxfp8(w)
    C = mx(R, N) if q8o else torch.empty(R, N, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * R * N * Kd
    line = f"{name:7s} M={R} N={N} K={Kd}:"
    for v in VARIANTS:
        f8 = lambda: K.gemm_fp8(R, N, Kd, A, Bq, C, N, bias=bias, residual=res, ldr=N, flags=flags, variant=v)
        ms8 = timeit(f8)
        line += f" fp8 v{v} {ms8 * 1e3:8.1f} us {fl / ms8 / 1e9:7.1f} TF/s |"
    if not q8o:
        Cb = torch.empty(R, N, device="cuda", dtype=torch.bfloat16)
        fb = lambda: K.gemm(R, N, Kd, x, Kd, True, w, Kd, True, Cb, N, bias=bias, residual=res, ldr=N, flags=flags)
        msb = timeit(fb)
        line += f" bf16 {msb * 1e3:8.1f} us {fl / msb / 1e9:7.1f} TF/s"
    print(line, flush=True)
    del x, w, A, Bq, C, res
    torch.cuda.empty_cache()

if ONLY:
    sys.exit(0)
x = torch.randn(R, D, device="cuda").to(torch.bfloat16)
wl = torch.ones(D, device="cuda", dtype=torch.bfloat16)
bl = torch.zeros(D, device="cuda", dtype=torch.bfloat16)
ms = timeit(lambda: K.quant_mxfp8(x))
print(f"quant_mxfp8 [{R}, {D}] bf16: {ms * 1e3:7.1f} us {R * D * (2 + 1 + 1 / 32) / ms / 1e6:7.1f} GB/s")
ms = timeit(lambda: K.layernorm_mxfp8(x, wl, bl))
print(f"layernorm_mxfp8 [{R}, {D}]: {ms * 1e3:7.1f} us {R * D * (2 + 1 + 1 / 32) / ms / 1e6:7.1f} GB/s")
