"""LayerNorm throughput (GPU): the in-tree library against an alternative build given as argv[1], interleaved
in one process.  Forward (clipmi_layernorm_fwd2) and backward (clipmi_layernorm_bwd2, with the residual
gradient and the affine-gradient partials) at the CLIP widths, with x in bf16 or fp32 (the bf16 mode's fp32
residual stream) and y / dy / dx / dres in bf16.  GB/s counts x, y (fwd) / dy, x, dres, dx (bwd) once."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch
from clipmi import _lib, kernels as K

libs = {"new": ctypes.CDLL(_lib.lib()._name, mode=os.RTLD_LOCAL)}
if len(sys.argv) > 1:
    libs["alt"] = ctypes.CDLL(os.path.abspath(sys.argv[1]), mode=os.RTLD_LOCAL)
vp, i64, i32, f = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
for L in libs.values():
    L.clipmi_layernorm_bwd2.argtypes = [vp, i32, i32, vp, i64, vp, i64, vp, vp, vp, vp, i64, vp, i64, vp, vp, i32, vp,
                                        i64, i32, i32]
    L.clipmi_layernorm_fwd2.argtypes = [vp, i32, i32, vp, i64, vp, i64, vp, vp, vp, vp, i32, i32, f, vp, vp, i32]
    L.clipmi_layernorm_bwd_ws.restype = ctypes.c_int64
s = K.stream()


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 10


for R, D in ((1024 * 197, 768), (1024 * 77, 512)):
    for xdt in (torch.float32, torch.bfloat16):
        xs = 4 if xdt == torch.float32 else 2
        xc = _lib.F32 if xdt == torch.float32 else _lib.BF16
        t = lambda dt=torch.bfloat16: torch.randn(R, D, device="cuda").to(dt)
        dy, x, dres, dx = t(), t(xdt), t(), t()
        mean, rstd = torch.zeros(R, device="cuda"), torch.ones(R, device="cuda")
        w = torch.ones(D, device="cuda").to(torch.bfloat16)
        bvec = torch.zeros(D, device="cuda").to(torch.bfloat16)
        dw, db = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
        ws = torch.empty(int(libs["new"].clipmi_layernorm_bwd_ws(R, D)), dtype=torch.uint8, device="cuda")
        for rep in range(3):
            for name, L in libs.items():
                fb = lambda: L.clipmi_layernorm_bwd2(s, xc, _lib.BF16, dy.data_ptr(), D, x.data_ptr(), D, mean.data_ptr(),
                                                     rstd.data_ptr(), w.data_ptr(), dx.data_ptr(), D, dres.data_ptr(), D,
                                                     dw.data_ptr(), db.data_ptr(), 0, ws.data_ptr(), ws.numel(), R, D)
                ff = lambda: L.clipmi_layernorm_fwd2(s, xc, _lib.BF16, x.data_ptr(), D, dx.data_ptr(), D, w.data_ptr(),
                                                     bvec.data_ptr(), mean.data_ptr(), rstd.data_ptr(), R, D, 1e-5,
                                                     None, None, 0)
                mb, mf = timed(fb), timed(ff)
                nb, nf = R * D * (3 * 2 + xs), R * D * (2 + xs)
                print(f"ln {name} R={R} D={D} x={str(xdt)[6:]}: bwd {mb * 1e3:7.1f} us {nb / mb / 1e6:6.0f} GB/s | "
                      f"fwd {mf * 1e3:7.1f} us {nf / mf / 1e6:6.0f} GB/s", flush=True)
