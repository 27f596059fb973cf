"""LayerNorm backward throughput (GPU), the in-tree library against an alternative build given as
argv[1] (e.g. the previous kernel), interleaved in one process; bytes = dy, x, dres read + dx
written (4 * R * D * 2 B)."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlm-clip_amd"))
import torch
from clipmi import _lib, kernels as K

libs = {"new": ctypes.CDLL(_lib.lib()._name, mode=os.RTLD_LOCAL)}
if len(sys.argv) > 1:
    libs["old"] = ctypes.CDLL(os.path.abspath(sys.argv[1]), mode=os.RTLD_LOCAL)
vp, i64, i32, f = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
for L in libs.values():
    L.clipmi_layernorm_bwd.argtypes = [vp, i32, vp, i64, vp, i64, vp, vp, vp, vp, i64, vp, i64, vp, vp, i32, vp, i64,
                                       i32, i32]
    L.clipmi_layernorm_bwd_ws.restype = ctypes.c_int64
s = K.stream()
for R, D in ((1024 * 197, 768), (1024 * 77, 512)):
    t = lambda: torch.randn(R, D, device="cuda").to(torch.bfloat16)
    dy, x, dres, dx = t(), t(), t(), t()
    mean, rstd = torch.zeros(R, device="cuda"), torch.ones(R, device="cuda")
    w = torch.ones(D, device="cuda").to(torch.bfloat16)
    dw, db = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    ws = torch.empty(int(libs["new"].clipmi_layernorm_bwd_ws(R, D)), dtype=torch.uint8, device="cuda")
    for rep in range(3):
        for name, L in libs.items():
            fn = lambda: L.clipmi_layernorm_bwd(s, _lib.BF16, dy.data_ptr(), D, x.data_ptr(), D, mean.data_ptr(),
                                                rstd.data_ptr(), w.data_ptr(), dx.data_ptr(), D, dres.data_ptr(), D,
                                                dw.data_ptr(), db.data_ptr(), 0, ws.data_ptr(), ws.numel(), R, D)
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            print(f"ln_bwd {name} R={R} D={D}: {ms * 1e3:7.1f} us {4 * R * D * 2 / ms / 1e6:6.0f} GB/s", flush=True)
