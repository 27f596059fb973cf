"""ctypes binding of libclipmi.so (the C ABI in include/clipmi.h).

The library is built in-tree (``make -C vlm-clip_amd``) and loaded from this package's
directory.  There is no fallback: if the library is missing, every op raises."""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CLIPMI_LIB: an alternative build of the same library (schedule A/B experiments only)
LIB_PATH = os.environ.get("CLIPMI_LIB") or os.path.join(_HERE, "libclipmi.so")

F32, BF16, FP8 = 0, 1, 2
EPI_BIAS, EPI_QGELU, EPI_GELU, EPI_RESID = 1, 2, 4, 8
EPI_DQGELU, EPI_DGELU, EPI_BETA, EPI_STORE_PRE = 16, 32, 64, 128
EPI_STORE_DACT, EPI_MUL_AUX = 256, 512
GEMM_SPLIT3 = 1024  # not an epilogue: fp32 operands as a bf16x3 split product (include/clipmi.h)

c_i64 = ctypes.c_int64
c_vp = ctypes.c_void_p


class GemmDesc(ctypes.Structure):
    _fields_ = [("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int),
                ("A", c_vp), ("lda", c_i64), ("a_kmajor", ctypes.c_int),
                ("B", c_vp), ("ldb", c_i64), ("b_kmajor", ctypes.c_int),
                ("C", c_vp), ("ldc", c_i64),
                ("bias", c_vp),
                ("residual", c_vp), ("ldr", c_i64),
                ("aux", c_vp), ("ldaux", c_i64),
                ("alpha", ctypes.c_float),
                ("flags", ctypes.c_int),
                ("ab_dtype", ctypes.c_int), ("c_dtype", ctypes.c_int), ("bias_dtype", ctypes.c_int),
                ("split_k", ctypes.c_int),
                ("workspace", c_vp), ("workspace_bytes", c_i64),
                ("bias_grad", c_vp), ("force_small_tile", ctypes.c_int),
                ("a_scale", c_vp), ("b_scale", c_vp), ("c_scale", c_vp)]


class ClipmiError(RuntimeError):
    pass


_lib = None
_PROTOS = {}


def _declare(name, restype, argtypes):
    _PROTOS[name] = (restype, argtypes)


_declare("clipmi_version", ctypes.c_int, [])
_declare("clipmi_build_digest", ctypes.c_char_p, [])
_declare("clipmi_last_error", ctypes.c_char_p, [])
_declare("clipmi_gemm", ctypes.c_int, [c_vp, ctypes.POINTER(GemmDesc)])
_declare("clipmi_gemm_split3_ws", ctypes.c_int64, [ctypes.c_int] * 6)
_declare("clipmi_gemm_x3out_ws", ctypes.c_int64, [ctypes.c_int] * 2)
_declare("clipmi_gemm_x3out_ok", ctypes.c_int, [ctypes.c_int] * 6)
_declare("clipmi_gemm_x3out", ctypes.c_int, [c_vp, ctypes.POINTER(GemmDesc), ctypes.c_int, c_vp, ctypes.c_int, c_vp,
                                             c_i64])
_declare("clipmi_gemm_batched", ctypes.c_int, [c_vp, ctypes.POINTER(GemmDesc), ctypes.c_int, ctypes.c_int]
         + [ctypes.c_int64] * 6)


def declare(name, argtypes, restype=ctypes.c_int):
    """Register an entry point's prototype (used by the modules that bind it)."""
    _declare(name, restype, argtypes)
    if _lib is not None:
        f = getattr(_lib, name)
        f.restype, f.argtypes = restype, argtypes


def source_digest() -> str:
    """sha256 of the library's sources as the Makefile computes it (sorted csrc/*.hip, *.cpp,
    *.h, then include/clipmi.h), from the tree this package sits in."""
    import hashlib
    pkg = os.path.dirname(_HERE)
    csrc = os.path.join(pkg, "csrc")
    names = sorted(f"csrc/{n}" for n in os.listdir(csrc) if n.endswith((".hip", ".cpp", ".h")))
    h = hashlib.sha256()
    for n in names:
        with open(os.path.join(pkg, n), "rb") as f:
            h.update(f.read())
    with open(os.path.join(os.path.dirname(pkg), "include", "clipmi.h"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def build_digest() -> str:
    return lib().clipmi_build_digest().decode()


def lib():
    global _lib
    if _lib is None:
        if not os.path.isfile(LIB_PATH):
            raise ImportError(f"libclipmi.so not built at {LIB_PATH}; run `make -C vlm-clip_amd` "
                              "(there is no CPU fallback on the product path)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _PROTOS.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        # provenance: the library must be built from the sources next to it (an alternative
        # CLIPMI_LIB build is an A/B experiment of other sources, so it is exempt)
        if not os.environ.get("CLIPMI_LIB") and not os.environ.get("CLIPMI_ALLOW_STALE"):
            built, src = L.clipmi_build_digest().decode(), source_digest()
            if built != src:
                raise ImportError(f"{LIB_PATH} was built from other sources (digest {built[:12]}, tree "
                                  f"{src[:12]}); rebuild with `make -C vlm-clip_amd`")
        _lib = L
    return _lib


def check(status: int, what: str = ""):
    if status != 0:
        msg = lib().clipmi_last_error().decode(errors="replace")
        if status == -1:
            raise ValueError(f"{what}: {msg}")
        raise ClipmiError(f"{what}: status {status}: {msg}")


def call(name, *args):
    check(getattr(lib(), name)(*args), name)
