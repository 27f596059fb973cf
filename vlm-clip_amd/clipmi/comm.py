"""RCCL communicator and the data-parallel exchanges as library calls (include/clipmi.h, csrc/collectives.cpp):
the C-ABI path for hosts that run one process per GPU without torch.distributed.  The PyTorch host uses
torch.distributed for the same exchanges (towers.ContrastiveFn, trainer.GradBucketReducer)."""
import ctypes

import torch

from . import _lib
from . import kernels as K

c_vp, c_int, c_i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_lib.declare("clipmi_comm_unique_id", [c_vp])
_lib.declare("clipmi_comm_init", [ctypes.POINTER(c_vp), c_vp, c_int, c_int])
_lib.declare("clipmi_comm_destroy", [c_vp])
_lib.declare("clipmi_allgather_embed", [c_vp, c_vp, c_int, c_vp, c_vp, c_i64])
_lib.declare("clipmi_reducescatter_grad", [c_vp, c_vp, c_int, c_vp, c_vp, c_i64])
_lib.declare("clipmi_allreduce_grads", [c_vp, c_vp, c_vp, c_i64])


def unique_id() -> bytes:
    """A fresh 128-byte communicator id (rank 0 creates it and hands it to every rank)."""
    buf = ctypes.create_string_buffer(128)
    _lib.check(_lib.lib().clipmi_comm_unique_id(buf), "clipmi_comm_unique_id")
    return buf.raw


def _dt(t):
    if t.dtype == torch.float32:
        return _lib.F32
    if t.dtype == torch.bfloat16:
        return _lib.BF16
    raise ValueError("float32 or bfloat16 tensors")


class Communicator:
    """One rank of an RCCL communicator on the current device."""

    def __init__(self, uid: bytes, nranks: int, rank: int):
        if len(uid) != 128:
            raise ValueError("the communicator id is 128 bytes (unique_id())")
        self.nranks, self.rank = nranks, rank
        self._c = c_vp()
        _lib.check(_lib.lib().clipmi_comm_init(ctypes.byref(self._c), ctypes.create_string_buffer(uid, 128), nranks,
                                               rank), "clipmi_comm_init")

    def close(self):
        if self._c:
            _lib.check(_lib.lib().clipmi_comm_destroy(self._c), "clipmi_comm_destroy")
            self._c = c_vp()

    def all_gather(self, local: torch.Tensor) -> torch.Tensor:
        """[n, ...] per rank -> [nranks * n, ...] in rank order."""
        local = local.contiguous()
        out = torch.empty((self.nranks * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        _lib.check(_lib.lib().clipmi_allgather_embed(K.stream(), self._c, _dt(local), local.data_ptr(),
                                                     out.data_ptr(), local.numel()), "clipmi_allgather_embed")
        return out

    def reduce_scatter(self, full: torch.Tensor) -> torch.Tensor:
        """[nranks * n, ...] per rank -> this rank's block of the sum over ranks, [n, ...]."""
        full = full.contiguous()
        if full.shape[0] % self.nranks:
            raise ValueError("leading dimension must be a multiple of nranks")
        out = torch.empty((full.shape[0] // self.nranks,) + tuple(full.shape[1:]), dtype=full.dtype,
                          device=full.device)
        _lib.check(_lib.lib().clipmi_reducescatter_grad(K.stream(), self._c, _dt(full), full.data_ptr(),
                                                        out.data_ptr(), out.numel()), "clipmi_reducescatter_grad")
        return out

    def all_reduce_(self, grads: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks of an fp32 (contiguous) gradient buffer."""
        if grads.dtype != torch.float32 or not grads.is_contiguous():
            raise ValueError("contiguous float32 gradients")
        _lib.check(_lib.lib().clipmi_allreduce_grads(K.stream(), self._c, grads.data_ptr(), grads.numel()),
                   "clipmi_allreduce_grads")
        return grads
