"""RCCL communicator and the data-parallel exchanges as library calls (include/clipmi.h, csrc/collectives.cpp).

A ``Communicator`` is accepted wherever the product path takes a data-parallel group
(``CLIPWithAdapters(process_group=...)``, ``FusedAdamW(process_group=...)``): the embedding all-gather and
gradient reduce-scatter around the contrastive loss (towers.ContrastiveFn) and the bucketed gradient
all-reduce (trainer.GradBucketReducer) then run as ``clipmi_allgather_embed`` / ``clipmi_reducescatter_grad`` /
``clipmi_allreduce`` on the caller's (or the reducer's communication) stream -- SURVEY §8e's "RCCL issued from
libclipmi on the compute stream".  A torch.distributed group works the same way through torch's RCCL (and gloo
for the CPU tests).  The helpers below dispatch on the group's kind."""
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from . import kernels as K

c_vp, c_int, c_i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_lib.declare("clipmi_comm_unique_id", [c_vp])
_lib.declare("clipmi_comm_init", [ctypes.POINTER(c_vp), c_vp, c_int, c_int])
_lib.declare("clipmi_comm_destroy", [c_vp])
_lib.declare("clipmi_allgather_embed", [c_vp, c_vp, c_int, c_vp, c_vp, c_i64])
_lib.declare("clipmi_reducescatter_grad", [c_vp, c_vp, c_int, c_vp, c_vp, c_i64])
_lib.declare("clipmi_allreduce_grads", [c_vp, c_vp, c_vp, c_i64])
_lib.declare("clipmi_allreduce", [c_vp, c_vp, c_int, c_vp, c_i64])


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


def _stream(stream):
    return K.stream() if stream is None else ctypes.c_void_p(stream.cuda_stream)


class Communicator:
    """One rank of an RCCL communicator on the current device."""

    def __init__(self, uid: bytes, nranks: int, rank: int):
        if len(uid) != 128:
            raise ValueError("the communicator id is 128 bytes (unique_id())")
        self.nranks, self.rank = nranks, rank
        self._c = c_vp()
        _lib.check(_lib.lib().clipmi_comm_init(ctypes.byref(self._c), ctypes.create_string_buffer(uid, 128), nranks,
                                               rank), "clipmi_comm_init")

    @classmethod
    def from_process_group(cls, group=None):
        """Bootstrap over an initialised torch.distributed group (its store): rank 0 creates the id, every
        rank of the group joins with the group's size and rank."""
        obj = [unique_id() if dist.get_rank(group) == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return cls(obj[0], dist.get_world_size(group), dist.get_rank(group))

    def close(self):
        if self._c:
            _lib.check(_lib.lib().clipmi_comm_destroy(self._c), "clipmi_comm_destroy")
            self._c = c_vp()

    def all_gather(self, local: torch.Tensor, stream=None) -> torch.Tensor:
        """[n, ...] per rank -> [nranks * n, ...] in rank order."""
        local = local.contiguous()
        out = torch.empty((self.nranks * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        _lib.check(_lib.lib().clipmi_allgather_embed(_stream(stream), self._c, _dt(local), local.data_ptr(),
                                                     out.data_ptr(), local.numel()), "clipmi_allgather_embed")
        return out

    def reduce_scatter(self, full: torch.Tensor, stream=None) -> torch.Tensor:
        """[nranks * n, ...] per rank -> this rank's block of the sum over ranks, [n, ...]."""
        full = full.contiguous()
        if full.shape[0] % self.nranks:
            raise ValueError("leading dimension must be a multiple of nranks")
        out = torch.empty((full.shape[0] // self.nranks,) + tuple(full.shape[1:]), dtype=full.dtype,
                          device=full.device)
        _lib.check(_lib.lib().clipmi_reducescatter_grad(_stream(stream), self._c, _dt(full), full.data_ptr(),
                                                        out.data_ptr(), out.numel()), "clipmi_reducescatter_grad")
        return out

    def all_reduce_(self, buf: torch.Tensor, stream=None) -> torch.Tensor:
        """In-place sum over ranks of a contiguous fp32 or bf16 buffer."""
        if not buf.is_contiguous():
            raise ValueError("contiguous buffer")
        _lib.check(_lib.lib().clipmi_allreduce(_stream(stream), self._c, _dt(buf), buf.data_ptr(), buf.numel()),
                   "clipmi_allreduce")
        return buf


# ---- the data-parallel group, either kind: None (single device), a Communicator or a torch.distributed group
def is_lib(group):
    return isinstance(group, Communicator)


def world_rank(group):
    if group is None:
        return 1, 0
    if is_lib(group):
        return group.nranks, group.rank
    return dist.get_world_size(group), dist.get_rank(group)


def all_reduce_(t, group):
    """In-place sum over the group on the current stream (the loss, a whole gradient arena)."""
    if is_lib(group):
        return group.all_reduce_(t)
    dist.all_reduce(t, group=group)
    return t
