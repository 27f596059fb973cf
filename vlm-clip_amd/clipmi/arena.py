"""Flat parameter arenas in HBM.

All parameters of one model part live in ONE fp32 buffer (``data``), with a matching
fp32 gradient buffer (``grad``) and, for the bf16 MFMA path, a bf16 shadow (``shadow``)
that the kernels read.  ``nn.Parameter`` objects handed to users are views into
``data`` (so ``state_dict``/``load_state_dict`` and torch optimizers work unchanged);
``p.grad`` are views into ``grad``.  One arena = one AdamW launch, one grad-norm launch,
one cast launch, and contiguous [q;k;v] blocks that the fused QKV GEMM reads directly.
"""
from __future__ import annotations

import torch

from . import _lib
from . import kernels as K

ALIGN = 64  # elements (256 B of fp32, 128 B of bf16): keeps every GEMM operand 16-B aligned


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class Arena:
    def __init__(self, specs, device, dtype_shadow=True):
        """specs: ordered (name, shape) list; names that must be adjacent (q/k/v) are listed
        consecutively and are checked to stay contiguous after alignment."""
        self.offsets = {}
        n = 0
        for name, shape in specs:
            numel = 1
            for s in shape:
                numel *= s
            n = _align(n)
            self.offsets[name] = (n, tuple(shape), numel)
            n += numel
        self.numel = _align(max(n, 1))
        self.device = torch.device(device)
        self.data = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.shadow = (torch.zeros(self.numel, dtype=torch.bfloat16, device=self.device)
                       if dtype_shadow else None)
        self._shadow_version = -1
        self.params = {}  # name -> nn.Parameter (set by the owner)

    # -- views ---------------------------------------------------------------------------
    def view(self, name, buf=None):
        off, shape, numel = self.offsets[name]
        b = self.data if buf is None else buf
        return b[off:off + numel].view(shape)

    def ptr(self, name, buf):
        off = self.offsets[name][0]
        return buf.data_ptr() + off * buf.element_size()

    def check_adjacent(self, names):
        off0 = self.offsets[names[0]][0]
        o = off0
        for n in names:
            off, _, numel = self.offsets[n]
            if off != o:
                raise AssertionError(f"arena layout: {n} not adjacent")
            o += numel

    # -- shadow --------------------------------------------------------------------------
    def sync_shadow(self):
        """Refresh the bf16 shadow if the fp32 master changed outside our optimizer."""
        if self.shadow is None:
            return
        v = self.data._version
        if v != self._shadow_version:
            _lib.check(_lib.lib().clipmi_cast_f32_bf16(K.stream(), K.ptr(self.data), K.ptr(self.shadow),
                                                      self.numel), "cast")
            self._shadow_version = self.data._version

    def mark_shadow_fresh(self):
        self._shadow_version = self.data._version

    # -- gradients -----------------------------------------------------------------------
    def prepare_grads(self):
        """Emulate AccumulateGrad on the arena: params whose .grad is None get a zeroed view
        of the grad arena attached; a foreign .grad tensor is copied in first."""
        for name, p in self.params.items():
            if not p.requires_grad:
                continue
            g = p.grad
            v = self.view(name, self.grad)
            if g is None:
                v.zero_()
                p.grad = v
            elif g.data_ptr() != v.data_ptr():
                v.copy_(g)
                p.grad = v

    def zero_grad(self):
        self.grad.zero_()
        for name, p in self.params.items():
            if p.requires_grad:
                p.grad = self.view(name, self.grad)

    def any_requires_grad(self):
        return any(p.requires_grad for p in self.params.values())

    def all_require_grad(self):
        return all(p.requires_grad for p in self.params.values())

    # -- device moves --------------------------------------------------------------------
    def apply_(self, fn):
        new = fn(self.data)
        if new.dtype != torch.float32:
            raise TypeError("clipmi parameters are fp32 masters; choose the compute precision with "
                            "CLIPWithAdapters(precision=...) instead of casting the module")
        if new.data_ptr() == self.data.data_ptr():
            return False
        self.data = new
        self.grad = fn(self.grad)
        if self.shadow is not None:
            self.shadow = self.shadow.to(self.data.device)
        self.device = self.data.device
        self._shadow_version = -1
        return True  # the owner re-creates its Parameter views
