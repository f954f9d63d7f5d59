"""Flat parameter / gradient storage.

Every trainable tensor of a parameter group is a VIEW into one contiguous bf16 buffer,
and its gradient a view into one contiguous bf16 gradient buffer laid out identically.
This is the memory plan the rest of the runtime is built around (288 GB of HBM per
MI355X, so we size for few, large, contiguous buffers):

* the optimizer is one streaming kernel over the flat buffers (ops/csrc/adamw.hip);
* data-parallel gradient buckets are plain slices of the flat gradient buffer, so a
  bucket all-reduce / reduce-scatter needs no packing copy;
* weight-gradient GEMMs write (or accumulate, beta=1) straight into their slice.

Parameters are registered in *reverse execution order* by the model (last layer first),
so during backward the finished gradients form a growing prefix of the buffer and
buckets can be launched as soon as the prefix crosses a bucket boundary.
"""
from __future__ import annotations

import zlib

from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import torch

ALIGN = 64  # elements; keeps every view 128-byte aligned for 16-byte vector loads


def _round(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


@dataclass
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    offset: int = 0
    numel: int = 0
    init: str = "normal"      # normal | ones | zeros
    std: float = 0.02
    decay: bool = True


@dataclass
class FlatGroup:
    """A group of parameters that share flat storage."""
    name: str
    specs: List[ParamSpec] = field(default_factory=list)
    numel: int = 0
    params: torch.Tensor = None   # bf16 [numel]
    grads: torch.Tensor = None    # bf16 [numel]
    _index: Dict[str, ParamSpec] = field(default_factory=dict)

    def add(self, name, shape, init="normal", std=0.02, decay=True) -> ParamSpec:
        n = 1
        for s in shape:
            n *= int(s)
        spec = ParamSpec(name, tuple(int(s) for s in shape), self.numel, n, init, std, decay)
        self.specs.append(spec)
        self._index[name] = spec
        self.numel = _round(self.numel + n)
        return spec

    def allocate(self, device, dtype=torch.bfloat16, pad_to: int = 1, grads: bool = True):
        """Allocate storage; ``pad_to`` rounds the total so it divides evenly into DP shards.
        ``grads=False`` (inference) allocates no gradient buffer."""
        total = _round(self.numel, max(ALIGN, pad_to))
        self.numel = total
        self.params = torch.zeros(total, device=device, dtype=dtype)
        self.grads = torch.zeros(total, device=device, dtype=dtype) if grads else None
        return self

    def param(self, name) -> torch.Tensor:
        s = self._index[name]
        return self.params[s.offset:s.offset + s.numel].view(s.shape)

    def grad(self, name) -> torch.Tensor:
        s = self._index[name]
        return self.grads[s.offset:s.offset + s.numel].view(s.shape)

    def spec(self, name) -> ParamSpec:
        return self._index[name]

    def end_offset(self, name) -> int:
        s = self._index[name]
        return s.offset + s.numel

    def init_(self, seed: int, full_shapes: Dict[str, Tuple[torch.Size, callable]] | None = None):
        """Deterministic init. ``full_shapes[name] = (full_shape, slicer)`` lets a TP shard
        be cut out of the same full matrix every TP degree would generate (used by the
        TP-equivalence tests); otherwise each tensor is drawn from its own seeded stream."""
        for i, s in enumerate(self.specs):
            p = self.param(s.name)
            if s.init == "ones":
                p.fill_(1.0)
            elif s.init == "zeros":
                p.zero_()
            else:
                # seed by NAME so every TP/PP partitioning draws identical weights
                key = seed * 1000003 + zlib.crc32(s.name.encode())
                g = torch.Generator(device="cpu").manual_seed(key)
                if full_shapes and s.name in full_shapes:
                    fshape, slicer = full_shapes[s.name]
                    full = torch.empty(fshape, dtype=torch.float32).normal_(0.0, s.std, generator=g)
                    p.copy_(slicer(full).to(p.dtype))
                elif p.device.type == "cpu":
                    p.copy_(torch.empty(s.shape, dtype=torch.float32).normal_(0.0, s.std, generator=g))
                else:
                    # GPU: Philox stream seeded by the same name key, drawn straight into the
                    # bf16 parameter on the device (8B params in well under a second -- this
                    # sits on the CRD-to-first-step path)
                    dg = torch.Generator(device=p.device).manual_seed(key)
                    p.normal_(0.0, s.std, generator=dg)
        return self

    def zero_grad(self):
        self.grads.zero_()
