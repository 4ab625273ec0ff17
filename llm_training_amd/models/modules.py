"""Building blocks shared by the model families (all tensor-parallel aware).

Activations are SEQUENCE-MAJOR ``[S, B, H]`` everywhere inside the models: the sequence-parallel
shard is then dim 0, every TP collective is one contiguous RCCL call, and the flash-attention kernels
read the fused QKV buffer through strided views without transposes (see ops/fused.py).
"""
from __future__ import annotations

import math

import os

import torch
import torch.nn as nn
from torch.autograd import Function

from ..ops import fused as F_
from ..parallel import tensor_parallel as tpl
from ..parallel.context import ParallelContext


class RMSNorm(nn.Module):
    def __init__(self, hidden_size: int, eps: float = 1e-6, dtype=None, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size, dtype=dtype, device=device))
        self.eps = eps

    def forward(self, x, residual=None):
        return F_.rms_norm(x, self.weight, self.eps, residual)

    def reset_parameters(self, gen=None):
        with torch.no_grad():
            self.weight.fill_(1.0)

    def extra_repr(self):
        return f"{tuple(self.weight.shape)}, eps={self.eps}"


class Linear(nn.Module):
    """y = x W^T (+ b) through the main-grad aware autograd function.

    Shapes are LOCAL (already divided by the TP degree when the layer is TP-sharded).
    """

    def __init__(self, in_features, out_features, bias=False, dtype=None, device=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, dtype=dtype, device=device))
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=dtype, device=device)) if bias else None

    def forward(self, x):
        return F_.linear(x, self.weight, self.bias)

    def reset_parameters(self, std=0.02, gen=None):
        with torch.no_grad():
            normal_(self.weight, std, gen)
            if self.bias is not None:
                self.bias.zero_()

    def extra_repr(self):
        return f"in={self.in_features}, out={self.out_features}, bias={self.bias is not None}"


def normal_(t: torch.Tensor, std: float, gen: torch.Generator | None = None):
    """In-place N(0, std) init; with a seeded generator of t's device it is deterministic per shard."""
    if gen is None:
        return t.normal_(0.0, std)
    if t.dtype in (torch.float32, torch.float64, torch.bfloat16, torch.float16):
        return t.normal_(0.0, std, generator=gen)
    tmp = torch.empty(t.shape, dtype=torch.float32, device=t.device).normal_(0.0, std, generator=gen)
    return t.copy_(tmp)


class _EmbeddingFn(Function):
    @staticmethod
    def forward(ctx, ids, w, v0, v1, sharded):
        ctx.save_for_backward(ids)
        ctx.v = (v0, v1)
        ctx.wshape = w.shape
        ctx.w = w
        local = ids - v0
        if sharded:  # vocab-sharded: rows owned by other ranks contribute zeros
            mask = (ids >= v0) & (ids < v1)
            local = torch.where(mask, local, torch.zeros_like(local))
            out = torch.nn.functional.embedding(local, w)
            out = out * mask.unsqueeze(-1).to(out.dtype)
        else:
            out = torch.nn.functional.embedding(local, w)
        return out

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        w = ctx.w
        v0, v1 = ctx.v
        if not ctx.needs_input_grad[1]:
            return None, None, None, None, None
        mask = (ids >= v0) & (ids < v1)
        local = (ids - v0).masked_fill(~mask, 0).reshape(-1)
        g2 = (g * mask.unsqueeze(-1).to(g.dtype)).reshape(-1, g.shape[-1])
        mg = getattr(w, "main_grad", None)
        if mg is None:
            dw = torch.zeros(ctx.wshape, dtype=g.dtype, device=g.device)
            dw.index_add_(0, local, g2)
            return None, dw, None, None, None
        if not getattr(w, "grad_added", False):
            mg.zero_()
        if g.is_cuda and deterministic_mode():
            # index_add_ scatters with atomics (order-dependent sums for repeated tokens); the sort-based
            # accumulate path of index_put_ sums each row's contributions in a fixed order
            mg.view(ctx.wshape).index_put_((local,), g2.to(mg.dtype), accumulate=True)
        else:
            mg.view(ctx.wshape).index_add_(0, local, g2.to(mg.dtype))
        w.grad_added = True
        return None, None, None, None, None


def deterministic_mode() -> bool:
    """``Trainer(deterministic=True)`` / ``LLMT_DETERMINISTIC=1``: bitwise-reproducible steps."""
    return torch.are_deterministic_algorithms_enabled() or os.environ.get("LLMT_DETERMINISTIC", "0") == "1"


class VocabParallelEmbedding(nn.Module):
    """Vocab-sharded embedding; output is reduce-scattered onto the sequence shard under TP+SP."""

    def __init__(self, vocab_size, hidden_size, pc: ParallelContext | None = None, dtype=None, device=None):
        super().__init__()
        pc = pc or ParallelContext.single()
        self.pc = pc
        self.vocab_size = vocab_size
        per = math.ceil(vocab_size / pc.tp_size)
        self.v0 = per * pc.tp_rank
        self.v1 = min(vocab_size, self.v0 + per)
        self.weight = nn.Parameter(torch.empty(per, hidden_size, dtype=dtype, device=device))

    def forward(self, ids_sb: torch.Tensor) -> torch.Tensor:
        out = _EmbeddingFn.apply(ids_sb, self.weight, self.v0, self.v1, self.pc.tp)
        if self.pc.tp:
            out = tpl.scatter_seq(out, self.pc.tp_group)
        return out

    def reset_parameters(self, std=0.02, gen=None, padding_idx=None):
        with torch.no_grad():
            normal_(self.weight, std, gen)
            if padding_idx is not None and self.v0 <= padding_idx < self.v1:
                self.weight[padding_idx - self.v0].zero_()
