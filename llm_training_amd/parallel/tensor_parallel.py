"""Megatron-style tensor + sequence parallel primitives on RCCL (torch.distributed, backend "nccl").

Reference plan (src/llm_training/models/llama/llama_model.py:197-244): colwise q/k/v
and gate/up, rowwise o/down, vocab-sharded embedding and lm_head, SequenceParallel norms with the
residual stream sharded on the sequence dim. The reference expresses it with DTensor
``parallelize_module``; here it is four explicit autograd collectives on SEQ-MAJOR activations
[S, B, H], so the sequence shard is dim 0 and every collective is a single contiguous
``all_gather_into_tensor`` / ``reduce_scatter_tensor`` (no DTensor dispatch, no layout copies).

- ``gather_seq``   fwd all-gather(seq)     bwd reduce-scatter(seq)   (enter attention / MLP)
- ``scatter_seq``  fwd reduce-scatter(seq) bwd all-gather(seq)       (leave o_proj / down_proj)
- ``copy_to_tp``   fwd identity            bwd all-reduce            (non-SP input)
- ``reduce_tp``    fwd all-reduce          bwd identity
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch.autograd import Function


def _ws(group) -> int:
    return dist.get_world_size(group) if group is not None else 1


def all_gather_seq(x: torch.Tensor, group) -> torch.Tensor:
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty((x.shape[0] * n, *x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=group)
    return out


def reduce_scatter_seq(x: torch.Tensor, group) -> torch.Tensor:
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    assert x.shape[0] % n == 0, "sequence length must be divisible by the tensor-parallel size"
    out = torch.empty((x.shape[0] // n, *x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x, group=group)
    return out


class _GatherSeq(Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return all_gather_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return reduce_scatter_seq(g, ctx.group), None


class _ScatterSeq(Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return reduce_scatter_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return all_gather_seq(g, ctx.group), None


class _SplitSeq(Function):
    """Take this rank's sequence shard (no communication); bwd all-gathers."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        n = _ws(group)
        r = dist.get_rank(group)
        c = x.shape[0] // n
        return x[r * c:(r + 1) * c].contiguous()

    @staticmethod
    def backward(ctx, g):
        return all_gather_seq(g, ctx.group), None


class _CopyToTP(Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceTP(Function):
    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous().clone()
        dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


def gather_seq(x, group):
    return _GatherSeq.apply(x, group) if _ws(group) > 1 else x


def scatter_seq(x, group):
    return _ScatterSeq.apply(x, group) if _ws(group) > 1 else x


def split_seq(x, group):
    return _SplitSeq.apply(x, group) if _ws(group) > 1 else x


def copy_to_tp(x, group):
    return _CopyToTP.apply(x, group) if _ws(group) > 1 else x


def reduce_tp(x, group):
    return _ReduceTP.apply(x, group) if _ws(group) > 1 else x


def shard_rows(w: torch.Tensor, rank: int, n: int) -> torch.Tensor:
    """Contiguous row shard (column-parallel output features)."""
    c = w.shape[0] // n
    return w[rank * c:(rank + 1) * c]


def shard_cols(w: torch.Tensor, rank: int, n: int) -> torch.Tensor:
    c = w.shape[1] // n
    return w[:, rank * c:(rank + 1) * c]


def shard_fused_rows(w: torch.Tensor, sizes: list[int], rank: int, n: int) -> torch.Tensor:
    """Interleaved shard of a fused weight [a; b; c] -> [a_r; b_r; c_r].

    Fixes the reference's contiguous sharding of Phi-3's fused qkv/gate_up (SURVEY Q7,
    src/llm_training/models/phi3/phi3_model.py:242,249), which mixes heads / gate with up.
    """
    parts = torch.split(w, sizes, dim=0)
    return torch.cat([shard_rows(p, rank, n) for p in parts], dim=0)


def unshard_fused_rows(shards: list[torch.Tensor], sizes: list[int]) -> torch.Tensor:
    """Inverse of :func:`shard_fused_rows` given every rank's shard (in rank order)."""
    n = len(shards)
    local = [s // n for s in sizes]
    per = [torch.split(s, local, dim=0) for s in shards]
    return torch.cat([torch.cat([per[r][i] for r in range(n)], 0) for i in range(len(sizes))], 0)
