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

With SP the collectives next to the projection GEMMs are overlapped with GEMM work instead of
running back to back with it (``ag_linear`` / ``linear_rs``, used by the decoder layers):

- ``ag_linear``  (q/k/v, gate/up):  forward all-gathers the sequence shards asynchronously while the GEMM
  of this rank's own rows runs, then the GEMM of the other ranks' rows; backward starts the
  reduce-scatter of the input gradient and runs the weight-gradient GEMM under it.
- ``linear_rs``  (o, down):  backward all-gathers the output gradient asynchronously while the
  input-gradient GEMM of this rank's own rows runs. (The forward reduce-scatter has no independent
  GEMM work beside it.)
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


def _rows(t: torch.Tensor) -> torch.Tensor:
    return t.reshape(-1, t.shape[-1])


class _AGLinear(Function):
    """y = all_gather_seq(x) @ W^T (+ b) for seq-major x [S/n, B, K] -> [S, B, N]."""

    @staticmethod
    def forward(ctx, x, w, b, group):
        from ..ops.fused import mm_nt
        n, r = _ws(group), dist.get_rank(group)
        x = x.contiguous()
        c = x.shape[0]
        full = torch.empty((c * n, *x.shape[1:]), dtype=x.dtype, device=x.device)
        work = dist.all_gather_into_tensor(full, x, group=group, async_op=True)
        y = torch.empty((c * n, *x.shape[1:-1], w.shape[0]), dtype=x.dtype, device=x.device)
        y2, f2 = _rows(y), _rows(full)
        per = y2.shape[0] // n
        mm_nt(_rows(x), w, out=y2[r * per:(r + 1) * per])  # own rows while the others arrive
        work.wait()
        if r > 0:
            mm_nt(f2[:r * per], w, out=y2[:r * per])
        if r < n - 1:
            mm_nt(f2[(r + 1) * per:], w, out=y2[(r + 1) * per:])
        if b is not None:
            y += b
        ctx.save_for_backward(full)
        ctx.w, ctx.group, ctx.has_bias = w, group, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops.fused import _wgrad_mm, drop_dy_t, mm_nn
        (full,) = ctx.saved_tensors
        w, group = ctx.w, ctx.group
        n = _ws(group)
        dy2 = _rows(dy.contiguous())
        dx = db = dw = None
        work = None
        if ctx.needs_input_grad[0]:
            dx_full = mm_nn(dy2, w).view(*full.shape)
            dx = torch.empty((full.shape[0] // n, *full.shape[1:]), dtype=full.dtype, device=full.device)
            work = dist.reduce_scatter_tensor(dx, dx_full, group=group, async_op=True)
        if ctx.needs_input_grad[1]:
            dw = _wgrad_mm(w, dy2.t(), _rows(full))  # runs under the reduce-scatter
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy2.sum(0)
        if work is not None:
            work.wait()
        drop_dy_t()  # a SwiGLU-produced dy^T is only used by the plain linear path
        return dx, dw, db, None


class _LinearRS(Function):
    """y = reduce_scatter_seq(x @ W^T) (+ b once) for seq-major x [S, B, K] -> [S/n, B, N]."""

    @staticmethod
    def forward(ctx, x, w, b, group):
        from ..ops.fused import mm_nt
        x = x.contiguous()
        y = mm_nt(_rows(x), w).view(*x.shape[:-1], w.shape[0])
        y = reduce_scatter_seq(y, group)
        if b is not None:
            y = y + b
        ctx.save_for_backward(x)
        ctx.w, ctx.group, ctx.has_bias = w, group, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops.fused import _wgrad_mm, drop_dy_t, mm_nn
        (x,) = ctx.saved_tensors
        w, group = ctx.w, ctx.group
        n, r = _ws(group), dist.get_rank(group)
        dy = dy.contiguous()
        full = torch.empty((dy.shape[0] * n, *dy.shape[1:]), dtype=dy.dtype, device=dy.device)
        work = dist.all_gather_into_tensor(full, dy, group=group, async_op=True)
        dx = dw = db = None
        f2 = _rows(full)
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            dx2 = _rows(dx)
            per = dx2.shape[0] // n
            mm_nn(_rows(dy), w, out=dx2[r * per:(r + 1) * per])  # own rows while the others arrive
            work.wait()
            if r > 0:
                mm_nn(f2[:r * per], w, out=dx2[:r * per])
            if r < n - 1:
                mm_nn(f2[(r + 1) * per:], w, out=dx2[(r + 1) * per:])
        else:
            work.wait()
        if ctx.needs_input_grad[1]:
            dw = _wgrad_mm(w, f2.t(), _rows(x))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _rows(dy).sum(0)
        drop_dy_t()  # a SwiGLU-produced dy^T is only used by the plain linear path
        return dx, dw, db, None


def ag_linear(x, w, b, group):
    """Column-parallel projection of the sequence-gathered input, gather overlapped with the GEMM."""
    if _ws(group) == 1:
        from ..ops.fused import linear
        return linear(x, w, b)
    return _AGLinear.apply(x, w, b, group)


def linear_rs(x, w, b, group):
    """Row-parallel projection reduce-scattered over the sequence, backward gather overlapped."""
    if _ws(group) == 1:
        from ..ops.fused import linear
        return linear(x, w, b)
    return _LinearRS.apply(x, w, b, group)


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
