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

With SP the collectives next to the projection GEMMs are pipelined with the GEMMs (``ag_linear`` /
``linear_rs``, used by the decoder layers) as a staged collective matmul sized for MI355X's xGMI: every
GPU of a node has a direct link to each of the other seven, so one RCCL all-gather / reduce-scatter keeps
all seven links busy, while a peer-by-peer ring of P2P transfers would move each step over a single link
(and P2P operations on one communicator run one after another on its stream). Each rank's sequence shard
is therefore cut into ``m`` sub-chunks (``LLMT_TP_STAGES``, default 4) and each collective into ``m``
full-mesh collectives of one sub-chunk each, issued together on the communicator's stream; the compute
stream waits only for the stage it is about to use:

- ``ag_linear``  (q/k/v, gate/up), forward: all-gather stage j+1 is in flight while the GEMMs of stage j's
  rows (one per source rank, written straight into their rows of the output) run; backward: the input
  gradient of stage j (one GEMM per destination rank) is reduce-scattered while stage j+1's is computed,
  and the weight gradient accumulates per (stage, rank) block beside them.
- ``linear_rs``  (o, down), forward: the output rows of stage j are reduce-scattered while stage j+1's are
  computed; backward: the staged all-gather of the output gradient feeds the input-gradient GEMMs stage by
  stage, as in ``ag_linear``'s forward.

Gathered tensors are kept stage-major ([m, n, S/(n m), ...]): each stage's all-gather writes one
contiguous block, and every GEMM reads or writes a contiguous row block of it, so no reordering copy is
made. The compute stream's waits are metered when ``TP_WAIT_METER`` holds a list (bench.py reports the
exposed tensor-parallel communication per step from it).
"""
from __future__ import annotations

import os

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


# compute-stream stalls on tensor-parallel collectives: a list of (start, end) CUDA events, or None
TP_WAIT_METER: list | None = None


def _tp_wait(work) -> None:
    m = TP_WAIT_METER
    if m is not None and torch.cuda.is_available() and torch.cuda.is_initialized():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        work.wait()
        b.record()
        m.append((a, b))
    else:
        work.wait()


def tp_stages(rows: int) -> int:
    """Pipeline stages for a sequence shard of ``rows`` rows: LLMT_TP_STAGES (default 4), reduced to divide it."""
    m = max(1, int(os.environ.get("LLMT_TP_STAGES", "4")))
    while rows % m:
        m -= 1
    return m


class _AGLinear(Function):
    """y = all_gather_seq(x) @ W^T (+ b) for seq-major x [S/n, B, K] -> [S, B, N], staged (module doc)."""

    @staticmethod
    def forward(ctx, x, w, b, group):
        from ..ops.fused import mm_nt
        n = _ws(group)
        x = x.contiguous()
        c = x.shape[0]
        m = tp_stages(c)
        cm = c // m
        tail = x.shape[1:]
        full = torch.empty((m, n, cm, *tail), dtype=x.dtype, device=x.device)  # stage-major gathered input
        works = [dist.all_gather_into_tensor(full[j].view(n * cm, *tail), x[j * cm:(j + 1) * cm], group=group,
                                             async_op=True) for j in range(m)]
        y = torch.empty((c * n, *tail[:-1], w.shape[0]), dtype=x.dtype, device=x.device)
        y5 = y.view(n, m, cm, *tail[:-1], w.shape[0])
        for j in range(m):
            _tp_wait(works[j])
            for d in range(n):  # rows of source rank d, stage j -> their place in the output
                mm_nt(_rows(full[j, d]), w, out=_rows(y5[d, j]), bias=b)
        ctx.save_for_backward(full)
        ctx.w, ctx.group, ctx.has_bias, ctx.m = w, group, b is not None, m
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops.fused import _wgrad_mm, drop_dy_t, mm_nn
        (full,) = ctx.saved_tensors
        w, group, m = ctx.w, ctx.group, ctx.m
        n, cm = full.shape[1], full.shape[2]
        tail = full.shape[3:]
        dy = dy.contiguous()
        dy5 = dy.view(n, m, cm, *dy.shape[1:])
        dx = dw = db = None
        works = []
        if ctx.needs_input_grad[0]:
            dx = torch.empty((m * cm, *tail), dtype=full.dtype, device=full.device)
            for j in range(m):  # stage j's input gradient is reduce-scattered while stage j+1's is computed
                part = torch.empty((n, cm, *tail), dtype=full.dtype, device=full.device)
                for d in range(n):
                    mm_nn(_rows(dy5[d, j]), w, out=_rows(part[d]))
                works.append(dist.reduce_scatter_tensor(dx[j * cm:(j + 1) * cm], part.view(n * cm, *tail), group=group,
                                                        async_op=True))
        if ctx.needs_input_grad[1]:
            # the weight gradient per (stage, rank) block, accumulated, under the last reduce-scatters
            for j in range(m):
                for d in range(n):
                    r = _wgrad_mm(w, _rows(dy5[d, j]).t(), _rows(full[j, d]))
                    dw = r if dw is None else (dw + r if r is not None else dw)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _rows(dy).sum(0)
        for wk in works:
            _tp_wait(wk)
        drop_dy_t()  # a SwiGLU-produced dy^T is only used by the plain linear path
        return dx, dw, db, None


class _LinearRS(Function):
    """y = reduce_scatter_seq(x @ W^T) (+ b once) for seq-major x [S, B, K] -> [S/n, B, N], staged."""

    @staticmethod
    def forward(ctx, x, w, b, group):
        from ..ops.fused import mm_nt
        n = _ws(group)
        x = x.contiguous()
        assert x.shape[0] % n == 0, "sequence length must be divisible by the tensor-parallel size"
        c = x.shape[0] // n
        m = tp_stages(c)
        cm = c // m
        x5 = x.view(n, m, cm, *x.shape[1:])
        y = torch.empty((c, *x.shape[1:-1], w.shape[0]), dtype=x.dtype, device=x.device)
        works, parts = [], []
        for j in range(m):  # stage j's rows are reduce-scattered while stage j+1's are computed
            part = torch.empty((n, cm, *x.shape[1:-1], w.shape[0]), dtype=x.dtype, device=x.device)
            for d in range(n):
                mm_nt(_rows(x5[d, j]), w, out=_rows(part[d]))
            works.append(dist.reduce_scatter_tensor(y[j * cm:(j + 1) * cm], part.view(n * cm, *part.shape[2:]),
                                                    group=group, async_op=True))
            parts.append(part)
        for wk in works:
            _tp_wait(wk)
        del parts
        if b is not None:
            y = y + b
        ctx.save_for_backward(x)
        ctx.w, ctx.group, ctx.has_bias, ctx.m = w, group, b is not None, m
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops.fused import _wgrad_mm, drop_dy_t, mm_nn
        (x,) = ctx.saved_tensors
        w, group, m = ctx.w, ctx.group, ctx.m
        n = _ws(group)
        dy = dy.contiguous()
        c = dy.shape[0]
        cm = c // m
        x5 = x.view(n, m, cm, *x.shape[1:])
        full = torch.empty((m, n, cm, *dy.shape[1:]), dtype=dy.dtype, device=dy.device)  # stage-major dy
        works = [dist.all_gather_into_tensor(full[j].view(n * cm, *dy.shape[1:]), dy[j * cm:(j + 1) * cm],
                                             group=group, async_op=True) for j in range(m)]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            dx5 = dx.view(n, m, cm, *x.shape[1:])
        for j in range(m):
            _tp_wait(works[j])
            for d in range(n):
                if ctx.needs_input_grad[0]:
                    mm_nn(_rows(full[j, d]), w, out=_rows(dx5[d, j]))
                if ctx.needs_input_grad[1]:
                    r = _wgrad_mm(w, _rows(full[j, d]).t(), _rows(x5[d, j]))
                    dw = r if dw is None else (dw + r if r is not None else dw)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _rows(dy).sum(0)
        drop_dy_t()  # a SwiGLU-produced dy^T is only used by the plain linear path
        return dx, dw, db, None


def ag_linear(x, w, b, group):
    """Column-parallel projection of the sequence-gathered input, staged gather overlapped with the GEMMs."""
    if _ws(group) == 1:
        from ..ops.fused import linear
        return linear(x, w, b)
    return _AGLinear.apply(x, w, b, group)


def linear_rs(x, w, b, group):
    """Row-parallel projection reduce-scattered over the sequence, staged with the GEMMs both ways."""
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
