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
all seven links busy, while a peer-by-peer ring of P2P transfers would move each step over a single link.
Each collective is therefore cut into ``m`` full-mesh collectives (``LLMT_TP_STAGES``, default 4),
issued together on the communicator's stream; the compute stream waits only for the chunks it is about
to use.

**Chunked sequence layout.** The sequence shard of rank d is not one contiguous run of S/n positions
but m chunks: with S = m * n * cm, rank d holds positions j * n * cm + d * cm + [0, cm) for j = 0..m-1.
Then the all-gather of chunk j from every rank is global rows [j n cm, (j+1) n cm) in sequence order,
and a reduce-scatter of such a block lands chunk j on every rank: the gathered tensor IS the sequence,
every stage reads or writes one contiguous row block, and a projection needs no per-rank GEMMs and no
reordering copy. The layout is a permutation of the tokens over the ranks; RMSNorm, the residual stream
and the embedding are per-token and do not care, and attention / the loss only ever see gathered
(sequence-ordered) tensors. Every collective of this module uses it (``seq_chunks`` of the sequence).

- ``ag_linear``  (q/k/v, gate/up), forward: the chunk all-gathers run while earlier chunks' rows are
  multiplied; backward: the input gradient of a group of chunks is reduce-scattered while the next group's
  is computed. The weight gradient is ONE GEMM over the gathered input and the full output gradient.
- ``linear_rs``  (o, down), forward: the output rows of a group are reduce-scattered while the next
  group's are computed; backward: the chunked all-gather of the output gradient feeds the input-gradient
  GEMMs group by group, and again one weight-gradient GEMM.

GEMM granularity: consecutive chunks are grouped so that each GEMM fills the chip with at least
``LLMT_TP_GEMM_TILES`` (default 1024 = four waves of 256 CUs) output tiles of 256 x 256; a projection whose
chunk already does runs one GEMM per chunk. The input-gradient GEMMs of all groups share one W^T (the TN
layout hipBLASLt runs fastest). On one GPU the staged sequences run within 0-7 % of the single unstaged GEMM
of the same FLOPs, against up to 5x for the per-(chunk, rank) GEMMs of round 5
(benchmarks/bench_tp_gemms.py, profiles/r6_tp_gemms.md). The compute stream's waits are
metered when ``TP_WAIT_METER`` holds a list (bench.py reports the exposed tensor-parallel communication
per step from it); ``STAGE_PLANS`` records the group sizes each projection ran with.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
from torch.autograd import Function


def _ws(group) -> int:
    return dist.get_world_size(group) if group is not None else 1


def tp_stages(rows: int) -> int:
    """Chunks of a sequence shard of ``rows`` rows: LLMT_TP_STAGES (default 4), reduced to divide it."""
    m = max(1, int(os.environ.get("LLMT_TP_STAGES", "4")))
    while rows % m:
        m -= 1
    return m


def all_gather_seq(x: torch.Tensor, group) -> torch.Tensor:
    """Sequence shard [c, ...] (chunked layout, module doc) -> the sequence [n c, ...] in order."""
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    c = x.shape[0]
    m = tp_stages(c)
    cm = c // m
    out = torch.empty((m, n * cm, *x.shape[1:]), dtype=x.dtype, device=x.device)
    for j in range(m):
        dist.all_gather_into_tensor(out[j], x[j * cm:(j + 1) * cm], group=group)
    return out.view(m * n * cm, *x.shape[1:])


def reduce_scatter_seq(x: torch.Tensor, group) -> torch.Tensor:
    """The sequence [S, ...] (partial sums) -> this rank's shard [S / n, ...] in the chunked layout."""
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    assert x.shape[0] % n == 0, "sequence length must be divisible by the tensor-parallel size"
    c = x.shape[0] // n
    m = tp_stages(c)
    cm = c // m
    out = torch.empty((c, *x.shape[1:]), dtype=x.dtype, device=x.device)
    for j in range(m):
        dist.reduce_scatter_tensor(out[j * cm:(j + 1) * cm], x[j * n * cm:(j + 1) * n * cm], group=group)
    return out


def shard_seq_local(x: torch.Tensor, rank: int, n: int) -> torch.Tensor:
    """This rank's chunked-layout shard of a full sequence (no communication)."""
    c = x.shape[0] // n
    m = tp_stages(c)
    cm = c // m
    return x.view(m, n, cm, *x.shape[1:])[:, rank].reshape(c, *x.shape[1:])


def unshard_seq_local(shards: list[torch.Tensor]) -> torch.Tensor:
    """Inverse of :func:`shard_seq_local` given every rank's shard (in rank order)."""
    n, c = len(shards), shards[0].shape[0]
    m = tp_stages(c)
    cm = c // m
    parts = [s.view(m, cm, *s.shape[1:]) for s in shards]
    return torch.stack(parts, 1).reshape(n * c, *shards[0].shape[1:])


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
    """Take this rank's sequence shard (chunked layout; no communication); bwd all-gathers."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return shard_seq_local(x, dist.get_rank(group), _ws(group)).contiguous()

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
# chunk-group sizes each staged projection ran with: "ag:<N>" / "rs:<N>" -> [chunks per GEMM, ...]
STAGE_PLANS: dict[str, list[int]] = {}


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


def gemm_groups(m: int, chunk_rows: int, ncols: int) -> list[tuple[int, int]]:
    """Consecutive chunk ranges [j0, j1) of the m chunks, one GEMM each: the smallest group size dividing m
    whose GEMM ([g * chunk_rows, ncols] output) has at least LLMT_TP_GEMM_TILES (default 1024) 256 x 256
    tiles."""
    want = max(1, int(os.environ.get("LLMT_TP_GEMM_TILES", "1024")))
    tiles = -(-chunk_rows // 256) * -(-ncols // 256)
    g = m
    for d in range(1, m + 1):
        if m % d == 0 and d * tiles >= want:
            g = d
            break
    return [(j, j + g) for j in range(0, m, g)]


def _plan(key: str, groups) -> None:
    STAGE_PLANS[key] = [j1 - j0 for j0, j1 in groups]


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
        per = n * cm  # sequence positions per chunk of the gathered input
        full = torch.empty((m * per, *tail), dtype=x.dtype, device=x.device)  # the gathered input, in order
        works = [dist.all_gather_into_tensor(full[j * per:(j + 1) * per], x[j * cm:(j + 1) * cm], group=group,
                                             async_op=True) for j in range(m)]
        y = torch.empty((m * per, *tail[:-1], w.shape[0]), dtype=x.dtype, device=x.device)
        rows = per * (x[0, ..., 0].numel())
        groups = gemm_groups(m, rows, w.shape[0])
        _plan(f"ag:{w.shape[0]}", groups)
        for j0, j1 in groups:
            for j in range(j0, j1):
                _tp_wait(works[j])
            mm_nt(_rows(full[j0 * per:j1 * per]), w, out=_rows(y[j0 * per:j1 * per]), bias=b)
        ctx.save_for_backward(full)
        ctx.w, ctx.group, ctx.has_bias, ctx.m, ctx.n = w, group, b is not None, m, n
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops.fused import _wgrad_mm, drop_dy_t, mm_nn, weight_t
        (full,) = ctx.saved_tensors
        w, group, m, n = ctx.w, ctx.group, ctx.m, ctx.n
        per = full.shape[0] // m
        cm = per // n
        tail = full.shape[1:]
        dy = dy.contiguous()
        dx = dw = db = None
        works, parts = [], []
        if ctx.needs_input_grad[0]:
            dx = torch.empty((m * cm, *tail), dtype=full.dtype, device=full.device)
            rows = per * (full[0, ..., 0].numel())
            wt = weight_t(w, m * rows)  # W^T once for every group's TN input-gradient GEMM (or None)
            for j0, j1 in gemm_groups(m, rows, w.shape[1]):
                # this group's input gradient is reduce-scattered chunk by chunk while the next one's is computed
                part = torch.empty(((j1 - j0) * per, *tail), dtype=full.dtype, device=full.device)
                mm_nn(_rows(dy[j0 * per:j1 * per]), w, out=_rows(part), wt=wt)
                for j in range(j0, j1):
                    works.append(dist.reduce_scatter_tensor(dx[j * cm:(j + 1) * cm],
                                                            part[(j - j0) * per:(j - j0 + 1) * per], group=group,
                                                            async_op=True))
                parts.append(part)
        if ctx.needs_input_grad[1]:
            # one weight-gradient GEMM over the whole gathered input, under the last reduce-scatters
            dw = _wgrad_mm(w, _rows(dy).t(), _rows(full))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _rows(dy).sum(0)
        for wk in works:
            _tp_wait(wk)
        del parts
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
        per = n * cm
        N = w.shape[0]
        y = torch.empty((c, *x.shape[1:-1], N), dtype=x.dtype, device=x.device)
        rows = per * (x[0, ..., 0].numel())
        groups = gemm_groups(m, rows, N)
        _plan(f"rs:{N}", groups)
        works, parts = [], []
        for j0, j1 in groups:  # a group's output rows are reduce-scattered while the next group's are computed
            part = torch.empty(((j1 - j0) * per, *x.shape[1:-1], N), dtype=x.dtype, device=x.device)
            mm_nt(_rows(x[j0 * per:j1 * per]), w, out=_rows(part))
            for j in range(j0, j1):
                works.append(dist.reduce_scatter_tensor(y[j * cm:(j + 1) * cm], part[(j - j0) * per:(j - j0 + 1) * per],
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
        from ..ops.fused import _wgrad_mm, drop_dy_t, mm_nn, weight_t
        (x,) = ctx.saved_tensors
        w, group, m = ctx.w, ctx.group, ctx.m
        n = _ws(group)
        dy = dy.contiguous()
        c = dy.shape[0]
        cm = c // m
        per = n * cm
        full = torch.empty((m * per, *dy.shape[1:]), dtype=dy.dtype, device=dy.device)  # the gathered dy, in order
        works = [dist.all_gather_into_tensor(full[j * per:(j + 1) * per], dy[j * cm:(j + 1) * cm], group=group,
                                             async_op=True) for j in range(m)]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
        rows = per * (x[0, ..., 0].numel())
        wt = weight_t(w, m * rows) if ctx.needs_input_grad[0] else None
        for j0, j1 in gemm_groups(m, rows, w.shape[1]):
            for j in range(j0, j1):
                _tp_wait(works[j])
            if ctx.needs_input_grad[0]:
                mm_nn(_rows(full[j0 * per:j1 * per]), w, out=_rows(dx[j0 * per:j1 * per]), wt=wt)
        if ctx.needs_input_grad[1]:
            dw = _wgrad_mm(w, _rows(full).t(), _rows(x))  # one weight-gradient GEMM
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
