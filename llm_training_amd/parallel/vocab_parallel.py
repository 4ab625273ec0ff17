"""Vocab-parallel fused linear + cross-entropy / token log-probs for tensor parallelism.

Reference: ``loss_parallel()`` around F.cross_entropy on vocab-sharded DTensor logits
(src/llm_training/lms/clm/clm.py:113-134) and the manual vocab-window gather + all_reduce of DPO/ORPO
log-probs (lms/dpo/dpo.py:89-108, lms/orpo/orpo.py:68-87) — SURVEY K10/P7.

Cross-entropy runs in ONE pass over the local logits, chunk by chunk: each TP rank multiplies its
(sequence-gathered) hidden-state chunk by its lm_head vocab shard, the HIP CE kernel produces the LOCAL
log-sum-exp and target logit per row, ONE small all-gather of the packed (lse, target) pairs of that chunk
(2 x rows fp32 per rank) gives the global values, and the same kernel then turns the chunk's logits into
d loss / d logits in place, which feed the chunk's dh rows and dW contribution right away: three GEMMs
per chunk (logits, dh, dW) and no second lm_head GEMM. dh is returned as a per-rank partial: the
sequence-gather that produced h reduce-scatters (sums) it on the way back.

Token log-probs (DPO / ORPO) need the upstream gradient, so their logits are either kept for the backward
(when the local logits of all rows fit ``keep_budget`` bytes) or recomputed there; the local (lse, target,
row sum) triples of all chunks meet in one all-gather.

When the vocabulary does not divide by the TP degree the last shard carries zero padding rows
(``ceil(V / tp)`` rows per rank); only the first ``n_valid`` rows of a shard are multiplied, so the
padding never enters the softmax normaliser and its gradient rows stay zero.
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist
from torch.autograd import Function

from ..ops.fused import _apply_weight_grad, dw_accumulator, dw_add_chunk, mm_nn, mm_nt, weight_t
from ..ops.native import lib, use_native

log = logging.getLogger("llm_training")


def _combine(stats: torch.Tensor, group, async_op: bool = False):
    """All-gather the [k, n] local row statistics of every TP rank -> [tp, k, n] (one collective); with
    ``async_op`` -> (result, work): the result is valid once the work completes."""
    n = dist.get_world_size(group)
    allv = torch.empty(n * stats.numel(), dtype=stats.dtype, device=stats.device)
    work = dist.all_gather_into_tensor(allv, stats.contiguous().view(-1), group=group, async_op=async_op)
    return (allv.view(n, *stats.shape), work) if async_op else allv.view(n, *stats.shape)


def _local_stats(lg, lab, v0, ignore_index, native, rowsum=None):
    """(lse_local, tgt_local) of logits lg [n, Vl] for global labels lab (+ local row sums into rowsum)."""
    if native:
        lse, tgt, _ = lib().cross_entropy_(lg, lab, v0, ignore_index, None, None, None, False, 0, rowsum)
        return lse, tgt
    lf = lg.float()
    lse = torch.logsumexp(lf, -1)
    loc = lab - v0
    hit = (lab != ignore_index) & (loc >= 0) & (loc < lg.shape[1])
    tgt = lf.gather(1, loc.clamp(0, lg.shape[1] - 1).unsqueeze(1)).squeeze(1) * hit
    if rowsum is not None:
        rowsum.copy_(lf.sum(-1))
    return lse, tgt


def _local_grad(lg, lab, v0, ignore_index, lse, coef_row, coef_scalar, native):
    """Overwrite lg with coef * (softmax_global - onehot)."""
    if native:
        lib().cross_entropy_(lg, lab, v0, ignore_index, lse, coef_row, coef_scalar, True, 0)
        return lg
    p = torch.exp(lg.float() - lse.unsqueeze(1))
    loc = lab - v0
    hit = (lab != ignore_index) & (loc >= 0) & (loc < lg.shape[1])
    p[hit, loc[hit]] -= 1.0
    c = (lab != ignore_index).float()
    if coef_row is not None:
        c = c * coef_row
    if coef_scalar is not None:
        c = c * coef_scalar
    lg.copy_((p * c.unsqueeze(1)).to(lg.dtype))
    return lg


class _VPFusedCE(Function):
    """Vocab-parallel fused linear + CE in one pass, memory bounded by two local logits chunks: per chunk
    the local logits, one all-gather of their (lse, target) rows, d loss / d logits in place, dh and dW.
    The chunks are software-pipelined: chunk i+1's logits GEMM and local statistics are issued while chunk
    i's all-gather is in flight, so the small collective does not stall the compute stream between GEMMs."""

    @staticmethod
    def forward(ctx, h, w_full, labels, v0, ignore_index, group, chunk, n_valid):
        native = use_native(h)
        N = h.shape[0]
        w = w_full[:n_valid]
        valid = labels != ignore_index
        inv_n = (1.0 / valid.sum().clamp(min=1).float()).reshape(1)
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dh = torch.empty_like(h) if need_h else None
        dw_full = dw_accumulator(w_full, N, chunk) if need_w else None
        dw = dw_full[:n_valid] if need_w else None
        if need_w and n_valid < w_full.shape[0]:
            dw_full[n_valid:].zero_()
        wt = weight_t(w, N) if need_h and native and N > chunk else None
        loss = torch.zeros((), device=h.device, dtype=torch.float32)

        def finish(s0, s1, lg, allv, work):
            nonlocal loss
            work.wait()
            lab = labels[s0:s1]
            lse = torch.logsumexp(allv[:, 0], dim=0)
            tgt = allv[:, 1].sum(0)  # the target logit lives in exactly one rank's vocabulary window
            loss += ((lse - tgt) * valid[s0:s1]).sum()
            if need_h or need_w:
                _local_grad(lg, lab, v0, ignore_index, lse.contiguous(), None, inv_n, native)
                if need_h:
                    mm_nn(lg, w, out=dh[s0:s1], wt=wt)
                if need_w:
                    dw_add_chunk(dw, lg, h[s0:s1], s0 == 0)

        pending = None
        for s0 in range(0, N, chunk):
            s1 = min(N, s0 + chunk)
            lg = mm_nt(h[s0:s1], w)
            lse_l, tgt_l = _local_stats(lg, labels[s0:s1], v0, ignore_index, native)
            allv, work = _combine(torch.stack([lse_l.float(), tgt_l.float()]), group, async_op=True)
            if pending is not None:
                finish(*pending)
            pending = (s0, s1, lg, allv, work)
            del lg
        if pending is not None:
            finish(*pending)
        del pending
        ctx.save_for_backward(*(t for t in (dh, dw_full) if t is not None))
        ctx.has = (need_h, need_w)
        ctx.w = w_full
        return loss * inv_n[0]

    @staticmethod
    def backward(ctx, g):
        saved = list(ctx.saved_tensors)
        need_h, need_w = ctx.has
        dh = saved.pop(0) if need_h else None
        dw = saved.pop(0) if need_w else None
        if dh is not None:
            dh = dh * g.to(dh.dtype)
        dwr = _apply_weight_grad(ctx.w, dw, g) if dw is not None else None
        return dh, dwr, None, None, None, None, None, None


class _VPLogps(Function):
    """Vocab-parallel token log-probs: local stats per chunk, one all-gather of every row's (lse, target,
    logit row sum), logits kept for the backward when they fit ``keep_budget`` bytes (else recomputed)."""

    @staticmethod
    def forward(ctx, h, w_full, labels, v0, ignore_index, group, chunk, n_valid, keep_budget):
        native = use_native(h)
        N = h.shape[0]
        w = w_full[:n_valid]
        need = N * n_valid * h.element_size()
        keep = ctx.needs_input_grad[0] and need <= _keep_budget(keep_budget, h)
        if ctx.needs_input_grad[0] and not keep and not _RECOMPUTE_LOGGED[0]:
            _RECOMPUTE_LOGGED[0] = True
            log.info("vocab-parallel log-probs: %.2f GiB of local logits exceed the keep budget; the backward "
                     "recomputes them (LLMT_LOGPS_KEEP_GIB)", need / 2 ** 30)
        stats = torch.zeros(3, N, device=h.device, dtype=torch.float32)
        kept = []
        for s0 in range(0, N, chunk):
            s1 = min(N, s0 + chunk)
            lg = mm_nt(h[s0:s1], w)
            lse, tgt = _local_stats(lg, labels[s0:s1], v0, ignore_index, native, stats[2, s0:s1])
            stats[0, s0:s1] = lse
            stats[1, s0:s1] = tgt
            if keep:
                kept.append(lg)
        allv = _combine(stats, group)
        lse = torch.logsumexp(allv[:, 0], dim=0)
        tgt, rowsum = allv[:, 1].sum(0), allv[:, 2].sum(0).contiguous()
        valid = labels != ignore_index
        ctx.save_for_backward(h, labels, lse)
        ctx.kept = kept if keep else None
        ctx.w = w_full
        ctx.cfg = (v0, ignore_index, chunk, n_valid)
        ctx.mark_non_differentiable(rowsum)
        return (tgt - lse) * valid, rowsum

    @staticmethod
    def backward(ctx, g, _g_rowsum=None):
        h, labels, lse = ctx.saved_tensors
        w_full = ctx.w
        v0, ignore_index, chunk, n_valid = ctx.cfg
        kept, ctx.kept = ctx.kept, None
        w = w_full[:n_valid]
        native = use_native(h)
        N = h.shape[0]
        dh = torch.empty_like(h)
        coef = (-g).float().contiguous()
        dw = dw_accumulator(w_full, N, chunk)
        if n_valid < w_full.shape[0]:
            dw[n_valid:].zero_()
        wt = weight_t(w, N) if native and N > chunk else None
        for i, s0 in enumerate(range(0, N, chunk)):
            s1 = min(N, s0 + chunk)
            lg = kept[i] if kept is not None else mm_nt(h[s0:s1], w)
            _local_grad(lg, labels[s0:s1], v0, ignore_index, lse[s0:s1].contiguous(), coef[s0:s1], None, native)
            mm_nn(lg, w, out=dh[s0:s1], wt=wt)
            dw_add_chunk(dw[:n_valid], lg, h[s0:s1], s0 == 0)
            if kept is not None:
                kept[i] = None
            del lg
        one = torch.ones((), device=dw.device, dtype=torch.float32)
        return dh, _apply_weight_grad(w_full, dw, one), None, None, None, None, None, None, None


def _n_valid(w_local, vocab_start, vocab_size):
    n = w_local.shape[0]
    return n if vocab_size is None else max(0, min(n, int(vocab_size) - int(vocab_start)))


def vocab_parallel_cross_entropy(h, w_local, labels, vocab_start, group, ignore_index=-100, chunk_size=8192,
                                 vocab_size: int | None = None):
    """``vocab_size``: the real vocabulary (rows of w_local past it are padding)."""
    h = h.reshape(-1, h.shape[-1]).contiguous()
    return _VPFusedCE.apply(h, w_local, labels.reshape(-1).contiguous(), int(vocab_start), ignore_index, group,
                            chunk_size, _n_valid(w_local, vocab_start, vocab_size))


# Local logits kept from the log-prob forward for its backward (no lm_head recompute) up to this many bytes.
# None = automatic: at most 8 GiB and at most a quarter of the device memory free when the forward runs, so
# a configuration that fits with the recompute path does not run out of HBM because of the kept logits.
# LLMT_LOGPS_KEEP_GIB=<float> pins the budget (0: always recompute).
_KEEP_ENV = os.environ.get("LLMT_LOGPS_KEEP_GIB", "auto").strip().lower()
LOGPS_KEEP_BYTES = [None if _KEEP_ENV in ("", "auto") else int(float(_KEEP_ENV) * 2 ** 30)]
_RECOMPUTE_LOGGED = [False]


def _keep_budget(budget, h: torch.Tensor) -> int:
    if budget is not None:
        return int(budget)
    cap = 8 << 30
    if h.is_cuda:
        # free in the driver PLUS what the caching allocator holds reserved but unused: after warm-up the
        # allocator owns most of HBM, and the driver's free alone would shrink the budget step after step
        free, _ = torch.cuda.mem_get_info(h.device)
        free += torch.cuda.memory_reserved(h.device) - torch.cuda.memory_allocated(h.device)
        cap = min(cap, free // 4)
    return cap


def vocab_parallel_token_logps(h, w_local, labels, vocab_start, group, ignore_index=-100, chunk_size=8192,
                               vocab_size: int | None = None, logit_sums: bool = False):
    shape = labels.shape
    h = h.reshape(-1, h.shape[-1]).contiguous()
    out, rs = _VPLogps.apply(h, w_local, labels.reshape(-1).contiguous(), int(vocab_start), ignore_index, group,
                             chunk_size, _n_valid(w_local, vocab_start, vocab_size), LOGPS_KEEP_BYTES[0])
    return (out.view(shape), rs.view(shape)) if logit_sums else out.view(shape)
