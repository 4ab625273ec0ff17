"""Plain-PyTorch reference ops: the CPU execution path and the numerics oracle for the HIP kernels.

Semantics follow the reference repo's torch ops:
- ``shift_labels``: src/llm_training/ops/cross_entropy_op.py:4-8
- ``rms_norm``: src/llm_training/ops/rms_norm_op.py:4-14
- ``rotate_half`` / ``apply_rope``: src/llm_training/ops/rope_op.py:4-20
- ``silu_mul`` / ``swiglu``: src/llm_training/ops/swiglu_op.py:5-29
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def shift_labels(labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    out = torch.empty_like(labels)
    out[..., :-1] = labels[..., 1:]
    out[..., -1] = ignore_index
    return out


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    dtype = x.dtype
    xf = x.float()
    xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return weight * xf.to(dtype)


def rotate_half(x: torch.Tensor) -> torch.Tensor:
    x1, x2 = x.chunk(2, dim=-1)
    return torch.cat((-x2, x1), dim=-1)


def apply_rope(q, k, cos, sin, unsqueeze_dim: int = 2):
    """q/k: [B, S, H, D]; cos/sin: [B, S, D] (full-width, HF layout)."""
    cos = cos.unsqueeze(unsqueeze_dim)
    sin = sin.unsqueeze(unsqueeze_dim)
    return (q * cos + rotate_half(q) * sin).to(q.dtype), (k * cos + rotate_half(k) * sin).to(k.dtype)


def silu_mul(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    return F.silu(gate) * up


def swiglu_fused(gate_up: torch.Tensor) -> torch.Tensor:
    g, u = gate_up.chunk(2, dim=-1)
    return silu_mul(g, u)


def attention(q, k, v, causal: bool = True, segment_ids=None, window: int = -1, scale: float | None = None):
    """Eager attention oracle. q: [B, S, Hq, D], k/v: [B, S, Hkv, D]; returns [B, S, Hq, D].

    A key is visible to a query iff seg[q] == seg[k] (if given), k <= q (causal), k >= q - window.
    """
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    rep = Hq // Hkv
    qh = q.transpose(1, 2).float()
    kh = k.transpose(1, 2).float().repeat_interleave(rep, dim=1)
    vh = v.transpose(1, 2).float().repeat_interleave(rep, dim=1)
    s = torch.matmul(qh, kh.transpose(-1, -2)) * scale
    mask = visibility_mask(S, q.device, causal, segment_ids, window, B)
    s = s.masked_fill(~mask[:, None], float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    o = torch.matmul(p, vh)
    return o.transpose(1, 2).to(q.dtype)


def dropout_keep_scale(seed: int, B: int, Hq: int, S: int, p: float, device=None) -> torch.Tensor:
    """[B, Hq, S(q), S(k)] fp32 multipliers (0 or 1 / (1 - p)) of the HIP kernels' attention-dropout mask:
    the same 32-bit counter hash of (seed, b * Hq + h, q, k) as csrc/flash_attn.hip drop_hash (uint32
    arithmetic emulated in int64, low 32 bits kept)."""
    M = 0xFFFFFFFF
    bh = torch.arange(B * Hq, device=device, dtype=torch.int64).view(B, Hq, 1, 1)
    q = torch.arange(S, device=device, dtype=torch.int64).view(1, 1, S, 1)
    k = torch.arange(S, device=device, dtype=torch.int64).view(1, 1, 1, S)
    x = (int(seed) ^ ((bh * 0x9E3779B1) & M)) & M
    x = x ^ ((q * 0x85EBCA6B) & M)
    x = ((x ^ (x >> 15)) * 0x2C1B3C6D) & M
    x = x ^ ((k * 0xC2B2AE35) & M)
    x = ((x ^ (x >> 12)) * 0x297A2D39) & M
    x = x ^ (x >> 15)
    t = p * 4294967296.0
    thresh = int(min(max(t, 1.0), 4294967295.0))
    scale = float(torch.tensor(1.0 / (1.0 - p), dtype=torch.float32))
    return (x >= thresh).float() * scale


def attention_dropout(q, k, v, causal=True, segment_ids=None, window=-1, scale=None, p=0.0, seed=0):
    """Eager attention with the kernels' dropout mask applied to the probabilities (oracle)."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    rep = Hq // Hkv
    qh = q.transpose(1, 2).float()
    kh = k.transpose(1, 2).float().repeat_interleave(rep, dim=1)
    vh = v.transpose(1, 2).float().repeat_interleave(rep, dim=1)
    s = torch.matmul(qh, kh.transpose(-1, -2)) * scale
    mask = visibility_mask(S, q.device, causal, segment_ids, window, B)
    s = s.masked_fill(~mask[:, None], float("-inf"))
    pr = torch.softmax(s, -1).nan_to_num(0.0) * dropout_keep_scale(seed, B, Hq, S, p, q.device)
    return torch.matmul(pr, vh).transpose(1, 2).to(q.dtype)


def visibility_mask(S, device, causal=True, segment_ids=None, window=-1, B=1):
    i = torch.arange(S, device=device)
    m = torch.ones(S, S, dtype=torch.bool, device=device)
    if causal:
        m &= i[None, :] <= i[:, None]
    if window is not None and window >= 0:
        m &= i[None, :] >= (i[:, None] - window)
    m = m[None].expand(B, S, S)
    if segment_ids is not None:
        m = m & (segment_ids[:, :, None] == segment_ids[:, None, :])
    return m


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100, reduction: str = "mean"):
    return F.cross_entropy(logits.float().flatten(0, -2), labels.flatten(), ignore_index=ignore_index,
                           reduction=reduction)


def token_logps(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Per-token log p(label); 0 where label == ignore_index."""
    lp = logits.float().log_softmax(-1)
    mask = labels != ignore_index
    safe = labels.masked_fill(~mask, 0)
    out = lp.gather(-1, safe.unsqueeze(-1)).squeeze(-1)
    return out * mask
