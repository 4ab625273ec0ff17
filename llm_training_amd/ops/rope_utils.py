"""RoPE parameterisations and precomputed cos/sin tables.

Same family of scalings as the reference (src/llm_training/ops/rope_utils.py:33-296: default, linear,
dynamic NTK, YaRN, LongRoPE, llama3), re-expressed as: ``inv_freq(config) -> (inv_freq, attention_factor)``
and ONE precomputed fp32 half-width table pair ``cos/sin [max_positions, D/2]`` per model and device
(the reference rebuilds its cache in 4096-token steps and syncs with ``.item()``,
models/llama/llama_model.py:367-412). The HIP RoPE kernel gathers rows of these
tables by position id, so packed sequences with restarting positions need no special casing.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any

import torch


def _default(base: float, dim: int, max_pos: int, cfg: dict, seq_len: int | None):
    inv = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.int64).double() / dim))
    return inv, 1.0


def _linear(base, dim, max_pos, cfg, seq_len):
    inv, f = _default(base, dim, max_pos, cfg, seq_len)
    return inv / float(cfg["factor"]), f


def _dynamic(base, dim, max_pos, cfg, seq_len):
    factor = float(cfg["factor"])
    seq_len = max(seq_len or max_pos, max_pos)
    base = base * ((factor * seq_len / max_pos) - (factor - 1)) ** (dim / (dim - 2))
    return _default(base, dim, max_pos, cfg, seq_len)


def _yarn(base, dim, max_pos, cfg, seq_len):
    factor = float(cfg["factor"])
    orig = int(cfg.get("original_max_position_embeddings") or max_pos)
    attention_factor = cfg.get("attention_factor")
    mscale, mscale_all = cfg.get("mscale"), cfg.get("mscale_all_dim")

    def get_mscale(scale, m=1.0):
        return 1.0 if scale <= 1 else 0.1 * m * math.log(scale) + 1.0

    if attention_factor is None:
        if mscale and mscale_all:
            attention_factor = float(get_mscale(factor, mscale) / get_mscale(factor, mscale_all))
        else:
            attention_factor = get_mscale(factor)
    beta_fast = float(cfg.get("beta_fast") or 32)
    beta_slow = float(cfg.get("beta_slow") or 1)

    def corr_dim(n_rot):
        return (dim * math.log(orig / (n_rot * 2 * math.pi))) / (2 * math.log(base))

    low = max(math.floor(corr_dim(beta_fast)), 0)
    high = min(math.ceil(corr_dim(beta_slow)), dim - 1)
    if low == high:
        high += 0.001
    pos_freqs = base ** (torch.arange(0, dim, 2).double() / dim)
    inv_extra = 1.0 / pos_freqs
    inv_inter = 1.0 / (factor * pos_freqs)
    ramp = ((torch.arange(dim // 2).double() - low) / (high - low)).clamp(0, 1)
    extra_factor = 1 - ramp
    inv = inv_inter * (1 - extra_factor) + inv_extra * extra_factor
    return inv, attention_factor


def _longrope(base, dim, max_pos, cfg, seq_len):
    long_factor = cfg["long_factor"]
    short_factor = cfg["short_factor"]
    orig = int(cfg.get("original_max_position_embeddings") or max_pos)
    factor = cfg.get("factor")
    attention_factor = cfg.get("attention_factor")
    if factor is None:
        factor = max_pos / orig
    if attention_factor is None:
        attention_factor = 1.0 if factor <= 1.0 else math.sqrt(1 + math.log(factor) / math.log(orig))
    seq_len = seq_len if seq_len is not None else max_pos
    ext = torch.tensor(long_factor if seq_len > orig else short_factor, dtype=torch.float64)
    inv = 1.0 / (ext * base ** (torch.arange(0, dim, 2, dtype=torch.int64).double() / dim))
    return inv, attention_factor


def _llama3(base, dim, max_pos, cfg, seq_len):
    inv, f = _default(base, dim, max_pos, cfg, seq_len)
    factor = float(cfg["factor"])
    low = float(cfg["low_freq_factor"])
    high = float(cfg["high_freq_factor"])
    orig = float(cfg["original_max_position_embeddings"])
    low_wl = orig / low
    high_wl = orig / high
    wavelen = 2 * math.pi / inv
    out = torch.where(wavelen > low_wl, inv / factor, inv)
    smooth = (orig / wavelen - low) / (high - low)
    smoothed = (1 - smooth) * out / factor + smooth * out
    is_medium = (wavelen >= high_wl) & (wavelen <= low_wl)
    out = torch.where(is_medium, smoothed, out)
    return out, f


ROPE_INIT_FUNCTIONS = {
    "default": _default,
    "linear": _linear,
    "dynamic": _dynamic,
    "yarn": _yarn,
    "longrope": _longrope,
    "llama3": _llama3,
}


def rope_type(scaling: dict[str, Any] | None) -> str:
    if not scaling:
        return "default"
    t = scaling.get("rope_type", scaling.get("type", "default"))
    return "longrope" if t in ("su", "longrope") else t


def compute_rope_tables(head_dim: int, max_positions: int, base: float = 10000.0,
                        scaling: dict[str, Any] | None = None, max_position_embeddings: int | None = None,
                        partial_rotary_factor: float = 1.0, device=None, seq_len: int | None = None):
    """Return fp32 (cos, sin) of shape [max_positions, rot_dim/2] with the attention factor folded in.
    ``seq_len``: the sequence length the length-dependent scalings (dynamic NTK, LongRoPE) see; default
    ``max_positions``."""
    dim = int(head_dim * partial_rotary_factor)
    kind = rope_type(scaling)
    fn = ROPE_INIT_FUNCTIONS[kind]
    mpe = max_position_embeddings or max_positions
    inv, attn_factor = fn(float(base), dim, mpe, dict(scaling or {}), seq_len if seq_len is not None else max_positions)
    t = torch.arange(max_positions, dtype=torch.float64)
    freqs = torch.outer(t, inv)
    cos = (freqs.cos() * attn_factor).float()
    sin = (freqs.sin() * attn_factor).float()
    if device is not None:
        cos, sin = cos.to(device), sin.to(device)
    return cos.contiguous(), sin.contiguous()


@dataclass
class RopeTables:
    """Lazily (re)built per device; grows to the next multiple of 8192 positions when exceeded."""

    head_dim: int
    base: float = 10000.0
    scaling: dict | None = None
    max_position_embeddings: int = 4096

    def __post_init__(self):
        self._cache: dict[str, tuple[torch.Tensor, torch.Tensor, int]] = {}
        # dynamic NTK state, as the reference's rotary module keeps it (llama_model.py:312-341, 367-371): its
        # constructor builds the cache for max_position_embeddings rounded up to a multiple of 4096, so both the
        # initial and the "original" (reset) frequencies are NTK-scaled for that length whenever
        # max_position_embeddings is not a multiple of 4096 (e.g. 2048 -> 4096)
        self._dyn_orig = reference_rope_seq_len(self.max_position_embeddings)
        self._dyn_cached = self._dyn_orig  # the reference's max_seq_len_cached
        self._dyn_freq = self._dyn_orig  # the length the current frequencies were computed for

    @property
    def dynamic(self) -> bool:
        return rope_type(self.scaling) == "dynamic"

    def get(self, device, min_positions: int, ntk_positions: int | None = None):
        """cos / sin tables covering ``min_positions``. Dynamic NTK follows the reference's stateful rule
        (models/llama/llama_model.py:328-341, 367-371): the rescale length is ``ntk_positions`` (max
        position + 1, default ``min_positions``) rounded up to a multiple of 4096; it only grows while
        lengths stay at or above max_position_embeddings, and falls back to the original frequencies once a
        shorter batch comes."""
        n = max(min_positions, self.max_position_embeddings)
        n = (n + 8191) // 8192 * 8192
        ntk = None
        if self.dynamic:
            L = min_positions if ntk_positions is None else int(ntk_positions)
            orig = self.max_position_embeddings
            if not (orig <= L <= self._dyn_cached):
                R = reference_rope_seq_len(L)
                if R > self._dyn_cached:  # growth
                    self._dyn_cached = self._dyn_freq = R
                if R < orig and self._dyn_cached > orig:  # reset to the original frequencies
                    self._dyn_cached, self._dyn_freq = orig, self._dyn_orig
            ntk = self._dyn_freq
        key = (str(device), ntk)
        hit = self._cache.get(key)
        if hit is not None and hit[2] >= min_positions:
            return hit[0], hit[1]
        cos, sin = compute_rope_tables(self.head_dim, n, self.base, self.scaling, self.max_position_embeddings,
                                       device=device, seq_len=ntk)
        self._cache[key] = (cos, sin, n)
        return cos, sin


def reference_rope_seq_len(max_position_plus_one: int) -> int:
    """The sequence length the reference's rotary cache is built for: max(position_ids) + 1 rounded up to a
    multiple of 4096 (models/llama/llama_model.py:367-371, the same code in phi3_model.py)."""
    return -(-int(max_position_plus_one) // 4096) * 4096
