"""Ops layer: fused HIP kernels (GPU) with torch reference fallbacks for CPU tensors only."""
from .fused import (cross_entropy, flash_attention, fused_linear_cross_entropy, linear, linear_token_logps,
                    rms_norm, rope_attention, swiglu, token_logps)
from .reference import apply_rope, rotate_half, shift_labels
from .rope_utils import ROPE_INIT_FUNCTIONS, RopeTables, compute_rope_tables

__all__ = [
    "cross_entropy", "flash_attention", "fused_linear_cross_entropy", "linear", "linear_token_logps", "rms_norm",
    "rope_attention", "swiglu", "token_logps", "apply_rope", "rotate_half", "shift_labels", "ROPE_INIT_FUNCTIONS",
    "RopeTables", "compute_rope_tables",
]
