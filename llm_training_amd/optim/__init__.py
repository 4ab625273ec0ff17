"""Optimizer specs. The update itself is the fused HIP AdamW of the parallel engine.

``FusedAdamW`` is what YAML ``optimizer_class`` names resolve to for ``torch.optim.AdamW``,
``torch.optim.Adam`` (with weight decay folded as L2-free AdamW only when decay is 0) and
DeepSpeed ``FusedAdam`` (reference examples). The engine keeps fp32 master weights
(reference MasterWeightsOptimizer, src/llm_training/optim/master_weight_wrapper.py).
"""
from __future__ import annotations

from dataclasses import dataclass

SUPPORTED = {
    "torch.optim.AdamW": "adamw",
    "torch.optim.adamw.AdamW": "adamw",
    "torch.optim.Adam": "adam",
    "torch.optim.adam.Adam": "adam",
    "llm_training_amd.optim.FusedAdamW": "adamw",
    "deepspeed.ops.adam.FusedAdam": "adamw",
    "deepspeed.ops.adam.fused_adam.FusedAdam": "adamw",
}


@dataclass
class FusedAdamW:
    lr: float = 1e-3
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.01


def resolve_optimizer(name: str, kwargs: dict) -> dict:
    """Map an optimizer class path + kwargs to the engine's AdamW hyper-parameters."""
    kind = SUPPORTED.get(name)
    if kind is None:
        raise ValueError(f"optimizer {name!r} is not supported by the fused engine (AdamW family only)")
    kw = dict(kwargs)
    lr = float(kw.pop("lr", 1e-3))
    betas = tuple(float(b) for b in kw.pop("betas", (0.9, 0.999)))
    eps = float(kw.pop("eps", 1e-8))
    default_wd = 0.01 if kind == "adamw" else 0.0
    if name.startswith("deepspeed"):
        default_wd = 0.0  # DeepSpeed FusedAdam default weight_decay
        kw.pop("adam_w_mode", None)
    wd = float(kw.pop("weight_decay", default_wd))
    if kind == "adam" and wd != 0.0:
        raise ValueError("torch.optim.Adam with L2 weight decay is not supported; use AdamW")
    for k in ("amsgrad", "foreach", "fused", "capturable", "maximize", "differentiable", "bias_correction"):
        kw.pop(k, None)
    if kw:
        raise ValueError(f"unsupported optimizer kwargs: {sorted(kw)}")
    return {"lr": lr, "betas": betas, "eps": eps, "weight_decay": wd}


__all__ = ["FusedAdamW", "resolve_optimizer", "SUPPORTED"]
