"""Optimizer resolution: the fused HIP AdamW for the AdamW family, any other torch optimizer generically.

Reference: ``BaseOptimizerConfig.optimizer_class`` / ``optimizer_kwargs`` (src/llm_training/lms/
base_lm_config.py:13-17) and ``MasterWeightsOptimizer``, which wraps ANY torch optimizer over fp32
shadows of the half-precision parameters (src/llm_training/optim/master_weight_wrapper.py:17-80).

* ``torch.optim.AdamW`` / ``torch.optim.Adam`` (no L2 decay) / DeepSpeed ``FusedAdam`` with default
  flags run as ONE fused HIP AdamW launch per engine unit (fp32 master + moments, bf16 param written in
  the same pass, device-side clip scale). SURVEY K9.
* Every other torch optimizer — and AdamW / Adam with a flag the fused kernel does not implement
  (``amsgrad``, ``maximize``, L2 ``weight_decay`` for Adam) — runs as the class itself over each unit's
  flat fp32 master shard with the scaled fp32 gradient shard as ``.grad`` (generic path; its
  element-wise state is sharded and checkpointed like the Adam moments).
* DeepSpeed ``FusedAdam`` options that change the math and have no torch class to fall back on
  (``amsgrad``, ``bias_correction: false``, ``adam_w_mode: false`` with decay) raise: a config must not
  silently train a different optimizer.
"""
from __future__ import annotations

import inspect
from dataclasses import dataclass

FUSED = {
    "torch.optim.AdamW": "adamw",
    "torch.optim.adamw.AdamW": "adamw",
    "torch.optim.Adam": "adam",
    "torch.optim.adam.Adam": "adam",
    "llm_training_amd.optim.FusedAdamW": "adamw",
    "llm_training.optim.FusedAdamW": "adamw",
    "deepspeed.ops.adam.FusedAdam": "deepspeed",
    "deepspeed.ops.adam.fused_adam.FusedAdam": "deepspeed",
    # DeepSpeed's host Adam (used with optimizer offload): the same math; with an offloading strategy
    # the engine runs its own threaded host AdamW (csrc/cpu_adam.cpp), on the GPU the fused kernel
    "deepspeed.ops.adam.DeepSpeedCPUAdam": "deepspeed",
    "deepspeed.ops.adam.cpu_adam.DeepSpeedCPUAdam": "deepspeed",
}
SUPPORTED = FUSED  # backwards-compatible name

# kwargs that only select an implementation (no effect on the math)
_IMPL_ONLY = ("foreach", "fused", "capturable", "differentiable", "set_grad_none")


@dataclass
class FusedAdamW:
    lr: float = 1e-3
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.01


def _truthy(v) -> bool:
    return str(v).lower() in ("1", "true", "yes") if isinstance(v, str) else bool(v)


def resolve_optimizer(name: str, kwargs: dict) -> dict:
    """``{"kind": "fused", lr, betas, eps, weight_decay}`` for the fused AdamW, or
    ``{"kind": "generic", "cls": <optimizer class>, "kwargs": {...}, "lr": base lr}``."""
    kind = FUSED.get(name)
    kw = dict(kwargs)
    if kind == "deepspeed":
        if _truthy(kw.get("amsgrad", False)):
            raise ValueError("deepspeed FusedAdam does not support amsgrad (neither does the fused AdamW)")
        if not _truthy(kw.pop("bias_correction", True)):
            raise ValueError("FusedAdam(bias_correction=False) is not supported by the fused AdamW")
        adam_w = _truthy(kw.pop("adam_w_mode", kw.pop("adamw_mode", True)))  # FusedAdam / DeepSpeedCPUAdam
        kw.pop("fp32_optimizer_states", None)  # DeepSpeedCPUAdam: states are fp32 here anyway
        kw.pop("amsgrad", None)
        if not adam_w and float(kw.get("weight_decay", 0.0)) != 0.0:
            raise ValueError("FusedAdam(adam_w_mode=False) with L2 weight decay is not supported; use AdamW")
        kw.setdefault("weight_decay", 0.0)  # DeepSpeed FusedAdam default
        kind = "adamw"
    if kind in ("adamw", "adam"):
        for k in _IMPL_ONLY:
            kw.pop(k, None)
        generic = _truthy(kw.get("amsgrad", False)) or _truthy(kw.get("maximize", False)) or \
            (kind == "adam" and float(kw.get("weight_decay", 0.0)) != 0.0)
        if not generic:
            kw.pop("amsgrad", None)
            kw.pop("maximize", None)
            lr = float(kw.pop("lr", 1e-3))
            betas = tuple(float(b) for b in kw.pop("betas", (0.9, 0.999)))
            eps = float(kw.pop("eps", 1e-8))
            wd = float(kw.pop("weight_decay", 0.01 if kind == "adamw" else 0.0))
            if kw:
                raise ValueError(f"unsupported optimizer kwargs for {name}: {sorted(kw)}")
            return {"kind": "fused", "lr": lr, "betas": betas, "eps": eps, "weight_decay": wd}
        name = "torch.optim.AdamW" if kind == "adamw" else "torch.optim.Adam"
    return _generic(name, kw)


def _num(v):
    """YAML 1.1 reads ``3e-5`` as a string: numeric strings become floats (tuples element-wise)."""
    if isinstance(v, tuple):
        return tuple(_num(x) for x in v)
    if isinstance(v, str):
        try:
            return float(v)
        except ValueError:
            return v
    return v


def _generic(name: str, kw: dict) -> dict:
    from ..utils.imports import import_object
    try:
        cls = import_object(name) if isinstance(name, str) else name
    except (ImportError, AttributeError) as e:
        raise ValueError(f"optimizer class {name!r} cannot be imported: {e}") from e
    import torch
    if not (inspect.isclass(cls) and issubclass(cls, torch.optim.Optimizer)):
        raise ValueError(f"{name!r} is not a torch.optim.Optimizer subclass")
    sig = inspect.signature(cls.__init__)
    bad = [k for k in kw if k not in sig.parameters and not any(
        p.kind == inspect.Parameter.VAR_KEYWORD for p in sig.parameters.values())]
    if bad:
        raise ValueError(f"{name} got unknown optimizer kwargs {sorted(bad)}")
    kw = {k: _num(tuple(v) if isinstance(v, list) else v) for k, v in kw.items()}
    lr = kw.get("lr", sig.parameters["lr"].default if "lr" in sig.parameters else 1e-3)
    if lr is inspect.Parameter.empty:
        raise ValueError(f"{name} needs an explicit lr")
    kw["lr"] = float(lr)
    cls(  # validate the arguments once on a dummy tensor (bad values raise here, not at step 1)
        [torch.zeros(1)], **kw)
    return {"kind": "generic", "cls": cls, "kwargs": kw, "lr": float(lr), "name": name,
            "betas": tuple(kw.get("betas", (0.9, 0.999))), "eps": float(kw.get("eps", 1e-8)),
            "weight_decay": float(kw.get("weight_decay", 0.0))}


__all__ = ["FusedAdamW", "resolve_optimizer", "SUPPORTED", "FUSED"]
