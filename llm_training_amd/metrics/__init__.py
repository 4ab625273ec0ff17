"""Training metrics with distributed reduction and checkpointable state.

Parity with the reference's torchmetrics-based metrics (src/llm_training/metrics/consumed_samples.py:5-20,
consumed_tokens.py:5-21, perplexity.py:8-39, metric.py in-place state load), without the torchmetrics
dependency: state tensors stay on the training device (no host sync per update), ``compute`` performs
one all-reduce over the metric's process group when asked for the global value, and
``load_state_dict`` copies into the existing tensors (so device placement and references survive a
resume, as the reference's ``Metric._load_from_state_dict`` override does).
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist


class Metric:
    higher_is_better: bool | None = None
    full_state_update: bool = False

    def __init__(self, process_group=None, device=None, sync_on_compute: bool = True):
        self.process_group = process_group
        self.sync_on_compute = sync_on_compute
        self._device = device
        self._defaults: dict[str, torch.Tensor] = {}
        self._reduce: dict[str, str] = {}
        self._persistent: dict[str, bool] = {}

    def add_state(self, name: str, default: torch.Tensor, dist_reduce_fx: str = "sum", persistent: bool = False):
        if dist_reduce_fx not in ("sum", "max", "min"):
            raise ValueError(f"unsupported reduction {dist_reduce_fx}")
        default = default.clone()
        if self._device is not None:
            default = default.to(self._device)
        self._defaults[name] = default.clone()
        self._reduce[name] = dist_reduce_fx
        self._persistent[name] = persistent
        setattr(self, name, default)

    def to(self, device):
        self._device = device
        for k in self._defaults:
            setattr(self, k, getattr(self, k).to(device))
            self._defaults[k] = self._defaults[k].to(device)
        return self

    def reset(self):
        for k, d in self._defaults.items():
            setattr(self, k, d.clone())

    def _synced(self) -> dict[str, torch.Tensor]:
        vals = {k: getattr(self, k) for k in self._defaults}
        if not (self.sync_on_compute and dist.is_available() and dist.is_initialized()):
            return vals
        if dist.get_world_size(self.process_group) == 1:
            return vals
        out = {}
        ops = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}
        for k, v in vals.items():
            t = v.detach().clone().to(torch.float64 if v.is_floating_point() else torch.int64)
            dist.all_reduce(t, op=ops[self._reduce[k]], group=self.process_group)
            out[k] = t.to(v.dtype)
        return out

    def update(self, *args, **kwargs):  # pragma: no cover - abstract
        raise NotImplementedError

    def _compute(self, state: dict[str, torch.Tensor]) -> torch.Tensor:  # pragma: no cover - abstract
        raise NotImplementedError

    def compute(self) -> torch.Tensor:
        return self._compute(self._synced())

    def __call__(self, *args, **kwargs):
        self.update(*args, **kwargs)
        return self

    def state_dict(self, prefix: str = "") -> dict[str, torch.Tensor]:
        return {prefix + k: getattr(self, k).detach().clone() for k in self._defaults if self._persistent[k]}

    def load_state_dict(self, sd: dict, prefix: str = "", strict: bool = False):
        for k in self._defaults:
            name = prefix + k
            if name in sd:
                getattr(self, k).copy_(torch.as_tensor(sd[name]))
            elif strict and self._persistent[k]:
                raise KeyError(name)


class ConsumedSamples(Metric):
    """Number of samples seen (persistent across resume)."""
    higher_is_better = True

    def __init__(self, **kw):
        super().__init__(**kw)
        self.add_state("n", torch.tensor(0), dist_reduce_fx="sum", persistent=True)

    def update(self, target: torch.Tensor) -> None:
        self.n += target.size(0)

    def _compute(self, st):
        return st["n"]


class ConsumedTokens(Metric):
    """Number of supervised tokens seen (labels != ignore_index), persistent across resume."""
    higher_is_better = True

    def __init__(self, ignore_index: int = -100, **kw):
        super().__init__(**kw)
        self.ignore_index = ignore_index
        self.add_state("n", torch.tensor(0), dist_reduce_fx="sum", persistent=True)

    def update(self, target: torch.Tensor) -> None:
        self.n = self.n + target.ne(self.ignore_index).sum().to(self.n.device)

    def _compute(self, st):
        return st["n"]


class Perplexity(Metric):
    """exp(mean NLL). ``update`` takes a scalar mean loss (counted as one observation, the reference's
    scalar path) or (log-probs [..., V], target [...]) for a token-level update."""
    higher_is_better = False

    def __init__(self, ignore_index: int | None = None, **kw):
        super().__init__(**kw)
        if ignore_index is not None and not isinstance(ignore_index, int):
            raise ValueError(f"ignore_index must be None or int, got {ignore_index!r}")
        self.ignore_index = ignore_index
        self.add_state("total_log_probs", torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("count", torch.tensor(0.0), dist_reduce_fx="sum")

    def update(self, preds_or_loss: torch.Tensor, target: torch.Tensor | None = None) -> None:
        if preds_or_loss.dim() == 0:
            self.total_log_probs = self.total_log_probs + preds_or_loss.detach().float().to(self.count.device)
            self.count = self.count + 1
            return
        if target is None:
            raise ValueError("token-level perplexity needs targets")
        probs = torch.softmax(preds_or_loss.detach().float().reshape(-1, preds_or_loss.shape[-1]), dim=-1)
        tgt = target.reshape(-1)
        mask = torch.ones_like(tgt, dtype=torch.bool) if self.ignore_index is None else tgt.ne(self.ignore_index)
        tgt = torch.where(mask, tgt, torch.zeros_like(tgt))
        p = probs.gather(1, tgt.unsqueeze(1)).squeeze(1)
        self.total_log_probs = self.total_log_probs + (-torch.log(p[mask])).sum().to(self.count.device)
        self.count = self.count + mask.sum().to(self.count.device)

    def _compute(self, st):
        return torch.exp(st["total_log_probs"] / st["count"].clamp(min=1))


__all__ = ["Metric", "ConsumedSamples", "ConsumedTokens", "Perplexity"]
