"""Learning-rate schedules (closed form in the optimizer step index).

Same names, arguments and values as the reference (src/llm_training/lr_schedulers/: warmup.py:7-43,
cosine.py:7-26, constant.py:7-26, linear.py:5-39): linear warmup ``(step + 1) / W * lr`` then the inner
schedule counted from the end of warmup. Closed forms make resume exact from the step counter alone.
"""
from __future__ import annotations

import inspect
import math

from ..utils.imports import import_object


class LRSchedule:
    def __init__(self, base_lr: float):
        self.base_lr = base_lr
        self.last_step = 0

    def lr_at(self, step: int) -> float:
        raise NotImplementedError

    def get_lr(self) -> float:
        return self.lr_at(self.last_step)

    def step(self):
        self.last_step += 1

    def state_dict(self):
        return {"last_step": self.last_step, "base_lr": self.base_lr}

    def load_state_dict(self, st):
        self.last_step = int(st["last_step"])


class WarmupLR(LRSchedule):
    def __init__(self, base_lr: float, num_warmup_steps: int = 0):
        super().__init__(base_lr)
        self.num_warmup_steps = int(num_warmup_steps)

    def inner(self, e: int) -> float:
        return self.base_lr

    def lr_at(self, step: int) -> float:
        W = self.num_warmup_steps
        if step < W:
            return (step + 1) / W * self.base_lr
        return self.inner(step - W)


class ConstantWarmupLR(WarmupLR):
    def __init__(self, base_lr: float, factor: float = 1.0, total_iters: int = 0, num_warmup_steps: int = 0,
                 num_total_steps: int | None = None):
        super().__init__(base_lr, num_warmup_steps)
        self.factor, self.total_iters = float(factor), int(total_iters)

    def inner(self, e):
        return self.base_lr * (self.factor if e < self.total_iters else 1.0)


class CosineAnnealingWarmupLR(WarmupLR):
    def __init__(self, base_lr: float, num_warmup_steps: int, num_total_steps: int, min_lr: float = 0.0):
        super().__init__(base_lr, num_warmup_steps)
        self.num_total_steps, self.min_lr = int(num_total_steps), float(min_lr)

    def inner(self, e):
        T = max(1, self.num_total_steps - self.num_warmup_steps)
        return self.min_lr + (self.base_lr - self.min_lr) * (1 + math.cos(math.pi * e / T)) / 2


class LinearWarmupLR(LRSchedule):
    def __init__(self, base_lr: float, num_warmup_steps: int, num_total_steps: int, min_lr: float = 0.0):
        super().__init__(base_lr)
        self.num_warmup_steps, self.num_total_steps, self.min_lr = int(num_warmup_steps), int(num_total_steps), \
            float(min_lr)

    def lr_at(self, step):
        W, T = self.num_warmup_steps, self.num_total_steps
        if step < W:
            return (step + 1) / (W + 1) * self.base_lr
        factor = (T - step) / max(1, T - W)
        m = self.min_lr / self.base_lr if self.base_lr else 0.0
        return self.base_lr * ((1.0 - m) * factor + m)


def build_scheduler(cls, base_lr: float, kwargs: dict, num_total_steps: int) -> LRSchedule:
    if isinstance(cls, str):
        cls = import_object(cls)
    kw = dict(kwargs)
    params = inspect.signature(cls).parameters
    if "num_total_steps" in params and "num_total_steps" not in kw:
        kw["num_total_steps"] = num_total_steps  # reference base_lm.py:274-280
    return cls(base_lr, **kw)


__all__ = ["LRSchedule", "WarmupLR", "ConstantWarmupLR", "CosineAnnealingWarmupLR", "LinearWarmupLR",
           "build_scheduler"]
