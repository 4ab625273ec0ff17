"""Collective-consistency checker (the reference has no race / ordering checks).

A rank that issues a different sequence of collectives than its peers (a data-dependent branch, a
unit skipped on one rank, mismatched shapes) hangs RCCL until the 30-minute process-group timeout
with no hint of where. With ``LLMT_CHECK_COLLECTIVES=1`` (or :func:`enable`) every collective issued
through ``torch.distributed`` is recorded per process group as (op, shape, dtype, group size); at
:meth:`CollectiveRecorder.verify` (the trainer calls it every ``LLMT_CHECK_COLLECTIVES_EVERY`` steps)
the ranks exchange a digest of their logs over a separate gloo group and, on mismatch, every rank
raises with the first diverging call of each rank — a desync becomes an immediate, located error.

Only metadata is recorded (no tensor data, no device sync), so the check is cheap enough for debug
runs at full scale.
"""
from __future__ import annotations

import hashlib
import logging
import os
import threading
from functools import wraps

import torch
import torch.distributed as dist

logger = logging.getLogger("llm_training")

_WRAPPED = ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "all_to_all_single", "broadcast",
            "all_gather", "reduce_scatter", "barrier", "reduce", "all_to_all")


def _describe(name: str, args, kwargs) -> tuple:
    tensors = []
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor):
            tensors.append((tuple(a.shape), str(a.dtype).replace("torch.", "")))
        elif isinstance(a, (list, tuple)) and a and all(isinstance(t, torch.Tensor) for t in a):
            tensors.append(("list", len(a), tuple(a[0].shape), str(a[0].dtype).replace("torch.", "")))
    group = kwargs.get("group")
    gsize = dist.get_world_size(group) if dist.is_initialized() else 1
    op = kwargs.get("op")
    return (name, tuple(tensors), gsize, str(op) if op is not None else "")


class CollectiveRecorder:
    """Records collectives issued through torch.distributed while installed."""

    def __init__(self):
        self.log: list[tuple] = []
        self._orig: dict[str, object] = {}
        self._lock = threading.Lock()
        self._gloo = None
        self.installed = False

    def install(self):
        if self.installed:
            return self
        for name in _WRAPPED:
            fn = getattr(dist, name, None)
            if fn is None:
                continue
            self._orig[name] = fn
            setattr(dist, name, self._wrap(name, fn))
        self.installed = True
        return self

    def uninstall(self):
        for name, fn in self._orig.items():
            setattr(dist, name, fn)
        self._orig.clear()
        self.installed = False

    def _wrap(self, name, fn):
        @wraps(fn)
        def inner(*args, **kwargs):
            with self._lock:
                self.log.append(_describe(name, args, kwargs))
            return fn(*args, **kwargs)
        return inner

    def digest(self, entries=None) -> str:
        h = hashlib.sha1()
        for e in (self.log if entries is None else entries):
            h.update(repr(e).encode())
        return h.hexdigest()

    def _group(self):
        if self._gloo is None:
            self._gloo = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD
        return self._gloo

    def verify(self, reset: bool = True) -> None:
        """All ranks compare their logs since the last verify; raise on any difference."""
        if not dist.is_initialized() or dist.get_world_size() == 1:
            if reset:
                self.log.clear()
            return
        with self._lock:
            entries = list(self.log)
            if reset:
                self.log.clear()
        ws = dist.get_world_size()
        mine = (len(entries), self.digest(entries))
        allv = [None] * ws
        gather = self._orig.get("all_gather_object", dist.all_gather_object)
        gather(allv, mine, group=self._group())
        if all(v == allv[0] for v in allv):
            return
        # mismatch: exchange the full logs (debug path only) and report the first divergence
        logs = [None] * ws
        gather(logs, entries, group=self._group())
        n = min(len(lg) for lg in logs)
        first = next((i for i in range(n) if any(lg[i] != logs[0][i] for lg in logs)), n)
        detail = "\n".join(f"  rank {r}: call #{first}: {lg[first] if first < len(lg) else '<no call>'} "
                           f"({len(lg)} calls)" for r, lg in enumerate(logs))
        raise RuntimeError(f"collective sequence differs across ranks at call #{first}:\n{detail}")


_RECORDER: CollectiveRecorder | None = None


def enable() -> CollectiveRecorder:
    global _RECORDER
    if _RECORDER is None:
        _RECORDER = CollectiveRecorder().install()
        logger.info("collective consistency checker enabled")
    return _RECORDER


def recorder() -> CollectiveRecorder | None:
    return _RECORDER


def maybe_enable_from_env() -> CollectiveRecorder | None:
    if os.environ.get("LLMT_CHECK_COLLECTIVES", "0") == "1":
        return enable()
    return None


def check_every() -> int:
    return max(1, int(os.environ.get("LLMT_CHECK_COLLECTIVES_EVERY", "1")))
