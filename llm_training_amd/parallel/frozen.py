"""Gather-only ZeRO-3 sharding of a frozen model (the DPO reference model).

Reference: the DPO reference model is parallelised with the same FSDP / TP plan as the policy
(src/llm_training/lms/dpo/dpo.py:59-71) — under FSDP2 its parameters are dp-sharded and all-gathered per
unit for each forward. Here the frozen model gets the engine's unit layout without any of the training
machinery: per unit ONE flat buffer of which each rank keeps only its 1/dp shard (no gradients, no
optimizer state, no fp32 master), an all-gather right before the unit's forward (the next decoder
layer's gather is issued on the communication stream while the current one computes) and the release
right after it. Decoder layers gather into a small ring of buffers of the largest layer's size; the
embedding and the final norm + lm_head unit (used by the loss head outside the norm's forward, and
tied weights) keep theirs until :meth:`release_all` after the reference log-probs are computed.

Resident bytes per rank: params / dp + the ring (2 decoder layers) while a forward runs.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from .engine import ALIGN, _hookable, _round_up

RING = 2


class _FUnit:
    def __init__(self, idx, module, params, offsets, shapes, numel, keep):
        self.idx, self.module, self.params, self.offsets, self.shapes = idx, module, params, offsets, shapes
        self.numel, self.keep = numel, keep
        self.shard: torch.Tensor | None = None
        self.full: torch.Tensor | None = None    # resident gathered buffer (keep units)
        self.slot = None
        self.gathered = False
        self.event = None


class FrozenShards:
    def __init__(self, model: nn.Module, group, dp_rank: int, dp_size: int, comm_stream=None):
        self.model, self.group, self.rank, self.dp = model, group, dp_rank, dp_size
        dev = next(model.parameters()).device
        self.device, self.cuda = dev, dev.type == "cuda"
        self.dtype = next(model.parameters()).dtype
        self.stream = comm_stream if self.cuda else None
        mods = model.fsdp_units() if hasattr(model, "fsdp_units") else [model]
        seen: set[int] = set()
        self.units: list[_FUnit] = []
        for i, m in enumerate(mods):
            keep = i == 0 or i == len(mods) - 1 or isinstance(m, tuple)
            if isinstance(m, tuple):
                m, srcs = m
                plist = [p for s in srcs for p in s.parameters()]
            else:
                plist = list(m.parameters())
            params = []
            for p in plist:
                if id(p) not in seen:
                    seen.add(id(p))
                    params.append(p)
            offs, n = [], 0
            for p in params:
                offs.append(n)
                n = _round_up(n + p.numel(), ALIGN)
            numel = _round_up(max(n, 1), ALIGN * dp_size)
            u = _FUnit(i, m, params, offs, [p.shape for p in params], numel, keep or not _hookable(m))
            full = torch.zeros(numel, device=dev, dtype=self.dtype)
            for p, o in zip(params, offs):
                full[o:o + p.numel()].copy_(p.detach().reshape(-1))
            sn = numel // dp_size
            u.shard = full[dp_rank * sn:(dp_rank + 1) * sn].clone()
            del full
            self._bind(u, None)
            self.units.append(u)
        self._ring = None
        for u in self.units:
            if not u.keep:
                u.module.register_forward_pre_hook(self._pre(u))
                u.module.register_forward_hook(self._post(u))
            elif u.module is not None and _hookable(u.module):
                u.module.register_forward_pre_hook(self._pre(u))

    # ---------------------------------------------------------------- buffers
    def _bind(self, u: _FUnit, flat: torch.Tensor | None):
        for p, o, shp in zip(u.params, u.offsets, u.shapes):
            p.data = flat[o:o + shp.numel()].view(shp) if flat is not None else u.shard.new_empty(0)

    def _slot(self):
        if self._ring is None:
            n = max((u.numel for u in self.units if not u.keep), default=0)
            self._ring = [{"buf": torch.empty(n, device=self.device, dtype=self.dtype), "owner": None, "event": None}
                          for _ in range(RING)]
        for sl in self._ring:
            if sl["owner"] is None:
                return sl
        return None

    def _gather(self, u: _FUnit, async_: bool = False):
        if u.gathered:
            if u.event is not None and not async_:
                torch.cuda.current_stream().wait_event(u.event)
                u.event = None
            return
        if u.keep:
            if u.full is None:
                u.full = torch.empty(u.numel, device=self.device, dtype=self.dtype)
            flat = u.full
        else:
            sl = self._slot()
            if sl is None:  # more layers in flight than the ring holds
                flat = torch.empty(u.numel, device=self.device, dtype=self.dtype)
            else:
                sl["owner"] = u.idx
                if sl["event"] is not None:
                    torch.cuda.current_stream().wait_event(sl["event"])
                    sl["event"] = None
                u.slot = sl
                flat = sl["buf"][:u.numel]
        if self.stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                dist.all_gather_into_tensor(flat, u.shard, group=self.group)
                done = torch.cuda.Event()
                done.record(self.stream)
            u.event = done
            if not async_:
                torch.cuda.current_stream().wait_event(done)
                u.event = None
        else:
            dist.all_gather_into_tensor(flat, u.shard, group=self.group)
        self._bind(u, flat)
        u.gathered = True

    def _release(self, u: _FUnit):
        if not u.gathered:
            return
        if u.event is not None:
            torch.cuda.current_stream().wait_event(u.event)
            u.event = None
        if u.slot is not None:
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream())
                u.slot["event"] = ev
            u.slot["owner"] = None
            u.slot = None
        self._bind(u, None)
        u.gathered = False

    # ---------------------------------------------------------------- hooks
    def _pre(self, u: _FUnit):
        def hook(mod, args):
            self._gather(u)
            if u.idx == 0:  # the tail unit is used by the loss head: gather it with the first unit
                self._gather(self.units[-1], async_=True)
            nxt = self.units[u.idx + 1] if u.idx + 1 < len(self.units) else None
            if nxt is not None and not nxt.keep:
                self._gather(nxt, async_=True)
            return None
        return hook

    def _post(self, u: _FUnit):
        def hook(mod, args, out):
            self._release(u)
            return None
        return hook

    def release_all(self):
        """Drop every gathered buffer (after the reference forward and its loss head): between two
        reference forwards a rank holds only its shards."""
        for u in self.units:
            self._release(u)
            if u.full is not None:
                if self.cuda:
                    u.full.record_stream(torch.cuda.current_stream())
                u.full = None

    def gather_all(self):
        for u in self.units:
            self._gather(u)

    def resident_bytes(self) -> int:
        """Bytes this rank holds permanently (the shards; gathered buffers are transient)."""
        return sum(u.shard.numel() * u.shard.element_size() for u in self.units)
