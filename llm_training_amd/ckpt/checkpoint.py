"""Sharded, resumable, reshard-able training checkpoints.

Reference behaviour: Lightning checkpoint dict with state_dict / optimizer / lr scheduler / loop
progress / config (src/llm_training/lightning/strategy/fsdp2/fsdp2_strategy.py:315-409,
callbacks/save_config_callback.py:42-44) and the resumable data loader (data/resumable_dataloader.py).

Layout of ``<dir>/``:
- ``meta.json``            step / epoch / batch_idx / consumed counters / scheduler / parallel layout /
                           the resolved YAML config (so ``convert-to-hf`` can rebuild the model)
- ``tp{t}.safetensors``    for every tensor-parallel rank t (written by data-parallel rank 0 of that
                           TP group): ``model.<param>`` (training dtype), ``master.<param>``,
                           ``exp_avg.<param>``, ``exp_avg_sq.<param>`` (fp32), keyed by parameter name
Keying by parameter name (not flat-buffer offset) makes the checkpoint independent of the
data-parallel size and ZeRO stage: a run saved at dp=8 / stage 3 resumes at dp=2 / stage 2. A change of
the tensor-parallel size is handled by merging the TP files with the model's shard rules.
"""
from __future__ import annotations

import json
import logging
import os
from pathlib import Path

import torch
import torch.distributed as dist
from safetensors.torch import load_file, save_file

logger = logging.getLogger("llm_training")


def _unit_full(engine, u, t: torch.Tensor) -> torch.Tensor:
    """All-gather a unit's DP shard into the full flat tensor (no-op when not sharded)."""
    dp = engine._udp(u)
    if engine._ustage(u) == 0 or dp == 1:
        return t
    full = torch.empty(u.numel, dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(full, t.contiguous(), group=engine.group)
    return full


def collect_state(trainer) -> dict[str, torch.Tensor]:
    """Per-parameter model / master / Adam state of this TP rank (full over DP), on CPU."""
    eng = trainer.engine
    model = trainer.lm.model
    names = {id(p): n for n, p in model.named_parameters()}
    out: dict[str, torch.Tensor] = {}
    with eng.full_params_context():
        for n, p in model.named_parameters():
            if not p.requires_grad:
                out["model." + n] = p.detach().cpu()
        for u in eng.units:
            fulls = {k: _unit_full(eng, u, getattr(u, k)) for k in ("master", "exp_avg", "exp_avg_sq")}
            pflat = u.pflat if u.pflat.untyped_storage().size() else None
            for p, o in zip(u.params, u.offsets):
                n = names[id(p)]
                sl = slice(o, o + p.numel())
                out["model." + n] = (pflat[sl] if pflat is not None else fulls["master"][sl].to(p.dtype)).view(
                    p.shape).cpu().clone()
                for k, f in fulls.items():
                    out[f"{k}.{n}"] = f[sl].view(p.shape).cpu().clone()
    return out


def save_checkpoint(trainer, path: str):
    pc = trainer.pc
    state = collect_state(trainer)
    if pc.dp_rank == 0:
        os.makedirs(path, exist_ok=True)
        save_file({k: v.contiguous() for k, v in state.items()}, os.path.join(path, f"tp{pc.tp_rank}.safetensors"))
    if pc.rank == 0:
        meta = {
            "format": "llm_training_amd/v1",
            "trainer": trainer.state.state_dict(),
            "scheduler": trainer.scheduler.state_dict() if trainer.scheduler else None,
            "optimizer_step": trainer.engine.step_count,
            "tp_size": pc.tp_size, "dp_size": pc.dp_size, "zero_stage": trainer.engine.stage,
            "config": trainer.config_dict,
            "model_class": f"{type(trainer.lm.model).__module__}.{type(trainer.lm.model).__qualname__}",
            "model_config": trainer.lm.model.config.model_dump(mode="json"),
        }
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1, default=str)
    if dist.is_initialized():
        dist.barrier()
    if pc.rank == 0:
        logger.info("saved checkpoint %s", path)


def read_meta(path: str) -> dict:
    with open(os.path.join(path, "meta.json")) as f:
        return json.load(f)


def load_tp_state(path: str, model, tp_rank: int, tp_size: int) -> dict[str, torch.Tensor]:
    """State of ``tp_rank`` under the current tp size (merging / re-sharding saved TP files if needed)."""
    meta = read_meta(path)
    saved_tp = int(meta.get("tp_size", 1))
    if saved_tp == tp_size:
        return load_file(os.path.join(path, f"tp{tp_rank}.safetensors"))
    parts = [load_file(os.path.join(path, f"tp{t}.safetensors")) for t in range(saved_tp)]
    return reshard_tp(parts, model, saved_tp)


def reshard_tp(parts: list[dict], model, saved_tp: int) -> dict[str, torch.Tensor]:
    from ..parallel import tensor_parallel as tpl
    full: dict[str, torch.Tensor] = {}
    for key in parts[0]:
        prefix, name = key.split(".", 1)
        kind, sizes = model._tp_rule(name) if hasattr(model, "_tp_rule") else ("rep", None)
        ts = [p[key] for p in parts]
        if saved_tp == 1 or kind == "rep":
            full[key] = ts[0]
        elif kind == "fused":
            full[key] = tpl.unshard_fused_rows(ts, sizes)
        elif kind == "cols":
            full[key] = torch.cat(ts, 1)
        else:
            full[key] = torch.cat(ts, 0)[: model.config.vocab_size]
    # re-shard for this rank with the model's own rules, per state kind
    out = {}
    for prefix in ("model", "master", "exp_avg", "exp_avg_sq"):
        sub = {k[len(prefix) + 1:]: v for k, v in full.items() if k.startswith(prefix + ".")}
        if sub:
            for k, v in model.shard_full_state_dict(sub).items():
                out[f"{prefix}.{k}"] = v
    return out


@torch.no_grad()
def load_checkpoint(trainer, path: str, load_optimizer: bool = True):
    if os.path.islink(path):
        path = os.path.join(os.path.dirname(path), os.readlink(path))
    pc, eng = trainer.pc, trainer.engine
    model = trainer.lm.model
    meta = read_meta(path)
    st = load_tp_state(path, model, pc.tp_rank, pc.tp_size)
    dev = next(model.parameters()).device
    params = dict(model.named_parameters())
    # parameters (frozen ones included)
    with eng.full_params_context():
        for n, p in params.items():
            k = "model." + n
            if k in st:
                p.data.copy_(st[k].to(dev, p.dtype))
    # optimizer state: fill full flats then take this rank's shard
    for u in eng.units:
        names = {id(p): n for n, p in params.items()}
        dp, stage = eng._udp(u), eng._ustage(u)
        r = pc.dp_rank if dp > 1 else 0
        sn = u.numel // dp
        for kind in ("master", "exp_avg", "exp_avg_sq"):
            full = torch.zeros(u.numel, dtype=torch.float32, device=dev)
            for p, o in zip(u.params, u.offsets):
                key = f"{kind}.{names[id(p)]}"
                if key in st and load_optimizer:
                    full[o:o + p.numel()] = st[key].reshape(-1).to(dev, torch.float32)
                elif kind == "master":
                    full[o:o + p.numel()] = st["model." + names[id(p)]].reshape(-1).to(dev, torch.float32)
            tgt = getattr(u, kind)
            tgt.copy_(full[r * sn:(r + 1) * sn] if stage >= 1 else full)
    eng.sync_params_from_master()
    if load_optimizer:
        eng.step_count = int(meta.get("optimizer_step", 0))
        trainer.state.load_state_dict(meta["trainer"])
        if trainer.scheduler is not None and meta.get("scheduler"):
            trainer.scheduler.load_state_dict(meta["scheduler"])
    if pc.rank == 0:
        logger.info("resumed from %s (step %d)", path, trainer.state.global_step)


def load_model_state_for_export(path: str) -> tuple[dict, dict[str, torch.Tensor]]:
    """(meta, full unsharded model state dict) from a checkpoint dir, without any process group."""
    meta = read_meta(path)
    tp = int(meta.get("tp_size", 1))
    parts = [load_file(os.path.join(path, f"tp{t}.safetensors")) for t in range(tp)]
    parts = [{k[6:]: v for k, v in p.items() if k.startswith("model.")} for p in parts]
    return meta, parts
