"""Checkpoint -> Hugging Face folder (reference scripts/convert_to_hf.py).

Accepts
* our sharded checkpoint directories (meta.json + per-rank shards, any TP / DP layout);
* checkpoints written by the reference framework (``--config_path`` = its YAML config):
  - DeepSpeed ZeRO-1/2/3 directories (``latest`` + ``<tag>/mp_rank_00_model_states.pt`` +
    ``zero_pp_rank_*_optim_states.pt``): the fp32 master weights are reassembled from every rank's
    flat partitions (the algorithm of DeepSpeed's zero_to_fp32, reference convert_to_hf.py:100-108);
  - FSDP2 / Fabric distributed checkpoints (``*.distcp`` + ``.metadata``): read with
    torch.distributed.checkpoint without a process group (reference :110-152);
  - plain state-dict files;
  their keys (the LightningModule's ``model.`` prefix over HF-style module names; ``ref_model.*`` of
  DPO is dropped) are mapped through the model class's HF conversion;
* plain state-dict files of our models (safetensors, or a torch file).
Torch pickles are read with ``weights_only=True`` only: a file that needs arbitrary unpickling is
refused with an explanation instead of executed. The model is rebuilt from the config stored in the
checkpoint (or ``--config_path``), TP shards are merged with the model's own shard rules, keys are
mapped to HF names and written with config.json (+ tokenizer when a local tokenizer is configured).
"""
from __future__ import annotations

import logging
import os
from pathlib import Path

import torch

logger = logging.getLogger("llm_training")


def _merge_tp(parts: list[dict], model_cls, config) -> dict:
    from ..parallel import tensor_parallel as tpl

    if len(parts) == 1:
        return parts[0]
    probe = model_cls.__new__(model_cls)
    probe.config = config
    full = {}
    for k in parts[0]:
        kind, sizes = model_cls._tp_rule(probe, k)
        ts = [p[k] for p in parts]
        if kind == "rep":
            full[k] = ts[0]
        elif kind == "fused":
            full[k] = tpl.unshard_fused_rows(ts, sizes)
        elif kind == "cols":
            full[k] = torch.cat(ts, 1)
        else:
            full[k] = torch.cat(ts, 0)[: config.vocab_size]
    return full


def _torch_load(path) -> dict:
    try:
        return torch.load(str(path), map_location="cpu", weights_only=True)
    except Exception as e:  # noqa: BLE001
        raise RuntimeError(f"{path}: cannot be read with torch.load(weights_only=True) ({e}); export it to a "
                           "plain tensor state dict first") from e


def is_deepspeed_checkpoint(p: Path) -> bool:
    return p.is_dir() and (p / "latest").is_file()


def is_dcp_checkpoint(p: Path) -> bool:
    return p.is_dir() and any(p.glob("*.distcp"))


def read_deepspeed_checkpoint(p: Path) -> dict[str, torch.Tensor]:
    """fp32 state dict of a DeepSpeed ZeRO-1/2/3 checkpoint directory (no DeepSpeed import)."""
    tag = (p / "latest").read_text().strip()
    d = p / tag
    model_files = sorted(d.glob("*mp_rank_00_model_states.pt"))
    if not model_files:
        raise FileNotFoundError(f"{d}: no *mp_rank_00_model_states.pt")
    ms = _torch_load(model_files[0])
    optim_files = sorted(d.glob("*zero_pp_rank_*_mp_rank_00_optim_states.pt"),
                         key=lambda f: int(f.name.split("zero_pp_rank_")[1].split("_")[0]))
    osds = [_torch_load(f)["optimizer_state_dict"] for f in optim_files]
    if not osds:
        raise FileNotFoundError(f"{d}: no zero_pp_rank_*_optim_states.pt")
    stage = int(osds[0]["zero_stage"])
    world = len(osds)
    shapes = ms["param_shapes"]
    shapes = shapes if isinstance(shapes, list) else [shapes]
    sd: dict[str, torch.Tensor] = {}
    module = ms.get("module") or {}
    for name in ms.get("buffer_names", []) or []:  # buffers are stored whole
        if name in module:
            sd[name] = module[name]
    if stage <= 2:
        for gi, group in enumerate(shapes):
            flat = torch.cat([o["single_partition_of_fp32_groups"][gi] for o in osds])
            off = 0
            for name, shape in group.items():
                n = int(torch.Size(shape).numel())
                sd[name] = flat[off:off + n].view(shape).clone()
                off += n
    else:
        flats = [torch.cat(list(o["fp32_flat_groups"])) for o in osds]
        off = 0
        for group in shapes:
            for name, shape in group.items():
                n = int(torch.Size(shape).numel())
                part = -(-n // world)  # each rank holds ceil(n / world) elements of every parameter
                sd[name] = torch.cat([f[off:off + part] for f in flats])[:n].view(shape).clone()
                off += part
    # frozen parameters: whole tensors in the module state dict (stage 1/2); at stage 3 every rank's
    # zero_pp_rank_<r>_mp_rank_00_model_states.pt holds its fragment (ceil(n / world) elements, padded),
    # merged in rank order as DeepSpeed's zero_to_fp32 does (_zero3_merge_frozen_params)
    frozen_shapes = ms.get("frozen_param_shapes") or {}
    if stage >= 3 and frozen_shapes:
        rank_files = sorted(d.glob("zero_pp_rank_*_mp_rank_00_model_states.pt"),
                            key=lambda f: int(f.name.split("zero_pp_rank_")[1].split("_")[0]))
        frags = [(_torch_load(f).get("frozen_param_fragments") or {}) for f in rank_files] or \
            [ms.get("frozen_param_fragments") or {}]
        for name, shape in frozen_shapes.items():
            n = int(torch.Size(shape).numel())
            pieces = [fr[name].reshape(-1) for fr in frags if name in fr]
            if pieces:
                sd[name] = torch.cat(pieces)[:n].view(shape).clone()
    else:
        for name, frag in (ms.get("frozen_param_fragments") or {}).items():
            sd.setdefault(name, frag)
    for name, t in module.items():
        if name not in sd and isinstance(t, torch.Tensor) and t.numel() > 0:
            sd[name] = t
    return sd


def read_dcp_checkpoint(p: Path) -> dict[str, torch.Tensor]:
    """Tensors of a torch.distributed.checkpoint directory, loaded in one process."""
    import torch.distributed.checkpoint as dcp
    from torch.distributed.checkpoint.metadata import TensorStorageMetadata

    reader = dcp.FileSystemReader(str(p))
    meta = reader.read_metadata()
    sd = {k: torch.empty(m.size, dtype=m.properties.dtype) for k, m in meta.state_dict_metadata.items()
          if isinstance(m, TensorStorageMetadata)}
    dcp.load(sd, storage_reader=reader, no_dist=True)
    return sd


def read_reference_checkpoint(p: Path) -> dict[str, torch.Tensor]:
    """Model weights of a reference-framework checkpoint with the LightningModule prefixes removed
    (HF-style module names, e.g. ``layers.0.self_attn.q_proj.weight``)."""
    if is_deepspeed_checkpoint(p):
        sd = read_deepspeed_checkpoint(p)
    elif is_dcp_checkpoint(p):
        sd = read_dcp_checkpoint(p)
    else:
        raw = _torch_load(p)
        sd = raw.get("state_dict", raw) if isinstance(raw, dict) else raw
    out = {}
    for k, v in sd.items():
        if not isinstance(v, torch.Tensor):
            continue
        k = k[len("state_dict."):] if k.startswith("state_dict.") else k
        if k.startswith("_forward_module."):
            k = k[len("_forward_module."):]
        if k.startswith("ref_model."):
            continue  # DPO's frozen reference model
        if k.startswith("model."):
            k = k[len("model."):]
        out[k] = v
    return out


def convert(checkpoint_path, output_dir=None, config_path=None, eos_token_id=None, dtype=None):
    import yaml

    from ..ckpt.checkpoint import load_model_state_for_export
    from ..ckpt.hf import load_safetensors_state_dict, save_hf_folder
    from ..models.base import to_dtype
    from ..utils.imports import import_object

    cp = Path(checkpoint_path)
    out = Path(output_dir) if output_dir else cp.parent / "hf" / cp.stem
    cfg = None
    foreign = False
    from ..ckpt.checkpoint import is_complete as _ours
    if (cp / "meta.json").exists() or (cp.is_file() and _ours(cp)):  # ours: shard dir or consolidated file
        meta, parts = load_model_state_for_export(str(cp))
        model_cls = import_object(meta["model_class"])
        mcfg = model_cls.config_class.model_validate({**meta["model_config"], "hf_path": None})
        cfg = meta.get("config")
        full = _merge_tp(parts, model_cls, mcfg)
    else:
        if config_path is None:
            raise ValueError("a checkpoint without meta.json needs --config_path")
        foreign = is_deepspeed_checkpoint(cp) or is_dcp_checkpoint(cp) or cp.suffix in (".ckpt", ".pt", ".pth")
        if foreign:
            full = read_reference_checkpoint(cp)  # HF-style names: mapped below
        else:
            sd = load_safetensors_state_dict(cp)
            full = {k[len("model."):] if k.startswith("model.") else k: v for k, v in sd.items()}
        cfg = None
    if config_path is not None:
        with open(config_path) as f:
            cfg = yaml.safe_load(f)
        from ..config.loader import expand_dotted
        cfg = expand_dotted(cfg)
        m = cfg["model"]["init_args"]["config"]["model"]
        model_cls = import_object(m["model_class"])
        mcfg = model_cls.config_class.model_validate(m.get("model_config") or {})
        if foreign:
            full = model_cls.convert_state_dict_from_hf(full, mcfg)
    if dtype is None:
        prec = ((cfg or {}).get("trainer") or {}).get("precision", "bf16-true")
        dtype = {"bf16-true": torch.bfloat16, "16-true": torch.float16, "32-true": torch.float32}.get(prec,
                                                                                                   torch.bfloat16)
    else:
        dtype = to_dtype(dtype)
    probe = model_cls.__new__(model_cls)
    probe.config = mcfg
    hf_cfg = model_cls.hf_config_dict(probe)
    if eos_token_id is not None:
        hf_cfg["eos_token_id"] = eos_token_id if isinstance(eos_token_id, (int, list)) else int(eos_token_id)
    tok = None
    try:
        tspec = cfg["data"]["init_args"]["config"]["tokenizer"] if cfg else None
        if tspec is not None:
            from ..config.loader import instantiate
            tok = instantiate(tspec)
    except Exception as e:  # noqa: BLE001 - tokenizer is optional for export
        logger.warning("tokenizer not exported: %r", e)
    save_hf_folder(model_cls, mcfg, full, str(out), dtype=dtype, tokenizer=tok, hf_config=hf_cfg)
    logger.info("wrote HF model to %s", out)
    return str(out)
