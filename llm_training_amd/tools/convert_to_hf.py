"""Checkpoint -> Hugging Face folder (reference scripts/convert_to_hf.py).

Accepts our sharded checkpoint directories (meta.json + tp*.safetensors, any TP size) and plain
state-dict files (safetensors or a torch file read with ``weights_only=True``). The model is rebuilt
from the config stored in the checkpoint (or ``--config_path``), TP shards are merged with the
model's own shard rules, keys are mapped to HF names and written with config.json (+ tokenizer when a
local tokenizer is configured).
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


def convert(checkpoint_path, output_dir=None, config_path=None, eos_token_id=None, dtype=None):
    import yaml

    from ..ckpt.checkpoint import load_model_state_for_export
    from ..ckpt.hf import load_safetensors_state_dict, save_hf_folder
    from ..models.base import to_dtype
    from ..utils.imports import import_object

    cp = Path(checkpoint_path)
    out = Path(output_dir) if output_dir else cp.parent / "hf" / cp.stem
    cfg = None
    if (cp / "meta.json").exists():
        meta, parts = load_model_state_for_export(str(cp))
        model_cls = import_object(meta["model_class"])
        mcfg = model_cls.config_class.model_validate({**meta["model_config"], "hf_path": None})
        cfg = meta.get("config")
        full = _merge_tp(parts, model_cls, mcfg)
    else:
        if config_path is None:
            raise ValueError("a plain state-dict checkpoint needs --config_path")
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
