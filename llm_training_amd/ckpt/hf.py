"""Hugging Face interop: load local HF weights into our models, export checkpoints as HF folders.

Reference: HFCompatModel.load_hf_model / convert_state_dict_{from,to}_hf / get_hf_model
(src/llm_training/models/hf_compat_model/hf_compat_model.py:48-119) and scripts/convert_to_hf.py
(DCP/DeepSpeed/plain checkpoint detection :100-161, re-instantiation from checkpoint['config']
:164-169, save_pretrained + tokenizer :68-97). Everything here reads LOCAL files only (no hub access
in this environment); weights are read with safetensors (or torch.load(weights_only=True)).
"""
from __future__ import annotations

import json
import logging
import os
from pathlib import Path

import torch
from safetensors.torch import load_file, save_file

logger = logging.getLogger("llm_training")


def load_safetensors_state_dict(path: str | os.PathLike) -> dict[str, torch.Tensor]:
    p = Path(path)
    if p.is_dir():
        idx = p / "model.safetensors.index.json"
        if idx.exists():
            files = sorted(set(json.loads(idx.read_text())["weight_map"].values()))
            sd = {}
            for f in files:
                sd.update(load_file(str(p / f)))
            return sd
        st = sorted(p.glob("*.safetensors"))
        if st:
            sd = {}
            for f in st:
                sd.update(load_file(str(f)))
            return sd
        binf = sorted(p.glob("pytorch_model*.bin"))
        if binf:
            sd = {}
            for f in binf:
                sd.update(torch.load(str(f), map_location="cpu", weights_only=True))
            return sd
        raise FileNotFoundError(f"no weights found in {p}")
    if p.suffix == ".safetensors":
        return load_file(str(p))
    return torch.load(str(p), map_location="cpu", weights_only=True)


def load_hf_weights(model, hf_path: str) -> bool:
    """Load a local HF checkpoint dir into ``model`` (TP-sharded as needed). False if not available."""
    p = Path(hf_path)
    if not p.is_dir():
        logger.warning("hf_path %s is not a local directory; weights not loaded (random init)", hf_path)
        return False
    try:
        sd = load_safetensors_state_dict(p)
    except FileNotFoundError:
        logger.warning("no weights under %s; random init", hf_path)
        return False
    full = type(model).convert_state_dict_from_hf(sd, model.config)
    model.load_full_state_dict(full, strict=False)
    logger.info("loaded HF weights from %s", hf_path)
    return True


def save_hf_folder(model_cls, config, full_sd: dict[str, torch.Tensor], out_dir: str, dtype=torch.bfloat16,
                   tokenizer=None, hf_config: dict | None = None, max_shard_bytes: int = 5 * 2 ** 30):
    """Write config.json + (sharded) model.safetensors in HF layout."""
    os.makedirs(out_dir, exist_ok=True)
    hf_sd = model_cls.convert_state_dict_to_hf(full_sd, config)
    hf_sd = {k: v.to(dtype).contiguous() for k, v in hf_sd.items()}
    # tied weights are stored once in safetensors
    if getattr(config, "tie_word_embeddings", False):
        hf_sd.pop("lm_head.weight", None)
    shards, cur, size = [], {}, 0
    for k, v in hf_sd.items():
        b = v.numel() * v.element_size()
        if cur and size + b > max_shard_bytes:
            shards.append(cur)
            cur, size = {}, 0
        cur[k] = v
        size += b
    shards.append(cur)
    if len(shards) == 1:
        save_file(shards[0], os.path.join(out_dir, "model.safetensors"), metadata={"format": "pt"})
    else:
        wm = {}
        for i, s in enumerate(shards):
            name = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
            save_file(s, os.path.join(out_dir, name), metadata={"format": "pt"})
            wm.update({k: name for k in s})
        with open(os.path.join(out_dir, "model.safetensors.index.json"), "w") as f:
            json.dump({"metadata": {"total_size": sum(v.numel() * v.element_size() for v in hf_sd.values())},
                       "weight_map": wm}, f, indent=1)
    cfg = dict(hf_config or {})
    cfg["torch_dtype"] = str(dtype).replace("torch.", "")
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(cfg, f, indent=1)
    if tokenizer is not None:
        tokenizer.save_pretrained(out_dir)
    return out_dir
