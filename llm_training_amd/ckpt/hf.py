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
import re
from collections import defaultdict
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


_LAYER = re.compile(r"(?:^|\.)layers\.(\d+)\.")


def _safetensors_files(p: Path) -> list[Path]:
    if p.is_file():
        return [p] if p.suffix == ".safetensors" else []
    idx = p / "model.safetensors.index.json"
    if idx.exists():
        return [p / f for f in sorted(set(json.loads(idx.read_text())["weight_map"].values()))]
    return sorted(p.glob("*.safetensors"))


def iter_weight_groups(path: str | os.PathLike):
    """Yield the checkpoint's tensors one decoder layer at a time (then everything outside the layers).

    safetensors files are memory-mapped and each group's tensors are materialised only while that group
    is loaded, so a rank's host memory holds one layer (~0.44 GB for Llama-3-8B) instead of the whole
    state dict (16 GB), and the ranks of a node share one page-cache copy of the files — the disk is read
    once per node however many ranks load (reference: rank-0 load + broadcast, lms/base_lm.py:147-191).
    ``pytorch_model*.bin`` checkpoints (no mmap format) are read whole with ``weights_only=True``.
    """
    from safetensors import safe_open

    p = Path(path)
    files = _safetensors_files(p)
    if not files:
        yield load_safetensors_state_dict(p)
        return
    handles = {f: safe_open(str(f), framework="pt", device="cpu") for f in files}
    groups: dict[int, list[tuple[Path, str]]] = defaultdict(list)
    for f, h in handles.items():
        for k in h.keys():
            m = _LAYER.search(k)
            groups[int(m.group(1)) if m else -1].append((f, k))
    for gid in sorted(groups, key=lambda g: (g < 0, g)):
        yield {k: handles[f].get_tensor(k) for f, k in groups[gid]}


def stream_load_weights(model, path: str | os.PathLike, convert=None) -> list[str]:
    """Load a (possibly sharded) checkpoint into ``model`` group by group (TP slicing per group);
    returns the model keys that no group provided."""
    own = set(model.state_dict().keys())
    seen: set[str] = set()
    for sd in iter_weight_groups(path):
        full = convert(sd) if convert is not None else sd
        model.load_full_state_dict(full, strict=False)
        seen.update(k for k in full if k in own)
        del sd, full
    return sorted(own - seen)


def load_hf_weights(model, hf_path: str) -> bool:
    """Load a local HF checkpoint dir into ``model`` (TP-sharded as needed). False if not available."""
    p = Path(hf_path)
    if not p.is_dir():
        logger.warning("hf_path %s is not a local directory; weights not loaded (random init)", hf_path)
        return False
    try:
        missing = stream_load_weights(model, p, lambda sd: type(model).convert_state_dict_from_hf(sd, model.config))
    except FileNotFoundError:
        logger.warning("no weights under %s; random init", hf_path)
        return False
    if missing:
        logger.warning("HF checkpoint %s did not provide %d tensors (kept initialised): %s", hf_path,
                       len(missing), missing[:8])
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
