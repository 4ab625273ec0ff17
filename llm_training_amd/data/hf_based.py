"""Hugging Face ``datasets``-based data module.

Reference: src/llm_training/data/hf_based/hf_based_datamodule.py (load_dataset :36-53, seeded
train_test_split :55-59, save/load pre-processed :77-83, stable cache fingerprints for tokenizer
functions :89-176) and hf_based_datamodule_config.py:4-8.
"""
from __future__ import annotations

import hashlib
import json
import logging
from typing import Any

from .base import BaseDataModule, BaseDataModuleConfig

logger = logging.getLogger("llm_training")


class HFBasedDataModuleConfig(BaseDataModuleConfig):
    dataset_kwargs: dict[str, Any] = {}
    num_proc: int | None = None
    cleanup_cache_files: bool = False
    enable_cache: bool = True


def tokenizer_fingerprint(tok) -> str:
    """Stable identity of a tokenizer for ``datasets`` cache fingerprints (vocab + special tokens + template)."""
    if tok is None:
        return "none"
    h = hashlib.sha256()
    h.update(str(getattr(tok, "name_or_path", "")).encode())
    try:
        h.update(json.dumps(sorted(tok.get_vocab().items())[:2000]).encode())
    except Exception:  # noqa: BLE001
        pass
    h.update(str(len(tok)).encode())
    h.update(json.dumps(getattr(tok, "special_tokens_map", {}), sort_keys=True, default=str).encode())
    h.update(str(getattr(tok, "chat_template", "")).encode())
    h.update(str(getattr(tok, "padding_side", "")).encode())
    return h.hexdigest()[:16]


class HFBasedDataModule(BaseDataModule):
    config_class = HFBasedDataModuleConfig

    def load_data(self):
        import datasets as hfd

        if not self.config.enable_cache:
            hfd.disable_caching()
        kw = dict(self.config.dataset_kwargs)
        ds = hfd.load_dataset(**kw)
        if isinstance(ds, hfd.Dataset):
            ds = hfd.DatasetDict({"train": ds})
        return ds

    def fingerprint(self, name: str, **parts) -> str:
        h = hashlib.sha256(name.encode())
        for k in sorted(parts):
            v = parts[k]
            h.update(k.encode())
            h.update((tokenizer_fingerprint(v) if hasattr(v, "get_vocab") else json.dumps(v, default=str)).encode())
        return h.hexdigest()[:32]

    def map_dataset_dict(self, dsd, fn, fn_kwargs: dict, remove_columns: bool = True, desc: str | None = None,
                         **kw):
        out = {}
        for split, d in dsd.items():
            fp = self.fingerprint(f"{type(self).__name__}.{fn.__name__}.{split}.{d._fingerprint}", **fn_kwargs)
            out[split] = d.map(fn, fn_kwargs=fn_kwargs, remove_columns=d.column_names if remove_columns else None,
                               num_proc=self.config.num_proc, new_fingerprint=fp, desc=desc, **kw)
        import datasets as hfd
        return hfd.DatasetDict(out)

    def split(self, ds):
        import datasets as hfd

        vs = self.config.validation_split
        if isinstance(ds, hfd.DatasetDict) and vs and "validation" not in ds and "train" in ds:
            parts = ds["train"].train_test_split(test_size=vs, seed=42)
            return {"train": parts["train"], "validation": parts["test"]}
        return dict(ds)

    def load_pre_processed_data(self, path):
        import datasets as hfd

        return hfd.load_from_disk(path)

    def save_pre_processed_data(self, path):
        import datasets as hfd

        hfd.DatasetDict(self.datasets).save_to_disk(path)
        if self.config.cleanup_cache_files:
            for d in self.datasets.values():
                d.cleanup_cache_files()
