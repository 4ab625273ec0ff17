"""Hugging Face ``datasets``-based data module.

Reference: src/llm_training/data/hf_based/hf_based_datamodule.py (load_dataset :36-53, seeded
train_test_split :55-59, save/load pre-processed :77-83, stable cache fingerprints for tokenizer
functions :89-176) and hf_based_datamodule_config.py:4-8.
"""
from __future__ import annotations

import hashlib
import json
import logging
import tempfile
from pathlib import Path
from typing import Any

from .base import BaseDataModule, BaseDataModuleConfig

logger = logging.getLogger("llm_training")


class HFBasedDataModuleConfig(BaseDataModuleConfig):
    dataset_kwargs: dict[str, Any] = {}
    num_proc: int | None = None
    cleanup_cache_files: bool = False
    enable_cache: bool = True


_TOK_HASH: dict[int, tuple[object, str]] = {}


def tokenizer_fingerprint(tok) -> str:
    """Stable identity of a tokenizer for ``datasets`` cache fingerprints: the bytes of every file
    ``save_pretrained`` writes (vocab, merges, special tokens, chat template, padding side), as the
    reference's hash_tokenizer (hf_based_datamodule.py:89-97). Memoised per tokenizer object."""
    if tok is None:
        return "none"
    hit = _TOK_HASH.get(id(tok))
    if hit is not None and hit[0] is tok:
        return hit[1]
    h = hashlib.sha256()
    try:
        with tempfile.TemporaryDirectory() as d:
            tok.save_pretrained(d)
            for p in sorted(Path(d).glob("*")):
                h.update(p.name.encode())
                h.update(p.read_bytes())
    except Exception:  # noqa: BLE001 — tokenizers that cannot serialise: hash their full observable state
        h.update(str(getattr(tok, "name_or_path", "")).encode())
        h.update(json.dumps(sorted(tok.get_vocab().items())).encode())
        h.update(json.dumps(getattr(tok, "special_tokens_map", {}), sort_keys=True, default=str).encode())
        h.update(str(getattr(tok, "chat_template", "")).encode())
        h.update(str(getattr(tok, "padding_side", "")).encode())
    digest = h.hexdigest()[:16]
    _TOK_HASH[id(tok)] = (tok, digest)
    return digest


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

    def prepare_data(self):
        """Warm the ``datasets`` cache: load + pre-process once (the Trainer calls this on one rank per
        node or per job, then every rank's ``setup`` hits the cache; reference :61-65)."""
        if self.config.pre_processed_data_path is None and self.config.enable_cache:
            self.pre_process_data(self.load_data())

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
