"""Pre-training data: tokenize (+BOS/EOS), stride truncation, naive or best-fit-decreasing packing,
per-source sampling, token tables, collator.

Reference: src/llm_training/data/pre_training/pre_training_datamodule.py (tokenize :30-59, truncate
:61-83, naive packing :85-142, best-fit bin packing :156-179, per-source BFD :181-211, sampling
:266-302, token tables :312-360), pre_training_datacollator.py:9-46, config :10-44.

Packing assignments come from the C++ packer (csrc/packing.cpp, O(n log n), same assignment as the
reference's O(n * bins) scan). Collator parity: by default the packed segment ids are discarded and
the mask is all ones (reference behaviour, SURVEY Q2: documents attend across boundaries);
``isolate_documents: true`` keeps the segment ids so the HIP attention kernel isolates documents
(no cross-contamination) and ``reset_position_ids: true`` restarts positions per document.
"""
from __future__ import annotations

import enum
import logging
import math
import random
from typing import Any

import torch
from pydantic import Field, ValidationInfo, field_validator

from .hf_based import HFBasedDataModule, HFBasedDataModuleConfig
from .packing import bfd_assign

logger = logging.getLogger("llm_training")


class PackingMethod(str, enum.Enum):
    NO_PACKING = "no_packing"
    NAIVE_PACKING = "naive_packing"
    BEST_FIT_BIN_PACKING = "best_fit_bin_packing"


class PreTrainingDataModuleConfig(HFBasedDataModuleConfig):
    tokenizer: Any = None
    max_length: int | None = None
    stride: int | None = None
    packing_method: PackingMethod | str = PackingMethod.NAIVE_PACKING
    sample_rate: dict[str, float] = Field(default_factory=dict)
    pre_processing_batch_size: int = 1000
    pad_to_multiple_of: int | None = None
    isolate_documents: bool = False
    reset_position_ids: bool = False

    @field_validator("packing_method")
    @classmethod
    def _pm(cls, v, info: ValidationInfo):
        v = PackingMethod(str(v.value if isinstance(v, PackingMethod) else v).lower())
        if v != PackingMethod.NO_PACKING and info.data.get("max_length") is None:
            raise ValueError("You must set `max_length` to pack data")
        return v

    @field_validator("stride")
    @classmethod
    def _stride(cls, v, info: ValidationInfo):
        ml = info.data.get("max_length")
        if v is None:
            return ml
        if ml is None:
            raise ValueError("You must also set `max_length` to use `stride`")
        if v > ml:
            raise ValueError("`stride` must be <= `max_length`")
        return v


# --------------------------------------------------------------------------- batch transforms (pure)
def tokenize_batch(batch: dict, tokenizer) -> dict:
    keep = [i for i, t in enumerate(batch["text"]) if t]
    texts = [batch["text"][i] for i in keep]
    sources = [batch["source"][i] for i in keep] if "source" in batch else [None] * len(keep)
    ids = tokenizer(texts, add_special_tokens=False, return_attention_mask=False,
                    return_token_type_ids=False)["input_ids"] if texts else []
    bos, eos = tokenizer.bos_token_id, tokenizer.eos_token_id
    out_ids = []
    for x in ids:
        x = list(x)
        if bos is not None:
            x.insert(0, bos)
        if eos is not None:
            x.append(eos)
        out_ids.append(x)
    return {"source": sources, "input_ids": out_ids, "length": [len(x) for x in out_ids]}


def truncate_batch(batch: dict, max_length: int, stride: int) -> dict:
    out = {"source": [], "input_ids": [], "length": []}
    for s, x in zip(batch["source"], batch["input_ids"]):
        for j in range(0, len(x), stride):
            piece = x[j:j + max_length]
            out["source"].append(s)
            out["input_ids"].append(piece)
            out["length"].append(len(piece))
    return out


def naive_pack_batch(batch: dict, max_length: int) -> dict:
    """Concatenate consecutive documents of the same source and cut into max_length rows.
    Segment ids number documents within a row (renumbered to start at 1)."""
    out = {"source": [], "input_ids": [], "attention_mask": [], "length": []}
    if not batch["input_ids"]:
        return out
    cur_src = batch["source"][0]
    cur_ids: list[int] = []
    cur_seg: list[int] = []

    def emit(src, ids, seg):
        off = seg[0] - 1
        out["source"].append(src)
        out["input_ids"].append(ids)
        out["attention_mask"].append([s - off for s in seg])
        out["length"].append(len(ids))

    for src, x in zip(batch["source"], batch["input_ids"]):
        if len(x) == max_length:
            emit(src, x, [1] * max_length)
            continue
        if src != cur_src:
            if cur_ids:
                emit(cur_src, cur_ids, cur_seg)
                cur_ids, cur_seg = [], []
            cur_src = src
        nxt = (cur_seg[-1] + 1) if cur_seg else 1
        cur_ids = cur_ids + x
        cur_seg = cur_seg + [nxt] * len(x)
        while len(cur_ids) >= max_length:
            emit(cur_src, cur_ids[:max_length], cur_seg[:max_length])
            cur_ids, cur_seg = cur_ids[max_length:], cur_seg[max_length:]
    if cur_ids:
        emit(cur_src, cur_ids, cur_seg)
    return out


def bfd_pack_batch(batch: dict, max_length: int) -> dict:
    """Best-fit-decreasing bin packing, per source (reference :181-211)."""
    out = {"input_ids": [], "attention_mask": [], "source": [], "length": []}
    by_src: dict[Any, list[int]] = {}
    for i, s in enumerate(batch["source"]):
        by_src.setdefault(s, []).append(i)
    for src, idx in by_src.items():
        # reference order: stable sort by length descending, then best fit over that order
        order = sorted(idx, key=lambda i: batch["length"][i], reverse=True)
        lengths = [batch["length"][i] for i in order]
        bins = bfd_assign(lengths, max_length)
        groups: dict[int, list[int]] = {}
        for pos, b in enumerate(bins):
            groups.setdefault(b, []).append(order[pos])
        for b in sorted(groups):
            ids, seg = [], []
            for d, i in enumerate(groups[b], start=1):
                ids += batch["input_ids"][i]
                seg += [d] * len(batch["input_ids"][i])
            out["input_ids"].append(ids)
            out["attention_mask"].append(seg)
            out["source"].append(src)
            out["length"].append(len(ids))
    return out


def pre_process_batch(batch: dict, tokenizer, max_length, stride, packing_method) -> dict:
    b = tokenize_batch(batch, tokenizer)
    if max_length is not None:
        b = truncate_batch(b, max_length, stride or max_length)
    pm = PackingMethod(packing_method)
    if pm == PackingMethod.NAIVE_PACKING:
        b = naive_pack_batch(b, max_length)
    elif pm == PackingMethod.BEST_FIT_BIN_PACKING:
        b = bfd_pack_batch(b, max_length)
    else:
        b["attention_mask"] = [[1] * n for n in b["length"]]
    return b


class PreTrainingDataCollator:
    def __init__(self, config: PreTrainingDataModuleConfig):
        self.config = config
        tok = config.tokenizer
        if tok is not None and tok.pad_token_id is None:
            raise ValueError("`pad_token` is not specified. Please set it manually.")

    def _target_len(self, n: int) -> int:
        m = self.config.pad_to_multiple_of
        if m is not None:
            n = (n // m + 1) * m  # reference rule: always at least one pad
        return n

    def __call__(self, batch: list[dict]) -> dict:
        tok = self.config.tokenizer
        left = getattr(tok, "padding_side", "right") == "left"
        n = self._target_len(max(len(x["input_ids"]) for x in batch))
        ids = torch.full((len(batch), n), -1, dtype=torch.long)
        seg = torch.zeros((len(batch), n), dtype=torch.long)
        pos = torch.zeros((len(batch), n), dtype=torch.long)
        for i, x in enumerate(batch):
            L = len(x["input_ids"])
            sl = slice(n - L, n) if left else slice(0, L)
            ids[i, sl] = torch.as_tensor(x["input_ids"], dtype=torch.long)
            s = torch.as_tensor(x.get("attention_mask") or [1] * L, dtype=torch.long)
            seg[i, sl] = s
            if self.config.reset_position_ids:
                starts = torch.ones(L, dtype=torch.long)
                starts[1:] = (s[1:] != s[:-1]).long()
                grp = torch.cumsum(starts, 0) - 1
                first = torch.nonzero(starts).flatten()
                pos[i, sl] = torch.arange(L) - first[grp]
        pad = ids == -1
        ids[pad] = tok.pad_token_id
        labels = ids.clone()
        if tok.bos_token_id is not None:
            labels[ids == tok.bos_token_id] = -100
        labels[pad] = -100
        if self.config.isolate_documents:
            mask = seg.masked_fill(pad, 0)
        else:
            mask = (~pad).long()
        out = {"input_ids": ids, "attention_mask": mask, "labels": labels,
               "position_ids": pos if self.config.reset_position_ids else torch.arange(n).unsqueeze(0)}
        out["attention_mask_trivial"] = bool((mask == 1).all())
        return out


class PreTrainingDataModule(HFBasedDataModule):
    config_class = PreTrainingDataModuleConfig

    def build_collator(self):
        return PreTrainingDataCollator(self.config)

    def pre_process_data(self, dsd):
        import datasets as hfd

        for k, d in list(dsd.items()):
            if "source" in d.column_names:
                dsd[k] = d.sort("source")
            else:
                dsd[k] = d.add_column("source", [None] * len(d))
        c = self.config
        feats = hfd.Features({"source": hfd.Value("string"), "input_ids": hfd.Sequence(hfd.Value("int32")),
                              "attention_mask": hfd.Sequence(hfd.Value("uint16")), "length": hfd.Value("uint32")})
        return self.map_dataset_dict(dsd, pre_process_batch,
                                     fn_kwargs=dict(tokenizer=c.tokenizer, max_length=c.max_length, stride=c.stride,
                                                    packing_method=PackingMethod(c.packing_method).value),
                                     batched=True, batch_size=c.pre_processing_batch_size, features=feats,
                                     desc="Pre-processing data")

    def sample_data(self, dataset):
        rates = self.config.sample_rate
        if all(v == 1.0 for v in rates.values()):
            return dataset
        src = dataset["source"]
        by: dict[Any, list[int]] = {}
        for i, s in enumerate(src):
            by.setdefault(s, []).append(i)
        r = random.Random(42)
        unused = dict(rates)
        picked: list[int] = []
        for s, idx in by.items():
            sr = rates.get(s, 1.0)
            unused.pop(s, None)
            frac, whole = math.modf(sr)
            picked += idx * int(whole)
            if frac > 0:
                picked += r.sample(idx, k=int(len(idx) * frac))
        if unused:
            logger.warning("sources in `sample_rate` not found in the dataset: %s", unused)
        return dataset.select(picked)

    def post_process_data(self, dsd):
        if "train" in dsd:
            dsd["train"] = self.sample_data(dsd["train"])
        return dsd

    @staticmethod
    def tokens_table(dsd) -> str:
        import pandas as pd
        from tabulate import tabulate

        rows = []
        for k, d in dsd.items():
            df = pd.DataFrame({"source": d["source"], "length": d["length"]})
            rows.append((k, "*", int(df["length"].sum())))
            for s, n in df.groupby("source", dropna=False)["length"].sum().items():
                rows.append((k, s, int(n)))
        rows.sort(key=lambda r: (r[0], str(r[1])))
        return tabulate(rows, headers=["Split", "Source", "Tokens"], tablefmt="orgtbl")

    def print_dataset_info(self):
        super().print_dataset_info()
        print("Original Tokens:\n")
        print(self.tokens_table(getattr(self, "pre_processed_datasets", self.datasets)))
        print("\nSampled Tokens:\n")
        print(self.tokens_table(self.datasets))
