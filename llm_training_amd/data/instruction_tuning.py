"""Instruction-tuning data: chat template -> tokens + assistant-only labels, overlong handling,
group-by-length packing with segment ids, collator.

Reference: src/llm_training/data/instruction_tuning/instruction_tuning_datamodule.py (template +
assistant mask -> labels :30-78, drop/truncate :80-100, GROUP_BY_LENGTH packing :102-145),
instruction_tuning_datacollator.py:12-72 and the config :15-57.

Deliberate fixes: truncation truncates the EXAMPLE (the reference slices the batch list).
Parity default kept: positions run continuously through a packed row; set
``reset_position_ids: true`` for per-segment positions. Packed segment ids always reach the HIP
attention kernel, which isolates them (no cross-contamination, independent of padding — SURVEY Q4).
"""
from __future__ import annotations

import enum
import logging
import random
from typing import Any

import torch
from pydantic import ValidationInfo, field_validator

from .chat_templates import get_chat_template
from .hf_based import HFBasedDataModule, HFBasedDataModuleConfig
from .packing import group_by_length

logger = logging.getLogger("llm_training")


class OverlongHandlingMethod(str, enum.Enum):
    DROP = "drop"
    TRUNCATE = "truncate"


class PackingMethod(str, enum.Enum):
    NO_PACKING = "no_packing"
    GROUP_BY_LENGTH = "group_by_length"


class InstructionTuningDataModuleConfig(HFBasedDataModuleConfig):
    tokenizer: Any = None
    chat_template: str | None = None
    max_length: int | None = None
    overlong_handling_method: OverlongHandlingMethod | str = OverlongHandlingMethod.DROP
    packing_method: PackingMethod | str = PackingMethod.NO_PACKING
    pad_to_multiple_of: int | None = None
    add_default_system_prompt_rate: float | None = None
    default_system_prompt: str | None = None
    reset_position_ids: bool = False

    @field_validator("chat_template")
    @classmethod
    def _tmpl(cls, v):
        return get_chat_template(v)

    @field_validator("overlong_handling_method")
    @classmethod
    def _olh(cls, v):
        return OverlongHandlingMethod(str(v.value if isinstance(v, enum.Enum) else v).lower())

    @field_validator("packing_method")
    @classmethod
    def _pm(cls, v, info: ValidationInfo):
        v = PackingMethod(str(v.value if isinstance(v, enum.Enum) else v).lower())
        if v == PackingMethod.GROUP_BY_LENGTH and info.data.get("max_length") is None:
            raise ValueError("group_by_length packing needs `max_length`")
        return v


def chat_tokenize_batch(batch: dict, tokenizer, chat_template, default_system_prompt, add_default_system_prompt_rate,
                        seed: int = 42) -> dict:
    rng = random.Random(seed)
    convs = []
    for msgs in batch["messages"]:
        msgs = [dict(m) for m in msgs]
        if (default_system_prompt is not None and add_default_system_prompt_rate is not None
                and not any(m["role"] == "system" for m in msgs) and rng.random() < add_default_system_prompt_rate):
            msgs.insert(0, {"role": "system", "content": default_system_prompt})
        convs.append(msgs)
    enc = tokenizer.apply_chat_template(convs, chat_template=chat_template, return_dict=True, tokenize=True,
                                        return_assistant_tokens_mask=True,
                                        tokenizer_kwargs={"return_attention_mask": False})
    out = {"input_ids": [], "attention_mask": [], "labels": [], "length": []}
    for ids, am in zip(enc["input_ids"], enc["assistant_masks"]):
        ids = list(ids)
        out["input_ids"].append(ids)
        out["labels"].append([t if a else -100 for t, a in zip(ids, am)])
        out["attention_mask"].append([1] * len(ids))
        out["length"].append(len(ids))
    return out


def handle_overlong(batch: dict, max_length: int, method: str) -> dict:
    if OverlongHandlingMethod(method) == OverlongHandlingMethod.DROP:
        keep = [i for i, n in enumerate(batch["length"]) if n <= max_length]
        return {k: [v[i] for i in keep] for k, v in batch.items()}
    out = {k: list(v) for k, v in batch.items()}
    for i, n in enumerate(out["length"]):
        if n > max_length:
            for k in ("input_ids", "labels", "attention_mask"):
                out[k][i] = out[k][i][:max_length]
            out["length"][i] = max_length
    return out


def group_pack_batch(batch: dict, max_length: int) -> dict:
    out = {"input_ids": [], "attention_mask": [], "labels": [], "length": []}
    for grp in group_by_length(batch["length"], max_length):
        ids, seg, lab = [], [], []
        for j, i in enumerate(grp, start=1):
            ids += batch["input_ids"][i]
            lab += batch["labels"][i]
            seg += [j] * batch["length"][i]
        out["input_ids"].append(ids)
        out["attention_mask"].append(seg)
        out["labels"].append(lab)
        out["length"].append(len(ids))
    return out


def it_pre_process_batch(batch, tokenizer, chat_template, default_system_prompt, add_default_system_prompt_rate,
                         max_length, overlong_handling_method, packing_method):
    b = chat_tokenize_batch(batch, tokenizer, chat_template, default_system_prompt, add_default_system_prompt_rate)
    if max_length is not None:
        b = handle_overlong(b, max_length, overlong_handling_method)
    if PackingMethod(packing_method) == PackingMethod.GROUP_BY_LENGTH:
        b = group_pack_batch(b, max_length)
    return b


def _pad(rows: list[list], n: int, value, left: bool) -> torch.Tensor:
    out = torch.full((len(rows), n), value, dtype=torch.long)
    for i, r in enumerate(rows):
        if r:
            t = torch.as_tensor(r, dtype=torch.long)
            if left:
                out[i, n - len(r):] = t
            else:
                out[i, :len(r)] = t
    return out


def segment_positions(seg_row: list[int]) -> list[int]:
    pos, prev, p = [], None, 0
    for s in seg_row:
        p = p + 1 if s == prev else 0
        prev = s
        pos.append(p)
    return pos


class InstructionTuningDataCollator:
    def __init__(self, config: InstructionTuningDataModuleConfig):
        self.config = config
        tok = config.tokenizer
        if tok is not None and tok.pad_token_id is None:
            raise ValueError("`pad_token` is not specified. Please set it manually.")

    def target_len(self, n: int) -> int:
        m = self.config.pad_to_multiple_of
        return (n // m + 1) * m if m is not None else n

    def __call__(self, batch: list[dict]) -> dict:
        c, tok = self.config, self.config.tokenizer
        left = getattr(tok, "padding_side", "right") == "left"
        packed = PackingMethod(c.packing_method) == PackingMethod.GROUP_BY_LENGTH
        ids, masks, poss, labs = [], [], [], []
        for x in batch:
            n = len(x["input_ids"])
            ids.append(list(x["input_ids"]))
            labs.append(list(x["labels"]))
            seg = list(x["attention_mask"]) if packed else [1] * n
            masks.append(seg)
            poss.append(segment_positions(seg) if (packed and c.reset_position_ids) else list(range(n)))
        n = self.target_len(max(len(r) for r in ids))
        out = {"input_ids": _pad(ids, n, tok.pad_token_id, left), "attention_mask": _pad(masks, n, 0, left),
               "position_ids": _pad(poss, n, 0, left), "labels": _pad(labs, n, -100, left)}
        out["attention_mask_trivial"] = bool((out["attention_mask"] == 1).all())
        return out


class InstructionTuningDataModule(HFBasedDataModule):
    config_class = InstructionTuningDataModuleConfig

    def build_collator(self):
        return InstructionTuningDataCollator(self.config)

    def pre_process_data(self, dsd):
        c = self.config
        return self.map_dataset_dict(
            dsd, it_pre_process_batch,
            fn_kwargs=dict(tokenizer=c.tokenizer, chat_template=c.chat_template,
                           default_system_prompt=c.default_system_prompt,
                           add_default_system_prompt_rate=c.add_default_system_prompt_rate, max_length=c.max_length,
                           overlong_handling_method=OverlongHandlingMethod(c.overlong_handling_method).value,
                           packing_method=PackingMethod(c.packing_method).value),
            batched=True, batch_size=1000, desc="Pre-processing data")
