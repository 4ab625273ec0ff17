"""Preference-tuning data (DPO / ORPO): paired chosen / rejected conversations.

Reference: src/llm_training/data/preference_tuning/preference_tuning_datamodule.py (paired tokenisation
:29-92, drop overlong :94-104), preference_tuning_datacollator.py:12-69, config :15-31.
Input rows carry ``chosen`` and ``rejected`` message lists (optionally a shared ``prompt`` list that
is prepended to both).
"""
from __future__ import annotations

import enum
from typing import Any

import torch
from pydantic import field_validator

from .chat_templates import get_chat_template
from .hf_based import HFBasedDataModule, HFBasedDataModuleConfig
from .instruction_tuning import _pad


class OverlongHandlingMethod(str, enum.Enum):
    DROP = "drop"


class PreferenceTuningDataModuleConfig(HFBasedDataModuleConfig):
    tokenizer: Any = None
    chat_template: str | None = None
    max_length: int | None = None
    overlong_handling_method: OverlongHandlingMethod | str = OverlongHandlingMethod.DROP
    pad_to_multiple_of: int | None = None

    @field_validator("chat_template")
    @classmethod
    def _tmpl(cls, v):
        return get_chat_template(v)


def _encode(tokenizer, convs, chat_template):
    enc = tokenizer.apply_chat_template(convs, chat_template=chat_template, return_dict=True, tokenize=True,
                                        return_assistant_tokens_mask=True,
                                        tokenizer_kwargs={"return_attention_mask": False})
    ids = [list(x) for x in enc["input_ids"]]
    labels = [[t if a else -100 for t, a in zip(x, m)] for x, m in zip(ids, enc["assistant_masks"])]
    return ids, labels


def pt_pre_process_batch(batch: dict, tokenizer, chat_template, max_length) -> dict:
    prompts = batch.get("prompt") or [[] for _ in batch["chosen"]]
    chosen = [list(p) + list(c) for p, c in zip(prompts, batch["chosen"])]
    rejected = [list(p) + list(r) for p, r in zip(prompts, batch["rejected"])]
    ci, cl = _encode(tokenizer, chosen, chat_template)
    ri, rl = _encode(tokenizer, rejected, chat_template)
    out = {"chosen_input_ids": ci, "chosen_labels": cl, "chosen_length": [len(x) for x in ci],
           "rejected_input_ids": ri, "rejected_labels": rl, "rejected_length": [len(x) for x in ri]}
    if max_length is not None:
        keep = [i for i in range(len(ci)) if len(ci[i]) <= max_length and len(ri[i]) <= max_length]
        out = {k: [v[i] for i in keep] for k, v in out.items()}
    return out


class PreferenceTuningDataCollator:
    def __init__(self, config: PreferenceTuningDataModuleConfig):
        self.config = config
        if config.tokenizer is not None and config.tokenizer.pad_token_id is None:
            raise ValueError("`pad_token` is not specified. Please set it manually.")

    def __call__(self, batch: list[dict]) -> dict:
        tok = self.config.tokenizer
        left = getattr(tok, "padding_side", "right") == "left"
        m = self.config.pad_to_multiple_of
        out = {}
        for side in ("chosen", "rejected"):
            ids = [list(x[f"{side}_input_ids"]) for x in batch]
            labs = [list(x[f"{side}_labels"]) for x in batch]
            n = max(len(r) for r in ids)
            if m is not None:
                n = (n // m + 1) * m
            out[f"{side}_input_ids"] = _pad(ids, n, tok.pad_token_id, left)
            out[f"{side}_attention_mask"] = _pad([[1] * len(r) for r in ids], n, 0, left)
            out[f"{side}_labels"] = _pad(labs, n, -100, left)
            out[f"{side}_position_ids"] = torch.arange(n).unsqueeze(0)
        return out


class PreferenceTuningDataModule(HFBasedDataModule):
    config_class = PreferenceTuningDataModuleConfig

    def build_collator(self):
        return PreferenceTuningDataCollator(self.config)

    def pre_process_data(self, dsd):
        c = self.config
        return self.map_dataset_dict(dsd, pt_pre_process_batch,
                                     fn_kwargs=dict(tokenizer=c.tokenizer, chat_template=c.chat_template,
                                                    max_length=c.max_length),
                                     batched=True, batch_size=1000, desc="Pre-processing data")
