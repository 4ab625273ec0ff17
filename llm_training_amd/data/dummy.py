"""Synthetic token data (the benchmark / long-context input).

Reference: src/llm_training/data/dummy/ (dataset :24-33 deterministic by base_seed + index, seed
broadcast from rank 0 dummy_datamodule.py:13-17, num_samples xor num_tokens dummy_datamodule_config.py).
"""
from __future__ import annotations

import math
import random

import torch
import torch.distributed as dist
from pydantic import Field, ValidationInfo, field_validator
from torch.utils.data import Dataset

from .base import BaseDataModule, BaseDataModuleConfig


class DummyDataModuleConfig(BaseDataModuleConfig):
    vocab_size: int
    max_length: int
    num_samples: int | None = None
    num_tokens: int | None = None
    base_seed: int | None = Field(None, validate_default=True)

    @field_validator("num_tokens")
    @classmethod
    def _excl(cls, v, info: ValidationInfo):
        if v is not None and info.data.get("num_samples") is not None:
            raise ValueError("num_samples and num_tokens are mutually exclusive")
        return v

    @field_validator("base_seed")
    @classmethod
    def _seed(cls, v):
        return random.randrange(0, 999999) if v is None else v


class DummyDataset(Dataset):
    def __init__(self, cfg: DummyDataModuleConfig):
        self.cfg = cfg
        if cfg.num_samples is not None:
            self.n = cfg.num_samples
        elif cfg.num_tokens is not None:
            self.n = math.ceil(cfg.num_tokens / cfg.max_length)
        else:
            raise ValueError("one of num_samples / num_tokens is required")

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.cfg.base_seed + int(i))
        ids = torch.randint(0, self.cfg.vocab_size, (self.cfg.max_length,), generator=g)
        return {"input_ids": ids, "attention_mask": torch.ones_like(ids), "position_ids": torch.arange(ids.numel()),
                "labels": ids}


class DummyDataModule(BaseDataModule):
    config_class = DummyDataModuleConfig

    def setup(self, stage=None):
        if dist.is_initialized() and dist.get_world_size() > 1:
            obj = [self.config.base_seed]
            dist.broadcast_object_list(obj, src=0)
            self.config.base_seed = obj[0]
        self.datasets = self.split(DummyDataset(self.config))
