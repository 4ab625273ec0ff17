"""Model base class, config base and the causal-LM output record.

Reference: BaseModel / BaseModelConfig (src/llm_training/models/base_model/base_model.py:15-74,
base_model_config.py:8-21), HFCompatModel (models/hf_compat_model/hf_compat_model.py:29-119) and
CausalLMOutput (models/utils/modeling_outputs.py:12-14).

Differences by design: models are built TP-aware (each rank allocates only its shards: no meta-device
materialise-then-shard step), weights are initialised after construction from a per-shard seeded
generator (the reference never re-initialises meta-built FSDP weights), and the loss heads
consume the post-norm hidden states with the fused linear+CE kernel instead of materialising fp32
logits (reference clm.py:147).
"""
from __future__ import annotations

import json
import logging
import os
from dataclasses import dataclass
from pathlib import Path
from typing import Any, ClassVar

import torch
import torch.nn as nn
from pydantic import BaseModel as PydanticModel
from pydantic import ConfigDict, field_validator

from ..parallel.context import ParallelContext

logger = logging.getLogger("llm_training")


def to_dtype(v):
    if v is None or isinstance(v, torch.dtype):
        return v
    if isinstance(v, str):
        if v == "auto":
            return v
        name = v.replace("torch.", "")
        aliases = {"bf16": "bfloat16", "fp16": "float16", "half": "float16", "fp32": "float32", "float": "float32"}
        return getattr(torch, aliases.get(name, name))
    raise ValueError(f"cannot convert {v!r} to a torch dtype")


class BaseModelConfig(PydanticModel):
    model_config = ConfigDict(extra="allow", arbitrary_types_allowed=True, protected_namespaces=())

    pre_trained_weights: str | None = None
    # HF-compat fields (reference hf_compat_config.py:9-20)
    hf_path: str | None = None
    hf_tokenizer_path: str | None = None
    torch_dtype: Any = "auto"
    trust_remote_code: bool = False
    low_cpu_mem_usage: bool = True
    revision: str = "main"
    attn_implementation: str | None = None
    hf_extra_kwargs: dict[str, Any] = {}
    load_hf_weights: bool = True

    @field_validator("torch_dtype", mode="before")
    @classmethod
    def _dtype(cls, v):
        return to_dtype(v)

    def resolved_attn_implementation(self, device_type: str) -> str:
        """Default: our HIP flash kernels on GPU, eager on CPU (reference crashes on CPU)."""
        impl = self.attn_implementation
        if impl in (None, "flash_attention_2", "flash", "hip"):
            return "flash" if device_type == "cuda" else "eager"
        return impl


@dataclass
class CausalLMOutput:
    logits: torch.Tensor | None = None
    last_hidden_states: torch.Tensor | None = None


def load_hf_config_dict(path: str | os.PathLike) -> dict | None:
    """Read ``config.json`` of a LOCAL HF model dir (no network in this build)."""
    p = Path(path)
    f = p / "config.json" if p.is_dir() else p
    if f.exists():
        return json.loads(f.read_text())
    return None


class BaseModel(nn.Module):
    config_class: ClassVar[type[BaseModelConfig]] = BaseModelConfig
    hf_model_type: ClassVar[str | None] = None

    def __init__(self, config: BaseModelConfig, pc: ParallelContext | None = None):
        super().__init__()
        self.config = config
        self.pc = pc or ParallelContext.single()

    # ---- weights
    def init_weights(self, seed: int = 0):
        raise NotImplementedError

    def get_input_embeddings(self):
        raise NotImplementedError

    def get_output_embeddings(self):
        raise NotImplementedError

    # ---- FSDP-style unit boundaries for the ZeRO engine (one unit per decoder layer + the ends)
    def fsdp_units(self) -> list[nn.Module]:
        return [self]

    # ---- HF conversion (full, unsharded state dicts)
    @classmethod
    def convert_state_dict_from_hf(cls, sd: dict[str, torch.Tensor], config) -> dict[str, torch.Tensor]:
        raise NotImplementedError

    @classmethod
    def convert_state_dict_to_hf(cls, sd: dict[str, torch.Tensor], config) -> dict[str, torch.Tensor]:
        raise NotImplementedError

    def hf_config_dict(self) -> dict:
        raise NotImplementedError

    # ---- TP (un)sharding of full state dicts
    def shard_full_state_dict(self, full: dict[str, torch.Tensor]) -> dict[str, torch.Tensor]:
        return full

    def load_full_state_dict(self, full: dict[str, torch.Tensor], strict: bool = True):
        local = self.shard_full_state_dict(full)
        own = self.state_dict()
        missing = [k for k in own if k not in local]
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:8]}")
        with torch.no_grad():
            for k, v in own.items():
                if k in local:
                    if tuple(v.shape) != tuple(local[k].shape):
                        raise ValueError(f"shape mismatch for {k}: {tuple(v.shape)} vs {tuple(local[k].shape)}")
                    v.copy_(local[k].to(v.dtype))
        return missing
