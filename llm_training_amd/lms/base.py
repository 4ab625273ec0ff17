"""Objective base class (the reference's BaseLightningModule, without Lightning).

Reference: src/llm_training/lms/base_lm.py (weight load/init decision :75-93, frozen modules :233-241,
configure_optimizers with auto-injected ``num_total_steps`` :269-288, grad-norm logging :290-300),
base_lm_config.py:13-43 (BaseOptimizerConfig / BaseLightningModuleConfig) and model_provider.py:9-22.

The objective owns the model(s) and the loss head; the Trainer owns the loop and the parallel engine.
Resume state is passed explicitly (no stack-frame inspection).
"""
from __future__ import annotations

import importlib
import inspect
import logging
from typing import Any, Callable

import torch
from pydantic import BaseModel as PydanticModel
from pydantic import ConfigDict, field_validator, model_validator

from ..models.base import BaseModel, to_dtype
from ..parallel.context import ParallelContext
from ..utils.imports import import_object

logger = logging.getLogger("llm_training")


class ModelProvider:
    """``model_class`` + ``model_config`` dict (validated with ``model_class.config_class``)."""

    def __init__(self, model_class: str | type, model_config: dict[str, Any] | None = None):
        self.model_class = import_object(model_class) if isinstance(model_class, str) else model_class
        self.model_config = self.model_class.config_class.model_validate(model_config or {})

    def __call__(self, pc: ParallelContext | None = None, dtype=None, device=None) -> BaseModel:
        return self.model_class(self.model_config, pc=pc, dtype=dtype, device=device)


class BaseOptimizerConfig(PydanticModel):
    model_config = ConfigDict(arbitrary_types_allowed=True, protected_namespaces=())

    optimizer_class: Any = "torch.optim.AdamW"
    optimizer_kwargs: dict[str, Any] = {}
    lr_scheduler_class: Any = "llm_training_amd.lr_schedulers.ConstantWarmupLR"
    lr_scheduler_kwargs: dict[str, Any] = {}


class BaseLMConfig(PydanticModel):
    model_config = ConfigDict(arbitrary_types_allowed=True, protected_namespaces=(), extra="forbid")

    model: Any = None
    init_weights: bool = False
    load_weights: bool = True
    pre_trained_weights: str | None = None
    optim: BaseOptimizerConfig | None = None
    frozen_modules: list[str] | None = None
    log_grad_norm: bool = True

    @field_validator("model", mode="before")
    @classmethod
    def _model(cls, v):
        if isinstance(v, dict) and "model_class" in v:
            return ModelProvider(v["model_class"], v.get("model_config"))
        return v


def build_model(spec, pc, dtype, device) -> BaseModel:
    if isinstance(spec, ModelProvider):
        return spec(pc=pc, dtype=dtype, device=device)
    if isinstance(spec, BaseModel):
        return spec.to(device)
    if callable(spec):
        return spec()
    raise TypeError(f"cannot build a model from {spec!r}")


class BaseLM:
    config_class = BaseLMConfig

    def __init__(self, config: BaseLMConfig | dict):
        if isinstance(config, dict):
            config = self.config_class.model_validate(config)
        self.config = config
        self.model: BaseModel | None = None
        self.training = True

    # ---------------------------------------------------------------- model setup
    def configure_model(self, pc: ParallelContext, device, dtype, seed: int = 0, resuming: bool = False):
        self.model = build_model(self.config.model, pc, dtype, device)
        self._load_or_init(self.model, seed, resuming)
        return self.model

    def _load_or_init(self, model: BaseModel, seed: int, resuming: bool):
        """Reference decision logic (base_lm.py:75-93): pre-trained weights unless resuming."""
        path = self.config.pre_trained_weights or getattr(model.config, "pre_trained_weights", None)
        hf_path = getattr(model.config, "hf_path", None)
        loaded = False
        if not resuming and self.config.load_weights:
            if path:
                from ..ckpt.hf import stream_load_weights
                own = set(model.state_dict().keys())
                stream_load_weights(model, path, lambda sd: {
                    k[len("model."):] if k.startswith("model.") and not k.startswith("model.layers") and
                    k[len("model."):] in own else k: v for k, v in sd.items()})
                loaded = True
            elif hf_path and getattr(model.config, "load_hf_weights", True):
                from ..ckpt.hf import load_hf_weights
                loaded = load_hf_weights(model, hf_path)
        if not loaded:
            model.init_weights(seed)

    def trainable_modules(self) -> list[torch.nn.Module]:
        return [self.model]

    # ---------------------------------------------------------------- optimisation config
    def optimizer_spec(self) -> dict:
        o = self.config.optim or BaseOptimizerConfig()
        cls = o.optimizer_class
        name = cls if isinstance(cls, str) else f"{cls.__module__}.{cls.__qualname__}"
        kw = dict(o.optimizer_kwargs)
        return {"name": name, "kwargs": kw}

    def build_lr_scheduler(self, base_lr: float, num_total_steps: int):
        from ..lr_schedulers import build_scheduler
        o = self.config.optim or BaseOptimizerConfig()
        return build_scheduler(o.lr_scheduler_class, base_lr, o.lr_scheduler_kwargs, num_total_steps)

    # ---------------------------------------------------------------- steps (override)
    def training_step(self, batch: dict, batch_idx: int):
        raise NotImplementedError

    def validation_step(self, batch: dict, batch_idx: int):
        raise NotImplementedError

    def train(self, mode: bool = True):
        self.training = mode
        for m in self.trainable_modules():
            m.train(mode)

    def eval(self):
        self.train(False)

    # ---------------------------------------------------------------- helpers shared by the heads
    @staticmethod
    def segment_ids_from_batch(batch: dict, key: str = "attention_mask"):
        """Packed segment ids for the attention kernel, or None when the mask is all ones.

        Collators attach ``<key>_trivial`` (computed on CPU in the loader worker) so this never
        synchronises with the GPU (reference checks ``0 in attention_mask`` on device).
        """
        m = batch.get(key)
        if m is None:
            return None
        triv = batch.get(key + "_trivial")
        if triv is None:
            return m
        return None if bool(triv) else m

    def hidden_and_head(self, model: BaseModel, input_ids, attention_mask_key, batch, embed_hook=None,
                        prefix: str = ""):
        seg = self.segment_ids_from_batch(batch, prefix + attention_mask_key)
        pos = batch.get(prefix + "position_ids")
        h = model.hidden_states(input_ids, pos, seg, embed_hook=embed_hook)
        return h

    def loss_from_hidden(self, model: BaseModel, h, labels_sb, ignore_index: int):
        """Mean token CE of the lm_head over seq-major hidden states h [S, B, H]."""
        from ..ops.fused import fused_linear_cross_entropy
        w = model.lm_head_weight()
        chunk = getattr(model.config, "loss_chunk_size", 8192)
        if model.pc.tp:
            from ..parallel.vocab_parallel import vocab_parallel_cross_entropy
            return vocab_parallel_cross_entropy(h, w, labels_sb, model.embed_tokens.v0, model.pc.tp_group,
                                                ignore_index, chunk, vocab_size=model.embed_tokens.vocab_size)
        return fused_linear_cross_entropy(h, w, labels_sb, ignore_index, chunk)

    def token_logps_from_hidden(self, model: BaseModel, h, labels_sb, ignore_index: int, logit_sums: bool = False):
        from ..ops.fused import linear_token_logps
        w = model.lm_head_weight()
        chunk = getattr(model.config, "loss_chunk_size", 8192)
        if model.pc.tp:
            from ..parallel.vocab_parallel import vocab_parallel_token_logps
            return vocab_parallel_token_logps(h, w, labels_sb, model.embed_tokens.v0, model.pc.tp_group,
                                              ignore_index, chunk, vocab_size=model.embed_tokens.vocab_size,
                                              logit_sums=logit_sums)
        return linear_token_logps(h, w, labels_sb, ignore_index, chunk, logit_sums=logit_sums)
