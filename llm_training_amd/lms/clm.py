"""Causal-LM objective (pre-training and instruction tuning), with optional NEFTune.

Reference: src/llm_training/lms/clm/clm.py (NEFTune hook :45-82, loss :113-134, training_step
:136-168, validation_step :170-185) and clm_config.py:5-9.

The loss is the fused lm_head + cross-entropy (HIP kernel; vocab-parallel under TP) on the post-norm
hidden states, so the fp32 [T, V] logits copy of the reference (clm.py:147) never exists. Metrics are
device tensors; the trainer reads them only at logging steps (no per-step host sync).
"""
from __future__ import annotations

import torch

from ..ops.reference import shift_labels
from .base import BaseLM, BaseLMConfig


class CLMConfig(BaseLMConfig):
    ignore_index: int = -100
    neftune_alpha: float | None = None
    log_perplexity: bool = True


class CLM(BaseLM):
    config_class = CLMConfig

    def _neftune_hook(self, attention_mask: torch.Tensor):
        """NEFTune noise (reference clm.py:45-78): uniform(-1, 1) * alpha / sqrt(L * d), L = tokens per row."""
        alpha = self.config.neftune_alpha
        pc = self.model.pc

        def hook(x):  # x: embeddings, seq-major [S_local, B, H]
            if not self.training:
                return x
            m = attention_mask.bool().to(x.dtype)  # [B, S]
            L = m.sum(1)
            mag = alpha / torch.sqrt(L * x.shape[-1])
            mt = m.t()
            if pc.tp:
                n = x.shape[0]
                if mt.shape[0] < n * pc.tp_size:  # sequence right-padded to a TP multiple: no noise on pads
                    mt = torch.nn.functional.pad(mt, (0, 0, 0, n * pc.tp_size - mt.shape[0]))
                from ..parallel.tensor_parallel import shard_seq_local
                mt = shard_seq_local(mt, pc.tp_rank, pc.tp_size)  # this rank's rows (chunked sequence layout)
            noise = torch.empty_like(x).uniform_(-1, 1) * mt.unsqueeze(-1) * mag.view(1, -1, 1)
            return x + noise.detach()

        return hook

    def forward_loss(self, batch: dict):
        labels = shift_labels(batch["labels"], self.config.ignore_index)
        hook = None
        if self.config.neftune_alpha is not None and self.training:
            am = batch.get("attention_mask")
            hook = self._neftune_hook(am if am is not None else torch.ones_like(batch["input_ids"]))
        h = self.hidden_and_head(self.model, batch["input_ids"], "attention_mask", batch, embed_hook=hook)
        loss = self.loss_from_hidden(self.model, h, labels.t().contiguous(), self.config.ignore_index)
        return loss, labels

    def training_step(self, batch: dict, batch_idx: int = 0):
        loss, labels = self.forward_loss(batch)
        metrics = {"Loss/Train/Step": loss.detach()}
        if self.config.log_perplexity:
            metrics["Perplexity/Train/Step"] = torch.exp(loss.detach())
        if self.config.neftune_alpha is not None:
            metrics["NEFTune Alpha"] = torch.tensor(self.config.neftune_alpha)
        counters = {"Consumed Samples": labels.shape[0],
                    "Consumed Tokens": (labels != self.config.ignore_index).sum()}
        return loss, metrics, counters

    @torch.no_grad()
    def validation_step(self, batch: dict, batch_idx: int = 0):
        loss, _ = self.forward_loss(batch)
        m = {"Loss/Val": loss.detach()}
        if self.config.log_perplexity:
            m["Perplexity/Val"] = torch.exp(loss.detach())
        return m
