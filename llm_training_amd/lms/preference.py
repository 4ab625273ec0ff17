"""Preference-tuning objectives: DPO and ORPO (paired chosen / rejected sequences).

Reference: src/llm_training/lms/dpo/dpo.py (reference model :59-71, get_logps :73-114, 4 forwards
:116-154, sigmoid loss + reward metrics :156-187), dpo_config.py:5-10; lms/orpo/orpo.py (mean logps
:61-93, 2 forwards :95-121, odds-ratio loss + CE on chosen :123-178, empty_cache :192-198),
orpo_config.py:5-9.

Per-token log-probs come from the fused lm_head + log-softmax-gather kernel (vocab-parallel under TP)
without materialising [T, V] log-softmax. Chosen and rejected are padded to a common length and run
as ONE batch through the model (one pass instead of two; the reference runs them separately).
DPO reference log-probs use the SHIFTED labels (the reference uses unshifted ones for the reference
model, dpo.py:134-146, SURVEY Q6 — a bug we do not reproduce).
"""
from __future__ import annotations

import copy

import torch
import torch.nn.functional as F

from ..ops.reference import shift_labels
from .base import BaseLM, BaseLMConfig, build_model


def _pad_to(x: torch.Tensor, S: int, value) -> torch.Tensor:
    if x.shape[1] == S:
        return x
    pad = torch.full((x.shape[0], S - x.shape[1]), value, dtype=x.dtype, device=x.device)
    return torch.cat([x, pad], 1)


def concat_pair(batch: dict, ignore_index: int, pad_id: int = 0, multiple: int = 1):
    """Stack chosen and rejected into one [2B, S] batch (right-padded)."""
    S = max(batch["chosen_input_ids"].shape[1], batch["rejected_input_ids"].shape[1])
    S = (S + multiple - 1) // multiple * multiple
    out = {}
    for key, val in (("input_ids", pad_id), ("labels", ignore_index), ("attention_mask", 0)):
        c, r = batch.get("chosen_" + key), batch.get("rejected_" + key)
        if c is None:
            continue
        out[key] = torch.cat([_pad_to(c, S, val), _pad_to(r, S, val)], 0)
    c, r = batch.get("chosen_position_ids"), batch.get("rejected_position_ids")
    if c is not None:
        B = batch["chosen_input_ids"].shape[0]
        c = c.expand(B, -1)
        r = r.expand(B, -1)
        out["position_ids"] = torch.cat([_pad_to(c, S, 0), _pad_to(r, S, 0)], 0)
    return out


class _PairMixin:
    def pair_token_logps(self, model, batch, pad_id=0, logit_means: bool = False):
        """Per-token log-probs of the chosen and rejected rows in one forward. ``logit_means``: also the
        mean logit of the chosen / rejected forwards over their own [B, S, V] (reference ORPO metrics
        "Chosen Logits" / "Rejected Logits", orpo.py:149-150), from the CE kernel's row sums."""
        cat = concat_pair(batch, self.config.ignore_index, pad_id)
        labels = shift_labels(cat["labels"], self.config.ignore_index)
        cat["attention_mask_trivial"] = False
        h = self.hidden_and_head(model, cat["input_ids"], "attention_mask", cat)
        res = self.token_logps_from_hidden(model, h, labels.t().contiguous(), self.config.ignore_index,
                                           logit_sums=logit_means)
        lp, rs = res if logit_means else (res, None)
        lp = lp.t()
        mask = labels != self.config.ignore_index
        B = batch["chosen_input_ids"].shape[0]
        if logit_means:
            V = getattr(model.config, "vocab_size", None) or model.lm_head_weight().shape[0]
            rs = rs.t()  # [2B, S]
            sc, sr = batch["chosen_input_ids"].shape[1], batch["rejected_input_ids"].shape[1]
            means = (rs[:B, :sc].sum() / (B * sc * V), rs[B:, :sr].sum() / (B * sr * V))
            return lp, mask, B, h, labels, means
        return lp, mask, B, h, labels


class DPOConfig(BaseLMConfig):
    ref_model: object | None = None
    beta: float = 0.1
    label_smoothing: float = 0.0
    ignore_index: int = -100

    @classmethod
    def _pre(cls, v):
        return v


class DPO(_PairMixin, BaseLM):
    config_class = DPOConfig

    def configure_model(self, pc, device, dtype, seed: int = 0, resuming: bool = False):
        super().configure_model(pc, device, dtype, seed, resuming)
        spec = self.config.ref_model
        if spec is None and not resuming:
            # the parallel context (process groups) is shared, not copied
            self.ref_model = copy.deepcopy(self.model, memo={id(self.model.pc): self.model.pc})
        elif spec is None:
            # resuming: the policy holds trained weights (and the checkpoint does not store the frozen
            # reference), so rebuild the reference from the pre-trained / initial weights instead
            self.ref_model = build_model(self.config.model, pc, dtype, device)
            self._load_or_init(self.ref_model, seed, False)
        else:
            if isinstance(spec, dict) and "model_class" in spec:
                from .base import ModelProvider
                spec = ModelProvider(spec["model_class"], spec.get("model_config"))
            self.ref_model = build_model(spec, pc, dtype, device)
            self._load_or_init(self.ref_model, seed, False)
        self.ref_model.requires_grad_(False)
        self.ref_model.eval()
        for p in self.ref_model.parameters():
            p.main_grad = None
        return self.model

    def logps(self, model, batch):
        lp, mask, B, _, _ = self.pair_token_logps(model, batch)
        seq = lp.sum(-1)  # DPO: summed log-probs
        return seq[:B], seq[B:]

    def compute_loss(self, pc_lp, pr_lp, rc_lp, rr_lp):
        beta, ls = self.config.beta, self.config.label_smoothing
        logits = (pc_lp - pr_lp) - (rc_lp - rr_lp)
        loss = (-F.logsigmoid(beta * logits) * (1 - ls) - F.logsigmoid(-beta * logits) * ls).mean()
        cr = beta * (pc_lp - rc_lp).detach()
        rr = beta * (pr_lp - rr_lp).detach()
        m = {"Chosen Reward": cr.mean(), "Rejected Reward": rr.mean(),
             "Reward Accuracy": (cr > rr).float().mean(), "Reward Margin": (cr - rr).mean(),
             "Chosen Log P": pc_lp.detach().mean(), "Rejected Log P": pr_lp.detach().mean(), "Loss": loss.detach()}
        return loss, m

    def on_engine_ready(self, engine):
        """With ZeRO-3 the frozen reference model is dp-sharded like the policy (reference dpo.py:59-71):
        gather-only units, 1/dp of its bytes per rank (parallel/frozen.py)."""
        self.ref_shards = None
        if engine.stage >= 3 and engine.sharded:
            from ..parallel.frozen import FrozenShards
            self.ref_shards = FrozenShards(self.ref_model, engine.group, engine.pc.dp_rank if engine.dp > 1 else 0,
                                           engine.dp, engine.comm_stream)

    def _step(self, batch):
        pc_lp, pr_lp = self.logps(self.model, batch)
        with torch.no_grad():
            rc_lp, rr_lp = self.logps(self.ref_model, batch)
        if getattr(self, "ref_shards", None) is not None:
            self.ref_shards.release_all()
        return self.compute_loss(pc_lp, pr_lp, rc_lp, rr_lp)

    def training_step(self, batch, batch_idx=0):
        loss, m = self._step(batch)
        B = batch["chosen_input_ids"].shape[0]
        return loss, {k + "/Train/Step": v for k, v in m.items()}, {"Consumed Samples": B}

    @torch.no_grad()
    def validation_step(self, batch, batch_idx=0):
        _, m = self._step(batch)
        return {k + "/Val": v for k, v in m.items()}


class ORPOConfig(BaseLMConfig):
    beta: float = 0.1
    ignore_index: int = -100
    empty_cache_threshold: int | None = None


class ORPO(_PairMixin, BaseLM):
    config_class = ORPOConfig

    def _step(self, batch):
        lp, mask, B, h, labels, (c_logits, r_logits) = self.pair_token_logps(self.model, batch, logit_means=True)
        n = mask.sum(-1).clamp(min=1)
        seq = lp.sum(-1) / n  # ORPO: length-normalised log-probs (reference orpo.py:93)
        c_lp, r_lp = seq[:B], seq[B:]
        beta = self.config.beta
        log_odds = (c_lp - r_lp) - (torch.log1p(-torch.exp(c_lp)) - torch.log1p(-torch.exp(r_lp)))
        ratio = F.logsigmoid(log_odds)
        or_loss = -(beta * ratio).mean()
        # CE on the chosen half: mean NLL over its valid tokens (= -sum lp / n_tokens)
        cmask = mask[:B]
        ce_loss = -(lp[:B] * cmask).sum() / cmask.sum().clamp(min=1)
        loss = or_loss + ce_loss
        cr, rr = beta * c_lp.detach(), beta * r_lp.detach()
        m = {"OR Loss": or_loss.detach(), "CE Loss": ce_loss.detach(), "Chosen Rewards": cr.mean(),
             "Rejected Rewards": rr.mean(), "Reward Accuracy": (cr > rr).float().mean(),
             "Reward Margin": (cr - rr).mean(), "Chosen Log P": c_lp.detach().mean(),
             "Rejected Log P": r_lp.detach().mean(), "Chosen Logits": c_logits, "Rejected Logits": r_logits,
             "Log Odds Ratio": ratio.detach().mean(),
             "Log Odds Chosen": log_odds.detach().mean(), "Loss": loss.detach()}
        return loss, m

    def training_step(self, batch, batch_idx=0):
        loss, m = self._step(batch)
        if self.config.empty_cache_threshold is not None and torch.cuda.is_available():
            S = batch["chosen_input_ids"].shape[1] + batch["rejected_input_ids"].shape[1]
            if S >= self.config.empty_cache_threshold:
                torch.cuda.empty_cache()
        B = batch["chosen_input_ids"].shape[0]
        return loss, {k + "/Train/Step": v for k, v in m.items()}, {"Consumed Samples": B}

    @torch.no_grad()
    def validation_step(self, batch, batch_idx=0):
        _, m = self._step(batch)
        return {k + "/Val": v for k, v in m.items()}
