"""Phi-3 / Phi-3.5 / Phi-4-mini for MI355X.

Reference: src/llm_training/models/phi3/phi3_model.py (fused qkv_proj / gate_up_proj :421-429,507-509,
LongRoPE :293-413, sliding window :169,690, residual / embedding dropout :47,797-823, TP plan
:212-256) and phi3_config.py:9-79.

Phi-3's HF checkpoints already store fused ``qkv_proj`` / ``gate_up_proj``, which is exactly our
Llama block layout, so this model reuses the Llama block (fused add+RMSNorm, in-place RoPE on the
QKV buffer, HIP flash attention with the sliding window, fused SwiGLU) and differs in config,
LongRoPE table selection (short factors up to ``original_max_position_embeddings``, long factors
beyond, with the attention scaling folded into the cos/sin tables) and dropout. Under TP the fused
weights are sharded per rank as [q_r; k_r; v_r] / [g_r; u_r] — the reference shards them contiguously
and mixes heads.
"""
from __future__ import annotations

import math
from typing import Any, Literal

import torch
import torch.nn.functional as F
from pydantic import field_validator, model_validator

from ..ops.rope_utils import RopeTables
from ..parallel import tensor_parallel as tpl
from .base import load_hf_config_dict, to_dtype
from .llama import Llama, LlamaConfig, LlamaDecoderLayer


class Phi3Config(LlamaConfig):
    vocab_size: int = 32064
    hidden_size: int = 3072
    intermediate_size: int = 8192
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int | None = None
    resid_pdrop: float = 0.0
    embd_pdrop: float = 0.0
    attention_dropout: float = 0.0
    max_position_embeddings: int = 4096
    original_max_position_embeddings: int = 4096
    initializer_range: float = 0.02
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    rope_scaling: dict[str, Any] | None = None
    partial_rotary_factor: float = 1.0
    bos_token_id: int = 1
    eos_token_id: int | list[int] = 32000
    pad_token_id: int | None = 32000
    sliding_window: int | None = None
    attention_compute_dtype: Any = None  # accepted for config parity; the HIP kernels accumulate in fp32

    @field_validator("rope_scaling")
    @classmethod
    def _longrope(cls, v):
        if v is None:
            return v
        t = v.get("type", v.get("rope_type"))
        if t not in ("longrope", "su"):
            raise ValueError(f"rope_scaling type must be 'longrope', got {t}")
        for k in ("short_factor", "long_factor"):
            if not isinstance(v.get(k), list):
                raise ValueError(f"rope_scaling.{k} must be a list of numbers")
        return v

    @model_validator(mode="after")
    def _check_factors(self):
        if self.rope_scaling is not None:
            half = int(self.head_dim * self.partial_rotary_factor) // 2
            for k in ("short_factor", "long_factor"):
                if len(self.rope_scaling[k]) != half:
                    raise ValueError(f"rope_scaling.{k} must have length {half}")
        return self

    def merge_hf_config(self, hf: dict):
        super().merge_hf_config(hf)
        for k in ("resid_pdrop", "embd_pdrop", "original_max_position_embeddings", "sliding_window",
                  "partial_rotary_factor"):
            if k in hf and hf[k] is not None:
                object.__setattr__(self, k, hf[k])


class Phi3DecoderLayer(LlamaDecoderLayer):
    def __init__(self, cfg: Phi3Config, pc, layer_idx, dtype=None, device=None):
        super().__init__(cfg, pc, layer_idx, dtype, device)
        self.resid_pdrop = cfg.resid_pdrop

    def forward(self, x, residual, rt):
        g = self.pc.tp_group if self.pc.tp else None
        drop = self.resid_pdrop if self.training else 0.0
        if residual is None:
            h, residual = self.input_layernorm(x), x
        else:
            h, residual = self.input_layernorm(x, residual)
        a = self.attn_block(h, rt, g)
        if drop > 0:
            a = F.dropout(a, drop, True)
        h, residual = self.post_attention_layernorm(a, residual)
        m = self.mlp_block(h, g)
        if drop > 0:
            m = F.dropout(m, drop, True)
        return m, residual


class Phi3(Llama):
    config_class = Phi3Config
    hf_model_type = "phi3"
    decoder_layer_class = Phi3DecoderLayer

    def __init__(self, config: Phi3Config, pc=None, dtype=None, device=None):
        super().__init__(config, pc, dtype, device)
        c = config
        rot = int(c.head_dim * c.partial_rotary_factor)
        if c.partial_rotary_factor != 1.0:
            raise NotImplementedError("partial rotary embeddings are not supported by the fused RoPE kernel")
        if c.rope_scaling is not None:
            base = dict(c.rope_scaling)
            base.setdefault("factor", c.max_position_embeddings / c.original_max_position_embeddings)
            base["original_max_position_embeddings"] = c.original_max_position_embeddings
            short = dict(base, long_factor=base["short_factor"], type="longrope")
            long = dict(base, short_factor=base["long_factor"], type="longrope")
            self.rope_short = RopeTables(rot, c.rope_theta, short, c.max_position_embeddings)
            self.rope_long = RopeTables(rot, c.rope_theta, long, c.max_position_embeddings)
        else:
            self.rope_short = self.rope_long = RopeTables(rot, c.rope_theta, None, c.max_position_embeddings)

    def _runtime(self, input_ids, position_ids, segment_ids, device, S, B):
        rt = super()._runtime(input_ids, position_ids, segment_ids, device, S, B)
        if self.rope_long is self.rope_short:
            rt["cos"], rt["sin"] = self.rope_short.get(device, S)
        else:
            # LongRoPE factor choice as in the reference (phi3_model.py rotary cache, the Llama code at
            # llama_model.py:343-352,367-371): long factors once max(position_ids) + 1, rounded up to a
            # multiple of 4096, exceeds original_max_position_embeddings. Decided on the device without a
            # host sync: the short and long tables are stacked and the positions shifted into the long half.
            cs, ss = self.rope_short.get(device, S)
            cl, sl = self.rope_long.get(device, S)
            key = (str(device), cs.shape[0])
            if getattr(self, "_rope_cat_key", None) != key:
                self._rope_cat = (torch.cat([cs, cl]), torch.cat([ss, sl]))
                self._rope_cat_key = key
            pos = rt["positions"]
            rounded = (pos.max() + 1 + 4095) // 4096 * 4096
            use_long = (rounded > self.config.original_max_position_embeddings).to(pos.dtype)
            rt["positions"] = pos + use_long * cs.shape[0]
            rt["cos"], rt["sin"] = self._rope_cat
        sw = self.config.sliding_window
        rt["window"] = -1 if (sw is None or sw >= S) else int(sw)
        return rt

    def hidden_states(self, input_ids=None, position_ids=None, segment_ids=None, inputs_embeds=None,
                      gather_sequence: bool = True, embed_hook=None):
        p = self.config.embd_pdrop
        if p > 0 and self.training:
            prev = embed_hook

            def embed_hook(x, _prev=prev):  # noqa: F811 - chain NEFTune (if any) then embedding dropout
                x = _prev(x) if _prev is not None else x
                return F.dropout(x, p, True)
        return super().hidden_states(input_ids, position_ids, segment_ids, inputs_embeds, gather_sequence,
                                     embed_hook)

    @classmethod
    def convert_state_dict_from_hf(cls, sd, config):
        out = {}
        for k, v in sd.items():
            out[k[len("model."):] if k.startswith("model.") else k] = v
        if config.tie_word_embeddings:
            out.pop("lm_head.weight", None)
        return out

    @classmethod
    def convert_state_dict_to_hf(cls, sd, config):
        out = {}
        for k, v in sd.items():
            out[k if k.startswith("lm_head.") else "model." + k] = v
        if config.tie_word_embeddings:
            out["lm_head.weight"] = out["model.embed_tokens.weight"]
        return out

    def hf_config_dict(self) -> dict:
        c = self.config
        d = super().hf_config_dict()
        d.update({"architectures": ["Phi3ForCausalLM"], "model_type": "phi3", "resid_pdrop": c.resid_pdrop,
                  "embd_pdrop": c.embd_pdrop, "original_max_position_embeddings": c.original_max_position_embeddings,
                  "sliding_window": c.sliding_window, "partial_rotary_factor": c.partial_rotary_factor})
        d.pop("mlp_bias", None)
        d.pop("head_dim", None)
        return d
