"""Wrapper for any Hugging Face ``AutoModelForCausalLM`` (e.g. the GPT-2 small CPU plumbing config).

Reference: src/llm_training/models/hf_causal_lm/hf_causal_lm.py (packed-mask patch :19-20, HF gradient
checkpointing :37-38, optional Liger patch :42-43, FSDP units by ``_no_split_modules`` plus
leftovers :88-114; no TP) and hf_causal_lm_config.py:8-17.

The model body runs through transformers; its attention is routed to our gfx950 flash kernels
(``ops.fused.flash_attention``) through transformers' ``AttentionInterface`` under the name
``llmt_hip``: the packed segment ids travel as a forward kwarg down to every attention call, so
packed rows take the varlen kernel instead of a dense [B, 1, S, S] mask — the reference reaches the
same end by patching ``_get_unpad_data`` for FA2 (hf_causal_lm.py:19-20). Calls the kernel cannot
serve (logit soft-capping, head dims other than 64/96/128, non-causal modules) run transformers'
SDPA with the equivalent dense mask; attention dropout runs in the kernels. The loss heads use our
fused lm_head + cross-entropy on the final hidden states, and the ZeRO engine shards the HF model by
its ``_no_split_modules`` blocks. ``hf_config`` builds a random-init model from a config dict (no
checkpoint needed); ``hf_path`` loads a LOCAL checkpoint.
"""
from __future__ import annotations

import logging
import types
from typing import Any

import torch
import torch.nn as nn

from ..parallel.context import ParallelContext
from .base import BaseModel, BaseModelConfig, CausalLMOutput


logger = logging.getLogger("llm_training")

HF_ATTN_IMPL = "llmt_hip"  # (a name containing "flash" would send transformers looking for a hub kernel)
_FALLBACK_WARNED: set[str] = set()


def _dense_mask(seg: torch.Tensor, S: int, dtype, window: int | None) -> torch.Tensor:
    i = torch.arange(S, device=seg.device)
    vis = (i[None, :] <= i[:, None])[None] & (seg[:, :, None] == seg[:, None, :])
    if window is not None:
        vis = vis & ((i[:, None] - i[None, :]) < window)[None]
    m = torch.zeros(seg.shape[0], 1, S, S, dtype=dtype, device=seg.device)
    return m.masked_fill(~vis[:, None], torch.finfo(dtype).min)


def hf_attention(module, query, key, value, attention_mask, scaling=None, dropout=0.0, sliding_window=None,
                 softcap=None, **kwargs):
    """transformers attention function: query [B, Hq, S, D], key/value [B, Hkv, S, D] ->
    ([B, S, Hq, D], None). Segment ids arrive as ``llmt_segment_ids`` [B, S] (None = one sequence)."""
    from ..ops.fused import flash_attention
    seg = kwargs.get("llmt_segment_ids")
    D = query.shape[-1]
    why = None
    if softcap is not None:
        why = "logit soft-capping"
    elif D not in (64, 96, 128) and query.is_cuda:
        why = f"head dim {D}"
    elif not getattr(module, "is_causal", True) or attention_mask is not None:
        why = "non-causal / explicit mask"
    if why is None:
        window = None if sliding_window is None else int(sliding_window) - 1  # HF: q - k < sliding_window
        o = flash_attention(query.transpose(1, 2), key.transpose(1, 2), value.transpose(1, 2), causal=True,
                            segment_ids=seg, window=window, scale=scaling, dropout_p=float(dropout or 0.0))
        return o, None
    if why not in _FALLBACK_WARNED:
        _FALLBACK_WARNED.add(why)
        logger.warning("HFCausalLM attention: %s is not served by the HIP flash kernel; using SDPA", why)
    from transformers.integrations.sdpa_attention import sdpa_attention_forward
    if attention_mask is None and seg is not None:
        attention_mask = _dense_mask(seg.to(query.device), query.shape[2], query.dtype, sliding_window)
    if softcap is not None:
        from transformers.integrations.sdpa_attention import repeat_kv
        n_rep = query.shape[1] // key.shape[1]
        k, v = repeat_kv(key, n_rep), repeat_kv(value, n_rep)
        s = torch.matmul(query, k.transpose(2, 3)) * (scaling if scaling is not None else D ** -0.5)
        s = torch.tanh(s / softcap) * softcap
        S = query.shape[2]
        if attention_mask is None:
            i = torch.arange(S, device=query.device)
            s = s.masked_fill(i[None, :] > i[:, None], float("-inf"))
        else:
            s = s + attention_mask
        p = torch.nn.functional.dropout(torch.softmax(s.float(), -1).to(query.dtype), dropout,
                                        training=module.training)
        return torch.matmul(p, v).transpose(1, 2).contiguous(), None
    return sdpa_attention_forward(module, query, key, value, attention_mask, scaling=scaling, dropout=dropout)


def _register_hf_attention():
    from transformers import AttentionInterface
    from transformers.masking_utils import AttentionMaskInterface
    AttentionInterface.register(HF_ATTN_IMPL, hf_attention)
    AttentionMaskInterface.register(HF_ATTN_IMPL, lambda *a, **k: None)  # masking is by segment ids


def _hf_auto_config(config):
    """The transformers config of an ``HFCausalLMConfig``: from ``hf_config`` or a local ``hf_path``."""
    from transformers import AutoConfig

    if config.hf_config is not None:
        d = dict(config.hf_config)
        mt = d.pop("model_type")
        return AutoConfig.for_model(mt, **d)
    if config.hf_path:
        return AutoConfig.from_pretrained(config.hf_path, local_files_only=True,
                                          trust_remote_code=config.trust_remote_code)
    raise ValueError("HFCausalLM needs `hf_config` or a local `hf_path`")


def _qkv_rows(hf_cfg) -> tuple[int, int, int]:
    """Output rows of q_proj, k_proj, v_proj."""
    nq = int(hf_cfg.num_attention_heads)
    nkv = int(getattr(hf_cfg, "num_key_value_heads", None) or nq)
    d = getattr(hf_cfg, "head_dim", None) or hf_cfg.hidden_size // nq
    return nq * d, nkv * d, nkv * d


class HFCausalLMConfig(BaseModelConfig):
    hf_config: dict[str, Any] | None = None
    enable_gradient_checkpointing: bool = False
    # reference hf_causal_lm.py:42-43 (Liger instance patch, rope=False): RMSNorm and the SiLU-gated MLP
    # of the transformers modules run on the HIP kernels (the loss head is always the fused one)
    enable_liger_kernel: bool = False
    loss_chunk_size: int = 8192


class HFCausalLM(BaseModel):
    config_class = HFCausalLMConfig
    writes_main_grad = False  # transformers modules produce ordinary .grad tensors

    def __init__(self, config: HFCausalLMConfig, pc: ParallelContext | None = None, dtype=None, device=None):
        super().__init__(config, pc)
        if self.pc.tp:
            raise NotImplementedError("HFCausalLM does not support tensor parallelism (as in the reference)")
        from transformers import AutoModelForCausalLM

        hf_cfg = _hf_auto_config(config)
        impl = config.attn_implementation
        if impl in (None, "flash_attention_2", "flash", "hip", HF_ATTN_IMPL):
            _register_hf_attention()
            impl = HF_ATTN_IMPL
        hf_cfg._attn_implementation = impl
        self.uses_hip_attention = impl == HF_ATTN_IMPL
        if dtype is None:
            dtype = config.torch_dtype if isinstance(config.torch_dtype, torch.dtype) else torch.float32
        if device is not None and torch.device(device).type == "cuda":
            # built on the GPU directly (an 8 B model's CPU construction + copy takes minutes)
            with torch.device(device):
                self.hf_model = AutoModelForCausalLM.from_config(hf_cfg, torch_dtype=dtype)
        else:
            self.hf_model = AutoModelForCausalLM.from_config(hf_cfg, torch_dtype=dtype)
            if device is not None:
                self.hf_model.to(device)
        if config.enable_gradient_checkpointing:
            self.hf_model.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
        self.fused_modules: dict[str, int] = {}
        if config.enable_liger_kernel:
            self.fused_modules = apply_fused_kernels(self.hf_model, attention=self.uses_hip_attention)
            logger.info("HFCausalLM: fused kernels patched into %s", self.fused_modules or "no module")

    @property
    def hf_config(self):
        return self.hf_model.config

    def init_weights(self, seed: int = 0):
        torch.manual_seed(seed)
        self.hf_model.apply(self.hf_model._init_weights)
        if getattr(self.hf_model.config, "tie_word_embeddings", False):
            self.hf_model.tie_weights()

    def lm_head_weight(self):
        return self.hf_model.get_output_embeddings().weight

    def get_input_embeddings(self):
        return self.hf_model.get_input_embeddings()

    def get_output_embeddings(self):
        return self.hf_model.get_output_embeddings()

    def fsdp_units(self):
        names = set(getattr(self.hf_model, "_no_split_modules", None) or [])
        units, seen = [], set()
        for m in self.hf_model.modules():
            if type(m).__name__ in names:
                units.append(m)
                seen.update(id(p) for p in m.parameters())
        rest = [p for p in self.hf_model.parameters() if id(p) not in seen]
        if rest:  # one more unit for the leftovers (embeddings, final norm, lm_head)
            units.insert(0, _ParamsUnit(rest))
        return units or [self.hf_model]

    @staticmethod
    def _hf_mask(segment_ids, B, S, dtype, device):
        """2-D padding mask when the ids are 0/1, else a 4-D block-diagonal causal mask (packed rows)."""
        if segment_ids is None:
            return None
        seg = segment_ids.to(device)
        if bool((seg <= 1).all()):
            return seg.long()
        i = torch.arange(S, device=device)
        vis = (i[None, :] <= i[:, None])[None] & (seg[:, :, None] == seg[:, None, :])
        m = torch.zeros(B, 1, S, S, dtype=dtype, device=device)
        return m.masked_fill(~vis[:, None], torch.finfo(dtype).min)

    def hidden_states(self, input_ids=None, position_ids=None, segment_ids=None, inputs_embeds=None,
                      gather_sequence: bool = True, embed_hook=None):
        if input_ids is not None:
            B, S = input_ids.shape
            dev = input_ids.device
        else:
            B, S = inputs_embeds.shape[:2]
            dev = inputs_embeds.device
        if embed_hook is not None:
            emb = self.get_input_embeddings()(input_ids) if inputs_embeds is None else inputs_embeds
            inputs_embeds = embed_hook(emb.transpose(0, 1)).transpose(0, 1)
            input_ids = None
        if self.uses_hip_attention:
            seg = None if segment_ids is None else segment_ids.to(dev)
            out = self.hf_model(input_ids=input_ids, inputs_embeds=inputs_embeds, position_ids=position_ids,
                                output_hidden_states=True, use_cache=False, llmt_segment_ids=seg)
        else:
            mask = self._hf_mask(segment_ids, B, S, next(self.parameters()).dtype, dev)
            out = self.hf_model(input_ids=input_ids, inputs_embeds=inputs_embeds, attention_mask=mask,
                                position_ids=position_ids, output_hidden_states=True, use_cache=False)
        return out.hidden_states[-1].transpose(0, 1)

    def forward(self, input_ids=None, attention_mask=None, position_ids=None, inputs_embeds=None,
                return_last_hidden_states: bool = False, segment_ids=None):
        h = self.hidden_states(input_ids, position_ids, segment_ids if segment_ids is not None else attention_mask,
                               inputs_embeds)
        logits = torch.nn.functional.linear(h, self.lm_head_weight()).transpose(0, 1)
        return CausalLMOutput(logits=logits, last_hidden_states=h.transpose(0, 1) if return_last_hidden_states
                              else None)

    @classmethod
    def convert_state_dict_from_hf(cls, sd, config):
        return {"hf_model." + k: v for k, v in sd.items()}

    @classmethod
    def convert_state_dict_to_hf(cls, sd, config):
        """Our names -> transformers keys. Checkpoints name tensors by ``named_parameters()``, so a model built
        with ``enable_liger_kernel`` stores its fused projections (``self_attn.qkv_weight`` / ``qkv_bias``,
        ``mlp.gate_up_weight``); they are split back into the per-projection HF keys here (rows
        [q | k | v] and [gate | up], as ``_fuse_linears`` concatenated them)."""
        out: dict[str, torch.Tensor] = {}
        qkv_rows = None
        for k, v in sd.items():
            if not k.startswith("hf_model."):
                continue
            k = k[len("hf_model."):]
            if k.endswith(".gate_up_weight"):
                base, half = k[:-len("gate_up_weight")], v.shape[0] // 2
                out[base + "gate_proj.weight"], out[base + "up_proj.weight"] = v[:half], v[half:]
            elif k.endswith((".self_attn.qkv_weight", ".self_attn.qkv_bias")):
                if qkv_rows is None:
                    qkv_rows = _qkv_rows(_hf_auto_config(config))
                base, suffix = k.rsplit(".", 1)
                kind = "weight" if suffix == "qkv_weight" else "bias"
                lo = 0
                for name, n in zip(("q_proj", "k_proj", "v_proj"), qkv_rows):
                    out[f"{base}.{name}.{kind}"] = v[lo:lo + n]
                    lo += n
                if lo != v.shape[0]:
                    raise ValueError(f"{k}: {v.shape[0]} rows, config gives q/k/v rows {qkv_rows}")
            else:
                out[k] = v
        return out

    def hf_config_dict(self) -> dict:
        hm = self.__dict__.get("_modules", {}).get("hf_model")
        if hm is not None:
            return hm.config.to_dict()
        # an unbuilt instance (convert_to_hf's config probe): from the model config alone
        d = _hf_auto_config(self.config).to_dict()
        d.pop("_attn_implementation_autoset", None)
        return d

    def _tp_rule(self, key):
        return "rep", None


# ---------------------------------------------------------------------------- fused-kernel instance patch
# RMSNorm classes computing w * (x / rms(x)) in fp32 then cast (Llama / Mistral / Qwen2 / Qwen3 / Phi-3 /
# Granite / OLMo-2 ...). Gemma-style (1 + w) norms are left alone.
_NORM_SKIP = ("Gemma",)


def _bind(m: nn.Module, fn) -> None:
    """Install ``fn(self, ...)`` as ``m``'s forward, bound to ``m``: ``copy.deepcopy`` rebinds a bound method
    to the copied module (a closure over ``m`` would keep calling the original module's weights, e.g. in
    DPO's deep-copied reference model)."""
    m.forward = types.MethodType(fn, m)


def _patch_norm(m: nn.Module) -> bool:
    if getattr(m, "weight", None) is None or type(m).__name__.startswith(_NORM_SKIP):
        return False
    eps = getattr(m, "variance_epsilon", getattr(m, "eps", None))
    if eps is None:
        return False

    def forward(self, hidden_states, _eps=float(eps)):
        from ..ops.fused import rms_norm
        return rms_norm(hidden_states, self.weight, _eps)

    _bind(m, forward)
    return True


def _is_silu(act) -> bool:
    return isinstance(act, nn.SiLU) or type(act).__name__ in ("SiLUActivation", "SiLU")


_SLICE_CLASSES: dict[tuple[type, bool], type] = {}


def _slice_linear(cls: type, with_bias: bool = False) -> type:
    """A subclass of ``cls`` (an nn.Linear) whose ``weight`` (and ``bias``) are row slices of a fused
    parameter of the owning module instead of parameters of its own."""
    sub = _SLICE_CLASSES.get((cls, with_bias))
    if sub is None:
        def weight(self):
            lo, hi = self._fused_rows
            return getattr(self._fused_owner, self._fused_w)[lo:hi]
        attrs = {"weight": property(weight)}
        if with_bias:
            def bias(self):
                lo, hi = self._fused_rows
                return getattr(self._fused_owner, self._fused_b)[lo:hi]
            attrs["bias"] = property(bias)
        sub = type(f"Fused{cls.__name__}", (cls,), attrs)
        _SLICE_CLASSES[(cls, with_bias)] = sub
    return sub


def _fuse_linears(owner: nn.Module, names: list[str], wname: str, bname: str | None = None) -> bool:
    """Re-home the weights (and biases, when every projection has one and ``bname`` is given) of the
    nn.Linear children ``names`` of ``owner`` into one parameter concatenated along the output rows: the
    patched forward multiplies by it directly (one GEMM, no per-call torch.cat of weights, no cat backward)
    and its gradient is written by the main-grad-aware linear kernel. The projections stay readable as
    views (``q_proj.weight`` ...); state dicts keep the transformers key names."""
    mods = [getattr(owner, n) for n in names]
    if any("weight" not in m._parameters for m in mods) or len({m.weight.shape[1] for m in mods}) != 1:
        return False
    has_b = [m.bias is not None for m in mods]
    fb = all(has_b)
    if any(has_b) and not (fb and bname):
        return False
    rows, lo = [], 0
    for m in mods:
        rows.append((lo, lo + m.weight.shape[0]))
        lo += m.weight.shape[0]
    owner.register_parameter(wname, nn.Parameter(torch.cat([m.weight.detach() for m in mods], 0),
                                                 requires_grad=any(m.weight.requires_grad for m in mods)))
    if fb:
        owner.register_parameter(bname, nn.Parameter(torch.cat([m.bias.detach() for m in mods], 0),
                                                     requires_grad=any(m.bias.requires_grad for m in mods)))
    for m, r in zip(mods, rows):
        del m._parameters["weight"]
        if fb:
            del m._parameters["bias"]
        m.__class__ = _slice_linear(type(m), fb)
        object.__setattr__(m, "_fused_owner", owner)  # plain attributes: not a child module
        object.__setattr__(m, "_fused_rows", r)
        object.__setattr__(m, "_fused_w", wname)
        if fb:
            object.__setattr__(m, "_fused_b", bname)
    groups = [("weight", wname)] + ([("bias", bname)] if fb else [])

    def split(module, state_dict, prefix, local_metadata):
        for suffix, fname in groups:
            w = state_dict.pop(prefix + fname, None)
            if w is not None:
                for n, (a, b) in zip(names, rows):
                    state_dict[f"{prefix}{n}.{suffix}"] = w[a:b]

    def fuse(module, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs):
        for suffix, fname in groups:
            keys = [f"{prefix}{n}.{suffix}" for n in names]
            if all(k in state_dict for k in keys):
                state_dict[prefix + fname] = torch.cat([state_dict.pop(k) for k in keys], 0)

    owner._register_state_dict_hook(split)
    owner._register_load_state_dict_pre_hook(fuse, with_module=True)
    return True


def _fuse_gate_up(m: nn.Module) -> bool:
    """gate_proj / up_proj weights as one [2I, h] parameter ``gate_up_weight`` (gate rows first)."""
    g, u = m.gate_proj, m.up_proj
    if g.bias is not None or u.bias is not None:
        return False
    return _fuse_linears(m, ["gate_proj", "up_proj"], "gate_up_weight")


# attention modules with separate q / k / v projections, full-width rotate-half RoPE and no extra q / k
# transforms: patched onto one fused QKV GEMM + the in-place RoPE kernel + flash attention (the native
# Llama layer's path) when the model routes its attention to the HIP kernels
_ATTN_PATCH = ("LlamaAttention", "MistralAttention", "Qwen2Attention", "Phi3Attention")


def _patch_attention(m: nn.Module) -> bool:
    name = type(m).__name__
    fused_proj = name == "Phi3Attention"  # already one [q | k | v] projection
    proj = ("qkv_proj", "o_proj") if fused_proj else ("q_proj", "k_proj", "v_proj", "o_proj")
    if name not in _ATTN_PATCH or not all(hasattr(m, n) for n in proj):
        return False
    cfg = getattr(m, "config", None)
    if cfg is None or getattr(m, "q_norm", None) is not None or getattr(cfg, "partial_rotary_factor", 1.0) != 1.0:
        return False
    D = int(m.head_dim)
    nq, nkv = int(cfg.num_attention_heads), int(cfg.num_key_value_heads)
    if D not in (64, 96, 128):
        return False
    if fused_proj:
        if m.qkv_proj.out_features != (nq + 2 * nkv) * D:
            return False
    elif (m.q_proj.out_features != nq * D or m.k_proj.out_features != nkv * D
          or not _fuse_linears(m, ["q_proj", "k_proj", "v_proj"], "qkv_weight", "qkv_bias")):
        return False
    # window as transformers hands it to the attention function (Mistral / Phi-3: the config's, Qwen2: per layer)
    win = getattr(cfg, "sliding_window", None) if name in ("MistralAttention", "Phi3Attention") else \
        getattr(m, "sliding_window", None)
    def forward(_m, hidden_states, position_embeddings=None, attention_mask=None, past_key_values=None,
                **kwargs):
        if (past_key_values is not None or attention_mask is not None or position_embeddings is None
                or position_embeddings[0].shape[-1] != D):  # (partial rotary: transformers' own path; still
            # valid after the fusion: q / k / v read slices of the fused parameter)
            return type(_m).forward(_m, hidden_states, position_embeddings, attention_mask, past_key_values,
                                    **kwargs)
        from ..ops.fused import linear, rope_attention_bm
        B, S = hidden_states.shape[:2]
        if fused_proj:
            w, b = _m.qkv_proj.weight, _m.qkv_proj.bias
        else:
            w, b = _m.qkv_weight, getattr(_m, "qkv_bias", None)
        qkv = linear(hidden_states, w, b).view(B, S, nq + 2 * nkv, D)
        cos, sin = position_embeddings
        o = rope_attention_bm(qkv, cos, sin, nq, nkv, segment_ids=kwargs.get("llmt_segment_ids"),
                              window=None if win is None else int(win) - 1, scale=_m.scaling,
                              dropout_p=float(_m.attention_dropout) if _m.training else 0.0)
        return linear(o.reshape(B, S, nq * D), _m.o_proj.weight, _m.o_proj.bias), None

    _bind(m, forward)
    return True


def _patch_mlp(m: nn.Module) -> bool:
    act = getattr(m, "act_fn", getattr(m, "activation_fn", None))
    if act is None or not _is_silu(act):
        return False
    if all(hasattr(m, n) for n in ("gate_proj", "up_proj", "down_proj")):
        # one GEMM for gate and up, the SwiGLU kernel on the fused [.., 2I] buffer, then down_proj
        # (Liger's LigerSwiGLUMLP); gate / up weights live in one fused parameter (no per-call concat)
        if _fuse_gate_up(m):
            def forward(_m, x):
                from ..ops.fused import linear, swiglu_down
                # down_proj's input-gradient GEMM carries the SwiGLU backward in its epilogue
                return swiglu_down(linear(x, _m.gate_up_weight), _m.down_proj.weight, _m.down_proj.bias,
                                   dy_t_consumer=True)
        else:  # biased projections: concatenated per call
            def forward(_m, x):
                from ..ops.fused import swiglu
                w = torch.cat([_m.gate_proj.weight, _m.up_proj.weight], 0)
                b = None
                if _m.gate_proj.bias is not None:
                    b = torch.cat([_m.gate_proj.bias, _m.up_proj.bias], 0)
                return _m.down_proj(swiglu(torch.nn.functional.linear(x, w, b)))
    elif hasattr(m, "gate_up_proj") and hasattr(m, "down_proj"):  # Phi-3: fused [gate | up] projection
        def forward(_m, x):
            from ..ops.fused import linear, swiglu_down
            gu = linear(x, _m.gate_up_proj.weight, _m.gate_up_proj.bias)
            return swiglu_down(gu, _m.down_proj.weight, _m.down_proj.bias, dy_t_consumer=True)
    else:
        return False
    _bind(m, forward)
    return True


_LAYER_PATCH = ("LlamaDecoderLayer", "MistralDecoderLayer", "Qwen2DecoderLayer")


def _patch_decoder_layer(m: nn.Module) -> bool:
    """Pre-norm decoder layer with the attention residual added inside the post-attention RMSNorm kernel
    (the native layer's fused add + norm: one pass writes both the sum and its norm)."""
    if type(m).__name__ not in _LAYER_PATCH or not all(hasattr(m, n) for n in
                                                      ("input_layernorm", "self_attn", "post_attention_layernorm", "mlp")):
        return False
    norm = m.post_attention_layernorm
    eps = getattr(norm, "variance_epsilon", getattr(norm, "eps", None))
    if eps is None or getattr(norm, "weight", None) is None or type(norm).__name__.startswith(_NORM_SKIP):
        return False

    def forward(_m, hidden_states, attention_mask=None, position_ids=None, past_key_values=None, use_cache=False,
                position_embeddings=None, _eps=float(eps), **kwargs):
        from ..ops.fused import rms_norm
        a, _ = _m.self_attn(hidden_states=_m.input_layernorm(hidden_states), attention_mask=attention_mask,
                            position_ids=position_ids, past_key_values=past_key_values, use_cache=use_cache,
                            position_embeddings=position_embeddings, **kwargs)
        h, res = rms_norm(a, _m.post_attention_layernorm.weight, _eps, residual=hidden_states)
        return res + _m.mlp(h)

    _bind(m, forward)
    return True


def apply_fused_kernels(model: nn.Module, attention: bool = False) -> dict[str, int]:
    """Patch every RMSNorm and SiLU-gated MLP instance of a transformers model onto the HIP kernels, and
    with ``attention`` (the model's attention already routed to the HIP flash kernels) the q / k / v
    projections, RoPE and attention of the supported attention classes; returns {class name: count}.
    On the CPU the same functions run their torch reference ops."""
    done: dict[str, int] = {}
    for m in list(model.modules()):
        name = type(m).__name__
        ok = False
        if name.endswith("RMSNorm"):
            ok = _patch_norm(m)
        elif name.endswith("MLP"):
            ok = _patch_mlp(m)
        elif attention and name.endswith("Attention"):
            ok = _patch_attention(m)
        elif name.endswith("DecoderLayer"):
            ok = _patch_decoder_layer(m)
        if ok:
            done[name] = done.get(name, 0) + 1
    return done


class _ParamsUnit(nn.Module):
    """Parameter container used as an engine unit (no forward hooks fire on it)."""

    def __init__(self, params):
        super().__init__()
        self._plist = list(params)

    def parameters(self, recurse: bool = True):
        return iter(self._plist)
