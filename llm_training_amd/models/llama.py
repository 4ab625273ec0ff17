"""Llama (2 / 3 / 3.x) for MI355X.

Reference: src/llm_training/models/llama/llama_model.py (module tree :32-58, forward :135-192, TP+SP
plan :197-244, FSDP plan :246-268, RMSNorm :271-286, rotary :289-412, MLP :415-427, attention
:434-744) and llama_config.py:7-32.

MI355X-first structure (not a translation):
- q/k/v are ONE fused GEMM (``qkv_proj``) and gate/up ONE fused GEMM (``gate_up_proj``): fewer, larger
  hipBLASLt calls. HF checkpoints are split / merged on conversion; under TP the fused weights are
  sharded per rank as [q_r; k_r; v_r] / [g_r; u_r].
- residual adds are fused into the following RMSNorm (one HIP kernel: add + norm, fwd and bwd).
- RoPE runs in place on the QKV GEMM output and the HIP flash kernels read q/k/v as strided views.
- activations are sequence-major [S, B, H]; under TP+SP the residual stream is the local sequence
  shard [S/tp, B, H] and attention/MLP see the all-gathered sequence.
- ``rope_scaling`` IS taken from the HF config (the reference drops it for Llama).
"""
from __future__ import annotations

import logging
import math
import zlib
from typing import Any, Literal

import torch
import torch.nn as nn
import torch.utils.checkpoint as ckpt
from pydantic import model_validator

from ..ops import fused as F_
from ..ops.rope_utils import RopeTables
from ..parallel import tensor_parallel as tpl
from ..parallel.context import ParallelContext
from .base import BaseModel, BaseModelConfig, CausalLMOutput, load_hf_config_dict, to_dtype
from .modules import Linear, RMSNorm, VocabParallelEmbedding, normal_
from .utils import keep_attention_context

logger = logging.getLogger("llm_training")


class LlamaConfig(BaseModelConfig):
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int | None = None
    head_dim: int | None = None
    max_position_embeddings: int = 4096
    initializer_range: float = 0.02
    rms_norm_eps: float = 1e-6
    pad_token_id: int | None = None
    bos_token_id: int = 1
    eos_token_id: int | list[int] = 2
    tie_word_embeddings: bool = False
    rope_theta: float = 10000.0
    rope_scaling: dict[str, Any] | None = None
    attention_bias: bool = False
    attention_dropout: float = 0.0
    # TP + SP: overlap the sequence all-gather / reduce-scatter with the projection GEMMs
    tp_comm_overlap: bool = True
    mlp_bias: bool = False
    enable_gradient_checkpointing: bool = False
    # "full_keep_attention": full layer recompute except the flash-attention forward, whose output and LSE
    # are kept (torch selective-checkpoint policy on llmt::flash_attn_fwd): + S*B*H*2 bytes per layer, one
    # attention forward less per step (the long-context cost: attention dominates at 128K)
    recompute_granularity: Literal["full", "selective", "full_keep_attention"] = "full"
    # loss-head chunking of the fused linear + cross-entropy (rows per lm_head GEMM)
    loss_chunk_size: int = 8192

    @model_validator(mode="after")
    def _post(self):
        if self.hf_path:
            hf = load_hf_config_dict(self.hf_path)
            if hf is None:
                logger.warning("hf_path %s has no local config.json; using the given architecture", self.hf_path)
            else:
                self.merge_hf_config(hf)
        if self.num_key_value_heads is None:
            self.num_key_value_heads = self.num_attention_heads
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_attention_heads
        return self

    def merge_hf_config(self, hf: dict):
        for k in ("vocab_size", "hidden_size", "intermediate_size", "num_hidden_layers", "num_attention_heads",
                  "num_key_value_heads", "head_dim", "max_position_embeddings", "initializer_range", "rms_norm_eps",
                  "pad_token_id", "bos_token_id", "eos_token_id", "tie_word_embeddings", "rope_theta",
                  "rope_scaling", "attention_bias", "attention_dropout", "mlp_bias"):
            if k in hf and hf[k] is not None:
                object.__setattr__(self, k, hf[k])
        if self.torch_dtype == "auto" and hf.get("torch_dtype"):
            object.__setattr__(self, "torch_dtype", to_dtype(hf["torch_dtype"]))


class LlamaAttention(nn.Module):
    def __init__(self, cfg: LlamaConfig, pc: ParallelContext, dtype=None, device=None):
        super().__init__()
        self.cfg, self.pc = cfg, pc
        tp = pc.tp_size
        assert cfg.num_attention_heads % tp == 0 and cfg.num_key_value_heads % tp == 0, \
            "heads must be divisible by the tensor-parallel size"
        self.nq = cfg.num_attention_heads // tp
        self.nkv = cfg.num_key_value_heads // tp
        self.hd = cfg.head_dim
        self.qkv_proj = Linear(cfg.hidden_size, (self.nq + 2 * self.nkv) * self.hd, cfg.attention_bias, dtype, device)
        self.o_proj = Linear(self.nq * self.hd, cfg.hidden_size, cfg.attention_bias, dtype, device)

    def forward(self, h, rt, sp_group=None):
        """h: [S, B, H]; with ``sp_group`` h is this rank's sequence shard and the gather / scatter run
        inside the projections, overlapped with their GEMMs (tensor_parallel.ag_linear / linear_rs)."""
        if sp_group is not None:
            qkv = tpl.ag_linear(h, self.qkv_proj.weight, self.qkv_proj.bias, sp_group)
        else:
            qkv = self.qkv_proj(h)
        S, B = qkv.shape[:2]
        qkv = qkv.view(S, B, self.nq + 2 * self.nkv, self.hd)
        def core(t):
            return F_.rope_attention(t, rt["positions"], rt["cos"], rt["sin"], self.nq, self.nkv, causal=True,
                                     segment_ids=rt["segment_ids"], window=rt.get("window", -1), impl=rt["impl"],
                                     seg_info=rt.get("seg_info"), rope_tok=rt.get("rope_tok"),
                                     dropout_p=self.cfg.attention_dropout if self.training else 0.0)

        if rt.get("selective") and rt["impl"] != "flash" and self.training and torch.is_grad_enabled():
            # selective recompute (reference llama_model.py:506-534): keep only the attention inputs and
            # recompute the score matrix in backward. The flash kernels never store it, so they skip this.
            a = ckpt.checkpoint(core, qkv, use_reentrant=False)
        else:
            a = core(qkv)
        a = a.reshape(S, B, self.nq * self.hd)
        if sp_group is not None:
            return tpl.linear_rs(a, self.o_proj.weight, self.o_proj.bias, sp_group)
        return self.o_proj(a)


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig, pc: ParallelContext, dtype=None, device=None):
        super().__init__()
        self.inter = cfg.intermediate_size // pc.tp_size
        self.gate_up_proj = Linear(cfg.hidden_size, 2 * self.inter, cfg.mlp_bias, dtype, device)
        self.down_proj = Linear(self.inter, cfg.hidden_size, cfg.mlp_bias, dtype, device)

    def forward(self, h, sp_group=None):
        if sp_group is not None:
            gu = tpl.ag_linear(h, self.gate_up_proj.weight, self.gate_up_proj.bias, sp_group)
            return tpl.linear_rs(F_.swiglu(gu), self.down_proj.weight, self.down_proj.bias, sp_group)
        gu = self.gate_up_proj(h)
        consumer = isinstance(self.gate_up_proj, Linear)
        if isinstance(self.down_proj, Linear):
            # the down projection's input-gradient GEMM carries the SwiGLU backward in its epilogue
            return F_.swiglu_down(gu, self.down_proj.weight, self.down_proj.bias, dy_t_consumer=consumer)
        return self.down_proj(F_.swiglu(gu, dy_t_consumer=consumer))


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig, pc: ParallelContext, layer_idx: int, dtype=None, device=None):
        super().__init__()
        self.pc = pc
        self.layer_idx = layer_idx
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, dtype, device)
        self.self_attn = LlamaAttention(cfg, pc, dtype, device)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, dtype, device)
        self.mlp = LlamaMLP(cfg, pc, dtype, device)
        self.sp_overlap = bool(getattr(cfg, "tp_comm_overlap", True))

    def attn_block(self, h, rt, g):
        """Attention on the (sequence-sharded when TP) normed input; returns the sharded output."""
        if g is None:
            return self.self_attn(h, rt)
        if self.sp_overlap:
            return self.self_attn(h, rt, sp_group=g)
        return tpl.scatter_seq(self.self_attn(tpl.gather_seq(h, g), rt), g)

    def mlp_block(self, h, g):
        if g is None:
            return self.mlp(h)
        if self.sp_overlap:
            return self.mlp(h, sp_group=g)
        return tpl.scatter_seq(self.mlp(tpl.gather_seq(h, g)), g)

    def forward(self, x, residual, rt):
        g = self.pc.tp_group if self.pc.tp else None
        if residual is None:
            h, residual = self.input_layernorm(x), x
        else:
            h, residual = self.input_layernorm(x, residual)
        a = self.attn_block(h, rt, g)
        h, residual = self.post_attention_layernorm(a, residual)
        return self.mlp_block(h, g), residual


def _pad_seq(pad: int, input_ids, position_ids, segment_ids, inputs_embeds):
    """Right-pad a batch by ``pad`` tokens along the sequence (see Llama.hidden_states)."""
    import torch.nn.functional as Fn
    if input_ids is not None:
        B, S = input_ids.shape
        input_ids = Fn.pad(input_ids, (0, pad), value=0)
    else:
        B, S = inputs_embeds.shape[:2]
        inputs_embeds = Fn.pad(inputs_embeds, (0, 0, 0, pad))
    dev = (input_ids if input_ids is not None else inputs_embeds).device
    if position_ids is None:
        position_ids = torch.arange(S, device=dev).unsqueeze(0).expand(B, S)
    position_ids = Fn.pad(position_ids.to(dev).long().expand(B, S), (0, pad), value=0)
    if segment_ids is not None:
        seg = segment_ids.to(dev)
        fresh = seg.max() + 1  # the padding forms a segment of its own (device op, no host sync)
        segment_ids = torch.cat([seg, fresh.expand(B, pad).to(seg.dtype)], 1)
    return input_ids, position_ids, segment_ids, inputs_embeds


class Llama(BaseModel):
    config_class = LlamaConfig
    hf_model_type = "llama"
    decoder_layer_class = LlamaDecoderLayer

    def __init__(self, config: LlamaConfig, pc: ParallelContext | None = None, dtype=None, device=None):
        super().__init__(config, pc)
        cfg = config
        if dtype is None:
            dtype = cfg.torch_dtype if isinstance(cfg.torch_dtype, torch.dtype) else torch.float32
        self.embed_tokens = VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, self.pc, dtype, device)
        self.layers = nn.ModuleList(
            [self.decoder_layer_class(cfg, self.pc, i, dtype, device) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, dtype, device)
        if cfg.tie_word_embeddings:
            self.lm_head = None
        else:
            self.lm_head = Linear(cfg.hidden_size, self.embed_tokens.weight.shape[0], False, dtype, device)
        self.rope = RopeTables(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling, cfg.max_position_embeddings)
        self.gradient_checkpointing = cfg.enable_gradient_checkpointing
        mark_tp_replicated(self)

    # ------------------------------------------------------------------ weights
    def lm_head_weight(self) -> torch.Tensor:
        return self.embed_tokens.weight if self.lm_head is None else self.lm_head.weight

    def get_input_embeddings(self):
        return self.embed_tokens

    def get_output_embeddings(self):
        return self.lm_head if self.lm_head is not None else self.embed_tokens

    def init_weights(self, seed: int = 0):
        """Normal(0, initializer_range) for matrices, ones for norms, zero pad row; per-shard seeded."""
        std = self.config.initializer_range
        for name, p in self.named_parameters():
            gen = torch.Generator(device=p.device).manual_seed(
                (seed * 1000003 + zlib.crc32(name.encode()) * 31 + self.pc.tp_rank) & 0x7FFFFFFFFFFFFFFF)
            with torch.no_grad():
                if name.endswith("layernorm.weight") or name == "norm.weight" or p.dim() == 1:
                    if "norm" in name:
                        p.fill_(1.0)
                    else:
                        p.zero_()
                else:
                    normal_(p, std, gen)
        pad = self.config.pad_token_id
        if pad is not None:
            e = self.embed_tokens
            if e.v0 <= pad < e.v1:
                with torch.no_grad():
                    e.weight[pad - e.v0].zero_()

    def fsdp_units(self):
        # last unit: final norm + lm_head, hooked on the norm (called first)
        tail = [m for m in (self.norm, self.lm_head) if m is not None]
        return [self.embed_tokens, *self.layers, (self.norm, tail)]

    # ------------------------------------------------------------------ forward
    def _runtime(self, input_ids, position_ids, segment_ids, device, S, B):
        if position_ids is None:
            position_ids = torch.arange(S, device=device).unsqueeze(0).expand(B, S)
        else:
            position_ids = position_ids.to(device).long().expand(B, S)
        n_pos = S
        if self.rope.dynamic:
            # dynamic NTK: the reference sizes the rescale by max(position_ids) + 1 (packed rows restart
            # their positions), llama_model.py:367-371; one host read, for this rope type only
            n_pos = int(position_ids.max()) + 1
        cos, sin = self.rope.get(device, max(S, n_pos), ntk_positions=n_pos)
        impl = self.config.resolved_attn_implementation(device.type)
        selective = self.gradient_checkpointing and self.config.recompute_granularity == "selective"
        seg_info = rope_tok = None
        if device.type == "cuda" and impl in ("flash", "flash_attention_2", "hip"):
            if segment_ids is not None:
                # run bounds and block orders, shared by every layer's attention
                seg_info = F_.segment_info(segment_ids, doc_major=(self.config.num_key_value_heads ==
                                                                   self.config.num_attention_heads))
            if F_.ROPE_FUSED[0] != "off":  # per-token RoPE table rows for the attention kernels, shared by every layer
                rope_tok = F_.rope_token_tables(position_ids, cos, sin)
        return {"positions": position_ids, "cos": cos, "sin": sin, "segment_ids": segment_ids, "impl": impl,
                "selective": selective, "seg_info": seg_info, "rope_tok": rope_tok}

    def hidden_states(self, input_ids=None, position_ids=None, segment_ids=None, inputs_embeds=None,
                      gather_sequence: bool = True, embed_hook=None):
        """Post-norm hidden states, sequence-major [S, B, H] (full sequence unless gather_sequence=False).

        Under TP + SP the sequence is sharded over the TP ranks: a length that does not divide by the TP
        size is right-padded to the next multiple (pad tokens: id 0 / zero embeddings, position 0, their
        own segment) and the padding is stripped again from the gathered output. Padding at the END
        never changes a real token's output (causal attention), so any S works, as with DTensor
        Shard(1) in the reference (llama_model.py:197-244)."""
        S_real = None
        if self.pc.tp:
            L = (input_ids if input_ids is not None else inputs_embeds).shape[1]
            pad = (-L) % self.pc.tp_size
            if pad:
                input_ids, position_ids, segment_ids, inputs_embeds = _pad_seq(
                    pad, input_ids, position_ids, segment_ids, inputs_embeds)
                S_real = L
        if input_ids is not None:
            B, S = input_ids.shape
            device = input_ids.device
            x = self.embed_tokens(input_ids.t().contiguous())
        else:
            B, S = inputs_embeds.shape[:2]
            device = inputs_embeds.device
            x = inputs_embeds.transpose(0, 1).contiguous()
            if self.pc.tp:
                x = tpl.split_seq(x, self.pc.tp_group)
        if embed_hook is not None:
            x = embed_hook(x)
        rt = self._runtime(input_ids, position_ids, segment_ids, device, S, B)
        residual = None
        gran = self.config.recompute_granularity
        for layer in self.layers:
            if (self.gradient_checkpointing and gran in ("full", "full_keep_attention") and self.training
                    and torch.is_grad_enabled()):
                kw = {"use_reentrant": False}
                if gran == "full_keep_attention":
                    kw["context_fn"] = keep_attention_context
                if residual is None:
                    x, residual = ckpt.checkpoint(lambda a, lay=layer: lay(a, None, rt), x, **kw)
                else:
                    x, residual = ckpt.checkpoint(lambda a, r, lay=layer: lay(a, r, rt), x, residual, **kw)
            else:
                x, residual = layer(x, residual, rt)
        h, _ = self.norm(x, residual)
        if gather_sequence and self.pc.tp:
            h = tpl.gather_seq(h, self.pc.tp_group)
            if S_real is not None:
                h = h[:S_real]
        return h

    def forward(self, input_ids=None, attention_mask=None, position_ids=None, inputs_embeds=None,
                return_last_hidden_states: bool = False, segment_ids=None) -> CausalLMOutput:
        """Reference-compatible forward returning logits [B, S, V_local] (vocab-sharded under TP)."""
        if segment_ids is None and attention_mask is not None:
            segment_ids = attention_mask
        h = self.hidden_states(input_ids, position_ids, segment_ids, inputs_embeds)
        logits = F_.linear(h, self.lm_head_weight()).transpose(0, 1)
        return CausalLMOutput(logits=logits, last_hidden_states=h.transpose(0, 1) if return_last_hidden_states
                              else None)

    # ------------------------------------------------------------------ HF conversion
    def _sizes(self):
        c = self.config
        return c.num_attention_heads * c.head_dim, c.num_key_value_heads * c.head_dim

    @classmethod
    def convert_state_dict_from_hf(cls, sd, config: LlamaConfig):
        out = {}
        L = config.num_hidden_layers
        for k, v in sd.items():
            k2 = k[len("model."):] if k.startswith("model.") else k
            out[k2] = v
        for i in range(L):
            p = f"layers.{i}."
            if p + "self_attn.q_proj.weight" not in out:
                continue  # a partial (streamed, one layer at a time) state dict
            q, kk, vv = (out.pop(p + f"self_attn.{n}_proj.weight") for n in ("q", "k", "v"))
            out[p + "self_attn.qkv_proj.weight"] = torch.cat([q, kk, vv], 0)
            if p + "self_attn.q_proj.bias" in out:
                out[p + "self_attn.qkv_proj.bias"] = torch.cat(
                    [out.pop(p + f"self_attn.{n}_proj.bias") for n in ("q", "k", "v")], 0)
            g, u = out.pop(p + "mlp.gate_proj.weight"), out.pop(p + "mlp.up_proj.weight")
            out[p + "mlp.gate_up_proj.weight"] = torch.cat([g, u], 0)
            if p + "mlp.gate_proj.bias" in out:
                out[p + "mlp.gate_up_proj.bias"] = torch.cat(
                    [out.pop(p + "mlp.gate_proj.bias"), out.pop(p + "mlp.up_proj.bias")], 0)
        out.pop("rotary_emb.inv_freq", None)
        if config.tie_word_embeddings:
            out.pop("lm_head.weight", None)
        return out

    @classmethod
    def convert_state_dict_to_hf(cls, sd, config: LlamaConfig):
        out = {}
        qd = config.num_attention_heads * config.head_dim
        kd = config.num_key_value_heads * config.head_dim
        for k, v in sd.items():
            if ".self_attn.qkv_proj." in k:
                pre, suf = k.split(".self_attn.qkv_proj.")
                q, kk, vv = torch.split(v, [qd, kd, kd], 0)
                for n, t in zip(("q", "k", "v"), (q, kk, vv)):
                    out[f"model.{pre}.self_attn.{n}_proj.{suf}"] = t
            elif ".mlp.gate_up_proj." in k:
                pre, suf = k.split(".mlp.gate_up_proj.")
                g, u = torch.chunk(v, 2, 0)
                out[f"model.{pre}.mlp.gate_proj.{suf}"] = g
                out[f"model.{pre}.mlp.up_proj.{suf}"] = u
            elif k.startswith("lm_head."):
                out[k] = v
            else:
                out["model." + k] = v
        if config.tie_word_embeddings:
            out["lm_head.weight"] = out["model.embed_tokens.weight"]
        return out

    def hf_config_dict(self) -> dict:
        c = self.config
        d = {
            "architectures": ["LlamaForCausalLM"], "model_type": "llama", "vocab_size": c.vocab_size,
            "hidden_size": c.hidden_size, "intermediate_size": c.intermediate_size,
            "num_hidden_layers": c.num_hidden_layers, "num_attention_heads": c.num_attention_heads,
            "num_key_value_heads": c.num_key_value_heads, "head_dim": c.head_dim, "hidden_act": "silu",
            "max_position_embeddings": c.max_position_embeddings, "initializer_range": c.initializer_range,
            "rms_norm_eps": c.rms_norm_eps, "pad_token_id": c.pad_token_id, "bos_token_id": c.bos_token_id,
            "eos_token_id": c.eos_token_id, "tie_word_embeddings": c.tie_word_embeddings,
            "rope_theta": c.rope_theta, "rope_scaling": c.rope_scaling, "attention_bias": c.attention_bias,
            "attention_dropout": c.attention_dropout, "mlp_bias": c.mlp_bias,
        }
        return d

    # ------------------------------------------------------------------ TP sharding of full state dicts
    def _tp_rule(self, key: str):
        """Return (kind, sizes) where kind in {rep, rows, cols, fused, vocab}."""
        c = self.config
        if key.endswith("qkv_proj.weight") or key.endswith("qkv_proj.bias"):
            qd, kd = self._sizes()
            return "fused", [qd, kd, kd]
        if key.endswith("gate_up_proj.weight") or key.endswith("gate_up_proj.bias"):
            return "fused", [c.intermediate_size, c.intermediate_size]
        if key.endswith("o_proj.weight") or key.endswith("down_proj.weight"):
            return "cols", None
        if key == "embed_tokens.weight" or key == "lm_head.weight":
            return "vocab", None
        return "rep", None

    def shard_full_state_dict(self, full):
        pc = self.pc
        if not pc.tp:
            return full
        out = {}
        for k, v in full.items():
            kind, sizes = self._tp_rule(k)
            if kind == "fused":
                out[k] = tpl.shard_fused_rows(v, sizes, pc.tp_rank, pc.tp_size)
            elif kind == "cols":
                out[k] = tpl.shard_cols(v, pc.tp_rank, pc.tp_size)
            elif kind == "vocab":
                per = math.ceil(v.shape[0] / pc.tp_size)
                s = v[per * pc.tp_rank: per * (pc.tp_rank + 1)]
                if s.shape[0] < per:
                    s = torch.cat([s, s.new_zeros(per - s.shape[0], *s.shape[1:])], 0)
                out[k] = s
            else:
                out[k] = v
        return out

    def gather_full_state_dict(self) -> dict[str, torch.Tensor]:
        """All-gather TP shards into a full (HF-convertible) state dict (CPU tensors)."""
        sd = {k: v.detach() for k, v in self.state_dict().items()}
        pc = self.pc
        if not pc.tp:
            return {k: v.to("cpu", copy=True) for k, v in sd.items()}
        import torch.distributed as dist
        out = {}
        for k, v in sd.items():
            kind, sizes = self._tp_rule(k)
            if kind == "rep":
                out[k] = v.to("cpu", copy=True)
                continue
            parts = [torch.empty_like(v) for _ in range(pc.tp_size)]
            dist.all_gather(parts, v.contiguous(), group=pc.tp_group)
            parts = [p.cpu() for p in parts]
            if kind == "fused":
                out[k] = tpl.unshard_fused_rows(parts, sizes)
            elif kind == "cols":
                out[k] = torch.cat(parts, 1)
            else:
                out[k] = torch.cat(parts, 0)[: self.config.vocab_size]
        return out


def mark_tp_replicated(model: BaseModel):
    """Tag parameters that are replicated across TP ranks (their grads need a TP all-reduce)."""
    if not model.pc.tp:
        return
    for n, p in model.named_parameters():
        if model._tp_rule(n)[0] == "rep":
            p.tp_replicated = True
