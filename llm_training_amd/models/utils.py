"""Model construction helpers (reference src/llm_training/models/utils/utils.py:8-64).

``init_on_device(dev)`` builds modules with their parameters (and optionally buffers) created on
``dev``; ``init_empty_weights()`` is the meta-device form used to instantiate large models without
allocating memory. Our own models take a ``device=`` argument and build weights in place on the GPU
(TP-sharded), so these are for user code and the HF wrapper.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn as nn


@contextlib.contextmanager
def init_on_device(device: torch.device | str, include_buffers: bool = False):
    device = torch.device(device)
    if include_buffers:
        # every tensor factory call inside defaults to `device`
        with device:
            yield
        return
    orig = nn.Module.register_parameter

    def register_parameter(module, name, param):
        orig(module, name, param)
        p = module._parameters.get(name)
        if p is not None and p.device != device:
            module._parameters[name] = type(p)(p.detach().to(device), requires_grad=p.requires_grad)

    nn.Module.register_parameter = register_parameter
    try:
        yield
    finally:
        nn.Module.register_parameter = orig


def init_empty_weights(include_buffers: bool = False):
    return init_on_device(torch.device("meta"), include_buffers=include_buffers)


def _keep_attention_policy(ctx, op, *args, **kwargs):
    from torch.utils.checkpoint import CheckpointPolicy
    if str(op).startswith("llmt.flash_attn_fwd"):  # the OpOverload llmt::flash_attn_fwd.default
        return CheckpointPolicy.MUST_SAVE
    return CheckpointPolicy.PREFER_RECOMPUTE


def keep_attention_context():
    """Selective-checkpoint contexts for ``recompute_granularity: full_keep_attention``: a checkpointed
    decoder layer saves the flash-attention forward's outputs (O and the LSE) and recomputes everything
    else in backward."""
    from torch.utils.checkpoint import create_selective_checkpoint_contexts
    return create_selective_checkpoint_contexts(_keep_attention_policy)
