"""The hand-allocated forward kernel (``fa_fwd4_kernel``, LLMT_FA_FWD_VARIANT=10: one wave per SIMD, 64 query
rows per wave, O^T / Q / K in asm-owned accumulator registers) against the fp32 torch oracle and the default
forward: causal, non-causal, sliding window, sequence ends inside a tile, GQA; the backward (which reads the
forward's LSE) must give the same gradients."""
import os

import pytest
import torch

from llm_training_amd.ops import fused as F_
from llm_training_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("B,S,Hq,Hkv,causal,window", [(2, 300, 8, 2, True, -1), (1, 64, 1, 1, True, -1),
                                                      (1, 300, 2, 1, False, -1), (1, 1000, 4, 1, True, 100),
                                                      (1, 1024, 4, 1, False, 300), (2, 2048, 8, 2, True, -1)])
def test_fwd4_matches_fp32_and_default(monkeypatch, B, S, Hq, Hkv, causal, window):
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16)
    outs = {}
    for var in ("4", "10"):
        monkeypatch.setenv("LLMT_FA_FWD_VARIANT", var)
        o = F_.flash_attention(q, k, v, causal, None, window)
        outs[var] = (o.detach(), torch.autograd.grad(o, (q, k, v), do))
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = ref.attention(qr, kr, vr, causal, None, window)
    gr = torch.autograd.grad(orf, (qr, kr, vr), do.float())
    o10, g10 = outs["10"]
    assert _rel(o10, orf) < 5e-3
    assert (o10.float() - outs["4"][0].float()).abs().max().item() < 2e-2
    for a, r in zip(g10, gr):
        assert _rel(a, r) < 5e-3
