"""The 64-keys-per-wave dK/dV kernel (``fa_bwd_dkdv6_kernel``, LLMT_FA_BWD_VARIANT=7: dV^T / dK^T of two
32-key halves in the asm-owned accumulator registers, V of the 256-key block in LDS) against the fp32 torch
oracle and the default dK/dV kernel: causal, non-causal, sliding window, sequence ends inside a tile and a
block, a block with fewer query tiles than the ring is deep, GQA and MHA."""
import pytest
import torch

from llm_training_amd.ops import fused as F_
from llm_training_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("B,S,Hq,Hkv,causal,window", [(1, 64, 1, 1, True, -1), (2, 300, 8, 2, True, -1),
                                                      (1, 300, 2, 1, False, -1), (1, 1000, 4, 1, True, 100),
                                                      (1, 1024, 4, 1, False, 300), (2, 2048, 8, 2, True, -1),
                                                      (1, 520, 4, 4, True, -1), (1, 96, 2, 2, False, -1)])
def test_dkdv6_matches_fp32_and_default(monkeypatch, B, S, Hq, Hkv, causal, window):
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, 128, device="cuda", dtype=torch.bfloat16)
    grads = {}
    for var in ("5", "7"):
        monkeypatch.setenv("LLMT_FA_BWD_VARIANT", var)
        o = F_.flash_attention(q, k, v, causal, None, window)
        grads[var] = torch.autograd.grad(o, (q, k, v), do)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = ref.attention(qr, kr, vr, causal, None, window)
    gr = torch.autograd.grad(orf, (qr, kr, vr), do.float())
    for a, r, d in zip(grads["7"], gr, grads["5"]):
        assert _rel(a, r) < 5e-3
        assert _rel(a, d) < 5e-3
    assert torch.equal(grads["7"][0], grads["5"][0])  # dQ comes from the same kernel
