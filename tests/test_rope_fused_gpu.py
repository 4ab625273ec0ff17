"""RoPE fused into the attention kernels (ops/fused.py _RopeFlashAttnFn, csrc/flash_attn.hip rope_frags /
rope_acc_inv): forward output and dQKV against the fp32 oracle (reference ops/rope_op.py:10-20 + eager
attention) and against the standalone-pass form (LLMT_ROPE_FUSED=0), for D = 64 / 96 / 128, GQA and MHA,
packed rows whose positions restart per document, tables longer than the sequence (LongRoPE-style offsets),
the batch-major HF layout, and the launch paths that fall back to the standalone rotation (generic kernels,
dropout, the opt-in forward / dK/dV variants)."""
import math

import pytest
import torch

from llm_training_amd.ops import fused as F_
from llm_training_amd.ops.rope_utils import compute_rope_tables

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _packed(B, S, gen):
    """segment ids of random documents per row and positions restarting at each document start"""
    seg = torch.zeros(B, S, dtype=torch.int64)
    pos = torch.zeros(B, S, dtype=torch.int64)
    for b in range(B):
        cuts = sorted(torch.randint(1, S, (5,), generator=gen).tolist())
        starts = [0] + cuts
        for i, s0 in enumerate(starts):
            s1 = starts[i + 1] if i + 1 < len(starts) else S
            seg[b, s0:s1] = i + 1
            pos[b, s0:s1] = torch.arange(s1 - s0)
    return seg.to(DEV), pos.to(DEV)


def _run(qkv0, pos, cos, sin, nq, nkv, seg, mode, do, dropout_p=0.0, tok=False):
    F_.ROPE_FUSED[0] = mode
    try:
        qkv = qkv0.detach().clone().requires_grad_(True)
        torch.manual_seed(1234)  # the dropout seed comes from torch's CPU generator
        # tok: per-token table rows (the model's runtime dict), else the kernels index through the positions
        rt = F_.rope_token_tables(pos, cos, sin) if (tok and mode != "off") else None
        o = F_.rope_attention(qkv * 1.0, pos, cos, sin, nq, nkv, True, seg, dropout_p=dropout_p, rope_tok=rt)
        (o.float() * do.float()).sum().backward()
        return o.detach(), qkv.grad
    finally:
        F_.ROPE_FUSED[0] = "auto"


def _oracle(qkv0, pos, cos, sin, nq, nkv, seg, do):
    D = qkv0.shape[-1]
    qr = qkv0.detach().float().requires_grad_(True)
    o = F_._ref_rope_attention(qr.transpose(0, 1), pos, cos, sin, nq, nkv, True, seg, -1, 1 / math.sqrt(D),
                               "eager").transpose(0, 1)
    (o * do.float()).sum().backward()
    return o.detach(), qr.grad


@pytest.mark.parametrize("D", [64, 96, 128])
@pytest.mark.parametrize("heads", [(8, 2), (4, 4)])
@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("tok", [False, True])
@pytest.mark.parametrize("mode", ["bwd", "full"])
def test_rope_fused_attention_matches_oracle(D, heads, packed, tok, mode):
    nq, nkv = heads
    gen = torch.Generator().manual_seed(D + nq + packed)
    torch.manual_seed(D + nq)
    S, B = 384, 2
    qkv0 = torch.randn(S, B, nq + 2 * nkv, D, device=DEV, dtype=torch.bfloat16)
    if packed:
        seg, pos = _packed(B, S, gen)
        pos = pos + 1000  # positions past the sequence length: the table row, not the token index, matters
    else:
        seg, pos = None, torch.arange(S, device=DEV).expand(B, S) + 37
    cos, sin = compute_rope_tables(D, 4096, 10000.0, device=DEV)
    do = torch.randn(S, B, nq, D, device=DEV, dtype=torch.bfloat16)
    o, g = _run(qkv0, pos, cos, sin, nq, nkv, seg, mode, do, tok=tok)
    ou, gu = _run(qkv0, pos, cos, sin, nq, nkv, seg, "off", do)
    orf, grf = _oracle(qkv0, pos, cos, sin, nq, nkv, seg, do)
    assert _rel(o, orf) < 2e-2 and _rel(g, grf) < 4e-2
    # the fused form rounds rotated q once (as the standalone pass) and un-rotates the fp32 gradient before
    # its one bf16 rounding: at least as close to the oracle as the standalone form
    assert _rel(o, ou) < 1e-2
    assert _rel(g, grf) <= _rel(gu, grf) * 1.05 + 1e-4
    for h0, h1 in ((0, nq), (nq, nq + nkv), (nq + nkv, nq + 2 * nkv)):  # q / k / v parts each
        assert _rel(g[:, :, h0:h1], grf[:, :, h0:h1]) < 4e-2


def test_rope_fused_leaves_queries_unrotated():
    # "full": the saved qkv buffer keeps unrotated q (rotated k): selective recompute that skips the attention
    # forward sees the same buffer as a full forward
    F_.ROPE_FUSED[0] = "full"
    torch.manual_seed(0)
    S, B, nq, nkv, D = 256, 1, 4, 2, 128
    qkv = torch.randn(S, B, nq + 2 * nkv, D, device=DEV, dtype=torch.bfloat16)
    ref = qkv.clone()
    cos, sin = compute_rope_tables(D, 1024, 500000.0, device=DEV)
    pos = torch.arange(S, device=DEV).expand(B, S)
    try:
        with torch.no_grad():
            F_.rope_attention(qkv, pos, cos, sin, nq, nkv)
    finally:
        F_.ROPE_FUSED[0] = "auto"
    assert torch.equal(qkv[:, :, :nq], ref[:, :, :nq])
    assert not torch.equal(qkv[:, :, nq:nq + nkv], ref[:, :, nq:nq + nkv])
    assert torch.equal(qkv[:, :, nq + nkv:], ref[:, :, nq + nkv:])


@pytest.mark.parametrize("env", [("LLMT_FA_GENERIC", "1"), ("LLMT_FA_RANGE_MASK", "0"), ("LLMT_FA_EARLY_DMA", "0")])
@pytest.mark.parametrize("mode", ["bwd", "full"])
def test_rope_fused_fallback_paths(env, mode, monkeypatch):
    # launch paths without the in-kernel rotation: the dispatcher rotates into the scratch copy / runs the
    # inverse passes itself, so the op's contract holds on every path
    monkeypatch.setenv(*env)
    D = 128
    torch.manual_seed(3)
    S, B, nq, nkv = 512, 2, 8, 2
    qkv0 = torch.randn(S, B, nq + 2 * nkv, D, device=DEV, dtype=torch.bfloat16)
    pos = torch.arange(S, device=DEV).expand(B, S)
    cos, sin = compute_rope_tables(D, 1024, 10000.0, device=DEV)
    do = torch.randn(S, B, nq, D, device=DEV, dtype=torch.bfloat16)
    o, g = _run(qkv0, pos, cos, sin, nq, nkv, None, mode, do, tok=True)
    orf, grf = _oracle(qkv0, pos, cos, sin, nq, nkv, None, do)
    assert _rel(o, orf) < 2e-2 and _rel(g, grf) < 4e-2


@pytest.mark.parametrize("mode", ["bwd", "full"])
def test_rope_fused_dropout_matches_standalone(mode):
    # dropout runs the generic kernels (fallback rotation); same seed -> same keep-mask in both forms
    torch.manual_seed(5)
    S, B, nq, nkv, D = 256, 2, 4, 2, 64
    qkv0 = torch.randn(S, B, nq + 2 * nkv, D, device=DEV, dtype=torch.bfloat16)
    pos = torch.arange(S, device=DEV).expand(B, S)
    cos, sin = compute_rope_tables(D, 512, 10000.0, device=DEV)
    do = torch.randn(S, B, nq, D, device=DEV, dtype=torch.bfloat16)
    o, g = _run(qkv0, pos, cos, sin, nq, nkv, None, mode, do, dropout_p=0.1)
    ou, gu = _run(qkv0, pos, cos, sin, nq, nkv, None, "off", do, dropout_p=0.1)
    assert _rel(o, ou) < 1e-2 and _rel(g, gu) < 2e-2


@pytest.mark.parametrize("per_batch", [False, True])
def test_rope_fused_batch_major_hf_tables(per_batch):
    # the HF layout: batch-major qkv and per-token full-width tables (any rope_type, e.g. LongRoPE's scaled
    # frequencies) through rope_attention_bm
    torch.manual_seed(7)
    B, S, nq, nkv, D = 2, 320, 4, 4, 96
    qkv0 = torch.randn(B, S, nq + 2 * nkv, D, device=DEV, dtype=torch.bfloat16)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=DEV).float() / D)) / torch.linspace(1, 4, D // 2, device=DEV)
    t = torch.arange(S, device=DEV).float()[None, :, None] + (torch.arange(B, device=DEV).float()[:, None, None] * 500
                                                              if per_batch else 0)
    ang = t * inv
    emb = torch.cat([ang, ang], -1)
    cos, sin = (emb.cos() * 1.1).bfloat16(), (emb.sin() * 1.1).bfloat16()  # LongRoPE's attention factor
    do = torch.randn(B, S, nq, D, device=DEV, dtype=torch.bfloat16)
    outs = []
    for mode in ("bwd", "full", "off"):
        F_.ROPE_FUSED[0] = mode
        try:
            qkv = qkv0.clone().requires_grad_(True)
            o = F_.rope_attention_bm(qkv * 1.0, cos, sin, nq, nkv)
            (o.float() * do.float()).sum().backward()
            outs.append((o.detach(), qkv.grad))
        finally:
            F_.ROPE_FUSED[0] = "auto"
    qr = qkv0.float().requires_grad_(True)
    ct, st, pos = F_._token_tables(cos, sin, B, S)
    orf = F_._ref_rope_attention(qr, pos, ct, st, nq, nkv, True, None, -1, 1 / math.sqrt(D), "eager")
    (orf * do.float()).sum().backward()
    (ou, gu) = outs[-1]
    for o, g in outs[:-1]:
        assert _rel(o, orf) < 2e-2 and _rel(g, qr.grad) < 4e-2
        assert _rel(o, ou) < 1e-2 and _rel(g, gu) < 2e-2
