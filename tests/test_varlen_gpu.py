"""Packed-document (varlen) flash attention: random contiguous segment layouts vs the fp32 oracle, and
the work it skips (reference: flash_attn_varlen_func, src/llm_training/ops/attention_op.py:606-619)."""
import time

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from llm_training_amd.ops import fused as F_
from llm_training_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    """Relative error, floored at an absolute 1e-3 per element: one-token documents have exactly zero
    dQ / dK (a query that sees only itself), where bf16 rounding noise would be "infinitely" relative."""
    a, b = a.float(), b.float()
    return ((a - b).norm() / max(b.norm().item(), 1e-3 * b.numel() ** 0.5)).item()


def _layout(S, lengths, pad, left_pad=False):
    """Segment ids 1..k as contiguous runs of the given lengths (cycled to fill S), then `pad` zeros."""
    ids, i, n = [], 0, 0
    body = S - pad
    while n < body:
        ln = min(lengths[i % len(lengths)], body - n)
        ids += [i + 1] * ln
        n += ln
        i += 1
    seg = [0] * pad + ids if left_pad else ids + [0] * pad
    return torch.tensor(seg, dtype=torch.int32, device=DEV)


def _check(B, S, Hq, Hkv, D, seg, causal=True, window=-1):
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = F_.flash_attention(q, k, v, causal, seg, window)
    do = torch.randn_like(o)
    (o.float() * do.float()).sum().backward()
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = ref.attention(qr, kr, vr, causal, seg, window)
    (orf * do.float()).sum().backward()
    real = (seg != 0).view(B, S, 1, 1)  # padding rows' outputs are unspecified
    errs = (_rel(o * real, orf * real), _rel(q.grad * real, qr.grad * real), _rel(k.grad, kr.grad),
            _rel(v.grad, vr.grad))
    assert errs[0] < 2e-2 and max(errs[1:]) < 4e-2, errs


@settings(max_examples=10, deadline=None, suppress_health_check=list(HealthCheck))
@given(S=st.sampled_from([257, 1000, 2048, 3001]),
       lengths=st.lists(st.integers(1, 1500), min_size=1, max_size=6),
       pad=st.integers(0, 200), left=st.booleans(),
       geo=st.sampled_from([(4, 4, 128), (8, 2, 128), (4, 2, 64), (4, 4, 96), (8, 2, 96)]), causal=st.booleans())
def test_varlen_random_layouts(S, lengths, pad, left, geo, causal):
    Hq, Hkv, D = geo
    pad = min(pad, S - 1)
    seg = torch.stack([_layout(S, lengths, pad, left), _layout(S, lengths[::-1], 0)])
    _check(2, S, Hq, Hkv, D, seg, causal=causal)


@pytest.mark.parametrize("D", [128, 96])
def test_varlen_8192_many_docs(D):
    """Production length: 8192 tokens, documents of 37..2900 tokens, GQA."""
    S = 8192
    seg = _layout(S, [1200, 37, 2900, 511, 640, 129], 100)[None]
    _check(1, S, 4 if D == 128 else 2, 2 if D == 128 else 2, D, seg)


def _time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def test_varlen_skips_cross_document_tiles():
    """8 equal documents in an 8192-token row cost ~1/8 of full causal attention: forward + backward at
    least 3x faster (Llama-3-8B head geometry)."""
    B, S, Hq, Hkv, D = 1, 8192, 32, 8, 128
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16)
    seg = (torch.arange(S, device=DEV, dtype=torch.int32) // (S // 8) + 1)[None]
    info = F_.segment_info(seg)

    def run(s):
        o = F_.flash_attention(q, k, v, True, s, seg_info=info if s is not None else None)
        o.backward(do)

    full = _time(lambda: run(None))
    packed = _time(lambda: run(seg))
    print(f"causal fwd+bwd {full:.3f} ms, 8 packed docs {packed:.3f} ms ({full / packed:.2f}x)")
    assert full / packed >= 3.0, (full, packed)


def _fwd_bwd(q, k, v, do, seg):
    qq, kk, vv = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    info = F_.segment_info(seg) if seg is not None else None
    o = F_.flash_attention(qq, kk, vv, causal=True, segment_ids=seg, seg_info=info)
    o.backward(do)
    return o.detach(), qq.grad, kk.grad, vv.grad


@pytest.mark.parametrize("Hq,Hkv,D", [(8, 2, 128), (4, 4, 128), (4, 4, 96), (4, 4, 64)])
@pytest.mark.parametrize("packed", [False, True])
def test_attention_kernel_variants_bitwise(Hq, Hkv, D, packed, monkeypatch):
    """The packed-block work orders (LLMT_SEG_ORDER 0 / 2), the batch-interleaved dense block order
    (LLMT_FA_BMAJOR=0) and the prologue issue order (LLMT_FA_EARLY_DMA=0) compute exactly what the default
    kernels compute: same per-head math, only the block -> workgroup assignment or the issue order differs."""
    torch.manual_seed(0)
    B, S = 2, 1024
    q = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16)
    do = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16)
    seg = _layout(S, [300, 17, 129, 64, 1, 200], 40).expand(B, S).contiguous() if packed else None
    base = _fwd_bwd(q, k, v, do, seg)
    forms = [] if packed else [("LLMT_FA_BMAJOR", "0")]
    if packed:  # index order, and document-major order (the MHA default of the models)
        forms += [("LLMT_SEG_ORDER", "0"), ("LLMT_SEG_ORDER", "2")]
    forms += [("LLMT_FA_EARLY_DMA", "0")]  # prologue issue order: row loads before the first ring tiles
    for env, val in forms:
        monkeypatch.setenv(env, val)
        got = _fwd_bwd(q, k, v, do, seg)
        monkeypatch.delenv(env)
        for name, x, y in zip(("o", "dq", "dk", "dv"), got, base):
            assert torch.equal(x, y), f"{env}={val}: {name} differs"


@pytest.mark.parametrize("Hq,Hkv,D", [(8, 2, 128), (8, 4, 64), (4, 4, 96)])
@pytest.mark.parametrize("packed", [False, True])
def test_backward_prep_inside_dq_matches_generic(Hq, Hkv, D, packed, monkeypatch):
    """The dQ kernel computes delta = rowsum(O * dO) and writes the per-32-row constants the dK/dV kernel
    reads, against the generic backward kernels (LLMT_FA_GENERIC=1: their own delta pass, no row constants):
    same gradients up to summation order. A ragged length (S = 300: the last 128-row dQ block has waves
    wholly past the sequence end, which must not write a tile) with several heads and batch rows, where a
    stray tile write would land in the next head's constants."""
    torch.manual_seed(0)
    B, S = 2, 300
    q = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device=DEV, dtype=torch.bfloat16)
    do = torch.randn(B, S, Hq, D, device=DEV, dtype=torch.bfloat16)
    seg = _layout(S, [90, 17, 130], 11).expand(B, S).contiguous() if packed else None
    fused = _fwd_bwd(q, k, v, do, seg)
    monkeypatch.setenv("LLMT_FA_GENERIC", "1")
    sep = _fwd_bwd(q, k, v, do, seg)
    monkeypatch.delenv("LLMT_FA_GENERIC")
    real = (seg != 0).view(B, S, 1, 1) if packed else torch.ones(B, S, 1, 1, dtype=torch.bool, device=DEV)
    for name, x, y in zip(("o", "dq", "dk", "dv"), fused, sep):
        assert _rel(x * real, y * real) < 1e-2, name
