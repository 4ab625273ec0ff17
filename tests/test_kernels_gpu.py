"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (GPU only)."""
import math

import pytest
import torch

from llm_training_amd.ops import fused as F_
from llm_training_amd.ops import reference as ref
from llm_training_amd.ops.native import lib
from llm_training_amd.ops.rope_utils import compute_rope_tables

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_native_loaded():
    L = lib()
    assert hasattr(L, "rmsnorm_fwd")


@pytest.mark.parametrize("H", [768, 3072, 4096, 5120])
@pytest.mark.parametrize("residual", [False, True])
def test_rmsnorm(H, residual):
    torch.manual_seed(0)
    T = 1000
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True) if residual else None
    w = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16().requires_grad_(True)
    if residual:
        y, s = F_.rms_norm(x, w, 1e-5, r)
    else:
        y = F_.rms_norm(x, w, 1e-5)
    dy = torch.randn_like(y)
    ds = torch.randn_like(y) if residual else None
    (y.float() * dy.float()).sum().add((s.float() * ds.float()).sum() if residual else 0).backward()
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if residual else None
    sr = xr + rr if residual else xr
    yr = ref.rms_norm(sr, wr, 1e-5)
    ((yr * dy.float()).sum() + ((sr * ds.float()).sum() if residual else 0)).backward()
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    if residual:
        assert _rel(s, sr) < 1e-2
        assert _rel(r.grad, rr.grad) < 2e-2


@pytest.mark.parametrize("H", [3072, 4096])
def test_rmsnorm_bwd_frozen_weight(H):
    """No weight gradient wanted (a frozen norm weight): the kernel writes no dW partials (it once wrote
    nblocks x H of them into an H-float buffer) and dx is the same as with the weight gradient."""
    torch.manual_seed(0)
    T = 4099  # several blocks, a ragged last one
    L = lib()
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    dy, dres = torch.randn_like(x), torch.randn_like(x)
    rstd = L.rmsnorm_fwd(x, None, w, 1e-5)[2]
    dx, dw = L.rmsnorm_bwd(dy, x, w, rstd, dres, None, False, True)
    dx2, _ = L.rmsnorm_bwd(dy, x, w, rstd, dres, None, False, False)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx2)
    xf, wf, dyf = x.float(), w.float(), dy.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)
    dn = dyf * wf
    dx_ref = r * (dn - xf * r * (dn * xf * r).mean(-1, keepdim=True)) + dres.float()
    assert _rel(dx, dx_ref) < 1e-2
    assert _rel(dw, (dyf * (xf * r).bfloat16().float()).sum(0)) < 1e-2


@pytest.mark.parametrize("I", [512, 14336])
def test_swiglu(I):
    torch.manual_seed(0)
    gu = torch.randn(300, 2 * I, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    c = F_.swiglu(gu)
    dc = torch.randn_like(c)
    (c.float() * dc.float()).sum().backward()
    gr = gu.detach().float().requires_grad_(True)
    cr = ref.swiglu_fused(gr)
    (cr * dc.float()).sum().backward()
    assert _rel(c, cr) < 1e-2
    assert _rel(gu.grad, gr.grad) < 2e-2


@pytest.mark.parametrize("T", [65536, 131071 + 300])
def test_swiglu_rows_split_over_launches(T, monkeypatch):
    """The row-blocked SwiGLU kernels split T > 65535 rows (grid.y) into equal launches: forward and backward
    bitwise equal to the flat grid-stride kernels (LLMT_EW_ROWS=0)."""
    torch.manual_seed(0)
    I = 64
    gu = torch.randn(T, 2 * I, device=DEV, dtype=torch.bfloat16)
    dc = torch.randn(T, I, device=DEV, dtype=torch.bfloat16)

    def run():
        g = gu.clone().requires_grad_(True)
        c = F_.swiglu(g)
        c.backward(dc)
        return c.detach(), g.grad

    rows = run()
    monkeypatch.setenv("LLMT_EW_ROWS", "0")
    flat = run()
    assert torch.equal(rows[0], flat[0]) and torch.equal(rows[1], flat[1])


@pytest.mark.parametrize("D", [64, 96, 128])
def test_rope_inplace_roundtrip(D):
    torch.manual_seed(0)
    S, B, H = 257, 2, 6
    qkv = torch.randn(S, B, H, D, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (B, S), device=DEV)
    cos, sin = compute_rope_tables(D, 4096, 500000.0, device=DEV)
    x = qkv.clone()
    lib().rope_(x, pos.t().contiguous().reshape(-1), cos, sin, 4, False)
    cf, sf = F_.rope_tables_to_full(cos, sin, pos.t())  # [S, B, D]
    q = qkv[:, :, :4].float()
    exp = q * cf[:, :, None] + ref.rotate_half(q) * sf[:, :, None]
    assert _rel(x[:, :, :4], exp) < 1e-2
    assert torch.equal(x[:, :, 4:], qkv[:, :, 4:])
    lib().rope_(x, pos.t().contiguous().reshape(-1), cos, sin, 4, True)
    assert _rel(x, qkv) < 2e-2


@pytest.mark.parametrize("D", [64, 96, 128])
def test_rope_token_blocked_equals_flat(D, monkeypatch):
    """The token-blocked and LDS-staged RoPE kernels are bitwise equal to the flat grid-stride one, on a
    token count that is not a multiple of their token blocks, int32 and int64 positions, forward and inverse;
    an out-of-table position is clamped and flagged by both."""
    from llm_training_amd.ops.native import check_kernel_errors
    torch.manual_seed(0)
    T, H = 1023, 10
    qkv = torch.randn(T, H, D, device=DEV, dtype=torch.bfloat16)
    cos, sin = compute_rope_tables(D, 2048, 10000.0, device=DEV)
    for pos in (torch.randint(0, 2048, (T,), device=DEV), torch.randint(0, 2048, (T,), device=DEV).int()):
        for inv in (False, True):
            out = {}
            for mode in ("rows", "flat", "lds"):
                monkeypatch.setenv("LLMT_ROPE_KERNEL", mode)
                x = qkv.clone()
                lib().rope_(x, pos, cos, sin, 6, inv)
                out[mode] = x
            assert torch.equal(out["rows"], out["flat"]) and torch.equal(out["lds"], out["flat"])
            assert torch.equal(out["rows"][:, 6:], qkv[:, 6:])
    bad = torch.randint(0, 2048, (T,), device=DEV)
    bad[7] = 5000
    res = {}
    for mode in ("rows", "flat", "lds"):
        monkeypatch.setenv("LLMT_ROPE_KERNEL", mode)
        x = qkv.clone()
        lib().rope_(x, bad, cos, sin, 6, False)
        assert check_kernel_errors(raise_error=False), f"out-of-table position not flagged ({mode})"
        res[mode] = x
    assert torch.equal(res["rows"], res["flat"]) and torch.equal(res["lds"], res["flat"])


def test_swiglu_bwd_with_transposed_gradient(monkeypatch):
    """swiglu_bwd_tr: dgu equal to swiglu_bwd bitwise and dgu^T its exact transpose; through the ops, the
    gate_up weight gradient takes it (TN) and matches the path without it."""
    import llm_training_amd.ops.fused as fused
    torch.manual_seed(0)
    T, I = 4096, 512
    gu = torch.randn(T, 2 * I, device=DEV).bfloat16()
    dc = torch.randn(T, I, device=DEV).bfloat16()
    dgu, dgu_t = lib().swiglu_bwd_tr(gu, dc)
    assert torch.equal(dgu, lib().swiglu_bwd(gu, dc))
    assert torch.equal(dgu_t, dgu.t().contiguous())
    monkeypatch.setattr(fused, "GEMM_MODES", {"fwd": "lt", "dgrad": "lt", "wgrad": "lt"})
    x = torch.randn(T, 256, device=DEV).bfloat16()
    w_gu = (0.05 * torch.randn(2 * I, 256, device=DEV)).bfloat16()
    w_dn = (0.05 * torch.randn(256, I, device=DEV)).bfloat16()
    grads = []
    for on in (True, False):
        monkeypatch.setattr(fused, "FUSED_DY_T", [on])
        monkeypatch.setattr(fused, "_LAYOUT_CACHE", {})
        a = x.clone().requires_grad_(True)
        g1, g2 = w_gu.clone().requires_grad_(True), w_dn.clone().requires_grad_(True)
        y = fused.linear(fused.swiglu(fused.linear(a, g1)), g2)
        y.float().square().mean().backward()
        assert not fused._DY_T  # consumed
        grads.append((a.grad, g1.grad, g2.grad))
    for u, v in zip(*grads):
        assert _rel(u, v) < 1e-2
    want = ((dgu.float().t() @ x.float()))
    got = torch.empty(2 * I, 256, device=DEV, dtype=torch.float32)
    fused._DY_T[dgu.data_ptr()] = dgu_t
    assert fused.wgrad_into(got, dgu, x, False)
    assert _rel(got, want) < 1e-4


def test_kernel_index_checks():
    """Data-dependent indices out of range: the RoPE kernel clamps a position past its cos/sin table and
    the CE kernel skips a label outside the vocabulary, both flag the device error word, and
    check_kernel_errors() raises once (then the words are clear)."""
    from llm_training_amd.ops.native import check_kernel_errors
    check_kernel_errors(raise_error=False)
    torch.manual_seed(0)
    S, H, D, P = 64, 4, 128, 128
    cos, sin = compute_rope_tables(D, P, 10000.0, device=DEV)
    qkv = torch.randn(S, H, D, device=DEV, dtype=torch.bfloat16)
    pos = torch.arange(S, device=DEV)
    x = qkv.clone()
    lib().rope_(x, pos, cos, sin, H, False)
    assert check_kernel_errors() == []  # in-range positions: clean
    bad = pos.clone()
    bad[5] = P + 1000  # clamped to the last table row
    y = qkv.clone()
    lib().rope_(y, bad, cos, sin, H, False)
    with pytest.raises(RuntimeError, match="RoPE"):
        check_kernel_errors()
    assert check_kernel_errors() == []  # cleared
    want = qkv.clone()
    lib().rope_(want, torch.full_like(pos, P - 1), cos, sin, H, False)
    assert torch.equal(y[5], want[5]) and torch.equal(y[:5], x[:5])
    V = 1000
    logits = torch.randn(16, V, device=DEV).bfloat16()
    labels = torch.randint(0, V, (16,), device=DEV)
    labels[3] = -100
    lib().cross_entropy_(logits.clone(), labels, 0, -100, None, None, None, False)
    assert check_kernel_errors() == []
    labels[7] = V + 3
    _, _, loss = lib().cross_entropy_(logits.clone(), labels, 0, -100, None, None, None, False)
    assert torch.isfinite(loss).all()
    with pytest.raises(RuntimeError, match="label"):
        check_kernel_errors()


@pytest.mark.parametrize("V", [32064, 128256, 50257, 152064])  # one-pass kernel up to 131072, two-pass above and for V % 8 != 0
def test_cross_entropy(V):
    torch.manual_seed(0)
    N = 257
    logits = (3 * torch.randn(N, V, device=DEV)).bfloat16().requires_grad_(True)
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[::7] = -100
    loss = F_.cross_entropy(logits, labels)
    loss.backward()
    lr_ = logits.detach().float().requires_grad_(True)
    lref = torch.nn.functional.cross_entropy(lr_, labels, ignore_index=-100)
    lref.backward()
    assert abs(loss.item() - lref.item()) < 1e-3 * max(1, abs(lref.item()))
    assert _rel(logits.grad, lr_.grad) < 2e-2


def test_fused_linear_cross_entropy():
    torch.manual_seed(0)
    N, H, V = 600, 256, 32064
    h = torch.randn(N, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (0.05 * torch.randn(V, H, device=DEV)).bfloat16().requires_grad_(True)
    lab = torch.randint(0, V, (N,), device=DEV)
    lab[:50] = -100
    loss = F_.fused_linear_cross_entropy(h, w, lab, chunk_size=256)
    loss.backward()
    hr = h.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    lref = torch.nn.functional.cross_entropy(hr @ wr.t(), lab, ignore_index=-100)
    lref.backward()
    assert abs(loss.item() - lref.item()) < 1e-2
    assert _rel(h.grad, hr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2


@pytest.mark.parametrize("head", ["flce", "logps"])
def test_loss_head_weight_grad_accumulates_in_fp32(head):
    """lm_head dW summed over 4 row chunks: with an fp32 gradient buffer (bf16-mixed) it equals the
    single-chunk GEMM (fp32 accumulate, one rounding) to fp32 precision; with bf16 gradients it is
    rounded once, not once per chunk."""
    torch.manual_seed(0)
    N, H, V = 2048, 256, 8192

    def run(chunk, fp32_buf):
        h = torch.randn(N, H, device=DEV, generator=torch.Generator(DEV).manual_seed(1)).bfloat16()
        w = (0.05 * torch.randn(V, H, device=DEV, generator=torch.Generator(DEV).manual_seed(2))).bfloat16()
        lab = torch.randint(0, V, (N,), device=DEV, generator=torch.Generator(DEV).manual_seed(3))
        w.requires_grad_(True)
        if fp32_buf:
            w.main_grad = torch.zeros(V, H, device=DEV, dtype=torch.float32)
            w.grad_added = False
        if head == "flce":
            F_.fused_linear_cross_entropy(h, w, lab, chunk_size=chunk).backward()
        else:
            lp = F_.linear_token_logps(h, w, lab, chunk_size=chunk)
            (lp * torch.linspace(-1, 1, N, device=DEV)).sum().backward()
        return (w.main_grad if fp32_buf else w.grad).float(), h, w, lab

    g4, *_ = run(N // 4, True)
    g1, *_ = run(N, True)
    assert _rel(g4, g1) < 1e-5
    gb, h, w, lab = run(N // 4, False)
    hr, wr = h.float(), w.detach().float().requires_grad_(True)
    if head == "flce":
        torch.nn.functional.cross_entropy(hr @ wr.t(), lab).backward()
    else:
        (ref.token_logps(hr @ wr.t(), lab) * torch.linspace(-1, 1, N, device=DEV)).sum().backward()
    assert _rel(gb, wr.grad) < 8e-3  # bf16 dlogits operand + one final rounding


def test_linear_token_logps():
    torch.manual_seed(0)
    N, H, V = 300, 128, 5000
    h = torch.randn(N, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (0.1 * torch.randn(V, H, device=DEV)).bfloat16().requires_grad_(True)
    lab = torch.randint(0, V, (N,), device=DEV)
    lab[::5] = -100
    lp = F_.linear_token_logps(h, w, lab, chunk_size=128)
    g = torch.randn_like(lp)
    (lp * g).sum().backward()
    hr = h.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    lpr = ref.token_logps(hr @ wr.t(), lab)
    (lpr * g).sum().backward()
    assert _rel(lp, lpr) < 1e-2
    assert _rel(h.grad, hr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2


def test_adamw_matches_torch():
    torch.manual_seed(0)
    n = 4096 * 3
    p0 = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV).bfloat16()
    p, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    pout = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    scale = torch.tensor([0.5], device=DEV)
    tp = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([tp], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(1, 4):
        lib().adamw_(p, m, v, g, pout, 1e-2, 0.9, 0.95, 1e-8, 0.1, step, scale)
        tp.grad = g.float() * 0.5
        opt.step()
    assert _rel(p, tp.detach()) < 1e-5
    assert _rel(pout, tp.detach()) < 1e-2
    out = torch.zeros(1, device=DEV)
    lib().sumsq_(g, out)
    assert abs(out.item() - g.float().pow(2).sum().item()) / out.item() < 1e-4
    # the 16-byte bf16 path (n % 8 == 0, aligned) incl. a grid-stride tail, the 8-byte path (odd offset)
    for m_ in (8 * 1024 * 300 + 8, 8 * 1024 * 256 * 3 + 8 * 17):
        gg = torch.randn(m_ + 4, device=DEV).bfloat16()
        for view in (gg[:m_], gg[4:4 + m_]):
            o = torch.zeros(1, device=DEV)
            lib().sumsq_(view, o)
            ref_ = view.float().pow(2).sum().item()
            assert abs(o.item() - ref_) / ref_ < 1e-4


def _attn_case(B, S, Hq, Hkv, D, causal=True, seg=None, window=-1, layout="bshd"):
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
    errs = (_rel(o, orf), _rel(q.grad, qr.grad), _rel(k.grad, kr.grad), _rel(v.grad, vr.grad))
    assert errs[0] < 2e-2, errs
    assert max(errs[1:]) < 4e-2, errs


@pytest.mark.parametrize("D", [64, 96, 128])
@pytest.mark.parametrize("Hq,Hkv", [(4, 4), (8, 2)])
def test_flash_attention_causal(D, Hq, Hkv):
    _attn_case(2, 300, Hq, Hkv, D)


def test_flash_attention_noncausal():
    _attn_case(1, 200, 4, 2, 128, causal=False)


def test_flash_attention_segments():
    B, S = 2, 384
    seg = torch.ones(B, S, dtype=torch.int32, device=DEV)
    seg[0, 100:250] = 2
    seg[0, 250:] = 3
    seg[1, 300:] = 0
    _attn_case(B, S, 4, 2, 128, seg=seg)


def test_flash_attention_window():
    _attn_case(1, 512, 4, 4, 96, window=100)


@pytest.mark.parametrize("causal,window", [(True, 100), (False, -1), (True, -1)])
def test_flash_attention_d128_pipeline(causal, window):
    # D = 128 backward runs the LDS-DMA ring kernels: long enough for several ring wraps and GQA head loops
    _attn_case(2, 1100, 8, 2, 128, causal=causal, window=window)


def test_flash_attention_d128_segments_gqa():
    B, S = 1, 777
    seg = torch.zeros(B, S, dtype=torch.int32, device=DEV)
    seg[0, 200:500] = 1
    seg[0, 500:] = 2
    _attn_case(B, S, 8, 1, 128, seg=seg)


_DKDV_CASES = [
    dict(B=2, S=300, Hq=4, Hkv=4, D=64),
    dict(B=2, S=300, Hq=8, Hkv=2, D=96),
    dict(B=2, S=300, Hq=8, Hkv=2, D=128),
    dict(B=1, S=200, Hq=4, Hkv=2, D=128, causal=False),
    dict(B=1, S=512, Hq=4, Hkv=4, D=96, window=100),
    dict(B=2, S=1100, Hq=8, Hkv=2, D=128, window=100),
    dict(B=2, S=1100, Hq=8, Hkv=2, D=128, causal=False),
]


@pytest.mark.parametrize("variant", ["default", "generic"])
@pytest.mark.parametrize("case", range(len(_DKDV_CASES) + 2))
def test_flash_attention_dkdv_variant(monkeypatch, variant, case):
    """The default (fa_bwd_dq3 + fa_bwd_dkdv5) and the generic backward kernels (LLMT_FA_GENERIC=1) against
    the fp32 oracle: causal / not, windows, GQA, D 64 / 96 / 128, several ring wraps, packed segments."""
    if variant == "generic":
        monkeypatch.setenv("LLMT_FA_GENERIC", "1")
    if case < len(_DKDV_CASES):
        _attn_case(**_DKDV_CASES[case])
        return
    if case == len(_DKDV_CASES):
        B, S = 2, 384
        seg = torch.ones(B, S, dtype=torch.int32, device=DEV)
        seg[0, 100:250] = 2
        seg[0, 250:] = 3
        seg[1, 300:] = 0
        _attn_case(B, S, 4, 2, 128, seg=seg)
    else:
        seg = torch.zeros(1, 777, dtype=torch.int32, device=DEV)
        seg[0, 200:500] = 1
        seg[0, 500:] = 2
        _attn_case(1, 777, 8, 1, 128, seg=seg)


def test_rope_attention_fused_matches_reference():
    torch.manual_seed(0)
    S, B, nq, nkv, D = 256, 2, 8, 2, 128
    qkv = torch.randn(S, B, nq + 2 * nkv, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    pos = torch.arange(S, device=DEV).expand(B, S)
    cos, sin = compute_rope_tables(D, 1024, 500000.0, device=DEV)
    o = F_.rope_attention(qkv * 1.0, pos, cos, sin, nq, nkv)
    do = torch.randn_like(o)
    (o.float() * do.float()).sum().backward()
    qr = qkv.detach().float().requires_grad_(True)
    orf = F_._ref_rope_attention(qr.transpose(0, 1), pos, cos, sin, nq, nkv, True, None, -1, 1 / math.sqrt(D),
                                 "eager").transpose(0, 1)
    (orf * do.float()).sum().backward()
    assert _rel(o, orf) < 2e-2
    assert _rel(qkv.grad, qr.grad) < 4e-2


# ----------------------------------------------------------------------------- GEMM (csrc/gemm.hip)
@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("out", ["bf16", "bf16_acc", "fp32", "fp32_acc"])
@pytest.mark.parametrize("M,N,K", [(520, 776, 352), (64, 128, 32), (8, 264, 96), (1024, 512, 4096)])
def test_gemm_layouts(layout, out, M, N, K):
    # nt = forward (x . W^T), nn = dgrad (dy . W), tn = wgrad (dy^T . x); partial tiles on every edge
    torch.manual_seed(0)
    xb = torch.randn(M, K, device=DEV).bfloat16()
    yb = torch.randn(N, K, device=DEV).bfloat16()
    a = xb.t().contiguous() if layout == "tn" else xb
    b = yb if layout == "nt" else yb.t().contiguous()
    dt = torch.float32 if out.startswith("fp32") else torch.bfloat16
    acc = out.endswith("acc")
    c0 = torch.randn(M, N, device=DEV).to(dt)
    c = c0.clone()
    lib().gemm_(a, b, c, layout == "tn", layout != "nt", acc)
    want = xb.float() @ yb.float().t() + (c0.float() if acc else 0.0)
    assert _rel(c, want) < (1e-4 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("M,N,K,ns", [(520, 776, 384, 2), (304, 1032, 4096, 4), (64, 128, 256, 4)])
def test_gemm_splitk(layout, M, N, K, ns):
    # fp32 slabs of the contraction slices (the weight-gradient split-K candidate) sum to the product
    torch.manual_seed(0)
    xb = torch.randn(M, K, device=DEV).bfloat16()
    yb = torch.randn(N, K, device=DEV).bfloat16()
    a = xb.t().contiguous() if layout == "tn" else xb
    b = yb if layout == "nt" else yb.t().contiguous()
    slabs = torch.full((ns, M, N), float("nan"), device=DEV)
    lib().gemm_splitk_(a, b, slabs, layout == "tn", layout != "nt")
    k = K // ns
    for s in range(ns):  # each slab holds exactly its own slice
        want = xb[:, s * k:(s + 1) * k].float() @ yb[:, s * k:(s + 1) * k].float().t()
        assert _rel(slabs[s], want) < 1e-4
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    lib().splitk_reduce_(slabs, out, False)
    assert _rel(out, xb.float() @ yb.float().t()) < 1e-2


def test_gemm_strided_operands():
    # row-strided views (leading dimension > row length), as the fused CE heads and TP slices pass them
    torch.manual_seed(0)
    M, N, K = 300, 200, 160
    xw = torch.randn(M, K + 64, device=DEV).bfloat16()
    yw = torch.randn(N, K + 32, device=DEV).bfloat16()
    cw = torch.zeros(M, N + 40, device=DEV, dtype=torch.bfloat16)
    x, y, c = xw[:, :K], yw[:, 8:K + 8], cw[:, :N]
    lib().gemm_(x, y, c, False, False, False)
    assert _rel(c, x.float() @ y.float().t()) < 1e-2
    assert cw[:, N:].abs().max().item() == 0


def test_transpose_kernel_strided():
    """csrc/elementwise.hip transpose: [R, C] (row-strided view) -> [C, R], bit exact."""
    torch.manual_seed(0)
    xw = torch.randn(320, 256 + 64, device=DEV).bfloat16()
    x = xw[:, 32:32 + 256]
    out = torch.empty(256, 320, device=DEV, dtype=torch.bfloat16)
    lib().transpose_(x, out)
    assert torch.equal(out, x.t().contiguous())


@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N,K", [(256, 192), (1024, 192)])
@pytest.mark.parametrize("forced", [None, "tn/nt", "nn/tt", "tn/nn", "tn/nt2", "nn/tt2", "tn/nn2", "tn/nn4"])
def test_backward_gemms_transposed_layouts(monkeypatch, out_dtype, N, K, forced):
    """dgrad (NN, or TN with W^T at M >= 16384) and wgrad (NT, NN with dy^T, TT with x^T, and each of them
    split-K in two: fp32 slabs + reduction), each layout forced and the timed per-shape choice, with and
    without accumulation, against fp32 products."""
    import llm_training_amd.ops.fused as fused
    monkeypatch.setattr(fused, "GEMM_MODES", {"fwd": "lt", "dgrad": "lt", "wgrad": "lt"})
    monkeypatch.setattr(fused, "_LAYOUT_CACHE", {})
    if forced is not None:
        dg, wg = forced.split("/")
        monkeypatch.setattr(fused, "_layout", lambda key, variants, default, can_time: dg if key[0] == "dgrad" else wg)
    torch.manual_seed(0)
    M = 16384
    dy = torch.randn(M, N, device=DEV).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    for tr in (True, False):
        monkeypatch.setattr(fused, "TRANSPOSE_LAYOUTS", [tr])
        dx = fused.mm_nn(dy, w)
        assert _rel(dx, dy.float() @ w.float()) < 1e-2
        dw = torch.empty(N, K, device=DEV, dtype=out_dtype)
        assert fused.wgrad_into(dw, dy, x, False)  # (times the layouts when not forced)
        assert _rel(dw, dy.float().t() @ x.float()) < (1e-4 if out_dtype == torch.float32 else 1e-2)
        c0 = torch.randn(N, K, device=DEV).to(out_dtype)
        dw = c0.clone()
        assert fused.wgrad_into(dw, dy, x, True)
        want = dy.float().t() @ x.float() + c0.float()
        assert _rel(dw, want) < (1e-4 if out_dtype == torch.float32 else 1e-2)
    if forced is None:
        assert any(k[0] == "wgrad" for k in fused._LAYOUT_CACHE)


@pytest.mark.parametrize("mode", ["hip", "lt", "blas"])
def test_linear_gemm_paths_grads_into_grad_buffer(monkeypatch, mode):
    """Every GEMM path (own kernel, tuned hipBLASLt, torch) through the linear op, with fp32 weight-grad
    accumulation into the flat gradient buffer across two micro-batches."""
    import llm_training_amd.ops.fused as fused
    monkeypatch.setattr(fused, "GEMM_MODES", {"fwd": mode, "dgrad": mode, "wgrad": mode})
    torch.manual_seed(0)
    T, K, N = 320, 256, 384
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16().requires_grad_(True)
    w.main_grad = torch.zeros(N, K, device=DEV, dtype=torch.float32)
    w.grad_added = False
    xs = [torch.randn(T, K, device=DEV, dtype=torch.bfloat16, requires_grad=True) for _ in range(2)]
    dys = [torch.randn(T, N, device=DEV, dtype=torch.bfloat16) for _ in range(2)]
    for x, dy in zip(xs, dys):
        y = F_.linear(x, w)
        assert _rel(y, x.float() @ w.float().t()) < 1e-2
        y.backward(dy)
    assert w.grad is None
    assert _rel(w.main_grad, sum(dy.float().t() @ x.float() for x, dy in zip(xs, dys))) < 1e-3
    for x, dy in zip(xs, dys):
        assert _rel(x.grad, dy.float() @ w.float()) < 1e-2


@pytest.mark.parametrize("bias_dtype", [torch.bfloat16, torch.float32])
def test_linear_bias_in_the_gemm_epilogue(monkeypatch, bias_dtype):
    """A biased linear on the hipBLASLt path adds the bias in the GEMM's BIAS epilogue (no elementwise add
    kernel after it) and matches x W^T + b; the bias gradient is the column sum of dy."""
    import llm_training_amd.ops.fused as fused
    monkeypatch.setattr(fused, "GEMM_MODES", {"fwd": "lt", "dgrad": "lt", "wgrad": "lt"})
    torch.manual_seed(0)
    T, K, N = 512, 256, 384
    x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16().requires_grad_(True)
    b = torch.randn(N, device=DEV).to(bias_dtype).requires_grad_(True)
    calls = []
    monkeypatch.setattr(fused, "lib", lambda: _Spy(torch.ops.llmt, calls))
    y = F_.linear(x, w, b)
    # (several calls on first sight of the problem: the stream-K / non-stream-K solutions are timed)
    assert calls and set(calls) == {"gemm_lt_bias"}
    assert y.dtype == torch.bfloat16
    assert _rel(y, x.float() @ w.float().t() + b.float()) < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    assert _rel(b.grad, dy.float().sum(0)) < 1e-2
    assert _rel(x.grad, dy.float() @ w.float()) < 1e-2


class _Spy:
    """Records which torch.ops.llmt GEMM entry points a call goes through."""

    def __init__(self, ops, calls):
        self._ops, self._calls = ops, calls

    def __getattr__(self, name):
        if name.startswith("gemm_lt"):
            self._calls.append(name)
        return getattr(self._ops, name)


# ----------------------------------------------------------------------------- int8 blockwise quant (ZeRO++)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_int8_quant_dequant_matches_torch(dtype):
    from llm_training_amd.parallel.engine import QBLOCK, dequant_sum, dequantize_int8, quantize_int8
    torch.manual_seed(0)
    n = 64 * 1000
    x = (torch.randn(n, device=DEV) * torch.rand(n // 64, device=DEV).repeat_interleave(64)).to(dtype)
    q, sc = quantize_int8(x)
    xb = x.float().reshape(-1, QBLOCK)
    am = xb.abs().amax(1)
    assert torch.allclose(sc, am / 127, rtol=1e-6)
    qr = torch.round(xb * (127 / am)[:, None]).clamp(-127, 127).to(torch.int8).reshape(-1)
    assert (q.int() - qr.int()).abs().max().item() <= 1  # round-half cases
    y = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    dequantize_int8(q, sc, y)
    assert (y.float() - x.float()).abs().max().item() <= (am.max() / 127).item() * 0.51 + 1e-2
    k = 3
    qs, ss = zip(*(quantize_int8(x * (j + 1)) for j in range(k)))
    out = torch.ones(n, device=DEV, dtype=torch.float32)
    dequant_sum(torch.cat(qs), torch.cat(ss), out, k, True)
    want = 1 + sum((qq.float().reshape(-1, QBLOCK) * s[:, None]).reshape(-1) for qq, s in zip(qs, ss))
    assert torch.allclose(out, want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("out", ["bf16", "bf16_acc", "fp32_acc"])
def test_gemm_lt_tuned_layouts(layout, out):
    """csrc/blaslt.cpp: tuned hipBLASLt solution per problem, all three linear layouts; the tuning pass
    must not disturb an accumulating output."""
    from llm_training_amd.ops.fused import mm_nn, mm_nt, wgrad_into
    torch.manual_seed(0)
    M, N, K = 1024, 768, 512
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16()
    dy = torch.randn(M, N, device=DEV).bfloat16()
    import llm_training_amd.ops.fused as fused
    old = dict(fused.GEMM_MODES)
    fused.GEMM_MODES.update(fwd="lt", dgrad="lt", wgrad="lt")
    try:
        if layout == "nt":
            assert _rel(mm_nt(x, w), x.float() @ w.float().t()) < 1e-2
        elif layout == "nn":
            assert _rel(mm_nn(dy, w), dy.float() @ w.float()) < 1e-2
        else:
            dt = torch.float32 if out.startswith("fp32") else torch.bfloat16
            acc = out.endswith("acc")
            c0 = torch.randn(N, K, device=DEV).to(dt)
            c = c0.clone()
            assert wgrad_into(c, dy, x, acc)
            want = dy.float().t() @ x.float() + (c0.float() if acc else 0)
            assert _rel(c, want) < (1e-4 if dt == torch.float32 else 1e-2)
    finally:
        fused.GEMM_MODES.update(old)
    assert "_acc" in lib().gemm_lt_export() or layout != "tn" or not out.endswith("acc")


def test_gemm_lt_adopt_replaces_choice():
    """csrc/blaslt.cpp gemm_lt_adopt (rank 0's choices broadcast by ops.fused.agree_layouts): a cached
    non-stream-K solution of this process is replaced by the adopted heuristic rank, the next call runs it
    (same result within GEMM reordering) and the export reports it."""
    torch.manual_seed(0)
    M, N, K = 1536, 640, 768  # a problem no other test uses: its cache entry starts here
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    # column-major c^T (N x M) = b (from K x N, op T) . a^T (K x M): the forward layout, non-stream-K (timed)
    lib().gemm_lt(b, a, c, True, False, N, M, K, K, K, N, False, False)
    want = a.float() @ b.float().t()
    assert _rel(c, want) < 1e-2
    line = next(l for l in lib().gemm_lt_export().splitlines() if l.startswith(f"tn_{N}_{M}_{K}_") and "_nosk" in l)
    key, rank = line.split()[:2]
    other = 1 if int(rank) == 0 else 0
    assert lib().gemm_lt_adopt(f"{key} {other} 0 adopted gsu0\n") == 1
    assert lib().gemm_lt_adopt(f"{key} {other} 0 adopted gsu0\n") == 0  # not cached yet: preset only
    c.zero_()
    lib().gemm_lt(b, a, c, True, False, N, M, K, K, K, N, False, False)
    assert _rel(c, want) < 1e-2
    now = next(l for l in lib().gemm_lt_export().splitlines() if l.startswith(key + " "))
    assert int(now.split()[1]) == other


@pytest.mark.parametrize("D,Hq,Hkv,segs", [(128, 4, 2, False), (64, 2, 2, True), (128, 2, 2, True)])
def test_flash_attention_dropout_matches_oracle(D, Hq, Hkv, segs):
    """Attention dropout inside the HIP kernels (generic fwd / dQ / dK-dV kernels): the keep mask is a
    counter hash of (seed, b, h, q, k); the fp32 oracle rebuilds the same mask (reference.py
    dropout_keep_scale), so output and all three gradients must match, and the backward must use the
    forward's mask (a different seed gives a different output)."""
    from llm_training_amd.ops import reference as ref
    from llm_training_amd.ops.fused import flash_attention
    torch.manual_seed(0)
    B, S, p = 2, 300, 0.3
    q = torch.randn(B, S, Hq, D, device=DEV).bfloat16().requires_grad_(True)
    k = torch.randn(B, S, Hkv, D, device=DEV).bfloat16().requires_grad_(True)
    v = torch.randn(B, S, Hkv, D, device=DEV).bfloat16().requires_grad_(True)
    seg = None
    if segs:
        seg = torch.repeat_interleave(torch.tensor([1, 2, 3]), torch.tensor([100, 120, 80])).expand(B, S).to(DEV)
    o = flash_attention(q, k, v, causal=True, segment_ids=seg, dropout_p=p, seed=1234)
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = ref.attention_dropout(qr, kr, vr, True, seg, -1, None, p, 1234)
    orf.backward(do.float())
    assert _rel(o, orf) < 2e-2
    for a_, b_ in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        assert _rel(a_, b_) < 3e-2
    o2 = flash_attention(q, k, v, causal=True, segment_ids=seg, dropout_p=p, seed=99)
    assert _rel(o2, orf) > 0.1
    o0 = flash_attention(q, k, v, causal=True, segment_ids=seg, dropout_p=0.0)
    assert _rel(o0, ref.attention(q.float(), k.float(), v.float(), True, seg, -1, None)) < 2e-2
