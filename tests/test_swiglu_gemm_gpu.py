"""The down-projection input-gradient GEMM with the SwiGLU backward in its epilogue (csrc/gemm.hip SwiArgs,
``ops.fused.swiglu_down``) against the fp32 oracle of the same op, and end to end against the unfused path
(hipBLASLt input gradient + the standalone swiglu_bwd_tr pass — the default; LLMT_SWIGLU_GEMM=1 opts in to the
fused kernel, which measured slower in-step, see ops/fused.py).

Reference op: src/llm_training/models/llama/llama_model.py:415-427 (down_proj(act(gate) * up)) through the
Liger SwiGLU of src/llm_training/ops/liger_kernel/swiglu_op.py:36-39."""
import pytest
import torch

from llm_training_amd.ops import fused as F_
from llm_training_amd.ops.native import lib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _oracle(dy, w, gu):
    I = w.shape[1]
    dc = (dy.float() @ w.float()).bfloat16().float()  # the unfused path rounds dc to bf16 (GEMM output)
    g, u = gu.float()[:, :I], gu.float()[:, I:]
    s = torch.sigmoid(g)
    dg = dc * u * s * (1 + g * (1 - s))
    du = dc * g * s
    return torch.cat([dg, du], 1)


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


# (T, H = contraction, I): Llama-3-8B and Phi-3-mini widths at small token counts, a ragged token count (not a
# multiple of the 256-row tile), an I that is not a multiple of the 256-column tile, a TP=8 shard width
@pytest.mark.parametrize("T,H,I", [(512, 4096, 14336), (256, 3072, 8192), (320, 256, 192), (192, 512, 1792),
                                   (1024, 4096, 1792), (64, 96, 64)])
@pytest.mark.parametrize("transposed", [True, False])
def test_gemm_swiglu_bwd_matches_fp32(T, H, I, transposed):
    torch.manual_seed(0)
    dy = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(H, I, device=DEV) * H ** -0.5).to(torch.bfloat16)
    gu = (torch.randn(T, 2 * I, device=DEV) * 2).to(torch.bfloat16)
    outs = lib().gemm_swiglu_bwd(dy, w, gu, transposed)
    ref = _oracle(dy, w, gu)
    assert _rel(outs[0], ref) < 1e-2
    # element-wise: within bf16 rounding of the oracle (the GEMM's fp32 accumulation order differs)
    assert float((outs[0].float() - ref).abs().max()) <= 0.02 * float(ref.abs().max()) + 1e-3
    if transposed:
        assert len(outs) == 2
        assert torch.equal(outs[1], outs[0].t().contiguous())
    else:
        assert len(outs) == 1


def test_gemm_swiglu_bwd_strided_dy():
    """dy as a row-strided view (a slice of a wider buffer) is read with its leading dimension."""
    torch.manual_seed(1)
    T, H, I = 256, 512, 256
    big = torch.randn(T, H + 64, device=DEV, dtype=torch.bfloat16)
    dy = big[:, :H]
    w = (torch.randn(H, I, device=DEV) * H ** -0.5).to(torch.bfloat16)
    gu = torch.randn(T, 2 * I, device=DEV, dtype=torch.bfloat16)
    got = lib().gemm_swiglu_bwd(dy, w, gu, False)[0]
    assert _rel(got, _oracle(dy, w, gu)) < 1e-2


@pytest.mark.parametrize("I,bias", [(1792, False), (512, True)])
def test_swiglu_down_matches_unfused(monkeypatch, I, bias):
    """swiglu_down (one autograd node, fused backward) == linear(swiglu(gu), W_down): forward bitwise, input
    gradient within GEMM reordering, weight / bias gradients bitwise (same kernels)."""
    torch.manual_seed(2)
    T, H = 512, 1024
    gu0 = torch.randn(T, 2 * I, device=DEV, dtype=torch.bfloat16)
    w0 = (torch.randn(H, I, device=DEV) * I ** -0.5).to(torch.bfloat16)
    b0 = torch.randn(H, device=DEV, dtype=torch.bfloat16) if bias else None
    dy = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)

    def run(fused):
        monkeypatch.setattr(F_, "SWIGLU_GEMM", [fused])
        gu = gu0.clone().requires_grad_(True)
        w = w0.clone().requires_grad_(True)
        b = b0.clone().requires_grad_(True) if bias else None
        y = F_.swiglu_down(gu, w, b)
        y.backward(dy)
        return y.detach(), gu.grad, w.grad, (b.grad if bias else None)

    yf, dgf, dwf, dbf = run(True)
    yu, dgu, dwu, dbu = run(False)
    assert torch.equal(yf, yu)
    assert _rel(dgf, dgu) < 1e-2
    assert torch.equal(dwf, dwu)
    if bias:
        assert torch.equal(dbf, dbu)


@pytest.mark.parametrize("fused", [True, False])
def test_llama_mlp_uses_fused_backward(monkeypatch, fused):
    """The Llama / Phi-3 MLP goes through swiglu_down: with LLMT_SWIGLU_GEMM on, one node whose backward is the
    fused GEMM kernel; off (the default), the unfused linear(swiglu(gu)) pair."""
    monkeypatch.setattr(F_, "SWIGLU_GEMM", [fused])
    from llm_training_amd.models.llama import LlamaConfig, LlamaMLP
    from llm_training_amd.parallel.context import ParallelContext
    cfg = LlamaConfig(vocab_size=128, hidden_size=256, intermediate_size=512, num_hidden_layers=1,
                      num_attention_heads=4, num_key_value_heads=2)
    mlp = LlamaMLP(cfg, ParallelContext.single(torch.device(DEV)), dtype=torch.bfloat16, device=DEV)
    for p in mlp.parameters():
        torch.nn.init.normal_(p, std=0.05)
    h = torch.randn(128, 2, 256, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = mlp(h)
    assert (type(y.grad_fn).__name__ == "_SwiGLUDownFnBackward") == fused
    y.float().sum().backward()
    assert h.grad is not None and torch.isfinite(h.grad.float()).all()
