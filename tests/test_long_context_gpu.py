"""Long-context attention on the GPU (the reference's 128K TP example config): the flash
kernels at S = 32K and 128K against an fp32 oracle evaluated on sampled query rows / key blocks (a full
S x S oracle would not fit). Forward output + LSE, dQ of sampled rows, dK / dV of sampled key blocks."""
import math

import pytest
import torch

from llm_training_amd.ops.fused import flash_attention
from llm_training_amd.ops.native import lib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _oracle_rows(q, k, v, rows, scale):
    """fp32 causal attention of the given query rows (one head): o [n, D], lse [n]."""
    qs = q[rows].float()
    s = (qs @ k.float().t()) * scale
    mask = torch.arange(k.shape[0], device=q.device)[None, :] > rows[:, None]
    s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, -1)
    return torch.softmax(s, -1) @ v.float(), lse


@pytest.mark.parametrize("S", [32768, 131072])
def test_flash_attention_long_context_sampled(S):
    torch.manual_seed(0)
    H, D = 2, 128
    scale = 1.0 / math.sqrt(D)
    q = torch.randn(1, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(1, S, 1, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(1, S, 1, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = flash_attention(q, k, v, causal=True)
    do = torch.randn_like(o)
    o.backward(do)
    _, lse = lib().flash_attn_fwd(q.detach(), k.detach(), v.detach(), None, scale, True, -1)
    rows = torch.cat([torch.arange(0, 64), torch.arange(S // 2 - 32, S // 2 + 32), torch.arange(S - 64, S)]).to(DEV)
    K, Vv = k[0, :, 0].detach(), v[0, :, 0].detach()
    for h in range(H):
        Q = q[0, :, h].detach()
        ro, rl = _oracle_rows(Q, K, Vv, rows, scale)
        got = o[0, rows, h].float()
        assert ((got - ro).norm() / ro.norm()).item() < 2e-2, h
        assert (lse[0, h, rows] - rl).abs().max().item() < 2e-2
        # dQ of the sampled rows: dS = P * (dP - delta), delta = rowsum(dO * O)
        s = (Q[rows].float() @ K.float().t()) * scale
        s = s.masked_fill(torch.arange(S, device=DEV)[None, :] > rows[:, None], float("-inf"))
        p = torch.softmax(s, -1)
        dOr = do[0, rows, h].float()
        dp = dOr @ Vv.float().t()
        delta = (dOr * ro).sum(-1, keepdim=True)
        dq_ref = (p * (dp - delta)) @ K.float() * scale
        dq = q.grad[0, rows, h].float()
        assert ((dq - dq_ref).norm() / dq_ref.norm()).item() < 3e-2, h
    # dK / dV of key blocks against a fully independent fp32 oracle: every query row that sees the block
    # gets its own fp32 softmax statistics (LSE) and output O from the whole key range (nothing taken
    # from the kernel's forward). Blocks: the start (all S queries see it) at 32K; at 128K the blocks
    # 8K and 256 keys before the end (the all-query block would be a 128K x 128K fp32 oracle per head).
    blocks = (0, S - 256) if S <= 32768 else (S - 8192, S - 256)
    for k0 in blocks:
        kb = torch.arange(k0, k0 + 256, device=DEV)
        dk_ref = torch.zeros(256, D, device=DEV)
        dv_ref = torch.zeros(256, D, device=DEV)
        for h in range(H):
            Q = q[0, :, h].detach().float()
            dO = do[0, :, h].float()
            for c0 in range(k0 // 4096 * 4096, S, 4096):  # query chunks that can see the block
                qi = torch.arange(c0, min(S, c0 + 4096), device=DEV)
                oi, lse_i = _oracle_rows(q[0, :, h].detach(), K, Vv, qi, scale)
                s = (Q[qi] @ K[kb].float().t()) * scale
                s = s.masked_fill(kb[None, :] > qi[:, None], float("-inf"))
                p = torch.exp(s - lse_i[:, None])
                dp = dO[qi] @ Vv[kb].float().t()
                delta = (dO[qi] * oi).sum(-1, keepdim=True)
                ds = p * (dp - delta)
                dv_ref += p.t() @ dO[qi]
                dk_ref += ds.t() @ Q[qi] * scale
        assert ((k.grad[0, kb, 0].float() - dk_ref).norm() / dk_ref.norm()).item() < 3e-2, k0
        assert ((v.grad[0, kb, 0].float() - dv_ref).norm() / dv_ref.norm()).item() < 3e-2, k0
