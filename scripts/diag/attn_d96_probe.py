"""Structured inputs for the head-dim-96 v3 forward: which part of the product (scores, softmax, P.V)
goes wrong, and for which query rows / k-slices."""
import sys

import torch

sys.path.insert(0, ".")
from llm_training_amd.ops import reference as ref  # noqa: E402
from llm_training_amd.ops.native import lib  # noqa: E402

D, S = 96, 64


def run(name, q, k, v, causal):
    o, lse = lib().flash_attn_fwd(q, k, v, None, D ** -0.5, causal, -1)
    want = ref.attention(q.float(), k.float(), v.float(), causal, None, -1, D ** -0.5)
    s = (q.float().transpose(1, 2) @ k.float().transpose(1, 2).transpose(-1, -2)) * D ** -0.5
    if causal:
        s = s.masked_fill(torch.ones(S, S, device="cuda", dtype=torch.bool).triu(1), float("-inf"))
    lref = torch.logsumexp(s, -1)
    err = (o.float() - want).abs()[0, :, 0].amax(-1)
    lerr = (lse[0, 0] - lref[0, 0]).abs()
    bad = [i for i in range(S) if err[i] > 0.05]
    lbad = [i for i in range(S) if not (lerr[i] < 1e-2)]
    print(f"{name:28s} o err {err.max().item():.3g} lse err {lerr.max().item():.3g} bad o rows {bad[:16]} bad lse rows {lbad[:16]}")
    if lbad:
        i = lbad[0]
        print(f"    row {i}: lse {lse[0, 0, i].item():.4f} want {lref[0, 0, i].item():.4f}")


torch.manual_seed(0)
rn = lambda: torch.randn(1, S, 1, D, device="cuda").bfloat16()  # noqa: E731
z = lambda: torch.zeros(1, S, 1, D, device="cuda").bfloat16()  # noqa: E731
for causal in (False, True):
    c = "causal" if causal else "full"
    run(f"{c} random", rn(), rn(), rn(), causal)
    run(f"{c} K=0", rn(), z(), rn(), causal)
    run(f"{c} Q=0", z(), rn(), rn(), causal)
    run(f"{c} V=1", rn(), rn(), torch.ones(1, S, 1, D, device="cuda").bfloat16(), causal)
    for kk in range(D // 16):
        q, k = z(), z()
        q[..., 16 * kk:16 * kk + 16] = rn()[..., :16]
        k[..., 16 * kk:16 * kk + 16] = rn()[..., :16]
        run(f"{c} QK only slice {kk}", q, k, rn(), causal)
    for h8 in range(2):
        q, k = z(), z()
        for kk in range(D // 16):
            q[..., 16 * kk + 8 * h8:16 * kk + 8 * h8 + 8] = rn()[..., :8]
            k[..., 16 * kk + 8 * h8:16 * kk + 8 * h8 + 8] = rn()[..., :8]
        run(f"{c} QK only half {h8}", q, k, rn(), causal)
