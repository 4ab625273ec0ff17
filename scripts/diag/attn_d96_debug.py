"""Where does a head-dim-96 flash forward differ from the fp32 oracle? (rows / columns / heads)"""
import sys

import torch

sys.path.insert(0, ".")
from llm_training_amd.ops import reference as ref  # noqa: E402
from llm_training_amd.ops.native import lib  # noqa: E402

torch.manual_seed(0)
for (B, S, H, D) in [(1, 64, 1, 96), (1, 200, 2, 96), (1, 64, 1, 128)]:
    q = torch.randn(B, S, H, D, device="cuda").bfloat16()
    k = torch.randn(B, S, H, D, device="cuda").bfloat16()
    v = torch.randn(B, S, H, D, device="cuda").bfloat16()
    o, lse = lib().flash_attn_fwd(q, k, v, None, D ** -0.5, True, -1)
    want = ref.attention(q.float(), k.float(), v.float(), True, None, -1, D ** -0.5)
    err = (o.float() - want).abs()
    print(B, S, H, D, "max err", err.max().item())
    print("  err by 32-col block:", [round(err[..., c:c + 32].max().item(), 3) for c in range(0, D, 32)])
    print("  err by 32-row block:", [round(err[:, r:r + 32].max().item(), 3) for r in range(0, S, 32)])
    print("  o sample", o[0, 5, 0, :8].float().tolist(), "want", want[0, 5, 0, :8].tolist())
    rowerr = err[0, :, 0].amax(-1)
    print("  bad rows (head 0):", [i for i in range(S) if rowerr[i] > 0.05][:64])
    colerr = err[0, :, 0].amax(0)
    print("  bad cols (head 0):", [i for i in range(D) if colerr[i] > 0.05][:96])
    s = (q.float().transpose(1, 2) @ k.float().transpose(1, 2).transpose(-1, -2)) * D ** -0.5
    s = s.masked_fill(torch.ones(S, S, device="cuda", dtype=torch.bool).triu(1), float("-inf"))
    print("  lse err", (lse - torch.logsumexp(s, -1)).abs().max().item())
