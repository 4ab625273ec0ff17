"""Compare flash-attention backward variants (LLMT_FA_BWD_VARIANT) on small shapes: per-gradient max abs
difference against variant 4 and relative error against the fp32 reference, one JSON line per case.
    python benchmarks/ab/attn_variant_check.py [variant]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402
from llm_training_amd.ops import reference as ref  # noqa: E402

var = sys.argv[1] if len(sys.argv) > 1 else "5"
cases = [(2, 300, 8, 2, 128, True, -1), (2, 300, 8, 2, 96, True, -1), (1, 300, 8, 2, 128, True, -1),
         (1, 300, 2, 2, 128, True, -1), (1, 256, 2, 2, 128, True, -1), (1, 128, 1, 1, 128, True, -1),
         (1, 64, 1, 1, 128, True, -1), (1, 288, 1, 1, 128, True, -1), (1, 300, 1, 1, 128, True, -1),
         (1, 300, 1, 1, 128, False, -1), (1, 1024, 4, 1, 128, True, -1), (2, 300, 8, 4, 64, True, -1),
         (4, 512, 8, 4, 64, True, "seg"), (2, 512, 8, 2, 128, True, "seg")]
for B, S, Hq, Hkv, D, causal, window in cases:
    seg = None
    if window == "seg":  # packed documents of 48-199 tokens (the convergence test's rows)
        g = torch.Generator().manual_seed(1)
        seg = torch.zeros(B, S, dtype=torch.int32)
        for r in range(B):
            pos, d = 0, 1
            while pos < S:
                ln = min(S - pos, int(torch.randint(48, 200, (1,), generator=g)))
                seg[r, pos:pos + ln] = d
                pos += ln
                d += 1
        seg = seg.cuda()
        window = -1
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    out = {"case": [B, S, Hq, Hkv, D, causal, window]}
    grads = {}
    for vv in ("4", var):
        os.environ["LLMT_FA_BWD_VARIANT"] = vv
        o = F_.flash_attention(q, k, v, causal, seg, window)
        grads[vv] = torch.autograd.grad(o, (q, k, v), do)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = ref.attention(qr, kr, vr, causal, seg, window)
    gr = torch.autograd.grad(orf, (qr, kr, vr), do.float())
    for name, a, b, r in zip("qkv", grads["4"], grads[var], gr):
        out[f"d{name}_maxdiff"] = float((a.float() - b.float()).abs().max())
        out[f"d{name}_rel_v{var}"] = float((b.float() - r).norm() / r.norm())
        # which key rows differ (dK / dV): first / last differing sequence index
        if name in "kv":
            bad = ((a.float() - b.float()).abs().amax(dim=(0, 2, 3)) > 1e-2).nonzero().flatten().tolist()
            out[f"d{name}_bad_rows"] = [bad[0], bad[-1], len(bad)] if bad else []
    print(json.dumps(out), flush=True)
