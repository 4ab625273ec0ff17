"""Compare flash-attention forward variants (LLMT_FA_FWD_VARIANT) against variant 4 and the fp32 reference
on small shapes: output and (through the backward, which reads the forward's LSE) gradient errors, one JSON
line per case.    python benchmarks/ab/fwd_variant_check.py [variant]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402
from llm_training_amd.ops import reference as ref  # noqa: E402

var = sys.argv[1] if len(sys.argv) > 1 else "10"
cases = [(2, 300, 8, 2, 128, True, -1), (1, 256, 2, 2, 128, True, -1), (1, 64, 1, 1, 128, True, -1),
         (1, 300, 1, 1, 128, False, -1), (1, 1000, 4, 1, 128, True, 100), (1, 1024, 4, 1, 128, False, 300),
         (2, 2048, 8, 2, 128, True, -1), (1, 4096, 4, 4, 128, True, -1)]
for B, S, Hq, Hkv, D, causal, window in cases:
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    res = {"case": [B, S, Hq, Hkv, D, causal, window]}
    outs = {}
    for vv in ("4", var):
        os.environ["LLMT_FA_FWD_VARIANT"] = vv
        o = F_.flash_attention(q, k, v, causal, None, window)
        outs[vv] = (o.detach(), torch.autograd.grad(o, (q, k, v), do))
    os.environ["LLMT_FA_FWD_VARIANT"] = "4"
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = ref.attention(qr, kr, vr, causal, None, window)
    gr = torch.autograd.grad(orf, (qr, kr, vr), do.float())
    for vv in ("4", var):
        o, g = outs[vv]
        res[f"o_rel_v{vv}"] = round(float((o.float() - orf).norm() / orf.norm()), 6)
        for name, a, r in zip("qkv", g, gr):
            res[f"d{name}_rel_v{vv}"] = round(float((a.float() - r).norm() / r.norm()), 6)
    res["o_maxdiff"] = float((outs["4"][0].float() - outs[var][0].float()).abs().max())
    print(json.dumps(res), flush=True)
