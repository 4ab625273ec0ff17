"""In-process A/B of RoPE fused into the attention kernels vs the standalone in-place passes
(ops/fused.py ROPE_FUSED: bwd / full / off): forward + backward of rope_attention on one fused QKV buffer, alternating windows.
    python benchmarks/ab/ab_rope_attention.py [S B nq nkv D docs]
docs > 0: packed rows of that many random documents (positions restart per document)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402
from llm_training_amd.ops.rope_utils import compute_rope_tables  # noqa: E402

S, B, nq, nkv, D, docs = (int(v) for v in (sys.argv[1:7] if len(sys.argv) > 6 else (8192, 4, 32, 8, 128, 0)))
torch.manual_seed(0)
qkv0 = torch.randn(S, B, nq + 2 * nkv, D, device="cuda", dtype=torch.bfloat16)
cos, sin = compute_rope_tables(D, max(S, 4096), 500000.0, device="cuda")
seg = info = None
pos = torch.arange(S, device="cuda").expand(B, S).contiguous()
if docs > 0:
    cuts = torch.sort(torch.randint(1, S, (B, docs - 1), device="cuda"), dim=1).values
    idx = torch.arange(S, device="cuda").expand(B, S)
    seg = 1 + (idx[:, :, None] >= cuts[:, None, :]).sum(-1)
    start = torch.where(torch.cat([torch.ones(B, 1, dtype=torch.bool, device="cuda"), seg[:, 1:] != seg[:, :-1]], 1),
                        idx, torch.zeros_like(idx))
    pos = idx - torch.cummax(start, 1).values
    info = F_.segment_info(seg)
do = torch.randn(S, B, nq, D, device="cuda", dtype=torch.bfloat16)


TOK = os.environ.get("LLMT_AB_TOK", "1") == "1"  # per-token tables, as the model passes them


def step():
    qkv = qkv0.clone().requires_grad_(True)
    tok = F_.rope_token_tables(pos, cos, sin) if (TOK and F_.ROPE_FUSED[0] != "off") else None
    o = F_.rope_attention(qkv * 1.0, pos, cos, sin, nq, nkv, True, seg, seg_info=info, rope_tok=tok)
    o.backward(do)
    return o.detach(), qkv.grad


out = {"shape": {"S": S, "B": B, "nq": nq, "nkv": nkv, "D": D, "docs": docs}}
modes = tuple(os.environ.get("LLMT_AB_ONLY", "bwd,full,off").split(","))
times = {m: [] for m in modes}
res = {}
for rnd in range(5):
    for fused in modes:
        F_.ROPE_FUSED[0] = fused
        step()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            r = step()
        b.record()
        torch.cuda.synchronize()
        times[fused].append(a.elapsed_time(b) / 5)
        res[fused] = r
F_.ROPE_FUSED[0] = "auto"
for m in modes:
    out[f"{m}_ms"] = round(sorted(times[m])[2], 4)
    if "off" in modes and m != "off":
        out[f"{m}_dqkv_rel_diff_vs_off"] = float((res[m][1].float() - res["off"][1].float()).norm() /
                                                 res["off"][1].float().norm())
print(json.dumps(out), flush=True)
