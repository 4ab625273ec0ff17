"""In-process A/B of a per-launch flash-attention knob in the backward (LLMT_FA_* is read on every launch):
alternating windows of each variant on the same operands, so box-to-box clock differences cancel.
    python benchmarks/ab/ab_attention_bwd.py [B S Hq Hkv D] [values, comma-separated] [env var]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402

B, S, Hq, Hkv, D = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (4, 8192, 32, 8, 128)))
variants = (sys.argv[6] if len(sys.argv) > 6 else "1,0").split(",")
ENV = sys.argv[7] if len(sys.argv) > 7 else "LLMT_FA_EARLY_DMA"  # or LLMT_FA_BMAJOR / LLMT_FA_GENERIC
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
o = F_.flash_attention(q, k, v, causal=True)
do = torch.randn_like(o)
grads = {}
times = {x: [] for x in variants}
for rnd in range(5):
    for var in variants:
        os.environ[ENV] = var
        for _ in range(2):
            g = torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            g = torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
        b.record()
        torch.cuda.synchronize()
        times[var].append(a.elapsed_time(b) / 10)
        grads[var] = g
ref = grads[variants[0]]
out = {"shape": [B, S, Hq, Hkv, D], "env": ENV}
for var in variants:
    out[f"v{var}_ms"] = round(sorted(times[var])[len(times[var]) // 2], 4)
    out[f"v{var}_max_abs_diff_vs_v{variants[0]}"] = max(float((x - y).abs().max()) for x, y in zip(grads[var], ref))
print(json.dumps(out), flush=True)
