"""In-process A/B of a per-launch flash-attention knob in the forward (LLMT_FA_* is read on every launch):
alternating windows of each variant on the same operands.
    python benchmarks/ab/ab_attention_fwd.py [B S Hq Hkv D] [variants, comma-separated] [env var]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402

B, S, Hq, Hkv, D = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (4, 8192, 32, 8, 128)))
variants = (sys.argv[6] if len(sys.argv) > 6 else "1,0").split(",")
ENV = sys.argv[7] if len(sys.argv) > 7 else "LLMT_FA_BMAJOR"  # or LLMT_FA_EARLY_DMA / LLMT_FA_GENERIC
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
outs, times = {}, {x: [] for x in variants}
with torch.no_grad():
    for rnd in range(5):
        for var in variants:
            os.environ[ENV] = var
            for _ in range(2):
                o = F_.flash_attention(q, k, v, causal=True)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                o = F_.flash_attention(q, k, v, causal=True)
            b.record()
            torch.cuda.synchronize()
            times[var].append(a.elapsed_time(b) / 10)
            outs[var] = o
res = {"shape": [B, S, Hq, Hkv, D], "env": ENV}
for var in variants:
    ms = sorted(times[var])[len(times[var]) // 2]
    res[f"v{var}_ms"] = round(ms, 4)
    res[f"v{var}_tflops"] = round(4 * B * Hq * S * S * D / 2 / ms / 1e9, 1)
    res[f"v{var}_max_abs_diff"] = float((outs[var].float() - outs[variants[0]].float()).abs().max())
print(json.dumps(res), flush=True)
