"""Forward attention only, a few calls (for PMC passes):
    rocprofv3 --pmc <counters> -- python benchmarks/probes/attn_fwd_probe.py [B S Hq Hkv D]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402

B, S, Hq, Hkv, D = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (4, 8192, 32, 8, 128)))
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
with torch.no_grad():
    for _ in range(4):
        F_.flash_attention(q, k, v, causal=True)
torch.cuda.synchronize()
