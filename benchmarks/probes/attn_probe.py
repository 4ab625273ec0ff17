"""Attention forward + backward at one shape, a few times (for PMC passes and per-kernel tables):
    rocprofv3 --pmc <counters> -- python benchmarks/probes/attn_probe.py [B S Hq Hkv D] [docs] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402

B, S, Hq, Hkv, D = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (4, 8192, 32, 8, 128)))
docs = int(sys.argv[6]) if len(sys.argv) > 6 else 1
iters = int(sys.argv[7]) if len(sys.argv) > 7 else 4
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
seg = None
if docs > 1:
    g = torch.Generator().manual_seed(0)
    cuts = sorted(torch.randperm(S - 1, generator=g)[: docs - 1].add(1).tolist())
    e = [0, *cuts, S]
    seg = torch.repeat_interleave(torch.arange(1, docs + 1, dtype=torch.int32),
                                  torch.tensor([b - a for a, b in zip(e[:-1], e[1:])])).expand(B, S).contiguous().cuda()
info = F_.segment_info(seg) if seg is not None else None
for _ in range(iters):
    o = F_.flash_attention(q, k, v, causal=True, segment_ids=seg, seg_info=info)
    o.backward(torch.ones_like(o))
torch.cuda.synchronize()
