"""One attention shape, forward + backward, N iterations (for rocprofv3 per-kernel tables):
    python benchmarks/attn_one_shape.py B S Hq Hkv D [docs] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_training_amd.ops import fused as F_  # noqa: E402

B, S, Hq, Hkv, D = (int(v) for v in sys.argv[1:6])
docs = int(sys.argv[6]) if len(sys.argv) > 6 else 1
iters = int(sys.argv[7]) if len(sys.argv) > 7 else 20
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
seg = info = None
if docs > 1:
    seg = (torch.arange(S, device="cuda") * docs // S + 1).to(torch.int32).expand(B, S).contiguous()
    info = F_.segment_info(seg)
for _ in range(iters):
    F_.flash_attention(q, k, v, causal=True, segment_ids=seg, seg_info=info).backward(do)
torch.cuda.synchronize()
print("done", flush=True)
