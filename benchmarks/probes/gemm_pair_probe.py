"""The hand-written GEMM and hipBLASLt (torch.mm) on the same problem, five calls each, for PMC passes that
compare the two kernels (MFMA busy, waits, clock):
    rocprofv3 --pmc <counters> -- python benchmarks/probes/gemm_pair_probe.py [T H I]
Problem: the down projection's input gradient dc [T, I] = dy [T, H] . W_down [H, I] (the fused SwiGLU GEMM's
main loop; hipBLASLt in its TN form with W_down^T, as the step runs it)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops.native import lib  # noqa: E402

T, H, I = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (32768, 4096, 14336)))
L = lib()
dy = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
w = (torch.randn(H, I, device="cuda") * H ** -0.5).to(torch.bfloat16)
wt = w.t().contiguous()
dc = torch.empty(T, I, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    L.gemm_(dy, w, dc, False, True, False)
torch.cuda.synchronize()
for _ in range(5):
    torch.mm(dy, wt.t(), out=dc)
torch.cuda.synchronize()
