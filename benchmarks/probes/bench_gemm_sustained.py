"""Sustained-clock GEMM rate: the Llama-3-8B gate_up forward (M=24576, N=28672, K=4096) run back to
back for ~N seconds, reported per window of 25 calls. A 10-call microbenchmark runs at boost clock;
inside a training step the GPU sits at its power limit, so this is the rate the step can expect."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import llm_training_amd.ops.fused as F  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
M, N, K = 24576, 28672, 4096
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
F.GEMM_MODES.update(fwd="lt")
F.mm_nt(x, w)
torch.cuda.synchronize()
t0 = time.time()
win = 0
while time.time() - t0 < secs:
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(25):
        F.mm_nt(x, w)
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b) / 25
    print(json.dumps({"window": win, "t": round(time.time() - t0, 2), "ms": round(ms, 3),
                      "pf": round(2 * M * N * K / ms / 1e12, 3)}), flush=True)
    win += 1
