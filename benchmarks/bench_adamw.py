"""Fused AdamW (csrc/optim.hip) alone on one decoder-layer unit of Llama-3-8B (218 M parameters):
fp32 master/m/v, bf16 gradient and bf16 parameter copy -> 28 bytes per parameter moved."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_training_amd.ops.native import lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 218_112_000
dev = torch.device("cuda", 0)
p = torch.randn(n, device=dev)
m = torch.zeros(n, device=dev)
v = torch.zeros(n, device=dev)
g = torch.randn(n, device=dev).bfloat16()
po = torch.empty(n, device=dev, dtype=torch.bfloat16)
gs = torch.ones(1, device=dev)


def run(step):
    lib().adamw_(p, m, v, g, po, 3e-5, 0.9, 0.95, 1e-8, 0.1, step, gs)


for s in range(1, 4):
    run(s)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 20
a.record()
for s in range(reps):
    run(4 + s)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / reps
print(json.dumps({"n": n, "ms": round(ms, 3), "tb_s": round(28 * n / ms / 1e9, 2)}), flush=True)
