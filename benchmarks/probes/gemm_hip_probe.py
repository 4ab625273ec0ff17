"""Run the hand-written gfx950 GEMM (csrc/gemm.hip) alone on one Llama-3-8B shape and layout, for PMC
passes:   rocprofv3 --pmc <counters> -- python benchmarks/probes/gemm_hip_probe.py [shape] [fwd|dgrad|wgrad] [T]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops.native import lib  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "gate_up"
kind = sys.argv[2] if len(sys.argv) > 2 else "fwd"
T = int(sys.argv[3]) if len(sys.argv) > 3 else 32768
N, K = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}[shape]
L = lib()
x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
W = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
out = {"fwd": torch.empty(T, N, device="cuda", dtype=torch.bfloat16),
       "dgrad": torch.empty(T, K, device="cuda", dtype=torch.bfloat16),
       "wgrad": torch.empty(N, K, device="cuda", dtype=torch.bfloat16)}[kind]
fn = {"fwd": lambda: L.gemm_(x, W, out, False, False, False),
      "dgrad": lambda: L.gemm_(dy, W, out, False, True, False),
      "wgrad": lambda: L.gemm_(dy, x, out, True, True, False)}[kind]
for _ in range(5):
    fn()
torch.cuda.synchronize()
