"""Attention kernels on contiguous q / k / v against the strided views the Llama layer passes (slices of
the fused QKV GEMM output, token stride (Hq + 2 Hkv) * D): forward and backward times, interleaved
rounds in one process.   python benchmarks/bench_attention_strided.py [B S Hq Hkv D]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_training_amd.ops import fused as F_  # noqa: E402

B, S, Hq, Hkv, D = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (4, 8192, 32, 8, 128)))
qkv = torch.randn(B, S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
views = {
    "strided": (qkv[..., :Hq * D].view(B, S, Hq, D), qkv[..., Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D),
                qkv[..., (Hq + Hkv) * D:].view(B, S, Hkv, D)),
}
views["contiguous"] = tuple(t.contiguous() for t in views["strided"])
do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)


def timed(fn, n=10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


res = {k: {"fwd": [], "bwd": []} for k in views}
for rnd in range(4):
    for name, (q, k, v) in views.items():
        q, k, v = (t.detach().requires_grad_(True) for t in (q, k, v))
        with torch.no_grad():
            res[name]["fwd"].append(timed(lambda: F_.flash_attention(q, k, v, causal=True)))
        o = F_.flash_attention(q, k, v, causal=True)
        res[name]["bwd"].append(timed(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True)))
out = {"shape": [B, S, Hq, Hkv, D]}
for name in views:
    for kind in ("fwd", "bwd"):
        out[f"{name}_{kind}_ms"] = round(sorted(res[name][kind])[len(res[name][kind]) // 2], 4)
print(json.dumps(out), flush=True)
