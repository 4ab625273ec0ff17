"""Attention microbenchmark: HIP flash kernels vs torch SDPA on MI355X (fwd and fwd+bwd TFLOP/s)."""
import argparse
import json
import sys
import os
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_training_amd.ops import fused as F_  # noqa: E402


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--S", type=int, default=8192)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--sdpa", action="store_true")
    ap.add_argument("--noncausal", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    B, S, Hq, Hkv, D = a.B, a.S, a.Hq, a.Hkv, a.D
    q = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    causal = not a.noncausal
    flops_f = 4 * B * Hq * S * S * D / (2 if causal else 1)
    res = {"shape": [B, S, Hq, Hkv, D], "causal": causal}
    o = F_.flash_attention(q, k, v, causal=causal)
    do = torch.randn_like(o)
    tf = timeit(lambda: F_.flash_attention(q, k, v, causal=causal))
    def fb():
        o = F_.flash_attention(q, k, v, causal=causal)
        o.backward(do)
    tfb = timeit(fb)
    res["hip_fwd_ms"] = tf * 1e3
    res["hip_fwd_tflops"] = flops_f / tf / 1e12
    res["hip_bwd_ms"] = (tfb - tf) * 1e3
    res["hip_bwd_tflops"] = 2.5 * flops_f / (tfb - tf) / 1e12
    if a.sdpa:
        qh, kh, vh = (t.detach().transpose(1, 2).contiguous().requires_grad_(True) for t in (q, k, v))
        f = lambda: torch.nn.functional.scaled_dot_product_attention(qh, kh, vh, is_causal=True, enable_gqa=True)
        try:
            o2 = f()
            do2 = torch.randn_like(o2)
            t2 = timeit(f)
            def fb2():
                o2 = f()
                o2.backward(do2)
            t2b = timeit(fb2)
            res["sdpa_fwd_ms"] = t2 * 1e3
            res["sdpa_fwd_tflops"] = flops_f / t2 / 1e12
            res["sdpa_bwd_ms"] = (t2b - t2) * 1e3
            res["sdpa_bwd_tflops"] = 2.5 * flops_f / (t2b - t2) / 1e12
        except Exception as e:  # noqa: BLE001
            res["sdpa_error"] = repr(e)[:200]
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
