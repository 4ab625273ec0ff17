"""GEMM roofline of a training step (Llama-3-8B micro-batch 4 x 8192 = 32768 tokens by default, or
Phi-3-mini with --model phi3-mini; one MI355X).

Every forward / input-gradient / weight-gradient GEMM of the step, timed standalone on random operands
through the framework's own dispatch (ops/fused.py: hipBLASLt with the per-shape layout choice —
transposed operands, split-K weight gradients — exactly as inside the step), with

  * ``ours``: the solution the step uses (hipBLASLt heuristic first choice unless tuned), and
  * ``best``: run with ``LLMT_GEMM_TUNE=1 LLMT_GEMM_TUNE_TOPK=<k>``, every one of the library's top-k
    solutions timed per problem and the fastest kept (the best standalone hipBLASLt solution).

Prints one JSON line per GEMM (ms, PF/s, layout chosen) and a summary line with the step's GEMM time
(sum over calls per step). Compare with the in-step GEMM kernel time of a rocprof step table to get the
in-step / standalone factor (profiles/r3_gemm_roofline.md).

    python benchmarks/gemm_roofline.py                 # ours
    LLMT_GEMM_TUNE=1 LLMT_GEMM_TUNE_TOPK=64 python benchmarks/gemm_roofline.py --tag best
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_training_amd.ops import fused as F_  # noqa: E402

# hidden, intermediate, vocabulary, layers, qkv width
MODELS = {"llama3-8b": (4096, 14336, 128256, 32, 4096 + 2 * 1024), "phi3-mini": (3072, 8192, 32064, 32, 3 * 3072)}


def shapes(model):
    H, I, V, L, QKV = MODELS[model]
    # name -> (N out features, K in features, calls per step per GEMM kind)
    return {"qkv": (QKV, H, L), "o": (H, H, L), "gate_up": (2 * I, H, L), "down": (H, I, L)}, H, V


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--chunk", type=int, default=8192, help="lm_head rows per GEMM (fused CE chunk)")
    ap.add_argument("--tag", default="ours")
    ap.add_argument("--model", default="llama3-8b", choices=sorted(MODELS))
    a = ap.parse_args()
    SHAPES, H, V = shapes(a.model)
    dev = "cuda"
    T = a.tokens
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape, scale=1.0):
        return (torch.randn(*shape, device=dev, generator=g) * scale).bfloat16()

    rows = []
    step_ms = 0.0
    problems = [(n, N, K, calls, T) for n, (N, K, calls) in SHAPES.items()]
    problems.append(("lm_head", V, H, T // a.chunk, a.chunk))
    for name, N, K, calls, M in problems:
        x = rnd(M, K)
        w = rnd(N, K, scale=0.02)
        dy = rnd(M, N, scale=0.01)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        wt = F_.weight_t(w, T) if name == "lm_head" else None  # the fused CE transposes W once per step
        # lm_head weight gradient: summed over chunks in fp32 (ops/fused.py dw_accumulator)
        dw = torch.empty(N, K, device=dev, dtype=torch.float32 if name == "lm_head" else torch.bfloat16)
        flops = 2.0 * M * N * K
        kinds = {
            "fwd": lambda: F_.mm_nt(x, w, out=y),
            "dgrad": lambda: F_.mm_nn(dy, w, out=dx, wt=wt),
            "wgrad": lambda: F_.wgrad_into(dw, dy, x, False),
        }
        for kind, fn in kinds.items():
            ms = timeit(fn)
            layout = [v for k, v in F_._LAYOUT_CACHE.items() if k[0] == kind and k[1] == M and k[2] == N][-1:] \
                if kind != "fwd" else ["nt"]
            r = {"tag": a.tag, "model": a.model, "gemm": name, "kind": kind, "M": M, "N": N, "K": K, "ms": round(ms, 4),
                 "pflops": round(flops / ms / 1e12, 3), "calls_per_step": calls,
                 "layout": layout[0] if layout else "direct"}
            rows.append(r)
            step_ms += ms * calls
            print(json.dumps(r), flush=True)
        del x, w, dy, y, dx, dw
        torch.cuda.empty_cache()
    total_flops = sum(2.0 * r["M"] * r["N"] * r["K"] * r["calls_per_step"] for r in rows)
    print(json.dumps({"tag": a.tag, "summary": True, "gemm_ms_per_step": round(step_ms, 1),
                      "gemm_pflop_per_step": round(total_flops / 1e15, 4),
                      "avg_pflops": round(total_flops / step_ms / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
