"""Hand-written gfx950 GEMM (csrc/gemm.hip) vs hipBLASLt (torch.mm) on the Llama-3-8B linear layers.

For each projection at T tokens: forward y = x W^T, dgrad dx = dy W, wgrad dW = dy^T x (bf16 output,
as into the bf16 gradient buffer). Random data; both back-ends timed in interleaved rounds with CUDA
events so clock drift hits both equally. One JSON line per shape, then totals.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from llm_training_amd.ops.native import lib
    L = lib()
    T, dev = args.tokens, "cuda"
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    tot = {"blas": 0.0, "hip": 0.0}
    for name, (N, K) in shapes.items():
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        gW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(T, K, device=dev, dtype=torch.bfloat16)
        fns = {
            "fwd": {"blas": lambda: torch.mm(x, W.t(), out=y), "hip": lambda: L.gemm_(x, W, y, False, False, False)},
            "dgrad": {"blas": lambda: torch.mm(dy, W, out=dx), "hip": lambda: L.gemm_(dy, W, dx, False, True, False)},
            "wgrad": {"blas": lambda: torch.mm(dy.t(), x, out=gW), "hip": lambda: L.gemm_(dy, x, gW, True, True, False)},
        }
        # numerics spot check of every layout against the library on this shape
        errs = {}
        for k, f in fns.items():
            f["hip"]()
            out = {"fwd": y, "dgrad": dx, "wgrad": gW}[k]
            got = out.float().clone()
            f["blas"]()
            errs[k] = round(((got - out.float()).norm() / out.float().norm()).item(), 5)
        res = {k: {"blas": [], "hip": []} for k in fns}
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for k, f in fns.items():
                for b, fn in f.items():
                    res[k][b].append(timeit(fn))
        fl = 2.0 * T * N * K
        r = {"shape": name, "N": N, "K": K, "T": T, "rel_err_vs_blas": errs}
        for k in fns:
            for b in ("blas", "hip"):
                ms = min(res[k][b])
                r[f"{k}_{b}_ms"] = round(ms, 4)
                r[f"{k}_{b}_tflops"] = round(fl / ms / 1e9, 1)
                tot[b] += ms
        print(json.dumps(r), flush=True)
        del x, dy, W, gW, y, dx
        torch.cuda.empty_cache()
    print(json.dumps({"total_ms_all_shapes": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
