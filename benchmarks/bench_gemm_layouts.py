"""Time the three GEMMs of a linear layer (fwd, dgrad, wgrad) for both weight storage layouts.

W stored [N, K] (PyTorch convention) or transposed [K, N]. hipBLASLt picks different kernels for
the different operand layouts; this measures which storage gives the lowest fwd+dgrad+wgrad time
per Llama-3-8B projection at T tokens.
"""
import argparse
import json

import torch


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
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
    args = ap.parse_args()
    T = args.tokens
    dev = "cuda"
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    for name, (N, K) in shapes.items():
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        Wt = W.t().contiguous()
        gW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        gWt = torch.empty(K, N, device=dev, dtype=torch.bfloat16)
        y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(T, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * N * K
        r = {"shape": name, "N": N, "K": K}
        r["fwd_W"] = timeit(lambda: torch.mm(x, W.t(), out=y))
        r["fwd_Wt"] = timeit(lambda: torch.mm(x, Wt, out=y))
        r["dgrad_W"] = timeit(lambda: torch.mm(dy, W, out=dx))
        r["dgrad_Wt"] = timeit(lambda: torch.mm(dy, Wt.t(), out=dx))
        r["wgrad_W"] = timeit(lambda: torch.mm(dy.t(), x, out=gW))
        r["wgrad_Wt"] = timeit(lambda: torch.mm(x.t(), dy, out=gWt))
        r["wgrad_W_acc"] = timeit(lambda: gW.addmm_(dy.t(), x))
        r["total_W"] = r["fwd_W"] + r["dgrad_W"] + r["wgrad_W"]
        r["total_Wt"] = r["fwd_Wt"] + r["dgrad_Wt"] + r["wgrad_Wt"]
        for k in list(r):
            if isinstance(r[k], float):
                r[k] = round(r[k], 4)
        r["pf_best"] = round(3 * fl / min(r["total_W"], r["total_Wt"]) / 1e12, 1)
        print(json.dumps(r), flush=True)
        del x, dy, W, Wt, gW, gWt, y, dx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
