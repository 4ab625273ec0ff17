"""Weight-gradient GEMM layouts on the Llama-3-8B step shapes (M = 24576 tokens), hipBLASLt via
csrc/blaslt.cpp, random operands, 25-call windows (sustained clock):
  nt  dW = dy^T . x straight from the token-major activations (the library's NT kernel)
  nn  dy transposed first (token-contiguous dy^T), then NN
  tn  dy and x both transposed first, then TN (the forward's layout)
Transpose time (torch copy) is reported separately and included in *_total."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_training_amd.ops.native import lib  # noqa: E402

M = 24576
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, reps=25):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


L = lib()
for name, (N, K) in SHAPES.items():
    x = torch.randn(M, K, device="cuda").bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    out = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    xT = x.t().contiguous()
    dyT = dy.t().contiguous()
    fl = 2 * M * N * K
    r = {"shape": name, "M": M, "N": N, "K": K}
    r["nt_ms"] = timeit(lambda: L.gemm_lt(x, dy, out, False, True, K, N, M, K, N, K, True))
    r["nn_ms"] = timeit(lambda: L.gemm_lt(x, dyT, out, False, False, K, N, M, K, M, K, True))
    r["tn_ms"] = timeit(lambda: L.gemm_lt(xT, dyT, out, True, False, K, N, M, M, M, K, True))
    r["tr_dy_ms"] = timeit(lambda: dyT.copy_(dy.t()))
    r["tr_x_ms"] = timeit(lambda: xT.copy_(x.t()))
    r["nn_total"] = r["nn_ms"] + r["tr_dy_ms"]
    r["tn_total"] = r["tn_ms"] + r["tr_dy_ms"] + r["tr_x_ms"]
    for k in ("nt", "nn", "tn"):
        r[k + "_pf"] = fl / r[k + "_ms"] / 1e12
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
