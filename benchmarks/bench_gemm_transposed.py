"""Linear-layer backward GEMMs at M = B*S tokens (Llama-3-8B projections), hipBLASLt in every layout
hipBLASLt offers once operands are transposed by the LDS-tiled HIP transpose (csrc/elementwise.hip):

  dgrad  NN (dy, W as stored)        vs  TN (W^T materialised: both operands contraction-contiguous)
  wgrad  NT (dy, x token-major)      vs  NN (dy^T)  /  TT (x^T)  /  TN (dy^T and x^T)

Each *_total adds the transposes that layout needs. Prints one JSON line per projection."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_training_amd.ops import fused  # noqa: E402
from llm_training_amd.ops.native import lib  # noqa: E402

M0 = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
PROJ = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
        ("lm_head_chunk8192", 128256, 4096)]
if len(sys.argv) > 2 and sys.argv[2] == "phi3":  # Phi-3-mini: hidden 3072, intermediate 8192, vocab 32064
    PROJ = [("qkv", 9216, 3072), ("o", 3072, 3072), ("gate_up", 16384, 3072), ("down", 3072, 8192),
            ("lm_head_chunk8192", 32064, 3072)]
dev = torch.device("cuda", 0)
sk = fused.ALLOW_STREAMK[0]
fused.TRANSPOSE_LAYOUTS[0] = False  # the *_nn / *_nt baselines below are the direct layouts


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def tr(x):
    out = torch.empty(x.shape[1], x.shape[0], device=x.device, dtype=x.dtype)
    lib().transpose_(x, out)
    return out


torch.manual_seed(0)
chk = torch.randn(192, 320, device=dev).bfloat16()
assert torch.equal(tr(chk), chk.t().contiguous()), "transpose mismatch"
for name, N, K in PROJ:
    M = 8192 if name.startswith("lm_head") else M0
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    wt, dyt, xt = tr(w), tr(dy), tr(x)
    r = {"shape": name, "M": M, "N": N, "K": K, "model": sys.argv[2] if len(sys.argv) > 2 else "llama3-8b"}
    f = 2 * M * N * K
    # dgrad
    r["dgrad_nn"] = timeit(lambda: fused.mm_nn(dy, w, dx))
    ref_dx = dx.float().clone()
    r["dgrad_tn"] = timeit(lambda: lib().gemm_lt(wt, dy, dx, True, False, K, M, N, N, N, K, False, sk))
    r["dgrad_tn_err"] = ((dx.float() - ref_dx).norm() / ref_dx.norm()).item()
    r["tr_w"] = timeit(lambda: lib().transpose_(w, wt))
    # wgrad
    r["wgrad_nt"] = timeit(lambda: fused.wgrad_into(dw, dy, x, False))
    ref_dw = dw.float().clone()
    r["wgrad_nn"] = timeit(lambda: lib().gemm_lt(x, dyt, dw, False, False, K, N, M, K, M, K, False, sk))
    r["wgrad_tt"] = timeit(lambda: lib().gemm_lt(xt, dy, dw, True, True, K, N, M, M, N, K, False, sk))
    r["wgrad_tn"] = timeit(lambda: lib().gemm_lt(xt, dyt, dw, True, False, K, N, M, M, M, K, False, sk))
    r["wgrad_tn_err"] = ((dw.float() - ref_dw).norm() / ref_dw.norm()).item()
    r["tr_dy"] = timeit(lambda: lib().transpose_(dy, dyt))
    r["tr_x"] = timeit(lambda: lib().transpose_(x, xt))
    r["tr_dy_tbs"] = 4 * M * N / r["tr_dy"] / 1e9
    r["dgrad_tn_total"] = r["dgrad_tn"] + r["tr_w"]
    r["wgrad_nn_total"] = r["wgrad_nn"] + r["tr_dy"]
    r["wgrad_tt_total"] = r["wgrad_tt"] + r["tr_x"]
    r["wgrad_tn_total"] = r["wgrad_tn"] + r["tr_dy"] + r["tr_x"]
    for k in ("dgrad_nn", "dgrad_tn", "wgrad_nt", "wgrad_nn", "wgrad_tt", "wgrad_tn"):
        r[k + "_pf"] = f / r[k] / 1e12
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    del dy, x, w, dx, dw, wt, dyt, xt
    torch.cuda.empty_cache()
