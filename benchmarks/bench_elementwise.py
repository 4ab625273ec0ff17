"""Memory-bound kernels of the Llama-3-8B step at 32768 tokens: SwiGLU forward / backward (row-blocked vs
flat grid-stride kernels, LLMT_EW_ROWS read per call, interleaved in one process) and RMSNorm forward /
backward (+ residual). Prints ms and achieved TB/s (bytes the kernel must move / time).
    python benchmarks/bench_elementwise.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_training_amd.ops.native import lib  # noqa: E402

L = lib()
T, H, I = 32768, 4096, 14336
gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16)
dc = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
res = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
w = torch.randn(H, device="cuda", dtype=torch.bfloat16)


def timed(fn, n=20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


out = {}
ref = {}
for rnd in range(3):
    for mode in ("1", "0"):
        os.environ["LLMT_EW_ROWS"] = mode
        tf = timed(lambda: L.swiglu_fwd(gu))
        tb = timed(lambda: L.swiglu_bwd(gu, dc))
        out.setdefault(f"swiglu_fwd_ms_rows{mode}", []).append(tf)
        out.setdefault(f"swiglu_bwd_ms_rows{mode}", []).append(tb)
        ref[mode] = (L.swiglu_fwd(gu), L.swiglu_bwd(gu, dc))
y, r_out, rstd = L.rmsnorm_fwd(x, res, w, 1e-5)
out["rmsnorm_fwd_res_ms"] = [timed(lambda: L.rmsnorm_fwd(x, res, w, 1e-5))]
dy = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
out["rmsnorm_bwd_res_ms"] = [timed(lambda: L.rmsnorm_bwd(dy, r_out, w, rstd, res, None, False, True))]
res_j = {k: round(sorted(v)[len(v) // 2], 4) for k, v in out.items()}
gb = {"swiglu_fwd": T * I * 2 * 3 / 1e9, "swiglu_bwd": T * I * 2 * 5 / 1e9, "rmsnorm_fwd_res": T * H * 2 * 4 / 1e9,
      "rmsnorm_bwd_res": T * H * 2 * 4 / 1e9}
for k, v in list(res_j.items()):
    base = next(n for n in gb if k.startswith(n))
    res_j[k.replace("_ms", "_tbs")] = round(gb[base] / v, 2)
res_j["rows_vs_flat_bitwise"] = bool(torch.equal(ref["1"][0], ref["0"][0]) and torch.equal(ref["1"][1], ref["0"][1]))
res_j["rmsnorm_bwd_blocks_env"] = os.environ.get("LLMT_RMSNORM_BWD_BLOCKS", "default")
print(json.dumps(res_j), flush=True)
