"""Memory-bound kernels of the Llama-3-8B step at 32768 tokens: SwiGLU forward / backward (row-blocked vs
flat grid-stride kernels, LLMT_EW_ROWS read per call, interleaved in one process) and RMSNorm forward /
backward (+ residual), RoPE in place on the q / k heads of the fused QKV buffer (token-blocked / flat / LDS-staged,
LLMT_ROPE_KERNEL; Llama-3-8B 32 + 8 heads of 128 and Phi-3-mini 32 + 32 heads of 96, packed positions).
Prints ms and achieved TB/s (bytes the kernel must move / time).
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
from llm_training_amd.ops.rope_utils import compute_rope_tables  # noqa: E402
rope_gb = {}
for name, hq, hkv, D in (("llama", 32, 8, 128), ("phi3", 32, 32, 96)):
    qkv = torch.randn(T, hq + 2 * hkv, D, device="cuda", dtype=torch.bfloat16)
    pos = (torch.arange(T, device="cuda") % 1024).contiguous()  # packed documents of 1024 tokens
    cos, sin = compute_rope_tables(D, 4096, 10000.0, device="cuda")
    rope_gb[f"rope_{name}"] = T * (hq + hkv) * D * 2 * 2 / 1e9
    for rnd in range(3):
        for mode in ("rows", "flat", "lds"):
            os.environ["LLMT_ROPE_KERNEL"] = mode
            out.setdefault(f"rope_{name}_ms_{mode}", []).append(
                timed(lambda: L.rope_(qkv, pos, cos, sin, hq + hkv, False)))
    os.environ.pop("LLMT_ROPE_KERNEL")
res_j = {k: round(sorted(v)[len(v) // 2], 4) for k, v in out.items()}
gb = {"swiglu_fwd": T * I * 2 * 3 / 1e9, "swiglu_bwd": T * I * 2 * 5 / 1e9, "rmsnorm_fwd_res": T * H * 2 * 4 / 1e9,
      "rmsnorm_bwd_res": T * H * 2 * 4 / 1e9, **rope_gb}
for k, v in list(res_j.items()):
    base = next(n for n in gb if k.startswith(n))
    res_j[k.replace("_ms", "_tbs")] = round(gb[base] / v, 2)
res_j["rows_vs_flat_bitwise"] = bool(torch.equal(ref["1"][0], ref["0"][0]) and torch.equal(ref["1"][1], ref["0"][1]))
res_j["rmsnorm_bwd_blocks_env"] = os.environ.get("LLMT_RMSNORM_BWD_BLOCKS", "default")
print(json.dumps(res_j), flush=True)
