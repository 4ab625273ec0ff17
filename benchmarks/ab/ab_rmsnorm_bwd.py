"""RMSNorm backward (+ residual gradient) at the Llama-3-8B (T 32768, H 4096) and Phi-3-mini IT (T 65536,
H 3072) step shapes: checked against an fp32 oracle, with and without the weight gradient, and timed. Prints one
JSON line.
    python benchmarks/ab/ab_rmsnorm_bwd.py

Round 6 ran this interleaved over three kernels (profiles/r6_rmsnorm_bwd_ab.jsonl): v0 = one wave per row
(240 VGPRs, two waves per SIMD, 512 blocks), v1 = two waves per row with the residual gradient read ahead of
the row reduction (768 blocks), v2 = read after it (128 VGPRs, four waves per SIMD, 1024 blocks). v2 won on
both shapes and is the only kernel kept."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops.native import lib  # noqa: E402

L = lib()


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
for name, T, H in (("llama", 32768, 4096), ("phi3", 65536, 3072)):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, generator=g)
    res = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(H, device="cuda", dtype=torch.bfloat16, generator=g)
    dy = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, generator=g)
    dres = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, generator=g)
    _, s, rstd = L.rmsnorm_fwd(x, res, w, 1e-5)
    # fp32 oracle of dx (+ dres) and dw from the bf16 residual sum s
    sf, wf, dyf = s.float(), w.float(), dy.float()
    r = torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + 1e-5)
    n = (sf * r).bfloat16().float()
    dn = dyf * wf
    dx_ref = r * (dn - sf * r * (dn * sf * r).mean(-1, keepdim=True)) + dres.float()
    dw_ref = (dyf * n).sum(0)
    gb = T * H * 2 * 4 / 1e9
    dx, dw = L.rmsnorm_bwd(dy, s, w, rstd, dres, None, False, True)
    out[f"{name}_dx_maxerr"] = round(float((dx.float() - dx_ref).abs().max()), 4)
    out[f"{name}_dw_relerr"] = float((dw.float() - dw_ref).abs().max() / dw_ref.abs().max())
    dx2, _ = L.rmsnorm_bwd(dy, s, w, rstd, dres, None, False, False)  # no weight gradient (frozen weight)
    out[f"{name}_dx_nodw_equal"] = bool(torch.equal(dx, dx2))
    ts = sorted(timed(lambda: L.rmsnorm_bwd(dy, s, w, rstd, dres, None, False, True)) for _ in range(5))
    out[f"{name}_ms"] = round(ts[2], 4)
    out[f"{name}_tbs"] = round(gb / ts[2], 2)
    del x, res, dy, dres, s, sf, dyf, dx_ref, n, dn
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
