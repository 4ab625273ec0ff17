"""Weight-gradient GEMM variants of ops/fused.py ``wgrad_into`` on the Llama-3-8B step shapes (M = 4 x 8192
tokens), each forced through the module's own launchers, transposes included: nt / tt / nn and their split-K
forms (nt2 / tt2 / nn2 and the 4-way nt4 / tt4 / nn4: contraction slices as a strided batch into fp32 slabs, then one reduction pass).
Output bf16 (the bench's main-grad dtype), random operands, 20-call windows."""
import json
import sys

import torch

sys.path.insert(0, ".")
import llm_training_amd.ops.fused as fused  # noqa: E402

M = 32768
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
fused.GEMM_MODES.update({"fwd": "lt", "dgrad": "lt", "wgrad": "lt"})


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for name, (N, K) in SHAPES.items():
    x = torch.randn(M, K, device="cuda").bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    ref = None
    r = {"shape": name, "M": M, "N": N, "K": K}
    for v in ("nt", "tt", "nn", "nt2", "tt2", "nn2", "nt4", "tt4", "nn4"):
        if v[-1].isdigit() and N * K > fused._SPLITK_MAX_OUT:
            continue
        fused._layout = (lambda vv: (lambda key, variants, default, can_time: vv))(v)
        ms = timeit(lambda: fused.wgrad_into(out, dy, x, False))
        if ref is None:
            ref = out.float().clone()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        r[v + "_ms"] = round(ms, 4)
        r[v + "_pf"] = round(2 * M * N * K / ms / 1e12, 3)
        r[v + "_err_vs_nt"] = round(err, 5)
    print(json.dumps(r), flush=True)
    del x, dy, out, ref
    torch.cuda.empty_cache()
