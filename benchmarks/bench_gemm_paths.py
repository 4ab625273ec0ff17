"""Per-projection GEMM timing of the three linear paths (torch/hipBLASLt default, tuned hipBLASLt via
csrc/blaslt.cpp, own gfx950 kernel) on the Llama-3-8B step shapes, random operands (rule: constant
data reads high). Prints one JSON line per (shape, layout, path) with ms and PF/s."""
import json
import sys

import torch

sys.path.insert(0, ".")
import llm_training_amd.ops.fused as F  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 24576
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head_chunk": (128256, 4096)}


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


for name, (N, K) in SHAPES.items():
    m = 8192 if name == "lm_head_chunk" else M
    x = torch.randn(m, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    dy = torch.randn(m, N, device="cuda").bfloat16()
    g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    fl = 2 * m * N * K
    for path in ("blas", "lt", "hip"):
        F.GEMM_MODES.update(fwd=path, dgrad=path, wgrad=path)
        res = {"shape": name, "M": m, "N": N, "K": K, "path": path}
        for lay, fn in (("fwd", lambda: F.mm_nt(x, w)), ("dgrad", lambda: F.mm_nn(dy, w)),
                        ("wgrad", lambda: F.wgrad_into(g, dy, x, True) or g.addmm_(dy.t(), x))):
            ms = timeit(fn)
            res[lay + "_ms"] = round(ms, 4)
            res[lay + "_pf"] = round(fl / ms / 1e12, 3)
        print(json.dumps(res), flush=True)
print(lib_export := F.lib().gemm_lt_export(), file=sys.stderr)
