"""Where the per-block cost of the attention kernels goes (LLMT_FA_PROBE diagnostic probes, wrong results by
design): forward with no tiles (1), no Q loads (2), no O / LSE stores (4), combinations; backward with no
tiles in dQ and dK/dV (8). Same process, alternating. Runs on the DIAGNOSTIC library (_C_diag.so, built on
first use or by `python -m llm_training_amd._build --diag`): the production library has no probe code.
    python benchmarks/probes/attn_block_probe.py B S Hq Hkv D"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["LLMT_NATIVE_DIAG"] = "1"  # before the package loads its native library
from llm_training_amd.ops import fused as F_  # noqa: E402
from llm_training_amd.ops.native import lib  # noqa: E402

assert lib().diag_build() == 1, "the probes need the diagnostic library"

B, S, Hq, Hkv, D = (int(v) for v in sys.argv[1:6])
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
o = F_.flash_attention(q, k, v, causal=True)


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


fw = {p: [] for p in (0, 1, 2, 4, 6, 7)}
bw = {p: [] for p in (0, 8)}
for _ in range(5):
    for p in fw:
        os.environ["LLMT_FA_PROBE"] = str(p)
        fw[p].append(timeit(lambda: F_.flash_attention(q, k, v, causal=True)))
    for p in bw:
        os.environ["LLMT_FA_PROBE"] = str(p)
        bw[p].append(timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True)))
os.environ.pop("LLMT_FA_PROBE")
med = lambda xs: round(sorted(xs)[len(xs) // 2], 4)  # noqa: E731
print(json.dumps({"shape": [B, S, Hq, Hkv, D], "early": os.environ.get("LLMT_FA_EARLY_DMA", "1"),
                  **{f"fwd_probe{p}_ms": med(x) for p, x in fw.items()},
                  **{f"bwd_probe{p}_ms": med(x) for p, x in bw.items()}}), flush=True)
