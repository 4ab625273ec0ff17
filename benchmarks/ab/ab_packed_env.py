"""Same-process A/B of a per-launch attention knob on packed (or dense) rows, fwd+bwd and bwd alone:
    python benchmarks/ab/ab_packed_env.py B S Hq Hkv D docs ENV v1,v2
docs = 0: dense causal rows; otherwise `docs` random-length documents per row in the models' block order
(document-major for MHA, heaviest-first for GQA). One JSON line with the median of 5 alternating windows."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402

B, S, Hq, Hkv, D, docs = (int(v) for v in sys.argv[1:7])
ENV, vals = sys.argv[7], sys.argv[8].split(",")
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
seg = info = None
if docs:
    g = torch.Generator().manual_seed(0)
    seg = torch.empty(B, S, dtype=torch.int32)
    for b in range(B):
        cuts = sorted(torch.randperm(S - 1, generator=g)[: docs - 1].add(1).tolist())
        e = [0, *cuts, S]
        seg[b] = torch.repeat_interleave(torch.arange(1, docs + 1, dtype=torch.int32),
                                         torch.tensor([y - x for x, y in zip(e[:-1], e[1:])]))
    seg = seg.cuda()
    info = F_.segment_info(seg, doc_major=(Hq == Hkv))


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


fwd = lambda: F_.flash_attention(q, k, v, causal=True, segment_ids=seg, seg_info=info)  # noqa: E731
o = fwd()
tfb = {x: [] for x in vals}
tb = {x: [] for x in vals}
grads = {}
for _ in range(5):
    for x in vals:
        os.environ[ENV] = x
        tfb[x].append(timeit(lambda: fwd().backward(do)))
        tb[x].append(timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True)))
        grads[x] = torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
os.environ.pop(ENV)
med = lambda xs: round(sorted(xs)[len(xs) // 2], 4)  # noqa: E731
same = all(torch.equal(a, b) for a, b in zip(grads[vals[0]], grads[vals[-1]]))
print(json.dumps({"shape": [B, S, Hq, Hkv, D], "docs": docs, "env": ENV, "grads_bitwise_equal": same,
                  **{f"fwd_bwd_ms_{x}": med(tfb[x]) for x in vals}, **{f"bwd_ms_{x}": med(tb[x]) for x in vals}}),
      flush=True)
