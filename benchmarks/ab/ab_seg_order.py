"""Block order of packed rows (ops/fused.py segment_info, LLMT_SEG_ORDER): 1 = heaviest block first over all
documents, 2 = document-major (a document's blocks back to back, heaviest first inside it), 0 = index order.
Same process, alternating, fwd and fwd+bwd:
    python benchmarks/ab/ab_seg_order.py B S Hq Hkv D docs [equal]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402

B, S, Hq, Hkv, D, docs = (int(v) for v in sys.argv[1:7])
equal = len(sys.argv) > 7 and sys.argv[7] == "equal"
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
g = torch.Generator().manual_seed(0)
seg = torch.empty(B, S, dtype=torch.int32)
for b in range(B):
    if equal:
        seg[b] = torch.arange(S) * docs // S + 1
    else:
        cuts = sorted(torch.randperm(S - 1, generator=g)[: docs - 1].add(1).tolist())
        e = [0, *cuts, S]
        seg[b] = torch.repeat_interleave(torch.arange(1, docs + 1, dtype=torch.int32),
                                         torch.tensor([y - x for x, y in zip(e[:-1], e[1:])]))
seg = seg.cuda()
orders = ("1", "2")
infos = {}
for o in orders:
    os.environ["LLMT_SEG_ORDER"] = o
    infos[o] = F_.segment_info(seg)
os.environ.pop("LLMT_SEG_ORDER")


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


tf = {o: [] for o in orders}
tb = {o: [] for o in orders}
for _ in range(5):
    for o in orders:
        fwd = lambda: F_.flash_attention(q, k, v, causal=True, segment_ids=seg, seg_info=infos[o])  # noqa: E731
        tf[o].append(timeit(fwd))
        tb[o].append(timeit(lambda: fwd().backward(do)))
med = lambda xs: round(sorted(xs)[len(xs) // 2], 4)  # noqa: E731
print(json.dumps({"shape": [B, S, Hq, Hkv, D], "docs": docs, "equal": equal,
                  **{f"fwd_ms_order{o}": med(tf[o]) for o in orders},
                  **{f"fwd_bwd_ms_order{o}": med(tb[o]) for o in orders}}), flush=True)
