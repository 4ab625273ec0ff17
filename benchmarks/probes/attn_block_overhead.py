"""Per-block fixed cost of the flash-attention kernels: the same token count as rows of S tokens
(dense, B = N / S) and as one row of N tokens packed with equal documents of S tokens, for S = 128 .. N.
A least-squares fit of time = blocks * c_blk + tiles * c_tile per kernel pass separates the per-block
prologue / epilogue cost from the per-tile cost (short packed documents are dominated by the former).
    python benchmarks/probes/attn_block_overhead.py [N Hq Hkv D]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops import fused as F_  # noqa: E402

N, Hq, Hkv, D = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (16384, 32, 32, 96)))


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best


rows = []
for S in (128, 256, 512, 1024, 2048, 4096, 8192):
    if S > N:
        break
    for packed in (False, True):
        if packed and S == N:
            continue
        B, L = (1, N) if packed else (N // S, S)
        q = torch.randn(B, L, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, L, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, L, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        do = torch.randn(B, L, Hq, D, device="cuda", dtype=torch.bfloat16)
        seg = info = None
        if packed:
            seg = (torch.arange(L, device="cuda") // S + 1).to(torch.int32).view(1, L)
            info = F_.segment_info(seg)

        def fwd():
            return F_.flash_attention(q, k, v, causal=True, segment_ids=seg, seg_info=info)

        tf = timeit(fwd)
        tfb = timeit(lambda: fwd().backward(do))
        nqb = S // 128
        blocks = (N // S) * nqb * Hq  # query blocks of 128 rows (one workgroup each)
        tiles64 = (N // S) * Hq * sum(2 * (i + 1) for i in range(nqb))  # 64-key tiles under the causal mask
        rows.append({"S": S, "packed": packed, "fwd_ms": round(tf, 4), "bwd_ms": round(tfb - tf, 4),
                     "blocks": blocks, "tiles64": tiles64})
        print(json.dumps(rows[-1]), flush=True)
for kind in ("fwd_ms", "bwd_ms"):
    for packed in (False, True):
        rs = [r for r in rows if r["packed"] == packed] + ([r for r in rows if r["S"] == N] if packed else [])
        A = np.array([[r["blocks"], r["tiles64"]] for r in rs], dtype=float)
        y = np.array([r[kind] for r in rs])
        (cb, ct), *_ = np.linalg.lstsq(A, y, rcond=None)
        print(json.dumps({"fit": kind, "packed": packed, "N": N, "Hq": Hq, "Hkv": Hkv, "D": D,
                          "us_per_block_per_slot": round(cb * 1e3 * 512, 3), "us_per_tile_per_slot": round(ct * 1e3 * 512, 4),
                          "resid_ms": [round(float(x), 4) for x in (A @ [cb, ct] - y)]}), flush=True)
