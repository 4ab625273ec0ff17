"""Packed (varlen) attention efficiency: HIP flash kernels on rows of K isolated documents vs dense causal.

For each documents-per-row count the rows are cut at random points (the bench.py pt-packed layout) or into
equal documents; the attended fraction of the causal work is computed exactly, and the reported
``attended_rate_vs_dense`` = (attended FLOPs / time) / (dense causal FLOPs / dense time) — 1.0 means a
packed row costs exactly its attended work (reference flash_attn_varlen_func cost).

    python benchmarks/bench_packed_attention.py --B 4 --S 8192
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_training_amd.ops import fused as F_  # noqa: E402


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def segments(B, S, n, equal, g):
    seg = torch.empty(B, S, dtype=torch.int32)
    frac = 0.0
    for b in range(B):
        if equal:
            lens = [S // n] * n
            lens[-1] += S - sum(lens)
        else:
            cuts = sorted(torch.randperm(S - 1, generator=g)[: n - 1].add(1).tolist()) if n > 1 else []
            e = [0, *cuts, S]
            lens = [y - x for x, y in zip(e[:-1], e[1:])]
        seg[b] = torch.repeat_interleave(torch.arange(1, n + 1, dtype=torch.int32), torch.tensor(lens))
        frac += sum(ln * (ln + 1) / 2 for ln in lens) / (S * (S + 1) / 2)
    return seg, frac / B


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=8192)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--docs", default="1,2,4,8,16,32")
    ap.add_argument("--equal", action="store_true")
    ap.add_argument("--ab", default="", help="in-process A/B of a per-launch env knob, e.g. LLMT_FA_RANGE_MASK:0,1")
    a = ap.parse_args()
    dev = "cuda"
    B, S = a.B, a.S
    q = torch.randn(B, S, a.Hq, a.D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, a.Hkv, a.D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, a.Hkv, a.D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, a.Hq, a.D, device=dev, dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(0)
    dense = None
    for n in [int(x) for x in a.docs.split(",")]:
        seg, frac = segments(B, S, n, a.equal, g)
        seg = seg.to(dev) if n > 1 else None
        info = F_.segment_info(seg) if seg is not None else None
        if seg is not None and os.environ.get("LLMT_SEG_ORDER_AB") == "1":
            os.environ["LLMT_SEG_ORDER"] = "0"
            info0 = F_.segment_info(seg)
            os.environ["LLMT_SEG_ORDER"] = "1"
            t_new, t_old = [], []
            for _ in range(3):
                t_new.append(timeit(lambda: F_.flash_attention(q, k, v, causal=True, segment_ids=seg, seg_info=info)))
                t_old.append(timeit(lambda: F_.flash_attention(q, k, v, causal=True, segment_ids=seg, seg_info=info0)))
            bn, bo = [], []
            for _ in range(3):
                bn.append(timeit(lambda: F_.flash_attention(q, k, v, causal=True, segment_ids=seg,
                                                            seg_info=info).backward(do)))
                bo.append(timeit(lambda: F_.flash_attention(q, k, v, causal=True, segment_ids=seg,
                                                            seg_info=info0).backward(do)))
            print(json.dumps({"docs": n, "B": B, "S": S, "D": a.D, "Hkv": a.Hkv, "fwd_ms_ordered": round(min(t_new), 4),
                              "fwd_ms_index_order": round(min(t_old), 4),
                              "fwd_bwd_ms_ordered": round(min(bn), 4), "fwd_bwd_ms_index_order": round(min(bo), 4)}),
                  flush=True)

        def fwd():
            return F_.flash_attention(q, k, v, causal=True, segment_ids=seg, seg_info=info)

        if a.ab:
            name, vals = a.ab.split(":")
            vals = vals.split(",")
            tf_ab, tb_ab = {x: [] for x in vals}, {x: [] for x in vals}
            for _ in range(3):
                for x in vals:
                    os.environ[name] = x
                    tf_ab[x].append(timeit(fwd))
                    tb_ab[x].append(timeit(lambda: fwd().backward(do)))
            os.environ.pop(name)
            print(json.dumps({"docs": n, "B": B, "S": S, "D": a.D, "Hq": a.Hq, "Hkv": a.Hkv, "ab": name,
                              **{f"fwd_ms_{x}": round(min(tf_ab[x]), 4) for x in vals},
                              **{f"fwd_bwd_ms_{x}": round(min(tb_ab[x]), 4) for x in vals}}), flush=True)

        def fb():
            fwd().backward(do)

        tf = timeit(fwd)
        tb = timeit(fb) - tf
        if dense is None:
            dense = (tf, tb)
        r = {"B": B, "S": S, "docs": n, "equal": a.equal, "attended_frac": round(frac, 4),
             "fwd_ms": round(tf, 3), "bwd_ms": round(tb, 3),
             "fwd_attended_rate_vs_dense": round(frac / tf * dense[0], 3),
             "bwd_attended_rate_vs_dense": round(frac / tb * dense[1], 3),
             "total_attended_rate_vs_dense": round(frac / (tf + tb) * (dense[0] + dense[1]), 3)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
