"""Compute-only timing of the staged tensor-parallel projection GEMMs on ONE GPU.

For tp in {2, 8} at (S=8192, micro-batch 4) and (S=131072, micro-batch 1) (the reference's TP examples,
/root/reference/config/examples/llama-3.1/llama-3.1-8b_tp_example.yaml:5-10), each Llama-3-8B projection's
per-rank GEMM sequence of one step is run exactly as parallel/tensor_parallel.py issues it, without the
collectives:

* ``staged``   the current scheme: m sequence chunks (LLMT_TP_STAGES), grouped into GEMMs of at least
               LLMT_TP_GEMM_TILES 256x256 output tiles (``gemm_groups``), one weight-gradient GEMM;
* ``old``      the round-5 scheme: one GEMM per (chunk, source rank) block of cm * B rows and n * m
               accumulating weight-gradient GEMMs;
* ``unstaged`` one GEMM per pass over all rows (the FLOP-equal reference).

One JSON line per (tp, shape, projection) with fwd / dgrad / wgrad ms of each scheme and staged / unstaged.
    python benchmarks/bench_tp_gemms.py [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

H, I, NQ, NKV, HD = 4096, 14336, 32, 8, 128


def projections(tp):
    # name: (kind, N_local, K_local); "ag" = column-parallel (input gathered), "rs" = row-parallel
    return {"qkv": ("ag", (NQ + 2 * NKV) * HD // tp, H), "o": ("rs", H, NQ * HD // tp),
            "gate_up": ("ag", 2 * I // tp, H), "down": ("rs", H, I // tp)}


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tp", default="2,8")
    ap.add_argument("--shapes", default="8192x4,131072x1")
    args = ap.parse_args()
    from llm_training_amd.ops.fused import mm_nn, mm_nt, weight_t, wgrad_into
    from llm_training_amd.parallel.tensor_parallel import gemm_groups, tp_stages
    dev = "cuda"
    for tp in (int(t) for t in args.tp.split(",")):
        for shp in args.shapes.split(","):
            S, B = (int(v) for v in shp.split("x"))
            c = S // tp
            m = tp_stages(c)
            cm = c // m
            per = tp * cm  # sequence positions per chunk
            rows_chunk = per * B
            T = S * B
            for name, (kind, N, K) in projections(tp).items():
                torch.manual_seed(0)
                x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
                w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
                dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
                y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
                dx = torch.empty(T, K, device=dev, dtype=torch.bfloat16)
                gw = torch.empty(N, K, device=dev, dtype=torch.float32)
                gf = gemm_groups(m, rows_chunk, N)    # forward groups (output width N)
                gd = gemm_groups(m, rows_chunk, K)    # input-gradient groups (output width K)
                rc = rows_chunk

                def fwd_staged():
                    for j0, j1 in gf:
                        mm_nt(x[j0 * rc:j1 * rc], w, out=y[j0 * rc:j1 * rc])

                def dgrad_staged():  # one W^T shared by the groups, as tensor_parallel does
                    wt = weight_t(w, T)
                    for j0, j1 in gd:
                        mm_nn(dy[j0 * rc:j1 * rc], w, out=dx[j0 * rc:j1 * rc], wt=wt)

                def wgrad_one():
                    wgrad_into(gw, dy, x, False)

                blk = cm * B  # rows of one (chunk, rank) block of the old scheme

                def fwd_old():
                    for i in range(m * tp):
                        mm_nt(x[i * blk:(i + 1) * blk], w, out=y[i * blk:(i + 1) * blk])

                def dgrad_old():
                    for i in range(m * tp):
                        mm_nn(dy[i * blk:(i + 1) * blk], w, out=dx[i * blk:(i + 1) * blk])

                def wgrad_old():
                    for i in range(m * tp):
                        wgrad_into(gw, dy[i * blk:(i + 1) * blk], x[i * blk:(i + 1) * blk], i > 0)

                fns = {"unstaged": (lambda: mm_nt(x, w, out=y), lambda: mm_nn(dy, w, out=dx), wgrad_one),
                       "staged": (fwd_staged, dgrad_staged, wgrad_one),
                       "old": (fwd_old, dgrad_old, wgrad_old)}
                res = {k: [[], [], []] for k in fns}
                for _ in range(args.rounds):
                    for k, trio in fns.items():
                        for i, f in enumerate(trio):
                            res[k][i].append(timeit(f))
                out = {"tp": tp, "S": S, "B": B, "proj": name, "kind": kind, "N": N, "K": K, "chunks": m,
                       "fwd_groups": [j1 - j0 for j0, j1 in gf], "dgrad_groups": [j1 - j0 for j0, j1 in gd],
                       "old_gemm_rows": blk}
                for k in fns:
                    for i, p in enumerate(("fwd", "dgrad", "wgrad")):
                        out[f"{k}_{p}_ms"] = round(min(res[k][i]), 4)
                    out[f"{k}_ms"] = round(sum(out[f"{k}_{p}_ms"] for p in ("fwd", "dgrad", "wgrad")), 4)
                out["staged_vs_unstaged"] = round(out["staged_ms"] / out["unstaged_ms"], 4)
                out["old_vs_unstaged"] = round(out["old_ms"] / out["unstaged_ms"], 4)
                print(json.dumps(out), flush=True)
                del x, w, dy, y, dx, gw
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
