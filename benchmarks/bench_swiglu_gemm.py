"""The down-projection input gradient + SwiGLU backward: fused (one hand-written GEMM whose epilogue writes
dgu and dgu^T, csrc/gemm.hip SwiArgs) against the unfused pair the step ran before (hipBLASLt dgrad through
ops.fused.mm_nn + the standalone swiglu_bwd_tr pass), interleaved in one process on the same operands.
    python benchmarks/bench_swiglu_gemm.py [--rounds 5]
One JSON line per shape: ms of each form and the saving per layer.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"llama3-8b mb4": (32768, 4096, 14336), "phi3-mini mb16": (65536, 3072, 8192),
          "llama3-8b tp2 mb4": (32768, 4096, 7168)}


def timeit(fn, iters=10):
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    from llm_training_amd.ops.fused import mm_nn
    from llm_training_amd.ops.native import lib
    L = lib()
    for name in args.shapes.split(","):
        T, H, I = SHAPES[name]
        torch.manual_seed(0)
        dy = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(H, I, device="cuda") * H ** -0.5).to(torch.bfloat16)
        gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16)
        dc = torch.empty(T, I, device="cuda", dtype=torch.bfloat16)

        def unfused():
            mm_nn(dy, w, out=dc)
            return L.swiglu_bwd_tr(gu, dc)

        def dgrad_only():
            mm_nn(dy, w, out=dc)

        def fused():
            return L.gemm_swiglu_bwd(dy, w, gu, True)

        def own_gemm_only():  # the same GEMM with a plain bf16 store of dc (no SwiGLU epilogue)
            L.gemm_(dy, w, dc, False, True, False)

        fns = {"unfused": unfused, "fused": fused, "hipblaslt_dgrad": dgrad_only, "own_dgrad": own_gemm_only,
               "swiglu_bwd_tr": lambda: L.swiglu_bwd_tr(gu, dc)}
        a = unfused()
        b = fused()
        err = float((a[0].float() - b[0].float()).norm() / a[0].float().norm())
        same_t = bool(torch.equal(b[1], b[0].t().contiguous()))
        del a, b
        res = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, f in fns.items():
                res[k].append(timeit(f))
        out = {"shape": name, "T": T, "H": H, "I": I, "rel_err_fused_vs_unfused": round(err, 5),
               "dgu_t_is_transpose": same_t}
        for k, v in res.items():
            out[f"{k}_ms"] = round(sorted(v)[len(v) // 2], 4)
        fl = 2.0 * T * H * I
        out["own_dgrad_pflops"] = round(fl / out["own_dgrad_ms"] / 1e12, 3)
        out["hipblaslt_dgrad_pflops"] = round(fl / out["hipblaslt_dgrad_ms"] / 1e12, 3)
        out["saving_ms_per_layer"] = round(out["unfused_ms"] - out["fused_ms"], 4)
        print(json.dumps(out), flush=True)
        del dy, w, gu, dc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
