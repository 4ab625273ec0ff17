"""Backward GEMMs of one Llama-3-8B decoder layer at M = B*S tokens (hipBLASLt via csrc/blaslt.cpp):
sequential (dgrad, wgrad per projection in backward order) vs the weight gradients on a side stream
overlapping the next projection's input gradient. Reports ms per layer and the effective PF/s."""
import json
import sys

import torch

sys.path.insert(0, ".")
from llm_training_amd.ops import fused  # noqa: E402
from llm_training_amd.ops.native import lib  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
# backward order: down, gate_up, o, qkv  (N = out features, K = in features)
PROJ = [("down", 4096, 14336), ("gate_up", 28672, 4096), ("o", 4096, 4096), ("qkv", 6144, 4096)]
dev = torch.device("cuda", 0)
torch.manual_seed(0)
ops = []
for name, N, K in PROJ:
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    ops.append((name, dy, x, w, dw, dx))
flops = sum(2 * 2 * M * N * K for _, N, K in PROJ)
side = torch.cuda.Stream(device=dev)


def seq():
    for _, dy, x, w, dw, dx in ops:
        fused.mm_nn(dy, w, dx)
        fused.wgrad_into(dw, dy, x, False)


def ovl():
    cur = torch.cuda.current_stream()
    for _, dy, x, w, dw, dx in ops:
        ev = torch.cuda.Event()
        ev.record(cur)
        fused.mm_nn(dy, w, dx)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            fused.wgrad_into(dw, dy, x, False)
    cur.wait_stream(side)


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


res = {"M": M}
for sk in (True, False):
    fused.ALLOW_STREAMK[0] = sk
    t_seq = timeit(seq)
    t_ovl = timeit(ovl)
    res[f"sk{int(sk)}"] = {"seq_ms": round(t_seq, 3), "ovl_ms": round(t_ovl, 3),
                           "seq_pf": round(flops / t_seq / 1e12, 3), "ovl_pf": round(flops / t_ovl / 1e12, 3)}
# per-projection breakdown (sequential, default stream-K setting)
fused.ALLOW_STREAMK[0] = True
for name, dy, x, w, dw, dx in ops:
    N, K = w.shape
    td = timeit(lambda: fused.mm_nn(dy, w, dx))
    tw = timeit(lambda: fused.wgrad_into(dw, dy, x, False))
    res[name] = {"dgrad_ms": round(td, 3), "wgrad_ms": round(tw, 3),
                 "dgrad_pf": round(2 * M * N * K / td / 1e12, 3), "wgrad_pf": round(2 * M * N * K / tw / 1e12, 3)}
print(json.dumps(res), flush=True)
