"""Cross-entropy with the gradient written in place, on the loss-head chunks of the Llama-3-8B step (8192 rows x
128256) and the Phi-3 step (8192 x 32064): checked against an fp32 oracle, with and without the gradient write,
and timed (the logits copy each call needs is timed alone and subtracted). Prints one JSON line.
    python benchmarks/ab/ab_ce.py

Round 6 ran it interleaved over two kernels selected per call (profiles/r6_ce_ab.jsonl): v0 = the two-pass
ce_kernel (256 threads, the row read twice), v1 = the one-pass ce_reg_kernel (1024 threads, the row in
registers). v1 is now used for every aligned row of up to 131072 logits; the switch is gone."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_training_amd.ops.native import lib  # noqa: E402

L = lib()


def timed(fn, n=10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


out = {}
for name, N, V in (("llama", 8192, 128256), ("phi3", 8192, 32064)):
    g = torch.Generator(device="cuda").manual_seed(0)
    logits = (3 * torch.randn(N, V, device="cuda", generator=g)).bfloat16()
    labels = torch.randint(0, V, (N,), device="cuda", generator=g)
    labels[::7] = -100
    inv_n = torch.full((1,), 1.0 / N, device="cuda")
    lf = logits[:512].float()
    lse_ref = torch.logsumexp(lf, -1)
    p = torch.softmax(lf, -1)
    lab = labels[:512]
    grad_ref = p.clone()
    ok = lab != -100
    grad_ref[ok, lab[ok]] -= 1
    grad_ref[~ok] = 0
    grad_ref /= N
    work = torch.empty_like(logits)
    for v in ("1",):
        x = logits.clone()
        lse, _, loss = L.cross_entropy_(x, labels, 0, -100, None, None, inv_n, True)
        out[f"{name}_v{v}_lse_maxerr"] = float((lse[:512] - lse_ref).abs().max())
        out[f"{name}_v{v}_grad_maxerr"] = float((x[:512].float() - grad_ref).abs().max())
        x2 = logits.clone()
        lse2, _, _ = L.cross_entropy_(x2, labels, 0, -100, None, None, None, False)
        out[f"{name}_v{v}_nograd_untouched"] = bool(torch.equal(x2, logits))
        out[f"{name}_v{v}_lse_same_without_grad"] = bool(torch.equal(lse, lse2))

    def run():
        work.copy_(logits)
        L.cross_entropy_(work, labels, 0, -100, None, None, inv_n, True)

    def copy_only():
        work.copy_(logits)

    tc = sorted(timed(copy_only) for _ in range(3))[1]
    times = {}
    for rnd in range(5):
        times.setdefault("1", []).append(timed(run) - tc)
    for v, ts in times.items():
        out[f"{name}_v{v}_ms"] = round(sorted(ts)[len(ts) // 2], 4)
    del logits, work, lf, p, grad_ref
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
