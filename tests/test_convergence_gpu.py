"""Multi-step loss-curve parity on LEARNABLE data: the bf16 HIP path must TRAIN like
the fp32 torch reference objective (reference clm.py:136-168, dpo.py:156-187), not only agree on one
forward / backward.

Data: an order-1 Markov source — every token has a fixed successor (a random permutation of the
vocabulary) that follows with probability 0.9, else a uniform token — cut into documents of random length
and packed into rows with segment ids (no cross-document attention, doc starts carry no loss). Its
per-token entropy is ~1.2 nats against ln V = 8.3 for random tokens, so the loss falls far only if the
optimizer, the gradients and the attention masking are all right.

Runs: a small Llama (h 512, 4 layers, 8 q / 4 kv heads, V 4096) from one fp32 init, on the same batches:
(a) bf16 weights on the HIP kernels (fused AdamW, fp32 master), (b) fp32 weights on the torch reference
ops, (c) (a) at dp 2 x ZeRO-2 with two ranks sharing this GPU over gloo; and DPO on learnable preference
pairs (chosen: Markov text, rejected: uniform tokens) for (a) vs (b)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = torch.device("cuda", 0)
V, S, B = 4096, 512, 4
STEPS = 300
LR = 2e-3
DPO_LR = 1e-4


def cfg():
    from llm_training_amd.models.llama import LlamaConfig
    return LlamaConfig(vocab_size=V, hidden_size=512, intermediate_size=1024, num_hidden_layers=4,
                       num_attention_heads=8, num_key_value_heads=4, max_position_embeddings=2048,
                       rope_theta=10000.0)


def markov_rows(n_rows: int, seed: int, p_follow: float = 0.9):
    """[n_rows, S] token rows of packed Markov documents, their segment ids and loss labels."""
    import numpy as np
    rng = np.random.default_rng(seed)
    succ = np.random.default_rng(1234).permutation(V)
    ids = np.empty((n_rows, S), dtype=np.int64)
    seg = np.empty((n_rows, S), dtype=np.int32)
    lab = np.empty((n_rows, S), dtype=np.int64)
    follow = rng.random((n_rows, S)) < p_follow
    noise = rng.integers(0, V, (n_rows, S))
    for r in range(n_rows):
        pos, d = 0, 1
        while pos < S:
            ln = min(S - pos, int(rng.integers(48, 200)))
            t = int(rng.integers(0, V))
            for j in range(pos, pos + ln):
                ids[r, j] = t
                t = int(succ[t]) if follow[r, j] else int(noise[r, j])
            seg[r, pos:pos + ln] = d
            lab[r, pos:pos + ln] = ids[r, pos:pos + ln]
            lab[r, pos] = -100  # a document's first token is not predictable from the previous document
            pos += ln
            d += 1
    return torch.from_numpy(ids), torch.from_numpy(seg), torch.from_numpy(lab)


def clm_batches(n_steps=STEPS, seed=7):
    ids, seg, lab = markov_rows(n_steps * B, seed)
    return [{"input_ids": ids[i * B:(i + 1) * B], "attention_mask": seg[i * B:(i + 1) * B],
             "labels": lab[i * B:(i + 1) * B]} for i in range(n_steps)]


def _init_state():
    from llm_training_amd.models.llama import Llama
    from llm_training_amd.parallel.context import ParallelContext
    m = Llama(cfg(), ParallelContext.single(), dtype=torch.float32)
    m.init_weights(3)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def train_clm(dtype, batches, init):
    from llm_training_amd.lms.clm import CLM
    from llm_training_amd.models.llama import Llama
    from llm_training_amd.parallel.context import ParallelContext
    from llm_training_amd.parallel.engine import DataParallelEngine
    pc = ParallelContext.single(DEV)
    m = Llama(cfg(), pc, dtype=dtype, device=DEV)
    m.load_state_dict({k: v.to(DEV, dtype) for k, v in init.items()})
    eng = DataParallelEngine(m, pc, 0, lr=LR, weight_decay=0.0)
    lm = CLM({"model": None})
    lm.model = m
    lm.train()
    losses = []
    for b in batches:
        b = {k: v.to(DEV) for k, v in b.items()}
        b["attention_mask_trivial"] = False
        eng.begin_step(1)
        eng.zero_grad()
        eng.begin_micro(0)
        loss, _, _ = lm.training_step(b)
        loss.backward()
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(LR)
        losses.append(loss.detach().float())
    return torch.stack(losses).cpu()


def _tail_rel(a, b, n=50):
    a, b = a[-n:].mean().item(), b[-n:].mean().item()
    return abs(a - b) / abs(b)


@pytest.fixture(scope="module")
def curves():
    # deterministic mode: the GEMM layouts come from the static rule, not from timing on this box, so the
    # curves (whose bf16 roundings a different GEMM algorithm would change) are the same on every box
    old = os.environ.get("LLMT_DETERMINISTIC")
    os.environ["LLMT_DETERMINISTIC"] = "1"
    try:
        init = _init_state()
        batches = clm_batches()
        hip = train_clm(torch.bfloat16, batches, init)
        ref = train_clm(torch.float32, batches, init)
    finally:
        if old is None:
            os.environ.pop("LLMT_DETERMINISTIC", None)
        else:
            os.environ["LLMT_DETERMINISTIC"] = old
    return init, batches, hip, ref


def _window_rel(hip, ref, i, n=25, lag=4):
    """Relative gap of hip's window [i, i+n) to the closest reference window within +-lag steps: on the
    steep part of the curve (~0.13 nats per step) a 1-2 step lag between two runs' roundings would read as
    ~8 % in a fixed window, while a path that learns slower or worse lags by far more than 4 steps."""
    h = hip[i:i + n].mean()
    best = min(abs(h - ref[j:j + n].mean()) for j in range(max(0, i - lag), min(len(ref) - n, i + lag) + 1))
    return float(best / ref[i:i + n].mean())


def test_clm_bf16_hip_trains_like_the_fp32_reference(curves):
    import math
    _, _, hip, ref = curves
    assert torch.isfinite(hip).all() and torch.isfinite(ref).all()
    assert hip[-50:].mean() <= 0.5 * math.log(V), hip[-50:].mean()  # it learned the source
    assert hip[-50:].mean() < 0.4 * hip[:5].mean()
    assert _tail_rel(hip, ref) < 0.02, (hip[-50:].mean(), ref[-50:].mean())
    # and along the way, not only at the end: every 25-step window within 5 % (of the reference within 4 steps)
    gaps = [_window_rel(hip, ref, i) for i in range(0, STEPS, 25)]
    print("window gaps", [round(g, 4) for g in gaps], "tail", round(_tail_rel(hip, ref), 4))
    assert max(gaps) < 0.05, gaps


def test_clm_dp2_zero2_matches_single_process(curves, tmp_path):
    """Two ranks on this GPU over gloo (RCCL refuses two ranks on one device), ZeRO-2 with the transient
    gradient ring: the averaged loss curve matches the single-process bf16 curve within 1 %."""
    init, batches, hip, _ = curves
    n = 160  # (the two runs' bf16 roundings differ, so compare where the curve flattens, over 50 steps)
    torch.save({"init": init, "batches": batches[:n]}, tmp_path / "in.pt")
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4", LLMT_DIST_BACKEND="gloo", LLMT_SHARED_DEVICE="1",
               LLMT_DETERMINISTIC="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29650", os.path.join(ROOT, "tests", "test_convergence_gpu.py"),
           str(tmp_path / "in.pt"), str(tmp_path / "out.pt")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=115)
    assert r.returncode == 0, r.stderr[-4000:]
    got = torch.load(tmp_path / "out.pt", weights_only=True)
    print("dp2 tail", round(_tail_rel(got, hip[:n], 50), 4))
    assert _tail_rel(got, hip[:n], 50) < 0.01, (got[-50:].mean(), hip[n - 50:n].mean())
    assert (got - hip[:n]).abs().max() < 0.05 * hip[:n].max()


def _dp2_rank_main(inp, out):
    """Rank process of test_clm_dp2_zero2_matches_single_process (run through torch.distributed.run)."""
    import torch.distributed as dist

    from llm_training_amd.lms.clm import CLM
    from llm_training_amd.models.llama import Llama
    from llm_training_amd.parallel.context import ParallelContext, init_distributed
    from llm_training_amd.parallel.engine import DataParallelEngine
    init_distributed()
    d = torch.load(inp, weights_only=True)
    pc = ParallelContext.create("auto", 1, DEV)
    m = Llama(cfg(), pc, dtype=torch.bfloat16, device=DEV)
    m.load_state_dict({k: v.to(DEV, torch.bfloat16) for k, v in d["init"].items()})
    eng = DataParallelEngine(m, pc, 2, lr=LR, weight_decay=0.0)
    lm = CLM({"model": None})
    lm.model = m
    lm.train()
    losses = []
    half = B // 2
    for b in d["batches"]:
        loc = {k: v[pc.dp_rank * half:(pc.dp_rank + 1) * half].to(DEV) for k, v in b.items()}
        loc["attention_mask_trivial"] = False
        eng.begin_step(1)
        eng.zero_grad()
        eng.begin_micro(0)
        loss, _, _ = lm.training_step(loc)
        loss.backward()
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(LR)
        # the full-batch loss is the token-weighted mean of the two halves
        n_tok = (loc["labels"][:, 1:] != -100).sum().float()
        t = torch.stack([loss.detach().float() * n_tok, n_tok]).cpu()
        dist.all_reduce(t)
        losses.append(float(t[0] / t[1]))
    if dist.get_rank() == 0:
        torch.save(torch.tensor(losses), out)
    dist.barrier()
    dist.destroy_process_group()


def dpo_batches(n_steps, seed=9, Bp=2, Sp=256):
    ids, _, _ = markov_rows(n_steps * Bp, seed, p_follow=1.0)
    g = torch.Generator().manual_seed(seed + 1)
    out = []
    for i in range(n_steps):
        c = ids[i * Bp:(i + 1) * Bp, :Sp]
        r_ = torch.randint(0, V, (Bp, Sp), generator=g)
        r_[:, :Sp // 4] = c[:, :Sp // 4]  # a shared prompt
        b = {}
        for side, t in (("chosen", c), ("rejected", r_)):
            lab = t.clone()
            lab[:, :Sp // 4] = -100
            b.update({f"{side}_input_ids": t, f"{side}_labels": lab,
                      f"{side}_attention_mask": torch.ones(Bp, Sp, dtype=torch.long)})
        out.append(b)
    return out


def train_dpo(dtype, batches, init):
    from llm_training_amd.lms.preference import DPO
    from llm_training_amd.models.llama import Llama
    from llm_training_amd.parallel.context import ParallelContext
    from llm_training_amd.parallel.engine import DataParallelEngine
    pc = ParallelContext.single(DEV)
    mk = lambda: Llama(cfg(), pc, dtype=dtype, device=DEV)  # noqa: E731
    m, ref = mk(), mk()
    for x in (m, ref):
        x.load_state_dict({k: v.to(DEV, dtype) for k, v in init.items()})
    ref.requires_grad_(False)
    ref.eval()
    lm = DPO({"model": None, "beta": 0.1})
    lm.model, lm.ref_model = m, ref
    eng = DataParallelEngine(m, pc, 0, lr=DPO_LR, weight_decay=0.0)
    lm.train()
    losses = []
    for b in batches:
        b = {k: v.to(DEV) for k, v in b.items()}
        eng.begin_step(1)
        eng.zero_grad()
        eng.begin_micro(0)
        loss, _, _ = lm.training_step(b)
        loss.backward()
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(DPO_LR)
        losses.append(loss.detach().float())
    return torch.stack(losses).cpu()


def test_dpo_bf16_hip_trains_like_the_fp32_reference(monkeypatch):
    monkeypatch.setenv("LLMT_DETERMINISTIC", "1")  # GEMM layouts by the static rule (see `curves`)
    import math
    init = _init_state()
    batches = dpo_batches(150)
    hip = train_dpo(torch.bfloat16, batches, init)
    ref = train_dpo(torch.float32, batches, init)
    print("dpo hip", [round(x, 4) for x in hip.tolist()])
    print("dpo ref", [round(x, 4) for x in ref.tolist()])
    assert abs(hip[0].item() - math.log(2)) < 1e-2  # policy == reference at step 0
    assert hip[-30:].mean() <= 0.5 * math.log(2), hip[-30:].mean()  # it learned the preference
    assert abs(hip[-30:].mean() - ref[-30:].mean()) < 0.02 * math.log(2) + 0.02 * ref[-30:].mean(), \
        (hip[-30:].mean(), ref[-30:].mean())


if __name__ == "__main__":
    _dp2_rank_main(sys.argv[1], sys.argv[2])
