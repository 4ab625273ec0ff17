"""Two rank processes on ONE MI355X over gloo (RCCL refuses two ranks on one GPU): ZeRO-2 and ZeRO-3 at
dp 2 and TP+SP at tp 2 run the engine's and the TP layers' rank > 0 paths with the HIP kernels and real
cross-rank data, and train like one process. (The 8-GPU RCCL run itself is the driver's scaling bench.)"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _single(tmp_path):
    from llm_training_amd.lms.clm import CLM
    from llm_training_amd.models.llama import Llama
    from llm_training_amd.parallel.context import ParallelContext
    from llm_training_amd.parallel.engine import DataParallelEngine
    from tests.multirank_gpu_common import CFG, batches
    dev = torch.device("cuda", 0)
    m = Llama(CFG, ParallelContext.single(dev), dtype=torch.bfloat16, device=dev)
    m.init_weights(3)
    full0 = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    torch.save(full0, tmp_path / "full0.pt")
    eng = DataParallelEngine(m, ParallelContext.single(dev), 0, lr=1e-3, weight_decay=0.0)
    lm = CLM({"model": None})
    lm.model = m
    lm.train()
    losses = []
    for ids in batches(dev):
        eng.begin_step(1)
        eng.zero_grad()
        eng.begin_micro(0)
        loss, _, _ = lm.training_step({"input_ids": ids, "labels": ids})
        loss.backward()
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(1e-3)
        losses.append(loss.item())
    eng.wait_params()
    return losses, {k: v.detach().float().cpu() for k, v in m.state_dict().items()}


@pytest.fixture(scope="module")
def reference(tmp_path_factory):
    d = tmp_path_factory.mktemp("mr")
    losses, params = _single(d)
    return d, losses, params


MODES = ["dp2_z2", "dp2_z3", "tp2", "tp2_stages1"]


def _run_worker(d, mode):
    """Run the two-rank worker once per mode (cached in the module's tmp dir). tp2_stages1: tp2 with the
    sequence collectives and GEMMs unstaged (LLMT_TP_STAGES=1)."""
    out = d / f"{mode}.pt"
    if not out.exists():
        env = dict(os.environ, FULL0=str(d / "full0.pt"), PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
        if mode == "tp2_stages1":
            env["LLMT_TP_STAGES"] = "1"
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(29600 + MODES.index(mode)),
               os.path.join(ROOT, "tests", "multirank_gpu_worker.py"), mode.split("_stages")[0], str(out)]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=100)
        assert r.returncode == 0, r.stderr[-4000:]
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("mode", MODES)
def test_two_ranks_on_one_gpu_match_single_process(reference, mode):
    d, ref_losses, ref_params = reference
    got = _run_worker(d, mode)
    # rank 1 runs rank 0's hipBLASLt solutions (ops.fused.agree_layouts -> gemm_lt_adopt)
    r0, r1 = got["lt_choices"]
    common = set(r0) & set(r1)
    assert common and all(r0[k] == r1[k] for k in common), {k: (r0[k], r1[k]) for k in common if r0[k] != r1[k]}
    # dp: the mean of the two half-batch losses is the full-batch loss (equal token counts); bf16 kernels
    for a, b in zip(got["losses"], ref_losses):
        assert abs(a - b) < 2e-2 * abs(b), (mode, got["losses"], ref_losses)
    num = den = 0.0
    for k, v in ref_params.items():
        num += (got["params"][k] - v).norm().item() ** 2
        den += v.norm().item() ** 2
    assert (num / den) ** 0.5 < 5e-3, mode


def test_tp_stages_do_not_change_the_bf16_training(reference):
    """The staged collective matmul (4 sequence chunks, grouped GEMMs, one weight-gradient GEMM over the whole
    gathered operands) trains like the unstaged form in bf16 on the GPU: the weight gradients are one GEMM in
    both, so no per-chunk bf16 rounding accumulates (round-5 advice)."""
    d = reference[0]
    a, b = _run_worker(d, "tp2"), _run_worker(d, "tp2_stages1")
    for x, y in zip(a["losses"], b["losses"]):
        assert abs(x - y) < 2e-3 * abs(y), (a["losses"], b["losses"])
    assert abs(a["grad_norm"] - b["grad_norm"]) < 1e-2 * b["grad_norm"]
    num = den = 0.0
    for k, v in b["params"].items():
        num += (a["params"][k] - v).norm().item() ** 2
        den += v.norm().item() ** 2
    # three AdamW steps at lr 1e-3 turn GEMM-order rounding (the staged forward GEMMs run other hipBLASLt
    # kernels) into ~1e-3 of the parameters; per-chunk bf16 accumulation of the weight gradients would show
    # as a loss / grad-norm gap first
    assert (num / den) ** 0.5 < 3e-3


def test_bench_two_ranks_through_the_launcher(tmp_path):
    """`bench.py --gpus 2` exactly as a user runs it (no torchrun): the in-process launcher starts two rank
    processes, they train the ZeRO-2 engine on the GPU (both on GPU 0 over gloo here) and rank 0 prints
    one JSON line with the whole-job tokens/s."""
    import json
    env = dict(os.environ, LLMT_DIST_BACKEND="gloo", LLMT_SHARED_DEVICE="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LLMT_LAUNCHED"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--layers", "2", "--seq", "1024", "--micro-batch", "1"],
                       env=env, capture_output=True, text=True, timeout=150, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["zero_stage"] == 2
    assert out["value"] > 0 and out["config"]["global_batch"] == 2
    assert out["config"]["force_sharded"] is False
    # the self-verification block: the process group that ran, the untimed collective probe, and the
    # compute stream's stalls on the comm / optimizer streams during the timed steps
    rc = out["rccl"]
    assert rc["backend"] == "gloo" and rc["world"] == 2 and rc["probe_group"] == 2
    assert rc["ag_busbw_gbs"] > 0 and rc["rs_busbw_gbs"] > 0
    assert rc["exposed_comm_ms_per_step"] >= 0 and rc["exposed_optimizer_wait_ms_per_step"] >= 0


def test_bench_hung_rank_ends_the_job_with_stacks(tmp_path):
    """A rank that stops inside step 2 (LLMT_BENCH_HANG) leaves the other blocked in a collective: the
    per-step watchdog dumps the ranks' stacks and the job exits non-zero within the limit instead of
    waiting for the driver's time-out."""
    import time
    env = dict(os.environ, LLMT_DIST_BACKEND="gloo", LLMT_SHARED_DEVICE="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="4",
               LLMT_BENCH_HANG="1:2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LLMT_LAUNCHED"):
        env.pop(k, None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--layers", "2", "--seq", "1024", "--micro-batch", "1", "--step-timeout", "15",
                        "--probe-mb", "8"],
                       env=env, capture_output=True, text=True, timeout=150, cwd=str(tmp_path))
    took = time.time() - t0
    assert r.returncode != 0, r.stdout[-2000:]
    assert "watchdog: timed step 1 exceeded 15 s" in r.stderr, r.stderr[-4000:]
    assert "File " in r.stderr and "bench.py" in r.stderr  # the Python stacks
    assert not any(x.startswith('{"metric"') for x in r.stdout.splitlines())
    assert took < 120


def test_dpo_zero3_sharded_reference_two_ranks_on_one_gpu(tmp_path):
    """DPO at dp2 x ZeRO-3 on the GPU: the frozen reference model is gather-only dp-sharded (half its
    bytes per rank, nothing held between steps) and training matches one process on the full batch."""
    from llm_training_amd.lms.preference import DPO
    from llm_training_amd.parallel.context import ParallelContext
    from llm_training_amd.parallel.engine import DataParallelEngine
    from tests.multirank_gpu_common import CFG, pref_batches
    dev = torch.device("cuda", 0)
    lm = DPO({"model": {"model_class": "llm_training.models.Llama", "model_config": CFG.model_dump()}, "beta": 0.1})
    lm.configure_model(ParallelContext.single(dev), dev, torch.bfloat16, seed=5)
    full_ref = sum(p.numel() * p.element_size() for p in lm.ref_model.parameters())
    eng = DataParallelEngine(lm.model, ParallelContext.single(dev), 0, lr=1e-3, weight_decay=0.0)
    lm.on_engine_ready(eng)
    lm.train()
    ref_losses = []
    for b in pref_batches(dev):
        eng.begin_step(1)
        eng.zero_grad()
        eng.begin_micro(0)
        loss, _, _ = lm.training_step(b)
        loss.backward()
        eng.finish_backward()
        eng.clip_and_scale(1.0)
        eng.step(1e-3)
        ref_losses.append(loss.item())
    eng.wait_params()
    ref_params = {k: v.detach().float().cpu() for k, v in lm.model.state_dict().items()}
    out = tmp_path / "dpo.pt"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29614",
           os.path.join(ROOT, "tests", "multirank_gpu_worker.py"), "dpo_z3", str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-4000:]
    got = torch.load(out, weights_only=True)
    assert got["ref_held"] == 0 and got["ref_shard_bytes"] <= full_ref / 2 * 1.05
    for a, b in zip(got["losses"], ref_losses):
        assert abs(a - b) < 2e-2 * max(1.0, abs(b)), (got["losses"], ref_losses)
    num = den = 0.0
    for k, v in ref_params.items():
        num += (got["params"][k] - v).norm().item() ** 2
        den += v.norm().item() ** 2
    assert (num / den) ** 0.5 < 5e-3
