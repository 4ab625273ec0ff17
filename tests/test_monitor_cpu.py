"""Observability / failure-handling helpers (runtime/monitor.py) and the collective-consistency checker
(parallel/debug.py). CPU only; the checker runs on 2 gloo ranks."""
import json
import os
import time

import pytest
import torch

from tests.helpers import run_gloo


def test_model_flops_per_token_llama3_8b():
    from types import SimpleNamespace

    from llm_training_amd.runtime.monitor import model_flops_per_token
    cfg = SimpleNamespace(hidden_size=4096, num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                          intermediate_size=14336, vocab_size=128256)
    f = model_flops_per_token(cfg, 8192)
    # 45.03 GF matmul + 6.44 GF attention = 51.5 GF/token
    assert abs(f / 1e9 - 51.5) < 0.2
    assert model_flops_per_token(None, 8192) == 0.0


def test_throughput_meter_rates():
    from llm_training_amd.runtime.monitor import ThroughputMeter
    m = ThroughputMeter(world_size=4, flops_per_token=1e9)
    assert m.metrics() == {}
    m.update(1000)
    time.sleep(0.05)
    m.update(1000)
    d = m.metrics()
    assert d["Throughput/tokens_per_sec"] == pytest.approx(4 * d["Throughput/tokens_per_sec_per_gpu"])
    assert 0 < d["Throughput/tokens_per_sec_per_gpu"] < 2000 / 0.05
    assert d["Throughput/tflops_per_gpu"] == pytest.approx(d["Throughput/tokens_per_sec_per_gpu"] * 1e9 / 1e12)
    assert m.steps == 0  # reset after reporting


def test_step_profiler_writes_trace(tmp_path):
    from llm_training_amd.runtime.monitor import StepProfiler
    p = StepProfiler("2-3", out_dir=str(tmp_path), rank=0)
    assert p.enabled
    for step in range(1, 5):
        p.before_step(step)
        torch.randn(64, 64) @ torch.randn(64, 64)
        p.after_step(step)
    assert p.trace_path is not None and os.path.isfile(p.trace_path)
    assert not p.enabled  # one window only
    with pytest.raises(ValueError):
        StepProfiler("abc")


def test_stall_watchdog_dumps_stack(tmp_path):
    from llm_training_amd.runtime.monitor import StallWatchdog
    path = tmp_path / "stall.txt"
    w = StallWatchdog(timeout=0.2, path=str(path))
    w.arm()
    time.sleep(0.6)
    w.close()
    text = path.read_text()
    assert "test_stall_watchdog_dumps_stack" in text
    assert not StallWatchdog(timeout=0).enabled


def _fake_ckpt(root, name, step, tp=1, complete=True, dp=2):
    d = root / name
    d.mkdir(parents=True)
    (d / "meta.json").write_text(json.dumps({"tp_size": tp, "dp_size": dp, "trainer": {"global_step": step}}))
    ranks = [(t, r) for t in range(tp) for r in range(dp)]
    for t, r in ranks[:len(ranks) if complete else -1]:  # an incomplete save lacks one rank's marker
        (d / f"shard-tp{t}-dp{r}.done").write_bytes(b"")
    return d


def test_find_last_checkpoint_skips_incomplete(tmp_path):
    from llm_training_amd.runtime.monitor import find_last_checkpoint
    assert find_last_checkpoint(tmp_path / "missing") is None
    _fake_ckpt(tmp_path, "epoch=0-step=10", 10)
    best = _fake_ckpt(tmp_path, "epoch=0-step=20", 20, tp=2)
    _fake_ckpt(tmp_path, "epoch=0-step=30", 30, tp=2, complete=False)  # crashed mid-save
    assert find_last_checkpoint(tmp_path) == str(best)


def test_record_failure(tmp_path):
    from llm_training_amd.runtime.monitor import record_failure
    try:
        raise ValueError("boom")
    except ValueError as e:
        path = record_failure(e, 3, str(tmp_path))
    assert path.endswith("failure_rank3.txt")
    text = open(path).read()
    assert "rank: 3" in text and "ValueError: boom" in text


def test_trainer_resumes_from_last(tmp_path):
    """fit(ckpt_path="last") picks the newest complete checkpoint the ModelCheckpoint callback wrote."""
    from llm_training_amd.runtime.callbacks import ModelCheckpoint
    from llm_training_amd.runtime.trainer import Trainer
    ckdir = tmp_path / "ck"
    _fake_ckpt(ckdir, "epoch=0-step=5", 5)
    best = _fake_ckpt(ckdir, "epoch=0-step=7", 7)
    t = Trainer(default_root_dir=str(tmp_path), callbacks=[ModelCheckpoint(dirpath=str(ckdir))])
    assert t.resolve_last_checkpoint() == str(best)
    t2 = Trainer(default_root_dir=str(tmp_path / "empty"))
    assert t2.resolve_last_checkpoint() is None


def _collective_worker(rank, world, diverge):
    import torch.distributed as dist

    from llm_training_amd.parallel.debug import CollectiveRecorder
    rec = CollectiveRecorder().install()
    try:
        t = torch.ones(4)
        dist.all_reduce(t)
        rec.verify()  # identical so far
        # rank 1 reduces with a different op: gloo completes it, but the sequences no longer agree
        op = dist.ReduceOp.MAX if (diverge and rank == 1) else dist.ReduceOp.SUM
        dist.all_reduce(torch.ones(8), op=op)
        try:
            rec.verify()
            return "ok"
        except RuntimeError as e:
            return str(e)
    finally:
        rec.uninstall()


def test_collective_checker_agrees_when_consistent():
    out = run_gloo(_collective_worker, world=2, args=(False,))
    assert out == {0: "ok", 1: "ok"}


def test_collective_checker_reports_divergence():
    out = run_gloo(_collective_worker, world=2, args=(True,))
    for r in (0, 1):
        assert "differs across ranks at call #0" in out[r]
        assert "MAX" in out[r] and "SUM" in out[r]


@pytest.mark.parametrize("gdtype", [torch.bfloat16, torch.float32])
def test_native_cpu_adamw_matches_reference(gdtype):
    """csrc/cpu_adam.cpp (optimizer offload) vs the torch AdamW reference used by the engine."""
    from llm_training_amd.ops.native import lib
    from llm_training_amd.parallel.engine import _adamw_ref
    torch.manual_seed(0)
    n = 100_003  # not a multiple of the thread-pool grain
    p = torch.randn(n)
    m = torch.randn(n) * 0.01
    v = torch.rand(n) * 1e-4
    g = torch.randn(n).to(gdtype)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    pout = torch.empty(n, dtype=torch.bfloat16)
    for step in (1, 2, 7):
        lib().adamw_cpu_(p, m, v, g, pout, 1e-3, 0.9, 0.95, 1e-8, 0.1, step, 0.5)
        _adamw_ref(pr, mr, vr, g.float() * 0.5, 1e-3, 0.9, 0.95, 1e-8, 0.1, step)
    assert torch.allclose(m, mr, rtol=1e-5, atol=1e-7)
    assert torch.allclose(v, vr, rtol=1e-5, atol=1e-9)
    assert torch.allclose(p, pr, rtol=1e-5, atol=1e-6)
    assert torch.equal(pout, p.bfloat16())  # round-to-nearest-even, as torch's cast


def test_strategies_map_offload_knobs():
    from llm_training_amd.runtime.strategies import DeepSpeedStrategy, FSDP2Strategy
    assert DeepSpeedStrategy(stage=2, offload_optimizer=True).offload_optimizer
    assert not DeepSpeedStrategy(stage=2).offload_optimizer
    assert FSDP2Strategy(offload_policy={"class_path": "torch.distributed.fsdp.CPUOffloadPolicy"}).offload_optimizer
    assert not FSDP2Strategy(offload_policy={"class_path": "torch.distributed.fsdp.OffloadPolicy"}).offload_optimizer
    assert not FSDP2Strategy().offload_optimizer


def test_csv_logger_one_header_across_resume_and_late_keys(tmp_path):
    """A resumed run appends under the existing header; a metric first logged later (validation loss)
    widens the header once and keeps every earlier row."""
    import csv

    from llm_training_amd.runtime.loggers import CSVLogger
    a = CSVLogger(save_dir=str(tmp_path), name="r")
    a.log_metrics({"loss": 1.0}, 1)
    a.log_metrics({"loss": 0.9}, 2)
    a.finalize("success")
    b = CSVLogger(save_dir=str(tmp_path), name="r")  # the resumed run, same directory
    b.log_metrics({"loss": 0.8}, 3)
    b.log_metrics({"loss": 0.7, "val": 0.75}, 4)
    b.log_metrics({"loss": 0.6}, 5)
    b.finalize("success")
    text = open(tmp_path / "r" / "metrics.csv").read()
    assert text.count("step") == 1
    rows = list(csv.DictReader(open(tmp_path / "r" / "metrics.csv")))
    assert [int(r["step"]) for r in rows] == [1, 2, 3, 4, 5]
    assert rows[3]["val"] == "0.75" and rows[0]["val"] == "" and rows[4]["loss"] == "0.6"


def test_validation_schedule_follows_lightning():
    """val_check_interval: an int counts training batches (accumulation does not stretch it), a float is a
    fraction of the epoch (None = 1.0 = every epoch end) gated by check_val_every_n_epoch."""
    from types import SimpleNamespace

    from llm_training_amd.runtime.trainer import Trainer

    def when(nbe=12, accum=1, epochs=2, **kw):
        t = Trainer(strategy="ddp", precision="32-true", accumulate_grad_batches=accum, **kw)
        t.datamodule = SimpleNamespace(datasets={"validation": [1]})
        t.state.epoch, out = 0, []
        for ep in range(epochs):
            t.state.epoch, t.state.batch_idx = ep, 0
            while t.state.batch_idx + accum <= nbe:
                t.state.batch_idx += accum
                if t._should_validate(nbe):
                    out.append((ep, t.state.batch_idx))
        return out

    assert when(val_check_interval=4, accum=2) == [(0, 4), (0, 8), (0, 12), (1, 4), (1, 8), (1, 12)]
    assert when() == [(0, 12), (1, 12)]                                  # default: every epoch end
    assert when(nbe=13, accum=2) == [(0, 12), (1, 12)]                   # the dropped remainder batch
    assert when(val_check_interval=0.5, accum=2) == [(0, 6), (0, 12), (1, 6), (1, 12)]
    assert when(check_val_every_n_epoch=2) == [(1, 12)]


def test_sanity_check_and_fractional_val_limit(monkeypatch):
    """num_sanity_val_steps (Lightning default 2) runs that many validation batches before training
    without logging them; limit_val_batches as a float is a fraction of the loader, 0 disables both."""
    from types import SimpleNamespace

    from llm_training_amd.runtime.trainer import Trainer

    t = Trainer(strategy="ddp", precision="32-true")
    dl = list(range(10))
    assert t._val_batch_limit(dl, sanity=True) == 2 and t._val_batch_limit(dl, sanity=False) is None
    t.limit_val_batches = 0.5
    assert t._val_batch_limit(dl, sanity=False) == 5
    t.limit_val_batches = 1.0
    assert t._val_batch_limit(dl, sanity=False) is None
    t.limit_val_batches = 3
    assert t._val_batch_limit(dl, sanity=False) == 3
    t.num_sanity_val_steps = -1
    assert t._val_batch_limit(dl, sanity=True) is None

    calls = []

    class LM:
        def eval(self):
            pass

        def train(self, mode=True):
            pass

        def validation_step(self, b, i):
            calls.append(i)
            return {"Loss/Val": __import__("torch").tensor(1.0)}

    t2 = Trainer(strategy="ddp", precision="32-true")
    t2.lm = LM()
    t2.pc = SimpleNamespace(dp_rank=0, dp_size=1, world_size=1, rank=0)
    t2.device = __import__("torch").device("cpu")
    t2.datamodule = SimpleNamespace(datasets={"validation": [0]}, val_dataloader=lambda r, s: [{"x": 1}] * 7)
    out = t2.validate(sanity=True)
    assert calls == [0, 1] and out == {"Loss/Val": 1.0} and "Loss/Val" not in t2.last_metrics
    t2.validate()
    assert len(calls) == 9 and t2.last_metrics["Loss/Val"] == 1.0


def test_step_watchdog_dumps_stacks_and_exits(tmp_path):
    """StepWatchdog (bench.py's hang guard): a phase that overruns its limit writes the rank, the phase and
    every thread's stack to stderr and ends the process with exit code 3; re-arming / disarming in time
    keeps it alive."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prog = ("import time\n"
            "from llm_training_amd.runtime.monitor import StepWatchdog\n"
            "wd = StepWatchdog(rank=5, timeout=1.0)\n"
            "for i in range(3):\n"
            "    wd.arm(f'step {i}')\n"
            "    time.sleep(0.3)\n"
            "wd.disarm()\n"
            "time.sleep(1.5)\n"
            "print('alive', flush=True)\n"
            "def stuck_in_a_collective():\n"
            "    time.sleep(60)\n"
            "wd.arm('step 3')\n"
            "stuck_in_a_collective()\n")
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", prog], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, PYTHONPATH=root))
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == "alive"
    assert "[rank 5] watchdog: step 3 exceeded 1 s" in r.stderr
    assert "stuck_in_a_collective" in r.stderr  # the main thread's stack
    assert time.time() - t0 < 30
