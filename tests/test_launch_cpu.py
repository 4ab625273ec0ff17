"""The in-process multi-rank launcher (llm_training_amd/launch.py): ``llm-training fit`` with
``trainer.devices: N`` and ``bench.py --gpus N`` start N rank processes themselves (reference:
Lightning's _SubprocessScriptLauncher, fsdp2_strategy.py:169-173). CPU ranks over gloo here."""
from __future__ import annotations

import csv
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TINY = """
seed_everything: 1
trainer:
  strategy: ddp
  precision: 32-true
  logger:
    class_path: llm_training.lightning.CSVLogger
    init_args: {{save_dir: {out}, name: t}}
  max_steps: 4
  log_every_n_steps: 1
  gradient_clip_val: 1.0
model:
  class_path: llm_training.lms.CLM
  init_args.config:
    model:
      model_class: llm_training.models.Llama
      model_config: {{vocab_size: 64, hidden_size: 32, intermediate_size: 64, num_hidden_layers: 2,
                      num_attention_heads: 2, num_key_value_heads: 1}}
    optim:
      optimizer_class: torch.optim.AdamW
      optimizer_kwargs: {{lr: 1e-2}}
data:
  class_path: llm_training.data.DummyDataModule
  init_args.config: {{batch_size: {bs}, vocab_size: 64, max_length: 16, num_samples: 32, base_seed: 3}}
"""


def _losses(path):
    rows = list(csv.DictReader(open(path)))
    return [float(r["Loss/Train/Step"]) for r in rows if r.get("Loss/Train/Step")], \
        [float(r["Gradient Norm"]) for r in rows if r.get("Gradient Norm")]


def _env():
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LLMT_LAUNCHED", "MASTER_PORT"):
        e.pop(k, None)
    e["OMP_NUM_THREADS"] = "2"
    return e


def test_fit_devices_2_spawns_two_gloo_ranks_matching_one_process(tmp_path):
    """dp2 x micro-batch 1 through the launcher == one process x micro-batch 2 (same global batch)."""
    one = tmp_path / "one.yaml"
    one.write_text(TINY.format(out=tmp_path / "one", bs=2))
    two = tmp_path / "two.yaml"
    two.write_text(TINY.format(out=tmp_path / "two", bs=1))
    from llm_training_amd.cli.main import main
    assert main(["fit", "--config", str(one), "--trainer.accelerator", "cpu"]) == 0
    r = subprocess.run([sys.executable, "-m", "llm_training_amd.cli.main", "fit", "--config", str(two),
                        "--trainer.devices", "2", "--trainer.accelerator", "cpu"],
                       env=_env(), cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "dp 2" in r.stderr, r.stderr[-3000:]  # the engine ran with two data-parallel ranks
    l1, g1 = _losses(tmp_path / "one" / "t" / "metrics.csv")
    l2, g2 = _losses(tmp_path / "two" / "t" / "metrics.csv")
    assert len(l1) == len(l2) == 4
    assert l2 == pytest.approx(l1, rel=1e-4, abs=1e-5)
    assert g2 == pytest.approx(g1, rel=1e-4, abs=1e-5)


def test_max_time_stops_every_rank_at_the_same_step(tmp_path):
    """max_time on two gloo ranks: rank 0's clock decides (broadcast), so both ranks stop after the
    same optimizer step and the job exits cleanly instead of one rank waiting in a collective."""
    cfg = tmp_path / "mt.yaml"
    cfg.write_text(TINY.format(out=tmp_path / "mt", bs=1).replace("max_steps: 4", "max_steps: 50\n  max_time: {seconds: 0}"))
    r = subprocess.run([sys.executable, "-m", "llm_training_amd.cli.main", "fit", "--config", str(cfg),
                        "--trainer.devices", "2", "--trainer.accelerator", "cpu"],
                       env=_env(), cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    losses, _ = _losses(tmp_path / "mt" / "t" / "metrics.csv")
    assert len(losses) == 1


def test_failing_rank_ends_the_job_without_orphans(tmp_path):
    """Rank 1 fails at once while rank 0 would block for minutes: the parent returns rank 1's code
    within the grace period and rank 0 is gone."""
    from llm_training_amd.launch import spawn
    prog = tmp_path / "p.py"
    prog.write_text(
        "import os, sys, time\n"
        f"open(os.path.join({str(tmp_path)!r}, 'pid' + os.environ['RANK']), 'w').write(str(os.getpid()))\n"
        "if os.environ['RANK'] == '1':\n"
        "    time.sleep(0.5); sys.exit(7)\n"
        "time.sleep(300)\n")
    t0 = time.time()
    rc = spawn(2, [sys.executable, str(prog)], grace=5.0)
    assert rc == 7
    assert time.time() - t0 < 60
    pid0 = int((tmp_path / "pid0").read_text())
    with pytest.raises(ProcessLookupError):
        os.kill(pid0, 0)


def test_rank_killed_by_signal_is_reported(tmp_path):
    from llm_training_amd.launch import spawn
    prog = tmp_path / "p.py"
    prog.write_text("import os, signal, time\n"
                    "if os.environ['RANK'] == '0':\n"
                    "    os.kill(os.getpid(), signal.SIGKILL)\n"
                    "time.sleep(300)\n")
    assert spawn(2, [sys.executable, str(prog)], grace=5.0) == 128 + 9


def test_children_get_rank_env_and_rccl_defaults(tmp_path):
    from llm_training_amd.launch import spawn
    prog = tmp_path / "p.py"
    prog.write_text("import os, json\n"
                    f"json.dump(dict(os.environ), open(os.path.join({str(tmp_path)!r}, 'env' + os.environ['RANK']), 'w'))\n")
    env = _env()
    env.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    assert spawn(3, [sys.executable, str(prog)], env=env) == 0
    import json
    envs = [json.load(open(tmp_path / f"env{r}")) for r in range(3)]
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) == (str(r), str(r), "3")
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_world_size_mismatch_is_an_error(monkeypatch):
    from llm_training_amd.launch import launch_for_trainer, maybe_launch
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit):
        maybe_launch(8, ["true"])
    assert maybe_launch(2, ["true"]) is None
    with pytest.raises(SystemExit):
        launch_for_trainer({"devices": 4}, ["true"])
    assert launch_for_trainer({"devices": "auto"}, ["true"]) is None


def test_bench_gpus_mismatch_under_torchrun_env_fails():
    """bench.py --gpus 2 inside a one-rank torchrun-style environment refuses to run one rank."""
    env = _env()
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29555")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE" in (r.stderr + r.stdout)


def test_device_list_pins_ranks_to_the_listed_gpus(tmp_path, monkeypatch):
    """trainer.devices [2, 3] (Lightning: those GPU indices) runs the ranks on GPUs 2 and 3: every child
    sees exactly the listed GPUs (HIP_VISIBLE_DEVICES), so LOCAL_RANK r is GPU devices[r]; an existing
    visibility mask is composed with the list."""
    import json

    from llm_training_amd.launch import launch_for_trainer, visible_devices_env
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LLMT_LAUNCHED", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    prog = tmp_path / "p.py"
    prog.write_text("import os, json\n"
                    f"json.dump(dict(os.environ), open(os.path.join({str(tmp_path)!r}, 'env' + os.environ['RANK']), 'w'))\n")
    assert launch_for_trainer({"devices": [2, 3]}, [sys.executable, str(prog)]) == 0
    envs = [json.load(open(tmp_path / f"env{r}")) for r in range(2)]
    assert [e["HIP_VISIBLE_DEVICES"] for e in envs] == ["2,3", "2,3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1"]
    assert [e["CUDA_VISIBLE_DEVICES"] for e in envs] == ["2,3", "2,3"]
    assert visible_devices_env([1, 3], {"HIP_VISIBLE_DEVICES": "4,5,6,7"}) == {"HIP_VISIBLE_DEVICES": "5,7",
                                                                             "CUDA_VISIBLE_DEVICES": "5,7"}
    # a parent selecting through CUDA_VISIBLE_DEVICES only: composed, and the child's alias agrees
    assert visible_devices_env([0, 2], {"CUDA_VISIBLE_DEVICES": "3,4,6"}) == {"HIP_VISIBLE_DEVICES": "3,6",
                                                                            "CUDA_VISIBLE_DEVICES": "3,6"}
    with pytest.raises(SystemExit):
        visible_devices_env([0, 0], {})
    with pytest.raises(SystemExit):
        visible_devices_env([5], {"HIP_VISIBLE_DEVICES": "0,1"})
