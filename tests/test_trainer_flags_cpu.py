"""Lightning Trainer flags that the reference gets for free from Lightning
(src/llm_training/lightning/cli/trainer.py:1-11): fast_dev_run, overfit_batches, min_steps / min_epochs,
EarlyStopping, profiler, detect_anomaly, barebones, use_distributed_sampler. Each either does what
Lightning does or raises; nothing is silently ignored."""

import pytest
import torch

from llm_training_amd.data.dummy import DummyDataModule
from llm_training_amd.lms.clm import CLM
from llm_training_amd.runtime.callbacks import EarlyStopping, ModelCheckpoint
from llm_training_amd.runtime.loggers import JSONLLogger
from llm_training_amd.runtime.trainer import IGNORED_TRAINER_ARGS, Trainer


def _lm():
    return CLM({"model": {"model_class": "llm_training.models.Llama",
                          "model_config": {"vocab_size": 96, "hidden_size": 32, "intermediate_size": 64,
                                           "num_hidden_layers": 2, "num_attention_heads": 4,
                                           "num_key_value_heads": 2}},
                "optim": {"optimizer_class": "torch.optim.AdamW", "optimizer_kwargs": {"lr": 5e-3}}})


def _dm(n=64, val=0.0):
    cfg = {"batch_size": 2, "vocab_size": 96, "max_length": 16, "num_samples": n, "base_seed": 5}
    if val:
        cfg["validation_split"] = val
    return DummyDataModule(cfg)


class _Count:
    """Counts the batches the trainer hands to training / validation."""

    def __init__(self):
        self.train, self.val, self.train_ids = 0, 0, []

    def on_train_batch_start(self, trainer, lm, batch, idx):
        self.train += 1
        self.train_ids.append(batch["input_ids"][:, :4].clone())

    def on_validation_end(self, trainer, lm, metrics):
        self.val += 1


def test_fast_dev_run_one_batch_no_loggers_no_checkpoints(tmp_path):
    cnt = _Count()
    log = JSONLLogger(str(tmp_path / "log"), "r")
    t = Trainer(strategy="ddp", precision="32-true", logger=log, max_epochs=5, fast_dev_run=True, seed=1,
                callbacks=[cnt, ModelCheckpoint(dirpath=str(tmp_path / "ck"), every_n_train_steps=1)],
                default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm(val=0.25))
    assert t.global_step == 1 and cnt.train == 1 and cnt.val == 1
    assert not (tmp_path / "ck").exists() and not (tmp_path / "log").exists()


def test_fast_dev_run_n(tmp_path):
    cnt = _Count()
    t = Trainer(strategy="ddp", precision="32-true", fast_dev_run=3, accumulate_grad_batches=2, seed=1,
                callbacks=[cnt], default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm(val=0.25))
    assert t.global_step == 3 and cnt.train == 3 and cnt.val == 1  # 3 optimizer steps of 2 micro-batches


def test_overfit_batches_repeats_the_same_unshuffled_batches(tmp_path):
    cnt = _Count()
    t = Trainer(strategy="ddp", precision="32-true", overfit_batches=2, max_epochs=3, seed=1, callbacks=[cnt],
                default_root_dir=str(tmp_path), num_sanity_val_steps=0)
    t.fit(_lm(), _dm())
    assert t.global_step == 6 and cnt.train == 6
    ids = cnt.train_ids
    for e in (1, 2):  # every epoch sees the same two batches in the same order
        assert torch.equal(ids[2 * e], ids[0]) and torch.equal(ids[2 * e + 1], ids[1])
    assert not torch.equal(ids[0], ids[1])


def test_min_steps_defers_a_stop_request(tmp_path):
    class StopAt2:
        def on_train_batch_end(self, trainer, lm, outputs, batch, idx):
            if trainer.global_step >= 2:
                trainer.should_stop = True
    t = Trainer(strategy="ddp", precision="32-true", max_steps=50, min_steps=5, seed=1, callbacks=[StopAt2()],
                default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    assert t.global_step == 5
    t2 = Trainer(strategy="ddp", precision="32-true", max_steps=50, seed=1, callbacks=[StopAt2()],
                 default_root_dir=str(tmp_path))
    t2.fit(_lm(), _dm())
    assert t2.global_step == 2


def test_min_epochs_extends_training(tmp_path):
    cnt = _Count()
    t = Trainer(strategy="ddp", precision="32-true", min_epochs=2, limit_train_batches=3, seed=1, callbacks=[cnt],
                default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    assert t.state.epoch == 2 and cnt.train == 6


def test_max_steps_is_not_deferred_by_min_steps(tmp_path):
    t = Trainer(strategy="ddp", precision="32-true", max_steps=3, min_steps=10, seed=1, default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    assert t.global_step == 3


def test_early_stopping_patience_and_state(tmp_path):
    es = EarlyStopping(monitor="Loss/Val", patience=2, min_delta=100.0)  # no check can improve by 100
    t = Trainer(strategy="ddp", precision="32-true", max_steps=40, val_check_interval=2, seed=1,
                callbacks=[es], default_root_dir=str(tmp_path), num_sanity_val_steps=0)
    t.fit(_lm(), _dm(val=0.25))
    # first check sets the best; two more without improvement -> stop after the third validation
    assert t.global_step == 6 and es.wait_count == 2 and "did not improve" in es.stopping_reason
    st = es.state_dict()
    es2 = EarlyStopping(monitor="Loss/Val")
    es2.load_state_dict(st)
    assert es2.wait_count == 2 and es2.best_score == es.best_score


def test_early_stopping_thresholds_and_strict(tmp_path):
    es = EarlyStopping(monitor="Loss/Val", stopping_threshold=100.0)
    t = Trainer(strategy="ddp", precision="32-true", max_steps=40, val_check_interval=2, seed=1,
                callbacks=[es], default_root_dir=str(tmp_path), num_sanity_val_steps=0)
    t.fit(_lm(), _dm(val=0.25))
    assert t.global_step == 2 and "stopping threshold" in es.stopping_reason
    es = EarlyStopping(monitor="Loss/Val", divergence_threshold=0.5)
    t = Trainer(strategy="ddp", precision="32-true", max_steps=40, val_check_interval=2, seed=1,
                callbacks=[es], default_root_dir=str(tmp_path), num_sanity_val_steps=0)
    t.fit(_lm(), _dm(val=0.25))
    assert t.global_step == 2 and "divergence" in es.stopping_reason
    es = EarlyStopping(monitor="no/such/metric")
    t = Trainer(strategy="ddp", precision="32-true", max_steps=4, val_check_interval=2, seed=1,
                callbacks=[es], default_root_dir=str(tmp_path), num_sanity_val_steps=0)
    with pytest.raises(RuntimeError, match="no/such/metric"):
        t.fit(_lm(), _dm(val=0.25))


def test_early_stopping_resolves_lightning_class_path():
    from llm_training_amd.utils.imports import import_object
    assert import_object("lightning.pytorch.callbacks.EarlyStopping") is EarlyStopping
    assert import_object("EarlyStopping") is EarlyStopping


def test_early_stopping_from_yaml_config(tmp_path):
    from llm_training_amd.config.loader import instantiate
    cb = instantiate({"class_path": "lightning.pytorch.callbacks.EarlyStopping",
                      "init_args": {"monitor": "Loss/Val", "patience": 4, "mode": "min", "min_delta": 0.01}})
    assert isinstance(cb, EarlyStopping) and cb.patience == 4 and cb.min_delta == -0.01


@pytest.mark.parametrize("kind", ["simple", "advanced", "pytorch"])
def test_profilers_write_their_reports(tmp_path, kind):
    t = Trainer(strategy="ddp", precision="32-true", max_steps=4, seed=1, profiler=kind,
                default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    rep = (tmp_path / "fit-profile-rank0.txt").read_text()
    if kind == "simple":
        for action in ("training_step", "backward", "optimizer_step", "get_train_batch"):
            assert action in rep
        row = next(line for line in rep.splitlines() if line.startswith("training_step"))
        assert int(row.split()[2]) == 4
    elif kind == "advanced":
        assert "cumulative" in rep and "train_step" in rep
    else:
        assert (tmp_path / "fit-profile-rank0.json").exists() and "Self CPU" in rep


def test_profiler_class_path_dict(tmp_path):
    t = Trainer(strategy="ddp", precision="32-true", max_steps=2, seed=1, default_root_dir=str(tmp_path),
                profiler={"class_path": "lightning.pytorch.profilers.SimpleProfiler",
                          "init_args": {"filename": "perf"}})
    t.fit(_lm(), _dm())
    assert (tmp_path / "perf-rank0.txt").exists()
    with pytest.raises(ValueError):
        Trainer(profiler="xla")


def test_detect_anomaly_raises_on_nan_backward(tmp_path):
    class NanGrad(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.clone()

        @staticmethod
        def backward(ctx, g):
            return g * float("nan")

    lm = _lm()
    orig = CLM.training_step

    def poisoned(self, batch, idx=0):
        loss, m, c = orig(self, batch, idx)
        return NanGrad.apply(loss), m, c
    lm.training_step = poisoned.__get__(lm)
    t = Trainer(strategy="ddp", precision="32-true", max_steps=2, seed=1, detect_anomaly=True,
                default_root_dir=str(tmp_path))
    with pytest.raises(RuntimeError, match="nan"):
        t.fit(lm, _dm())
    t = Trainer(strategy="ddp", precision="32-true", max_steps=2, seed=1, default_root_dir=str(tmp_path))
    lm2 = _lm()
    lm2.training_step = poisoned.__get__(lm2)
    t.fit(lm2, _dm())  # without the flag the NaN step goes through


def test_barebones_and_plugins(tmp_path):
    log = JSONLLogger(str(tmp_path / "log"), "r")
    t = Trainer(strategy="ddp", precision="32-true", max_steps=2, seed=1, barebones=True, logger=log,
                callbacks=[ModelCheckpoint(dirpath=str(tmp_path / "ck"), every_n_train_steps=1)],
                default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    assert t.global_step == 2 and not (tmp_path / "ck").exists() and not (tmp_path / "log").exists()
    with pytest.raises(ValueError, match="plugins"):
        Trainer(plugins=["something"])
    with pytest.raises(ValueError, match="barebones"):
        Trainer(barebones=True, profiler="simple")


def test_every_ignored_argument_is_accepted_and_unknown_raises():
    t = Trainer(**{k: True for k in IGNORED_TRAINER_ARGS})
    assert set(t.unused) == IGNORED_TRAINER_ARGS - {"benchmark", "enable_model_summary"}
    with pytest.raises(TypeError, match="fast_dev_runs"):
        Trainer(fast_dev_runs=1)
    assert {"fast_dev_run", "overfit_batches", "profiler", "detect_anomaly", "min_steps",
            "min_epochs"}.isdisjoint(IGNORED_TRAINER_ARGS)


def test_use_distributed_sampler_false_gives_every_rank_the_whole_set(tmp_path):
    t = Trainer(strategy="ddp", precision="32-true", max_steps=1, seed=1, use_distributed_sampler=False,
                default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    assert t._dp() == (0, 1)


@pytest.mark.parametrize("precision,path", [("32-true", "torch-reference"), ("16-mixed", "torch-reference"),
                                            ("bf16-true", "hip"), ("bf16-mixed", "hip")])
def test_gpu_precision_kernel_path_is_announced(precision, path):
    """The HIP kernels are bf16-only: a GPU run at 32-true / 16-* takes the torch reference ops. The trainer
    says so (a warning) and records it in its run metadata instead of switching paths silently; bf16
    precisions record the kernel path without a warning (device mocked: no GPU needed)."""
    import logging

    class _Keep(logging.Handler):
        def __init__(self):
            super().__init__(logging.WARNING)
            self.msgs = []

        def emit(self, record):
            self.msgs.append(record.getMessage())
    h = _Keep()
    lg = logging.getLogger("llm_training")  # the package logger (it does not propagate to the root)
    lg.addHandler(h)
    try:
        t = Trainer(precision=precision)
        meta = t.compute_path_meta(torch.device("cuda", 0))
        assert meta["compute_kernels"] == path and meta["device"] == "cuda"
        assert any("torch reference ops" in m for m in h.msgs) == (path != "hip")
        h.msgs.clear()
        assert t.compute_path_meta(torch.device("cpu"))["compute_kernels"] == "torch-reference"
        assert not h.msgs  # the CPU reference path is the expected one there
    finally:
        lg.removeHandler(h)


def test_run_meta_reaches_the_logger(tmp_path):
    import json
    t = Trainer(strategy="ddp", precision="32-true", max_steps=1, seed=1, logger=JSONLLogger(str(tmp_path), "r"),
                enable_checkpointing=False)
    t.fit(_lm(), _dm())
    hp = json.load(open(tmp_path / "r" / "hparams.json"))
    meta = hp["run_meta"]
    assert {k: meta[k] for k in ("device", "precision", "compute_kernels")} == {
        "device": "cpu", "precision": "32-true", "compute_kernels": "torch-reference"}
    assert meta["native_lib"] == "production"
    assert isinstance(meta["llmt_env"], dict) and all(k.startswith("LLMT_") for k in meta["llmt_env"])


def test_run_meta_records_llmt_knobs(tmp_path, monkeypatch):
    """Every LLMT_* knob of the environment is recorded with the run (bench JSON and Trainer run_meta)."""
    import json
    monkeypatch.setenv("LLMT_FA_BMAJOR", "0")
    monkeypatch.setenv("LLMT_TP_STAGES", "2")
    t = Trainer(strategy="ddp", precision="32-true", max_steps=1, seed=1, logger=JSONLLogger(str(tmp_path), "r"),
                enable_checkpointing=False)
    t.fit(_lm(), _dm())
    env = json.load(open(tmp_path / "r" / "hparams.json"))["run_meta"]["llmt_env"]
    assert env["LLMT_FA_BMAJOR"] == "0" and env["LLMT_TP_STAGES"] == "2"


@pytest.mark.parametrize("var", ["LLMT_FA_PROBE", "LLMT_FA_D6_PROBE"])
def test_trainer_refuses_wrong_result_probes(tmp_path, monkeypatch, var):
    """A diagnostic probe variable (kernels that compute wrong results on purpose) makes a training run
    refuse to start with the production library; the native loader refuses it too."""
    from llm_training_amd.ops import native
    monkeypatch.setenv(var, "1")
    t = Trainer(strategy="ddp", precision="32-true", max_steps=1, seed=1, enable_checkpointing=False,
                default_root_dir=str(tmp_path))
    with pytest.raises(RuntimeError, match="diagnostic probes"):
        t.fit(_lm(), _dm())
    with pytest.raises(RuntimeError, match="diagnostic probes"):
        native.check_probe_env()
    monkeypatch.setenv(var, "0")
    native.check_probe_env()  # "0" = off


def test_use_native_counts_reference_ops_on_gpu(monkeypatch):
    """use_native on a non-bf16 GPU tensor warns once per dtype and counts the calls (mocked device)."""
    from llm_training_amd.ops import native
    monkeypatch.setattr(native, "lib", lambda: None)
    monkeypatch.setattr(native, "REFERENCE_ON_GPU", {})

    class _T:
        def __init__(self, dtype):
            self.device, self.dtype = torch.device("cuda", 0), dtype
    assert native.use_native(_T(torch.bfloat16))
    assert not native.use_native(_T(torch.float32)) and not native.use_native(_T(torch.float32))
    assert native.REFERENCE_ON_GPU == {"float32": 2}
