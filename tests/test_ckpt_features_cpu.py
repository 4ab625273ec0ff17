"""Checkpoint features: safe rotation with async writes, best-k by a monitored metric, background write
errors surfacing, consolidated single-file checkpoints (save_distributed_checkpoint: false), reading
v1 checkpoints, and exact resume of random streams (NEFTune noise + dropout)."""
import json
import os

import pytest
import torch
from safetensors.torch import save_file

from llm_training_amd.ckpt import checkpoint as ckpt
from llm_training_amd.data.dummy import DummyDataModule
from llm_training_amd.lms.clm import CLM
from llm_training_amd.runtime.callbacks import ModelCheckpoint
from llm_training_amd.runtime.loggers import JSONLLogger
from llm_training_amd.runtime.strategies import FSDP2Strategy
from llm_training_amd.runtime.trainer import Trainer

MC = {"vocab_size": 96, "hidden_size": 32, "intermediate_size": 64, "num_hidden_layers": 2,
      "num_attention_heads": 4, "num_key_value_heads": 2}


def _lm(model_class="llm_training.models.Llama", mc=None, **kw):
    return CLM({"model": {"model_class": model_class, "model_config": dict(mc or MC)},
                "optim": {"optimizer_class": "torch.optim.AdamW", "optimizer_kwargs": {"lr": 5e-3}}, **kw})


def _dm(n=64):
    return DummyDataModule({"batch_size": 2, "vocab_size": 96, "max_length": 16, "num_samples": n, "base_seed": 5})


def _losses(d):
    rows = [json.loads(line) for line in open(os.path.join(d, "metrics.jsonl"))]
    return {r["step"]: r["Loss/Train/Step"] for r in rows if "Loss/Train/Step" in r}


def test_async_save_top_k_1_keeps_only_complete_checkpoints(tmp_path):
    ck = tmp_path / "ck"
    cb = ModelCheckpoint(dirpath=str(ck), every_n_train_steps=2, save_top_k=1, save_last=True, async_save=True)
    t = Trainer(strategy="ddp", precision="32-true", max_steps=6, seed=1, callbacks=[cb],
                default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    names = sorted(p.name for p in ck.iterdir())
    assert names == ["epoch=0-step=6.ckpt", "last.ckpt"]
    assert ckpt.is_complete(ck / "epoch=0-step=6.ckpt")
    assert os.readlink(ck / "last.ckpt") == "epoch=0-step=6.ckpt"


def test_failed_background_write_raises_and_keeps_previous(tmp_path, monkeypatch):
    ck = tmp_path / "ck"
    calls = {"n": 0}
    real = ckpt._write_files

    def flaky(path, base, tensors, index):
        calls["n"] += 1
        if calls["n"] == 2:
            raise OSError("disk full (simulated)")
        real(path, base, tensors, index)

    monkeypatch.setattr(ckpt, "_write_files", flaky)
    cb = ModelCheckpoint(dirpath=str(ck), every_n_train_steps=2, save_top_k=1, async_save=True)
    t = Trainer(strategy="ddp", precision="32-true", max_steps=6, seed=1, callbacks=[cb],
                default_root_dir=str(tmp_path))
    with pytest.raises(RuntimeError, match="disk full"):
        t.fit(_lm(), _dm())
    # the step-2 checkpoint survived: the failed step-4 one never replaced it
    assert ckpt.is_complete(ck / "epoch=0-step=2.ckpt")
    assert not ckpt.is_complete(ck / "epoch=0-step=4.ckpt")


@pytest.mark.parametrize("mode", ["min", "max"])
def test_monitor_keeps_best_k(tmp_path, mode):
    ck = tmp_path / "ck"
    cb = ModelCheckpoint(dirpath=str(ck), every_n_train_steps=1, save_top_k=2, monitor="Loss/Train/Step", mode=mode)
    log = tmp_path / "log"
    t = Trainer(strategy="ddp", precision="32-true", max_steps=6, seed=1, callbacks=[cb],
                logger=JSONLLogger(str(log), "r"), log_every_n_steps=1, default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    losses = _losses(log / "r")
    best = sorted(losses, key=lambda s: losses[s], reverse=(mode == "max"))[:2]
    kept = sorted(int(p.name.split("step=")[1].split(".")[0]) for p in ck.iterdir())
    assert kept == sorted(best)


def test_consolidated_single_file_checkpoint_resumes_and_exports(tmp_path):
    st = FSDP2Strategy(save_distributed_checkpoint=False)
    ck = tmp_path / "ck"
    log1 = tmp_path / "a"
    t1 = Trainer(strategy=st, precision="32-true", max_steps=6, seed=3, log_every_n_steps=1,
                 logger=JSONLLogger(str(log1), "r"),
                 callbacks=[ModelCheckpoint(dirpath=str(ck), every_n_train_steps=3, save_top_k=-1)])
    t1.fit(_lm(), _dm())
    f = ck / "epoch=0-step=3.ckpt"
    assert f.is_file() and ckpt.is_complete(f)  # one file, no shard directory left behind
    assert not (ck / "epoch=0-step=3.ckpt.parts").exists()
    meta = ckpt.read_meta(str(f))
    assert meta["trainer"]["global_step"] == 3 and meta.get("consolidated")
    log2 = tmp_path / "b"
    t2 = Trainer(strategy=FSDP2Strategy(), precision="32-true", max_steps=6, seed=3, log_every_n_steps=1,
                 logger=JSONLLogger(str(log2), "r"))
    t2.fit(_lm(), _dm(), ckpt_path=str(f))
    a, b = _losses(log1 / "r"), _losses(log2 / "r")
    for s in (4, 5, 6):
        assert abs(a[s] - b[s]) < 1e-6, (s, a[s], b[s])
    from llm_training_amd.tools.convert_to_hf import convert
    out = convert(str(f), str(tmp_path / "hf"), dtype="float32")
    assert os.path.exists(os.path.join(out, "config.json"))


def test_reads_v1_checkpoints(tmp_path):
    """A format-v1 checkpoint (tp0.safetensors keyed by parameter name, full tensors) resumes."""
    t = Trainer(strategy="ddp", precision="32-true", max_steps=2, seed=1, default_root_dir=str(tmp_path))
    lm = _lm()
    t.fit(lm, _dm())
    d = tmp_path / "v1"
    d.mkdir()
    names = {id(p): n for n, p in lm.model.named_parameters()}
    out = {}
    for u in t.engine.units:
        for p, o, shp in zip(u.params, u.offsets, u.shapes):
            n = names[id(p)]
            out["model." + n] = p.detach().clone()
            for kind in ckpt.KINDS:
                out[f"{kind}.{n}"] = getattr(u, kind)[o:o + shp.numel()].view(shp).clone()
    save_file(out, str(d / "tp0.safetensors"))
    meta = {"format": "llm_training_amd/v1", "trainer": t.state.state_dict(), "scheduler": t.scheduler.state_dict(),
            "optimizer_step": t.engine.step_count, "tp_size": 1, "dp_size": 1, "zero_stage": 0}
    (d / "meta.json").write_text(json.dumps(meta))
    assert ckpt.is_complete(d)
    t2 = Trainer(strategy="ddp", precision="32-true", max_steps=2, seed=1, default_root_dir=str(tmp_path))
    lm2 = _lm()
    t2.setup(lm2, _dm(), str(d))
    for (n, p), q in zip(lm.model.named_parameters(), lm2.model.parameters()):
        assert torch.equal(p, q), n
    for u, v in zip(t.engine.units, t2.engine.units):
        assert torch.equal(u.exp_avg_sq, v.exp_avg_sq)
    assert t2.global_step == 2 and t2.engine.step_count == 2
    _, parts = ckpt.load_model_state_for_export(str(d))
    assert set(parts[0]) == {n for n, _ in lm.model.named_parameters()}


def test_resume_replays_neftune_and_dropout_streams_exactly(tmp_path):
    """Phi-3 with embedding / residual / attention dropout and NEFTune: the resumed run's random
    streams continue from the checkpointed generator states, so losses match bitwise."""
    mc = dict(MC, vocab_size=96, embd_pdrop=0.1, resid_pdrop=0.1, attention_dropout=0.1, pad_token_id=0)

    def lm():
        return _lm("llm_training.models.Phi3", mc, neftune_alpha=5.0)

    ck = tmp_path / "ck"
    log1 = tmp_path / "a"
    t1 = Trainer(strategy="ddp", precision="32-true", max_steps=6, seed=7, log_every_n_steps=1,
                 logger=JSONLLogger(str(log1), "r"),
                 callbacks=[ModelCheckpoint(dirpath=str(ck), every_n_train_steps=3, save_top_k=-1)])
    t1.fit(lm(), _dm())
    log2 = tmp_path / "b"
    t2 = Trainer(strategy="ddp", precision="32-true", max_steps=6, seed=7, log_every_n_steps=1,
                 logger=JSONLLogger(str(log2), "r"))
    t2.fit(lm(), _dm(), ckpt_path=str(ck / "epoch=0-step=3.ckpt"))
    a, b = _losses(log1 / "r"), _losses(log2 / "r")
    assert sorted(b) == [4, 5, 6]
    for s in (4, 5, 6):
        assert a[s] == b[s], (s, a[s], b[s])
    # and the streams matter: a resume without the generator states diverges
    os.remove(ck / "epoch=0-step=3.ckpt" / "rng-tp0-dp0.safetensors")
    log3 = tmp_path / "c"
    t3 = Trainer(strategy="ddp", precision="32-true", max_steps=6, seed=7, log_every_n_steps=1,
                 logger=JSONLLogger(str(log3), "r"))
    t3.fit(lm(), _dm(), ckpt_path=str(ck / "epoch=0-step=3.ckpt"))
    c = _losses(log3 / "r")
    assert any(a[s] != c[s] for s in (4, 5, 6))


def test_optimizer_resolution():
    from llm_training_amd.optim import resolve_optimizer
    assert resolve_optimizer("torch.optim.AdamW", {"lr": 1e-3})["kind"] == "fused"
    assert resolve_optimizer("deepspeed.ops.adam.FusedAdam", {"lr": 1e-3})["weight_decay"] == 0.0
    cpu_adam = resolve_optimizer("deepspeed.ops.adam.DeepSpeedCPUAdam",
                                 {"lr": 1e-3, "adamw_mode": True, "weight_decay": 0.1, "fp32_optimizer_states": True})
    assert cpu_adam["kind"] == "fused" and cpu_adam["weight_decay"] == 0.1
    with pytest.raises(ValueError):
        resolve_optimizer("deepspeed.ops.adam.DeepSpeedCPUAdam", {"lr": 1e-3, "adamw_mode": False, "weight_decay": 0.1})
    hp = resolve_optimizer("torch.optim.AdamW", {"lr": 1e-3, "amsgrad": True})
    assert hp["kind"] == "generic" and hp["cls"] is torch.optim.AdamW and hp["kwargs"]["amsgrad"] is True
    assert resolve_optimizer("torch.optim.Adam", {"lr": 1e-3, "weight_decay": 0.1})["kind"] == "generic"
    for bad in ({"amsgrad": True}, {"bias_correction": False}, {"adam_w_mode": False, "weight_decay": 0.1}):
        with pytest.raises(ValueError):
            resolve_optimizer("deepspeed.ops.adam.FusedAdam", {"lr": 1e-3, **bad})
    with pytest.raises(ValueError, match="unknown optimizer kwargs"):
        resolve_optimizer("torch.optim.SGD", {"lr": 0.1, "betas": (0.9, 0.9)})
    with pytest.raises(ValueError):
        resolve_optimizer("torch.optim.SGD", {"lr": 0.1, "momentum": -1.0})  # validated up front
    hp = resolve_optimizer("torch.optim.RMSprop", {"lr": "3e-4", "alpha": 0.9})
    assert hp["kind"] == "generic" and hp["lr"] == 3e-4


@pytest.mark.parametrize("opt,kw", [("torch.optim.SGD", {"lr": 0.05, "momentum": 0.9}),
                                    ("torch.optim.AdamW", {"lr": 5e-3, "amsgrad": True}),
                                    ("torch.optim.Adafactor", {"lr": 1e-2})])
def test_generic_optimizer_resume_is_exact(tmp_path, opt, kw):
    def lm():
        return CLM({"model": {"model_class": "llm_training.models.Llama", "model_config": dict(MC)},
                    "optim": {"optimizer_class": opt, "optimizer_kwargs": dict(kw)}})

    ck = tmp_path / "ck"
    log1 = tmp_path / "a"
    t1 = Trainer(strategy="ddp", precision="32-true", max_steps=6, seed=3, log_every_n_steps=1,
                 logger=JSONLLogger(str(log1), "r"),
                 callbacks=[ModelCheckpoint(dirpath=str(ck), every_n_train_steps=3, save_top_k=-1)])
    t1.fit(lm(), _dm())
    assert type(t1.engine.units[0].opt).__name__ == opt.rsplit(".", 1)[1]
    log2 = tmp_path / "b"
    t2 = Trainer(strategy="ddp", precision="32-true", max_steps=6, seed=3, log_every_n_steps=1,
                 logger=JSONLLogger(str(log2), "r"))
    t2.fit(lm(), _dm(), ckpt_path=str(ck / "epoch=0-step=3.ckpt"))
    a, b = _losses(log1 / "r"), _losses(log2 / "r")
    for s in (4, 5, 6):
        assert abs(a[s] - b[s]) < 1e-6, (s, a[s], b[s])


@pytest.mark.parametrize("precision", ["16-mixed", "16-true"])
def test_fp16_precisions_with_dynamic_loss_scaler(tmp_path, precision):
    """fp16 params with the loss scaler (reference FSDP2Precision 16-true / 16-mixed): an absurd initial
    scale overflows, those steps are skipped and the scale backs off until training proceeds; the
    scaler state is checkpointed."""
    log = tmp_path / "log"
    t = Trainer(strategy="ddp", precision=precision, max_steps=8, seed=1, log_every_n_steps=1,
                logger=JSONLLogger(str(log), "r"), default_root_dir=str(tmp_path))
    t.scaler.scale = 2.0 ** 100  # overflows fp16 gradients at once
    lm = _lm()
    t.fit(lm, _dm())
    assert next(lm.model.parameters()).dtype == torch.float16
    assert t.scaler.skipped >= 1 and t.scaler.scale < 2.0 ** 100
    rows = [json.loads(line) for line in open(log / "r" / "metrics.jsonl")]
    assert rows[-1]["Skipped Steps"] == t.scaler.skipped
    losses = [r["Loss/Train/Step"] for r in rows if "Loss/Train/Step" in r]
    assert all(x == x for x in losses)
    t.save_checkpoint(str(tmp_path / "ck"))
    assert ckpt.read_meta(str(tmp_path / "ck"))["loss_scaler"]["scale"] == t.scaler.scale


def test_fp16_with_optimizer_offload(tmp_path):
    """fp16 gradients reach the host AdamW (which reads bf16 / fp32) upcast to fp32: 16-mixed / 16-true
    with offload_optimizer train instead of failing in the first step."""
    from llm_training_amd.runtime.strategies import DeepSpeedStrategy
    for precision in ("16-true", "16-mixed"):
        t = Trainer(strategy=DeepSpeedStrategy(stage=2, offload_optimizer=True), precision=precision, max_steps=3,
                    seed=1, default_root_dir=str(tmp_path))
        lm = _lm()
        t.fit(lm, _dm())
        assert t.global_step == 3
        assert all(u.g_host.dtype == torch.float32 for u in t.engine.units)
        assert all(torch.isfinite(p).all() for p in lm.model.parameters())
