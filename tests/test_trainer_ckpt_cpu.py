"""Trainer loop, LR schedules, checkpoint save -> resume (exact continuation), HF export round trip."""
import math
import os

import pytest
import torch

from llm_training_amd.data.dummy import DummyDataModule
from llm_training_amd.lms.clm import CLM
from llm_training_amd.lr_schedulers import ConstantWarmupLR, CosineAnnealingWarmupLR, LinearWarmupLR
from llm_training_amd.runtime.callbacks import ModelCheckpoint
from llm_training_amd.runtime.loggers import JSONLLogger
from llm_training_amd.runtime.strategies import DeepSpeedStrategy, FSDP2Strategy
from llm_training_amd.runtime.trainer import Trainer


def test_lr_schedules_match_reference_formulas():
    c = CosineAnnealingWarmupLR(1.0, num_warmup_steps=4, num_total_steps=14, min_lr=0.1)
    assert [round(c.lr_at(s), 6) for s in range(4)] == [0.25, 0.5, 0.75, 1.0]
    assert abs(c.lr_at(4) - 1.0) < 1e-9 and abs(c.lr_at(14) - 0.1) < 1e-9
    assert abs(c.lr_at(9) - (0.1 + 0.9 * (1 + math.cos(math.pi * 5 / 10)) / 2)) < 1e-9
    k = ConstantWarmupLR(2.0, factor=0.5, total_iters=3, num_warmup_steps=2)
    assert [k.lr_at(s) for s in range(7)] == [1.0, 2.0, 1.0, 1.0, 1.0, 2.0, 2.0]
    lin = LinearWarmupLR(1.0, num_warmup_steps=3, num_total_steps=13, min_lr=0.0)
    assert abs(lin.lr_at(0) - 0.25) < 1e-9 and abs(lin.lr_at(13)) < 1e-9 and abs(lin.lr_at(8) - 0.5) < 1e-9


def _lm(seed=0, total_steps=None):
    sched = {"num_warmup_steps": 2, "min_lr": 1e-4}
    if total_steps is not None:
        sched["num_total_steps"] = total_steps
    return CLM({"model": {"model_class": "llm_training.models.Llama",
                          "model_config": {"vocab_size": 96, "hidden_size": 32, "intermediate_size": 64,
                                           "num_hidden_layers": 2, "num_attention_heads": 4,
                                           "num_key_value_heads": 2}},
                "optim": {"optimizer_class": "torch.optim.AdamW", "optimizer_kwargs": {"lr": 5e-3},
                          "lr_scheduler_class": "llm_training.lr_schedulers.CosineAnnealingWarmupLR",
                          "lr_scheduler_kwargs": sched}})


def _dm():
    return DummyDataModule({"batch_size": 2, "vocab_size": 96, "max_length": 16, "num_samples": 64, "base_seed": 5})


def _losses(tmp):
    rows = [__import__("json").loads(l) for l in open(os.path.join(tmp, "metrics.jsonl"))]
    return {r["step"]: r["Loss/Train/Step"] for r in rows if "Loss/Train/Step" in r}


@pytest.mark.parametrize("strategy", [FSDP2Strategy(), DeepSpeedStrategy(stage=2)], ids=["fsdp2", "zero2"])
def test_resume_is_exact(tmp_path, strategy):
    log1 = tmp_path / "a"
    t1 = Trainer(strategy=strategy, precision="32-true", logger=JSONLLogger(str(log1), "r"), max_steps=6,
                 log_every_n_steps=1, accumulate_grad_batches=2, gradient_clip_val=1.0, seed=11,
                 callbacks=[ModelCheckpoint(dirpath=str(tmp_path / "ck"), every_n_train_steps=3, save_top_k=-1,
                                            async_save=True)])
    t1.fit(_lm(), _dm())
    full = _losses(log1 / "r")
    ck = tmp_path / "ck" / "epoch=0-step=3.ckpt"
    assert (ck / "meta.json").exists() and (ck / "shard-tp0-dp0.safetensors").exists()
    log2 = tmp_path / "b"
    t2 = Trainer(strategy=strategy, precision="32-true", logger=JSONLLogger(str(log2), "r"), max_steps=6,
                 log_every_n_steps=1, accumulate_grad_batches=2, gradient_clip_val=1.0, seed=11)
    t2.fit(_lm(), _dm(), ckpt_path=str(ck))
    resumed = _losses(log2 / "r")
    assert sorted(resumed) == [4, 5, 6]
    for s in (4, 5, 6):
        assert abs(resumed[s] - full[s]) < 1e-5, (s, resumed[s], full[s])


def test_convert_to_hf_roundtrip(tmp_path):
    from transformers import AutoModelForCausalLM

    from llm_training_amd.tools.convert_to_hf import convert
    t = Trainer(strategy="ddp", precision="32-true", max_steps=2, log_every_n_steps=1, seed=1,
                default_root_dir=str(tmp_path))
    lm = _lm()
    t.fit(lm, _dm())
    ck = tmp_path / "ck"
    t.save_checkpoint(str(ck))
    out = convert(str(ck), str(tmp_path / "hf"), dtype="float32")
    hf = AutoModelForCausalLM.from_pretrained(out, local_files_only=True)
    hf.eval()
    lm.model.eval()
    ids = torch.randint(0, 96, (2, 16))
    with torch.no_grad():
        a = lm.model(input_ids=ids).logits
        b = hf(input_ids=ids).logits
    assert torch.allclose(a, b, atol=1e-4), (a - b).abs().max()


def test_reference_style_convert_script(tmp_path):
    """``python scripts/convert_to_hf.py <ckpt> <out> --dtype float32`` (the reference's script interface)."""
    import subprocess
    import sys
    t = Trainer(strategy="ddp", precision="32-true", max_steps=1, seed=1, default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    ck = tmp_path / "ck"
    t.save_checkpoint(str(ck))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "convert_to_hf.py"), str(ck),
                        str(tmp_path / "hf"), "--dtype", "float32"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (tmp_path / "hf" / "config.json").exists()


def test_training_time_estimator_stops(tmp_path):
    from llm_training_amd.runtime.callbacks import TrainingTimeEstimator
    est = TrainingTimeEstimator(num_test_steps=4, num_warmup_steps=2)
    t = Trainer(strategy="ddp", precision="32-true", max_steps=50, callbacks=[est], seed=1,
                default_root_dir=str(tmp_path))
    t.fit(_lm(), _dm())
    assert t.global_step == 4 and est.result is not None and est.result["steps_per_sec"] > 0


def test_dpo_resume_rebuilds_reference_from_pretrained(tmp_path):
    """Resuming a DPO run must not copy the (trained) policy into the frozen reference model: the
    reference is rebuilt from the pre-trained weights, exactly as in the original run."""
    from safetensors.torch import save_file

    from llm_training_amd.lms.preference import DPO
    from llm_training_amd.parallel.context import ParallelContext
    mcfg = {"vocab_size": 96, "hidden_size": 32, "intermediate_size": 64, "num_hidden_layers": 2,
            "num_attention_heads": 4, "num_key_value_heads": 2}
    src = DPO({"model": {"model_class": "llm_training.models.Llama", "model_config": mcfg}})
    src.configure_model(ParallelContext.single(), torch.device("cpu"), torch.float32, seed=11)
    path = str(tmp_path / "pre.safetensors")
    save_file({k: v.contiguous() for k, v in src.model.state_dict().items()}, path)
    refs = []
    for resuming in (False, True):
        lm = DPO({"model": {"model_class": "llm_training.models.Llama", "model_config": mcfg},
                  "pre_trained_weights": path})
        lm.configure_model(ParallelContext.single(), torch.device("cpu"), torch.float32, seed=3, resuming=resuming)
        refs.append({k: v.clone() for k, v in lm.ref_model.state_dict().items()})
    for k, v in src.model.state_dict().items():
        assert torch.equal(refs[0][k], v) and torch.equal(refs[1][k], v), k


def _reference_style_state(seed=0):
    """A tiny Llama's weights under the reference LightningModule's names (``model.`` + HF-style module
    names, lm_head inside the model), plus the YAML config that describes it."""
    from collections import OrderedDict

    from llm_training_amd.models.llama import Llama, LlamaConfig
    from llm_training_amd.parallel.context import ParallelContext
    mc = {"vocab_size": 96, "hidden_size": 32, "intermediate_size": 64, "num_hidden_layers": 2,
          "num_attention_heads": 4, "num_key_value_heads": 2}
    m = Llama(LlamaConfig(**mc), ParallelContext.single(), dtype=torch.float32)
    m.init_weights(seed)
    hf = Llama.convert_state_dict_to_hf({k: v.detach().clone() for k, v in m.state_dict().items()}, m.config)
    lm_keys = OrderedDict(("model." + (k[len("model."):] if k.startswith("model.") else k), v) for k, v in hf.items())
    cfg = {"trainer": {"precision": "32-true"},
           "model": {"class_path": "llm_training.lms.CLM",
                     "init_args": {"config": {"model": {"model_class": "llm_training.models.Llama",
                                                        "model_config": mc}}}}}
    return hf, lm_keys, cfg


def _write_deepspeed(d, lm_keys, stage, world):
    """Synthetic DeepSpeed ZeRO checkpoint with DeepSpeed's on-disk layout (param_shapes + per-rank flat
    fp32 partitions), parameter names as Lightning's DeepSpeed wrapper records them."""
    from collections import OrderedDict
    names = ["_forward_module." + k for k in lm_keys]
    tensors = [v.float() for v in lm_keys.values()]
    shapes = OrderedDict((n, t.shape) for n, t in zip(names, tensors))
    tag = d / "checkpoint"
    tag.mkdir(parents=True)
    (d / "latest").write_text("checkpoint")
    torch.save({"module": {}, "buffer_names": [], "param_shapes": [shapes], "ds_version": "0.14.0"},
               tag / "mp_rank_00_model_states.pt")
    if stage <= 2:
        flat = torch.cat([t.reshape(-1) for t in tensors])
        align = 2 * world
        flat = torch.cat([flat, flat.new_zeros((-flat.numel()) % align)])
        parts = flat.chunk(world)
        key = "single_partition_of_fp32_groups"
    else:
        per_rank = [[] for _ in range(world)]
        for t in tensors:
            f = t.reshape(-1)
            f = torch.cat([f, f.new_zeros((-f.numel()) % world)])
            for r, c in enumerate(f.chunk(world)):
                per_rank[r].append(c)
        parts = [torch.cat(p) for p in per_rank]
        key = "fp32_flat_groups"
    for r in range(world):
        torch.save({"optimizer_state_dict": {"zero_stage": stage, "partition_count": world, key: [parts[r].clone()]}},
                   tag / f"zero_pp_rank_{r}_mp_rank_00_optim_states.pt")


@pytest.mark.parametrize("fmt", ["zero2_w2", "zero3_w3", "dcp", "plain_pt"])
def test_convert_to_hf_from_reference_checkpoints(tmp_path, fmt):
    """convert-to-hf on checkpoints in the reference framework's formats (DeepSpeed ZeRO-2/3 directories,
    FSDP2 distributed checkpoints, plain Lightning state dicts): the HF export equals the weights."""
    import yaml
    from safetensors.torch import load_file

    from llm_training_amd.tools.convert_to_hf import convert
    hf, lm_keys, cfg = _reference_style_state()
    (tmp_path / "cfg.yaml").write_text(yaml.safe_dump(cfg))
    ck = tmp_path / "ck"
    if fmt.startswith("zero"):
        _write_deepspeed(ck, lm_keys, int(fmt[4]), int(fmt[-1]))
    elif fmt == "dcp":
        import torch.distributed.checkpoint as dcp
        dcp.save({"state_dict." + k: v for k, v in lm_keys.items()}, checkpoint_id=str(ck), no_dist=True)
    else:
        ck = tmp_path / "ck.pt"
        torch.save({"state_dict": dict(lm_keys), "global_step": 3}, ck)
    out = convert(str(ck), str(tmp_path / "hf"), config_path=str(tmp_path / "cfg.yaml"), dtype="float32")
    got = load_file(os.path.join(out, "model.safetensors"))
    assert set(got) == set(hf)
    for k, v in hf.items():
        assert torch.equal(got[k], v.float()), k


def test_convert_deepspeed_zero3_merges_frozen_fragments(tmp_path):
    """ZeRO-3 keeps frozen parameters as per-rank fragments in every rank's model-states file; the
    converter concatenates them in rank order (DeepSpeed zero_to_fp32 _zero3_merge_frozen_params)."""
    from collections import OrderedDict

    import yaml
    from safetensors.torch import load_file

    from llm_training_amd.tools.convert_to_hf import convert
    hf, lm_keys, cfg = _reference_style_state()
    (tmp_path / "cfg.yaml").write_text(yaml.safe_dump(cfg))
    frozen = "model.embed_tokens.weight"
    world = 3
    trainable = OrderedDict((k, v) for k, v in lm_keys.items() if k != frozen)
    ck = tmp_path / "ck"
    _write_deepspeed(ck, trainable, 3, world)
    tag = ck / "checkpoint"
    fz = lm_keys[frozen].float().reshape(-1)
    fz = torch.cat([fz, fz.new_zeros((-fz.numel()) % world)])
    name = "_forward_module." + frozen
    base = torch.load(tag / "mp_rank_00_model_states.pt", weights_only=False)
    for r, frag in enumerate(fz.chunk(world)):
        st = dict(base, frozen_param_shapes=OrderedDict([(name, lm_keys[frozen].shape)]),
                  frozen_param_fragments={name: frag.clone()})
        torch.save(st, tag / f"zero_pp_rank_{r}_mp_rank_00_model_states.pt")
    torch.save(dict(base, frozen_param_shapes=OrderedDict([(name, lm_keys[frozen].shape)]),
                    frozen_param_fragments={name: fz.chunk(world)[0].clone()}),
               tag / "mp_rank_00_model_states.pt")
    out = convert(str(ck), str(tmp_path / "hf"), config_path=str(tmp_path / "cfg.yaml"), dtype="float32")
    got = load_file(os.path.join(out, "model.safetensors"))
    for k, v in hf.items():
        assert torch.equal(got[k], v.float()), k


def test_early_stop_runs_epoch_end_checkpoint_and_resumes_mid_epoch(tmp_path):
    """max_steps stopping mid-epoch still runs the epoch-end hooks (Lightning), so a reference-style
    ModelCheckpoint(save_on_train_epoch_end=True) writes the final state; resuming from it continues in
    the same epoch, step for step equal to an uninterrupted run."""
    log_full, log_a, log_b = tmp_path / "full", tmp_path / "a", tmp_path / "b"
    Trainer(strategy="ddp", precision="32-true", logger=JSONLLogger(str(log_full), "r"), max_steps=8,
            log_every_n_steps=1, seed=3).fit(_lm(total_steps=8), _dm())
    t = Trainer(strategy="ddp", precision="32-true", logger=JSONLLogger(str(log_a), "r"), max_steps=5,
                log_every_n_steps=1, seed=3,
                callbacks=[ModelCheckpoint(dirpath=str(tmp_path / "ck"), save_on_train_epoch_end=True)])
    t.fit(_lm(total_steps=8), _dm())
    ck = tmp_path / "ck" / "epoch=0-step=5.ckpt"
    assert (ck / "meta.json").exists() and t.state.epoch == 0 and t.state.batch_idx == 5
    Trainer(strategy="ddp", precision="32-true", logger=JSONLLogger(str(log_b), "r"), max_steps=8,
            log_every_n_steps=1, seed=3).fit(_lm(total_steps=8), _dm(), ckpt_path=str(ck))
    full, resumed = _losses(log_full / "r"), _losses(log_b / "r")
    assert sorted(resumed) == [6, 7, 8]
    for s in resumed:
        assert abs(resumed[s] - full[s]) < 1e-5, (s, resumed[s], full[s])


def test_max_time():
    import datetime

    from llm_training_amd.runtime.trainer import parse_max_time
    assert parse_max_time("00:12:00:00") == 12 * 3600
    assert parse_max_time({"days": 1, "minutes": 30}) == 86400 + 1800
    assert parse_max_time(datetime.timedelta(seconds=90)) == 90
    assert parse_max_time(None) is None
    with pytest.raises(ValueError):
        parse_max_time("12:00")
    t = Trainer(strategy="ddp", precision="32-true", max_steps=20, max_time={"seconds": 0}, seed=1)
    t.fit(_lm(total_steps=8), _dm())
    assert t.global_step == 1  # time is checked after each optimizer step, as Lightning's Timer does


def test_convert_to_hf_roundtrip_phi3_longrope(tmp_path):
    """A trained Phi-3 (fused qkv / gate_up, LongRoPE, sliding window) exported by convert-to-hf loads in
    transformers' Phi3ForCausalLM with the same logits, past the original context (long factors)."""
    from transformers import AutoModelForCausalLM

    from llm_training_amd.tools.convert_to_hf import convert
    rs = {"type": "longrope", "short_factor": [1.0 + 0.1 * i for i in range(8)],
          "long_factor": [2.0 + 0.3 * i for i in range(8)]}
    lm = CLM({"model": {"model_class": "llm_training.models.Phi3",
                        "model_config": {"vocab_size": 96, "hidden_size": 64, "intermediate_size": 96,
                                         "num_hidden_layers": 2, "num_attention_heads": 4,
                                         "num_key_value_heads": 4, "max_position_embeddings": 16384,
                                         "original_max_position_embeddings": 4096, "rope_scaling": rs,
                                         "sliding_window": 48, "pad_token_id": 0, "eos_token_id": 1,
                                         "bos_token_id": 2}},
              "optim": {"optimizer_class": "torch.optim.AdamW", "optimizer_kwargs": {"lr": 5e-3}}})
    t = Trainer(strategy="ddp", precision="32-true", max_steps=2, seed=1, default_root_dir=str(tmp_path))
    t.fit(lm, DummyDataModule({"batch_size": 2, "vocab_size": 96, "max_length": 64, "num_samples": 16,
                               "base_seed": 5}))
    ck = tmp_path / "ck"
    t.save_checkpoint(str(ck))
    out = convert(str(ck), str(tmp_path / "hf"), dtype="float32")
    import json
    exported = json.loads((tmp_path / "hf" / "config.json").read_text())
    assert exported["sliding_window"] == 48  # the config value is exported unchanged, as the reference does
    # the window counts like flash-attn's window_size=(W, W) in the reference (attention_op.py:588, and its
    # eager mask :160-163): keys q-W..q, W+1 of them; transformers 5 counts W keys (kv > q - W), so
    # the same model needs W+1 there
    hf = AutoModelForCausalLM.from_pretrained(out, local_files_only=True, attn_implementation="eager",
                                              sliding_window=49)
    assert type(hf).__name__ == "Phi3ForCausalLM"
    hf.eval()
    lm.model.eval()
    for S in (24, 4100):  # inside and past original_max_position_embeddings
        ids = torch.randint(3, 96, (2, S))
        with torch.no_grad():
            a = lm.model(input_ids=ids).logits
            b = hf(input_ids=ids).logits
        assert torch.allclose(a, b, atol=2e-4), (S, (a - b).abs().max())


@pytest.mark.parametrize("model_type", ["llama", "qwen2"])
def test_convert_to_hf_splits_fused_hf_projections(tmp_path, model_type):
    """HFCausalLM with ``enable_liger_kernel`` trains with fused q/k/v (Qwen2: and their biases) and gate/up
    parameters, and checkpoints name them as such; the HF export splits them back into the per-projection
    keys, so transformers loads every projection (none randomly initialised) and reproduces the logits."""
    from transformers import AutoModelForCausalLM

    from llm_training_amd.tools.convert_to_hf import convert
    hc = {"model_type": model_type, "num_hidden_layers": 2, "num_attention_heads": 4, "num_key_value_heads": 2,
          "hidden_size": 64, "intermediate_size": 96, "vocab_size": 96, "max_position_embeddings": 64}
    lm = CLM({"model": {"model_class": "llm_training.models.HFCausalLM",
                        "model_config": {"hf_config": hc, "enable_liger_kernel": True,
                                         "attn_implementation": "flash"}},
              "optim": {"optimizer_class": "torch.optim.AdamW", "optimizer_kwargs": {"lr": 5e-3}}})
    t = Trainer(strategy="ddp", precision="32-true", max_steps=2, log_every_n_steps=1, seed=1,
                default_root_dir=str(tmp_path))
    t.fit(lm, _dm())
    names = {n for n, _ in lm.model.named_parameters()}
    assert any(n.endswith("mlp.gate_up_weight") for n in names), sorted(names)[:8]
    ck = tmp_path / "ck"
    t.save_checkpoint(str(ck))
    out = convert(str(ck), str(tmp_path / "hf"), dtype="float32")
    from safetensors.torch import load_file
    keys = set(load_file(os.path.join(out, "model.safetensors")))
    assert not any("qkv_" in k or "gate_up_weight" in k for k in keys), sorted(keys)
    for proj in ("self_attn.q_proj.weight", "self_attn.k_proj.weight", "self_attn.v_proj.weight",
                 "mlp.gate_proj.weight", "mlp.up_proj.weight"):
        assert f"model.layers.1.{proj}" in keys, proj
    assert ("model.layers.0.self_attn.k_proj.bias" in keys) == (model_type == "qwen2")
    hf = AutoModelForCausalLM.from_pretrained(out, local_files_only=True)
    hf.eval()
    lm.model.eval()
    sd = lm.model.state_dict()  # transformers key view of the fused parameters
    for k, v in hf.state_dict().items():
        if "hf_model." + k in sd:
            assert torch.equal(v, sd["hf_model." + k].float()), k
    ids = torch.randint(0, 96, (2, 16))
    with torch.no_grad():
        a = lm.model(input_ids=ids).logits
        b = hf(input_ids=ids).logits
    assert torch.allclose(a, b, atol=1e-4), (a - b).abs().max()


@pytest.mark.parametrize("model_type", ["llama", "qwen2"])
def test_hf_fused_qkv_names_convert_to_hf_keys(model_type):
    """The fused q/k/v parameters (built when the attention runs on the flash path) of a parameter-named
    state dict (what checkpoints hold) convert to exactly the unpatched model's transformers state dict."""
    from llm_training_amd.models.hf_causal_lm import HFCausalLM, HFCausalLMConfig
    hc = {"model_type": model_type, "num_hidden_layers": 2, "num_attention_heads": 4, "num_key_value_heads": 2,
          "hidden_size": 256, "intermediate_size": 96, "vocab_size": 96, "max_position_embeddings": 64}
    cfg = HFCausalLMConfig(hf_config=hc, enable_liger_kernel=True, attn_implementation="flash")
    m = HFCausalLM(cfg)
    m.init_weights(0)
    named = {n: p.detach() for n, p in m.named_parameters()}
    assert any(n.endswith("self_attn.qkv_weight") for n in named)
    assert any(n.endswith("self_attn.qkv_bias") for n in named) == (model_type == "qwen2")
    hf = HFCausalLM.convert_state_dict_to_hf(named, cfg)
    want = {k[len("hf_model."):]: v for k, v in m.state_dict().items()}
    want.pop("lm_head.weight", None) if "lm_head.weight" not in hf else None
    assert set(hf) == set(want), sorted(set(hf) ^ set(want))
    for k in want:
        assert torch.equal(hf[k], want[k]), k
