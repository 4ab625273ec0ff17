"""Config loader / CLI surface: every reference example YAML parses and its objects instantiate."""
import glob
import os

import pytest

from llm_training_amd.config.loader import expand_dotted, instantiate, load_config
from llm_training_amd.lms import CLM, DPO, ORPO
from llm_training_amd.runtime.strategies import DeepSpeedStrategy, FSDP2Strategy

REF = "/root/reference/config/examples"
OURS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "config", "examples")
EXAMPLES = sorted(glob.glob(f"{REF}/*/*.yaml")) + sorted(glob.glob(f"{OURS}/*/*.yaml"))


def test_dotted_keys_expand():
    d = expand_dotted({"a.b.c": 1, "a": {"b": {"d": 2}}, "x": [{"y.z": 3}]})
    assert d == {"a": {"b": {"c": 1, "d": 2}}, "x": [{"y": {"z": 3}}]}


def test_overrides_and_interpolation(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("trainer:\n  max_steps: 5\n  val: ${trainer.max_steps}\nmodel:\n  lr: 1e-5\n")
    c = load_config(p, ["trainer.max_steps=7", "--model.extra=abc"])
    assert c["trainer"]["max_steps"] == 7 and c["trainer"]["val"] == 7
    assert c["model"]["lr"] == 1e-5 and c["model"]["extra"] == "abc"


@pytest.mark.skipif(not EXAMPLES, reason="reference configs not mounted")
@pytest.mark.parametrize("path", EXAMPLES, ids=lambda p: os.path.basename(p))
def test_reference_examples_parse_and_instantiate(path):
    cfg = load_config(path)
    assert {"trainer", "model", "data"} <= set(cfg)
    tcfg = dict(cfg["trainer"])
    strat = instantiate(tcfg["strategy"])
    assert isinstance(strat, (FSDP2Strategy, DeepSpeedStrategy))
    if isinstance(strat, FSDP2Strategy) and "tp" in os.path.basename(path):
        assert strat.tensor_parallel_size in (2, 4, 8)
    cbs = instantiate(tcfg.get("callbacks", []))
    assert isinstance(cbs, list)
    logger = instantiate(tcfg["logger"])
    assert logger.log_dir.startswith("logs")
    lm = instantiate(cfg["model"])
    assert isinstance(lm, (CLM, DPO, ORPO))
    assert lm.config.optim is not None
    # data modules need the (remote) tokenizer: check the class path resolves instead
    from llm_training_amd.utils.imports import import_object
    import_object(cfg["data"]["class_path"])


def test_fused_adam_alias_resolves():
    from llm_training_amd.optim import resolve_optimizer
    hp = resolve_optimizer("deepspeed.ops.adam.FusedAdam", {"lr": 1e-5})
    assert hp["lr"] == 1e-5 and hp["weight_decay"] == 0.0
    hp = resolve_optimizer("torch.optim.AdamW", {"lr": "3e-5", "betas": [0.9, 0.95]})
    assert hp["lr"] == 3e-5 and hp["betas"] == (0.9, 0.95) and hp["weight_decay"] == 0.01


def test_cli_fit_tiny_cpu(tmp_path):
    from llm_training_amd.cli.main import main
    cfg = tmp_path / "tiny.yaml"
    cfg.write_text(f"""
seed_everything: 1
trainer:
  strategy: ddp
  precision: 32-true
  logger:
    class_path: llm_training.lightning.CSVLogger
    init_args: {{save_dir: {tmp_path}/logs, name: t}}
  max_steps: 4
  log_every_n_steps: 1
  gradient_clip_val: 1.0
  callbacks:
    - class_path: lightning.pytorch.callbacks.LearningRateMonitor
      init_args: {{logging_interval: step, log_momentum: true}}
model:
  class_path: llm_training.lms.CLM
  init_args.config:
    model:
      model_class: llm_training.models.Llama
      model_config: {{vocab_size: 64, hidden_size: 32, intermediate_size: 64, num_hidden_layers: 1,
                      num_attention_heads: 2, num_key_value_heads: 1}}
    optim:
      optimizer_class: torch.optim.AdamW
      optimizer_kwargs: {{lr: 1e-2}}
data:
  class_path: llm_training.data.DummyDataModule
  init_args.config: {{batch_size: 2, vocab_size: 64, max_length: 16, num_samples: 32, base_seed: 3}}
""")
    assert main(["fit", "--config", str(cfg)]) == 0
    assert os.path.exists(tmp_path / "logs" / "t" / "metrics.csv")
    assert os.path.exists(tmp_path / "logs" / "t" / "config.yaml")
    # LearningRateMonitor: Lightning's lr-<Optimizer> / -momentum columns, equal to the step's lr
    import csv
    rows = list(csv.DictReader(open(tmp_path / "logs" / "t" / "metrics.csv")))
    assert rows and "lr-AdamW" in rows[-1] and "lr-AdamW-momentum" in rows[-1]
    assert float(rows[-1]["lr-AdamW"]) == pytest.approx(float(rows[-1]["lr"]))
    assert float(rows[-1]["lr-AdamW-momentum"]) == pytest.approx(0.9)


def test_fsdp2_mp_policy_and_int_reshard_map_to_the_engine():
    """FSDP2Strategy(mp_policy=MixedPrecisionPolicy(...), reshard_after_forward=<int>) (reference
    fsdp2_strategy.py:56-58,94-99): param/reduce dtypes reach the engine; an int reshard size becomes the
    engine's secondary (hpZ) partition."""
    import torch
    from torch.distributed.fsdp import MixedPrecisionPolicy

    from llm_training_amd.runtime.strategies import FSDP2Strategy
    from llm_training_amd.runtime.trainer import Trainer
    s = FSDP2Strategy(mp_policy=MixedPrecisionPolicy(param_dtype=torch.bfloat16, reduce_dtype=torch.float32),
                      reshard_after_forward=4)
    assert (s.param_dtype, s.grad_reduce_dtype, s.zero_hpz_partition_size, s.zero_stage) == \
        ("bfloat16", "float32", 4, 3)
    assert s.engine_kwargs()["hpz_partition_size"] == 4
    s2 = FSDP2Strategy(mp_policy={"class_path": "torch.distributed.fsdp.MixedPrecisionPolicy",
                                  "init_args": {"param_dtype": "bf16", "reduce_dtype": "float32"}})
    assert (s2.param_dtype, s2.grad_reduce_dtype, s2.zero_hpz_partition_size) == ("bfloat16", "float32", 1)
    t = Trainer(strategy=s2, precision="32-true", max_steps=1)
    assert t.param_dtype == torch.bfloat16 and t.grad_dtype is None
    with pytest.raises(ValueError):
        FSDP2Strategy(mp_policy={"param_dtype": "float16"})


def test_container_recipes_reference_existing_files():
    """docker/Dockerfile, Singularity.def and install.sh: the files they copy / run exist and the build
    step is the in-tree gfx950 builder."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    df = open(os.path.join(root, "docker", "Dockerfile")).read()
    assert "docker/requirements.txt" in df and "docker/install.sh" in df and "HSA_ENABLE_IPC_MODE_LEGACY=0" in df
    for f in ("docker/requirements.txt", "docker/install.sh", "docker/Singularity.def", "setup.py"):
        assert os.path.exists(os.path.join(root, f)), f
    sh = open(os.path.join(root, "docker", "install.sh")).read()
    assert "python -m llm_training_amd._build" in sh and "gfx950" in sh


def test_pre_process_then_fit_from_the_saved_data(tmp_path):
    """`llm-training pre-process` on a YAML (local JSON data, a local HF tokenizer directory) writes the
    processed datasets and info.txt; `llm-training fit` with the same YAML then trains from the saved data
    (reference scripts/pre_process_data.py + pre_processed_data_path)."""
    import json
    import random
    import sys

    sys.path.insert(0, os.path.dirname(__file__))
    from helpers import toy_tokenizer

    from llm_training_amd.cli.main import main
    tok_dir = tmp_path / "tok"
    toy_tokenizer().save_pretrained(str(tok_dir))
    rng = random.Random(0)
    words = "hello world how are you the a of to and is it in that good bad yes no".split()
    data = tmp_path / "d.jsonl"
    data.write_text("\n".join(json.dumps({"text": " ".join(rng.choice(words) for _ in range(rng.randint(5, 40)))})
                              for _ in range(80)))
    cfg = tmp_path / "pt.yaml"
    cfg.write_text(f"""
seed_everything: 2
trainer:
  strategy: ddp
  precision: 32-true
  logger:
    class_path: llm_training.lightning.CSVLogger
    init_args: {{save_dir: {tmp_path}/logs, name: p}}
  max_steps: 3
  log_every_n_steps: 1
model:
  class_path: llm_training.lms.CLM
  init_args.config:
    model:
      model_class: llm_training.models.Llama
      model_config: {{vocab_size: 64, hidden_size: 32, intermediate_size: 64, num_hidden_layers: 1,
                      num_attention_heads: 2, num_key_value_heads: 1}}
    optim:
      optimizer_class: torch.optim.AdamW
      optimizer_kwargs: {{lr: 1e-2}}
data:
  class_path: llm_training.data.PreTrainingDataModule
  init_args.config:
    dataset_kwargs: {{path: json, data_files: {data}}}
    tokenizer:
      class_path: HFTokenizer
      init_args: {{path: {tok_dir}}}
    max_length: 32
    packing_method: BEST_FIT_BIN_PACKING
    batch_size: 2
    pre_processed_data_path: {tmp_path}/processed
""")
    assert main(["pre-process", "--config", str(cfg)]) == 0
    assert (tmp_path / "processed" / "info.txt").exists()
    # a second run keeps the existing output (the reference skips a non-empty directory) and rewrites info.txt
    train_files = sorted(p.name for p in (tmp_path / "processed" / "train").iterdir())
    stamp = (tmp_path / "processed" / "train" / train_files[0]).stat().st_mtime_ns
    (tmp_path / "processed" / "info.txt").unlink()
    assert main(["pre-process", "--config", str(cfg)]) == 0
    assert (tmp_path / "processed" / "info.txt").exists()
    assert (tmp_path / "processed" / "train" / train_files[0]).stat().st_mtime_ns == stamp
    assert main(["fit", "--config", str(cfg)]) == 0
    import csv
    rows = list(csv.DictReader(open(tmp_path / "logs" / "p" / "metrics.csv")))
    assert len(rows) == 3 and all(float(r["Loss/Train/Step"]) == float(r["Loss/Train/Step"]) for r in rows)


def test_cli_validate_from_checkpoint_matches_fit(tmp_path):
    """``llm-training validate --ckpt_path <ckpt>`` restores the trained weights and reproduces the
    validation loss the fit logged at the same step."""
    import json

    from llm_training_amd.cli.main import cmd_validate, main
    cfg = tmp_path / "tiny.yaml"
    cfg.write_text(f"""
seed_everything: 1
trainer:
  strategy: ddp
  precision: 32-true
  logger:
    class_path: JSONLLogger
    init_args: {{save_dir: {tmp_path}/logs, name: v}}
  max_steps: 3
  log_every_n_steps: 1
  val_check_interval: 3
  callbacks:
    - class_path: ModelCheckpoint
      init_args: {{dirpath: {tmp_path}/ck, every_n_train_steps: 3}}
model:
  class_path: llm_training.lms.CLM
  init_args.config:
    model:
      model_class: llm_training.models.Llama
      model_config: {{vocab_size: 64, hidden_size: 32, intermediate_size: 64, num_hidden_layers: 1,
                      num_attention_heads: 2, num_key_value_heads: 1}}
    optim:
      optimizer_class: torch.optim.AdamW
      optimizer_kwargs: {{lr: 1e-2}}
data:
  class_path: llm_training.data.DummyDataModule
  init_args.config: {{batch_size: 2, vocab_size: 64, max_length: 16, num_samples: 48, base_seed: 3,
                     validation_split: 8}}
""")
    assert main(["fit", "--config", str(cfg)]) == 0
    rows = [json.loads(x) for x in open(tmp_path / "logs" / "v" / "metrics.jsonl")]
    fit_val = [r["Loss/Val"] for r in rows if "Loss/Val" in r]
    assert len(fit_val) == 1
    ck = tmp_path / "ck" / "epoch=0-step=3.ckpt"
    out = cmd_validate(["--config", str(cfg), "--ckpt_path", str(ck)])
    assert out["Loss/Val"] == pytest.approx(fit_val[0], rel=1e-5)
