"""``llm-training`` command line: ``fit`` / ``validate`` / ``convert-to-hf`` / ``pre-process``.

Reference: console script ``llm-training = llm_training.cli.main:main`` (pyproject.toml:31-32) running
LightningCLI (src/llm_training/lightning/cli/cli.py:17-83) with the SLURM launch of
scripts/train.sh:17-22 (``llm-training fit --config $CONFIG --trainer.num_nodes $NODES --ckpt_path $CKPT``),
plus the two tools scripts/convert_to_hf.py and scripts/pre_process_data.py.

Launch: one process per GPU via ``torchrun`` / ``srun`` (RANK / WORLD_SIZE / LOCAL_RANK from the
environment); single-task SLURM jobs drop the SLURM variables as the reference does (cli.py:79-81).
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

logger = logging.getLogger("llm_training")

TOP_LEVEL = {"seed_everything", "float32_matmul_precision", "logging_level", "trainer", "model", "data",
             "ckpt_path", "output_redirection", "tqdm_progress", "world_size", "slurm"}


def _split_args(argv: list[str]):
    configs, overrides, rest = [], [], []
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ("--config", "-c"):
            configs.append(argv[i + 1])
            i += 2
            continue
        if a.startswith("--config="):
            configs.append(a.split("=", 1)[1])
        elif a.startswith("--"):
            if "=" in a:
                overrides.append(a[2:])
            elif i + 1 < len(argv) and not argv[i + 1].startswith("--"):
                overrides.append(f"{a[2:]}={argv[i + 1]}")
                i += 1
            else:
                overrides.append(f"{a[2:]}=true")
        else:
            rest.append(a)
        i += 1
    return configs, overrides, rest


def check_top_level(cfg: dict):
    """Reject unknown top-level keys (jsonargparse does, cli.py:17-83): a typo must not be ignored."""
    import difflib
    bad = [k for k in cfg if k not in TOP_LEVEL]
    if bad:
        hints = {k: difflib.get_close_matches(k, sorted(TOP_LEVEL), n=1) for k in bad}
        msg = ", ".join(f"{k!r}" + (f" (did you mean {h[0]!r}?)" if h else "") for k, h in hints.items())
        raise ValueError(f"unknown top-level config key(s): {msg}; allowed: {sorted(TOP_LEVEL)}")


def build_from_config(cfg: dict):
    """(trainer, lm, datamodule) from a resolved config dict."""
    from ..config.loader import instantiate
    from ..runtime.callbacks import ExtraConfig, OutputRedirection, SaveConfigCallback, TQDMProgressBar
    from ..runtime.trainer import Trainer

    check_top_level(cfg)
    ExtraConfig(cfg.get("float32_matmul_precision"), cfg.get("logging_level", "INFO"))
    if os.environ.get("SLURM_NTASKS") == "1":
        for k in ("SLURM_JOB_ID", "SLURM_NTASKS"):
            os.environ.pop(k, None)
    tcfg = dict(cfg.get("trainer") or {})
    tcfg = instantiate(tcfg)
    callbacks = list(tcfg.pop("callbacks", None) or [])
    callbacks.insert(0, SaveConfigCallback(cfg))
    # on by default, as in the reference (cli.py:67 adds OutputRedirection with enabled=True)
    orc = cfg.get("output_redirection", {})
    if orc is None or orc is True:
        orc = {}
    if orc is not False and (orc.get("enabled", True) if isinstance(orc, dict) else True):
        callbacks.insert(1, OutputRedirection(**(orc if isinstance(orc, dict) else {})))
    tq = cfg.get("tqdm_progress")
    if isinstance(tq, dict):
        callbacks.append(TQDMProgressBar(**tq))
    seed = cfg.get("seed_everything")
    trainer = Trainer(callbacks=callbacks, seed=seed if isinstance(seed, int) else None, **tcfg)
    lm = instantiate(cfg["model"])
    dm = instantiate(cfg["data"])
    return trainer, lm, dm


def cmd_fit(argv):
    from ..config.loader import load_config

    configs, overrides, _ = _split_args(argv)
    if not configs:
        raise SystemExit("llm-training fit: --config is required")
    cfg = load_config(configs, overrides)
    # trainer.devices ranks on this node, one process each (Lightning's subprocess launcher); the
    # parent only supervises and returns the job's exit code
    from ..launch import launch_for_trainer
    rc = launch_for_trainer(dict(cfg.get("trainer") or {}),
                            [sys.executable, "-m", "llm_training_amd.cli.main", "fit", *argv])
    if rc is not None:
        if rc:
            raise SystemExit(rc)
        return 0
    ckpt = cfg.pop("ckpt_path", None)
    trainer, lm, dm = build_from_config(cfg)
    trainer.fit(lm, dm, ckpt_path=ckpt)
    return trainer


def cmd_validate(argv):
    from ..config.loader import load_config

    configs, overrides, _ = _split_args(argv)
    cfg = load_config(configs, overrides)
    ckpt = cfg.pop("ckpt_path", None)
    trainer, lm, dm = build_from_config(cfg)
    trainer.setup(lm, dm, ckpt)
    return trainer.validate()


def cmd_convert(argv):
    ap = argparse.ArgumentParser(prog="llm-training convert-to-hf")
    ap.add_argument("checkpoint_path")
    ap.add_argument("output_dir", nargs="?")
    ap.add_argument("--config_path", default=None)
    ap.add_argument("--eos_token_id", default=None)
    ap.add_argument("--dtype", default=None)
    a = ap.parse_args(argv)
    from ..tools.convert_to_hf import convert

    return convert(a.checkpoint_path, a.output_dir, a.config_path, a.eos_token_id, a.dtype)


def cmd_pre_process(argv):
    from ..tools.pre_process_data import pre_process

    configs, overrides, _ = _split_args(argv)
    return pre_process(configs, overrides)


COMMANDS = {"fit": cmd_fit, "validate": cmd_validate, "convert-to-hf": cmd_convert, "convert_to_hf": cmd_convert,
            "pre-process": cmd_pre_process, "pre_process": cmd_pre_process}


def main(argv: list[str] | None = None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help") or argv[0] not in COMMANDS:
        print("usage: llm-training {fit,validate,convert-to-hf,pre-process} [--config cfg.yaml] [--a.b.c value ...]")
        return 0 if argv and argv[0] in ("-h", "--help") else 2
    r = COMMANDS[argv[0]](argv[1:])
    return r if isinstance(r, int) else 0


if __name__ == "__main__":
    r = main()
    sys.exit(r if isinstance(r, int) else 0)
