"""Import-path resolution for YAML ``class_path`` / ``*_class`` strings.

Reference YAML configs name classes under ``llm_training.*`` (e.g. ``llm_training.models.Llama``,
``llm_training.lightning.FSDP2Strategy``) and short names (``HFTokenizer``, ``LearningRateMonitor``)
(src/llm_training/lightning/cli/cli.py:17-83, docs/config.md). Those resolve here unchanged:
``llm_training.`` maps to this package, short names map to the registry below, and optimizers the
reference pulls from DeepSpeed map to our fused AdamW.
"""
from __future__ import annotations

import importlib

ALIASES = {
    "deepspeed.ops.adam.FusedAdam": "llm_training_amd.optim.FusedAdamW",
    "deepspeed.ops.adam.DeepSpeedCPUAdam": "llm_training_amd.optim.FusedAdamW",
    "lightning.pytorch.callbacks.LearningRateMonitor": "llm_training_amd.runtime.callbacks.LearningRateMonitor",
    "lightning.pytorch.callbacks.ModelCheckpoint": "llm_training_amd.runtime.callbacks.ModelCheckpoint",
    "lightning.pytorch.callbacks.EarlyStopping": "llm_training_amd.runtime.callbacks.EarlyStopping",
    "lightning.pytorch.callbacks.early_stopping.EarlyStopping": "llm_training_amd.runtime.callbacks.EarlyStopping",
    "lightning.pytorch.callbacks.TQDMProgressBar": "llm_training_amd.runtime.callbacks.TQDMProgressBar",
    "lightning.pytorch.profilers.SimpleProfiler": "llm_training_amd.runtime.profilers.SimpleProfiler",
    "lightning.pytorch.profilers.AdvancedProfiler": "llm_training_amd.runtime.profilers.AdvancedProfiler",
    "lightning.pytorch.profilers.PyTorchProfiler": "llm_training_amd.runtime.profilers.PyTorchProfiler",
}

SHORT_NAMES = {
    "HFTokenizer": "llm_training_amd.data.tokenizer.HFTokenizer",
    "LearningRateMonitor": "llm_training_amd.runtime.callbacks.LearningRateMonitor",
    "ModelCheckpoint": "llm_training_amd.runtime.callbacks.ModelCheckpoint",
    "EarlyStopping": "llm_training_amd.runtime.callbacks.EarlyStopping",
    "TrainingTimeEstimator": "llm_training_amd.runtime.callbacks.TrainingTimeEstimator",
    "OutputRedirection": "llm_training_amd.runtime.callbacks.OutputRedirection",
    "CSVLogger": "llm_training_amd.runtime.loggers.CSVLogger",
    "JSONLLogger": "llm_training_amd.runtime.loggers.JSONLLogger",
    "WandbLogger": "llm_training_amd.runtime.loggers.WandbLogger",
}


def normalize_path(path: str) -> str:
    if path in ALIASES:
        return ALIASES[path]
    if path in SHORT_NAMES:
        return SHORT_NAMES[path]
    if path.startswith("llm_training."):
        return "llm_training_amd." + path[len("llm_training."):]
    return path


def import_object(path: str):
    path = normalize_path(path)
    mod, _, name = path.rpartition(".")
    if not mod:
        raise ImportError(f"not an import path: {path!r}")
    try:
        m = importlib.import_module(mod)
        return getattr(m, name)
    except (ImportError, AttributeError):
        # nested attribute (e.g. package.Class.inner)
        parts = path.split(".")
        for i in range(len(parts) - 1, 0, -1):
            try:
                obj = importlib.import_module(".".join(parts[:i]))
            except ImportError:
                continue
            for p in parts[i:]:
                obj = getattr(obj, p)
            return obj
        raise
