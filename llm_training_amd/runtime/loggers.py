"""Metric loggers. JSONL / CSV always work; ``WandbLogger`` keeps the reference's directory layout
(``save_dir/project/name``, src/llm_training/lightning/loggers/wandb.py:49-72) and streams to W&B when the
``wandb`` package exists (it is not installed in this image), otherwise to a local JSONL file."""
from __future__ import annotations

import csv
import json
import logging
import os
import time

logger = logging.getLogger("llm_training")


class JSONLLogger:
    def __init__(self, save_dir: str = "logs", name: str = "run", version: str | None = None, **kw):
        self.save_dir, self.name = save_dir, name
        self.version = version
        self._f = None

    @property
    def log_dir(self):
        return os.path.join(self.save_dir, self.name) + (f"/{self.version}" if self.version else "")

    def setup(self, trainer):
        pass

    def log_metrics(self, metrics: dict, step: int):
        if self._f is None:
            os.makedirs(self.log_dir, exist_ok=True)
            self._f = open(os.path.join(self.log_dir, "metrics.jsonl"), "a", buffering=1)
        self._f.write(json.dumps({"step": step, "time": time.time(), **metrics}) + "\n")

    def log_hyperparams(self, params: dict):
        os.makedirs(self.log_dir, exist_ok=True)
        with open(os.path.join(self.log_dir, "hparams.json"), "w") as f:
            json.dump(params, f, default=str, indent=1)

    def finalize(self, status: str):
        if self._f:
            self._f.close()
            self._f = None


class CSVLogger(JSONLLogger):
    def __init__(self, save_dir: str = "logs", name: str = "run", version: str | None = None, **kw):
        super().__init__(save_dir, name, version)
        self._keys = None
        self._w = None

    def log_metrics(self, metrics: dict, step: int):
        row = {"step": step, **metrics}
        if self._w is None:
            os.makedirs(self.log_dir, exist_ok=True)
            self._f = open(os.path.join(self.log_dir, "metrics.csv"), "a", newline="")
            self._keys = list(row)
            self._w = csv.DictWriter(self._f, fieldnames=self._keys, extrasaction="ignore")
            self._w.writeheader()
        self._w.writerow(row)
        self._f.flush()


class WandbLogger(JSONLLogger):
    def __init__(self, name: str | None = None, project: str = "llm-training", save_dir: str = "logs",
                 job_type: str | None = None, save_code: bool = False, offline: bool = False, **kw):
        super().__init__(save_dir, name or "run")
        self.project, self.job_type, self.save_code, self.offline = project, job_type, save_code, offline
        self.kw = kw
        self._run = None
        try:
            import wandb  # noqa: F401
            self._wandb = wandb
        except ImportError:
            self._wandb = None

    @property
    def log_dir(self):
        return os.path.join(self.save_dir, self.project, self.name)

    def setup(self, trainer):
        if self._wandb is not None and trainer.is_global_zero:
            os.makedirs(self.log_dir, exist_ok=True)
            self._run = self._wandb.init(project=self.project, name=self.name, dir=self.log_dir,
                                         job_type=self.job_type, mode="offline" if self.offline else None,
                                         config=trainer.config_dict)

    def log_metrics(self, metrics: dict, step: int):
        if self._run is not None:
            self._run.log(metrics, step=step)
        super().log_metrics(metrics, step)

    def finalize(self, status: str):
        if self._run is not None:
            self._run.finish()
        super().finalize(status)
