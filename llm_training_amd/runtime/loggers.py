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
    """``metrics.csv`` with one header: a resumed run appends to the existing file under its header, and
    a metric that appears later (the first validation loss) rewrites the file once with the widened
    header instead of being dropped (Lightning's CSVLogger keeps every key as well)."""

    def __init__(self, save_dir: str = "logs", name: str = "run", version: str | None = None, **kw):
        super().__init__(save_dir, name, version)
        self._keys: list[str] | None = None
        self._w = None

    @property
    def path(self) -> str:
        return os.path.join(self.log_dir, "metrics.csv")

    def _open(self, keys: list[str]):
        """(Re)open for appending with header ``keys``; existing rows are rewritten under it if the file's
        header is narrower."""
        if self._f is not None:
            self._f.close()
        old_keys, rows = [], []
        if os.path.exists(self.path) and os.path.getsize(self.path) > 0:
            with open(self.path, newline="") as f:
                r = csv.DictReader(f)
                old_keys = list(r.fieldnames or [])
                if any(k not in old_keys for k in keys):
                    rows = list(r)
        merged = old_keys + [k for k in keys if k not in old_keys]
        if rows or not old_keys:
            with open(self.path, "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=merged)
                w.writeheader()
                w.writerows(rows)
        self._keys = merged
        self._f = open(self.path, "a", newline="")
        self._w = csv.DictWriter(self._f, fieldnames=self._keys)

    def log_metrics(self, metrics: dict, step: int):
        row = {"step": step, **metrics}
        if self._w is None:
            os.makedirs(self.log_dir, exist_ok=True)
            self._open(list(row))
        elif any(k not in self._keys for k in row):
            self._f.flush()
            self._open(self._keys + [k for k in row if k not in self._keys])
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
