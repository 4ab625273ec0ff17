"""Training callbacks with the reference's names and knobs.

Reference: src/llm_training/lightning/callbacks/ — ModelCheckpoint (model_checkpoint.py:13-18, plus
Lightning's every_n_train_steps / save_top_k / save_on_train_epoch_end), OutputRedirection
(output_redirection.py:16-101), SaveConfigCallback (save_config_callback.py:14-49: resolved YAML +
world size + SLURM env, config stored in every checkpoint), TQDMProgressBar (tqdm_progress.py:6-11),
TrainingTimeEstimator (training_time_estimator.py:12-83), ExtraConfig (extra_config.py:27-45) and
Lightning's LearningRateMonitor.
"""
from __future__ import annotations

import io
import json
import logging
import math
import os
import re
import shutil
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist
import yaml

logger = logging.getLogger("llm_training")


class Callback:
    pass


class LearningRateMonitor(Callback):
    """Lightning's LearningRateMonitor keys on top of the trainer's own ``lr``: ``lr-<Optimizer>`` (e.g.
    ``lr-AdamW``) and, with ``log_momentum``, ``lr-<Optimizer>-momentum`` (Adam beta1), logged every step
    (``logging_interval: step`` or None) or once per epoch (``epoch``) through the trainer's buffered
    metrics (host values: no device sync)."""

    def __init__(self, logging_interval: str | None = "step", log_momentum: bool = False,
                 log_weight_decay: bool = False, **kw):
        if logging_interval not in (None, "step", "epoch"):
            raise ValueError(f"LearningRateMonitor: logging_interval must be 'step', 'epoch' or None, "
                             f"got {logging_interval!r}")
        self.logging_interval = logging_interval
        self.log_momentum = log_momentum
        self.log_weight_decay = log_weight_decay

    def _values(self, trainer) -> dict[str, float]:
        name = getattr(trainer, "optimizer_name", "AdamW")
        eng = getattr(trainer, "engine", None)
        out = {f"lr-{name}": float(trainer.last_lr)}  # the rate the optimizer step just used
        if self.log_momentum and eng is not None:
            grp = eng.units[0].opt.param_groups[0] if eng.units and eng.units[0].opt is not None else {}
            mom = grp.get("momentum", grp["betas"][0] if "betas" in grp else eng.betas[0])
            out[f"lr-{name}-momentum"] = float(mom)
        if self.log_weight_decay and eng is not None:
            out[f"lr-{name}-weight_decay"] = float(eng.weight_decay)
        return out

    def on_step_metrics(self, trainer, lm):
        if self.logging_interval != "epoch":
            trainer.add_step_metrics(self._values(trainer))

    def on_train_epoch_end(self, trainer, lm):
        if self.logging_interval == "epoch":
            trainer.add_step_metrics(self._values(trainer))
            trainer._flush_logs(force=True)


class ModelCheckpoint(Callback):
    """Lightning ModelCheckpoint surface (reference model_checkpoint.py:13-18): every_n_train_steps /
    epoch-end cadence, ``save_top_k`` (the newest k, or the best k by ``monitor`` / ``mode``),
    ``save_last`` (``last.ckpt`` symlink), ``async_save`` (shard files written on a background thread).

    Old checkpoints are deleted and ``last.ckpt`` is moved only once the NEW checkpoint is complete on
    every rank: with async writes that happens at the start of the next save (or at fit end), after
    the pending writes are joined, a barrier, and ``is_complete`` — a crash mid-write always leaves the
    previous complete checkpoint in place."""

    def __init__(self, dirpath: str | None = None, filename: str | None = None, every_n_train_steps: int | None = None,
                 save_on_train_epoch_end: bool | None = None, save_top_k: int = 1, save_last: bool | None = None,
                 monitor: str | None = None, mode: str = "min", async_save: bool = False, **kw):
        if mode not in ("min", "max"):
            raise ValueError(f"ModelCheckpoint mode must be 'min' or 'max', got {mode!r}")
        self.dirpath = dirpath
        self.async_save = async_save  # write the shard files on a background thread
        self.filename = filename or "epoch={epoch}-step={step}"
        self.every_n_train_steps = every_n_train_steps
        self.save_on_train_epoch_end = save_on_train_epoch_end
        self.save_top_k = save_top_k
        self.save_last = save_last
        self.monitor = monitor
        self.mode = mode
        self.saved: list[str] = []              # complete checkpoints kept, oldest first
        self.scores: dict[str, float] = {}      # monitored value of each kept checkpoint
        self._pending: str | None = None        # saved, not yet known complete on every rank

    def _dir(self, trainer) -> str:
        # reference: <log_dir>/checkpoints when logging to a run directory (model_checkpoint.py:13-18)
        return self.dirpath or os.path.join(trainer.log_dir, "checkpoints")

    def _score(self, trainer) -> float | None:
        if self.monitor is None:
            return None
        trainer._flush_logs(force=True)  # the step's metrics, DP-averaged (one host sync per save)
        v = trainer.last_metrics.get(self.monitor)
        if v is None or v != v:
            logger.warning("ModelCheckpoint: monitored metric %r not available at step %d; the checkpoint is "
                           "kept but not ranked", self.monitor, trainer.global_step)
            return None
        return float(v)

    def _save(self, trainer):
        if self.save_top_k == 0:
            return
        name = self.filename.format(epoch=trainer.state.epoch, step=trainer.global_step) + ".ckpt"
        path = os.path.join(self._dir(trainer), name)
        if path in self.saved or path == self._pending:
            return
        self.finalize(trainer)  # the previous save is complete everywhere before anything is removed
        score = self._score(trainer)
        trainer.save_checkpoint(path, async_write=self.async_save)
        if score is not None:
            self.scores[path] = score
        self._pending = path
        if not self.async_save:
            self.finalize(trainer)

    def finalize(self, trainer):
        """Promote the pending checkpoint once it is complete on every rank: rotate old ones, move
        ``last.ckpt``."""
        path = self._pending
        if path is None:
            return
        from ..ckpt.checkpoint import is_complete, wait_for_pending_saves
        err = None
        try:
            wait_for_pending_saves()
        except Exception as e:  # noqa: BLE001 - re-raised below on every rank
            err = e
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            # a background write that failed on one rank fails the save on every rank (instead of the
            # others waiting in the barrier for a rank that has already raised)
            dev = getattr(trainer, "device", None)
            flag = torch.tensor([1.0 if err is not None else 0.0],
                                device=dev if dev is not None and dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(flag)
            if err is None and float(flag.item()) > 0:
                err = RuntimeError(f"checkpoint {path}: a background write failed on another rank")
        self._pending = None
        if err is not None:
            raise err
        if not is_complete(path):
            logger.error("checkpoint %s is incomplete; keeping the previous checkpoints", path)
            return
        self.saved.append(path)
        for old in self._to_remove():
            self.saved.remove(old)
            self.scores.pop(old, None)
            if trainer.is_global_zero:
                _remove_checkpoint(old)
        if self.save_last and trainer.is_global_zero:
            link = os.path.join(self._dir(trainer), "last.ckpt")
            try:
                if os.path.islink(link) or os.path.exists(link):
                    os.remove(link)
                os.symlink(os.path.basename(path), link)
            except OSError:
                pass

    def _to_remove(self) -> list[str]:
        k = self.save_top_k
        if k < 0 or len(self.saved) <= k:
            return []
        if self.monitor is None:
            return self.saved[:len(self.saved) - k]
        # best k by the monitored value; unranked checkpoints go first, ties keep the newer one
        sign = 1.0 if self.mode == "min" else -1.0
        order = sorted(range(len(self.saved)), key=lambda i: (
            self.saved[i] not in self.scores, sign * self.scores.get(self.saved[i], 0.0), -i))
        keep = {self.saved[i] for i in order[:k]}
        return [p for p in self.saved if p not in keep]

    def on_train_batch_end(self, trainer, lm, outputs, batch, batch_idx):
        n = self.every_n_train_steps
        if n and trainer.global_step > 0 and trainer.global_step % n == 0:
            self._save(trainer)

    def on_train_epoch_end(self, trainer, lm):
        if self.save_on_train_epoch_end or (self.save_on_train_epoch_end is None and not self.every_n_train_steps):
            self._save(trainer)

    def on_fit_end(self, trainer, lm):
        self.finalize(trainer)


class EarlyStopping(Callback):
    """Lightning's EarlyStopping: stop when ``monitor`` has not improved by more than ``min_delta`` for
    ``patience`` consecutive checks (validation ends, or training epoch ends with
    ``check_on_train_epoch_end``). ``check_finite`` stops on a NaN / inf value, ``stopping_threshold``
    once the value is good enough, ``divergence_threshold`` once it is hopeless. The stop is a request
    (``trainer.should_stop``) that ``min_steps`` / ``min_epochs`` can defer; the counters are saved in
    checkpoints. Every rank reads the same DP-averaged metric, so every rank decides alike."""

    def __init__(self, monitor: str, min_delta: float = 0.0, patience: int = 3, verbose: bool = False,
                 mode: str = "min", strict: bool = True, check_finite: bool = True,
                 stopping_threshold: float | None = None, divergence_threshold: float | None = None,
                 check_on_train_epoch_end: bool | None = None, log_rank_zero_only: bool = False):
        if mode not in ("min", "max"):
            raise ValueError(f"EarlyStopping mode must be 'min' or 'max', got {mode!r}")
        self.monitor, self.patience, self.verbose, self.mode, self.strict = monitor, int(patience), verbose, mode, strict
        self.min_delta = abs(float(min_delta)) * (-1.0 if mode == "min" else 1.0)
        self.check_finite = check_finite
        self.stopping_threshold, self.divergence_threshold = stopping_threshold, divergence_threshold
        self.check_on_train_epoch_end = check_on_train_epoch_end
        self.wait_count = 0
        self.best_score = float("inf") if mode == "min" else -float("inf")
        self.stopped_epoch = 0
        self.stopping_reason: str | None = None

    def _better(self, a: float, b: float) -> bool:
        return a < b if self.mode == "min" else a > b

    def _check(self, trainer, metrics: dict):
        if self.monitor not in metrics:
            if self.strict:
                raise RuntimeError(f"EarlyStopping: monitored metric {self.monitor!r} is not available; have "
                                   f"{sorted(metrics)} (set strict=False to skip)")
            return
        cur = float(metrics[self.monitor])
        reason = None
        if self.check_finite and not math.isfinite(cur):
            reason = f"{self.monitor} = {cur} is not finite"
        elif self.stopping_threshold is not None and self._better(cur, self.stopping_threshold):
            reason = f"{self.monitor} = {cur:.6g} reached the stopping threshold {self.stopping_threshold}"
        elif self.divergence_threshold is not None and self._better(self.divergence_threshold, cur):
            reason = f"{self.monitor} = {cur:.6g} is past the divergence threshold {self.divergence_threshold}"
        elif self._better(cur - self.min_delta, self.best_score):
            self.best_score, self.wait_count = cur, 0
            if self.verbose:
                logger.info("EarlyStopping: %s improved to %.6g", self.monitor, cur)
        else:
            self.wait_count += 1
            if self.wait_count >= self.patience:
                reason = (f"{self.monitor} did not improve by more than {abs(self.min_delta)} in the last "
                          f"{self.wait_count} checks; best {self.best_score:.6g}")
        if reason is not None:
            self.stopping_reason = reason
            self.stopped_epoch = trainer.state.epoch
            trainer.should_stop = True
            logger.info("EarlyStopping at step %d: %s", trainer.global_step, reason)

    def on_validation_end(self, trainer, lm, metrics: dict):
        if not self.check_on_train_epoch_end:
            self._check(trainer, metrics)

    def on_train_epoch_end(self, trainer, lm):
        if self.check_on_train_epoch_end:
            trainer._flush_logs(force=True)
            self._check(trainer, trainer.last_metrics)

    def state_dict(self) -> dict:
        return {"wait_count": self.wait_count, "best_score": self.best_score, "stopped_epoch": self.stopped_epoch,
                "patience": self.patience}

    def load_state_dict(self, st: dict):
        self.wait_count = int(st["wait_count"])
        self.best_score = float(st["best_score"])
        self.stopped_epoch = int(st.get("stopped_epoch", 0))


def _remove_checkpoint(path: str):
    if os.path.isdir(path) and not os.path.islink(path):
        shutil.rmtree(path, ignore_errors=True)
    elif os.path.exists(path):
        os.remove(path)


class SaveConfigCallback(Callback):
    """Saves the resolved config (+ world size / SLURM env) and embeds it in every checkpoint."""

    def __init__(self, config: dict | None = None, config_filename: str = "config.yaml", overwrite: bool = True):
        self.config = config or {}
        self.config_filename = config_filename
        self.overwrite = overwrite

    def setup(self, trainer, lm, stage):
        cfg = dict(self.config)
        cfg["world_size"] = trainer.world_size if trainer.pc else int(os.environ.get("WORLD_SIZE", 1))
        slurm = {k: v for k, v in os.environ.items() if k.startswith("SLURM_")}
        if slurm:
            cfg["slurm"] = slurm
        trainer.config_dict = cfg
        if trainer.is_global_zero:
            os.makedirs(trainer.log_dir, exist_ok=True)
            p = os.path.join(trainer.log_dir, self.config_filename)
            if self.overwrite or not os.path.exists(p):
                with open(p, "w") as f:
                    yaml.safe_dump(_plain(cfg), f, sort_keys=False)


def _plain(x):
    if isinstance(x, dict):
        return {str(k): _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    if isinstance(x, (str, int, float, bool)) or x is None:
        return x
    return str(x)


class _Tee(io.TextIOBase):
    def __init__(self, stream, buf):
        self.stream, self.buf = stream, buf

    def write(self, s):
        self.stream.write(s)
        self.buf.write(s)
        return len(s)

    def flush(self):
        self.stream.flush()
        self.buf.flush()


class OutputRedirection(Callback):
    """Tee stdout/stderr into ``<log_dir>/<log_file_name>.log`` (file name agreed from rank 0)."""

    def __init__(self, log_file_name: str = "{index}-{version}", redirect_stdout: bool = True,
                 redirect_stderr: bool = True, enabled: bool = True):
        self.log_file_name, self.redirect_stdout, self.redirect_stderr, self.enabled = \
            log_file_name, redirect_stdout, redirect_stderr, enabled
        self._f = None
        self._orig = (sys.stdout, sys.stderr)

    def setup(self, trainer, lm, stage):
        if not self.enabled:
            return
        d = trainer.log_dir
        name = [None]
        if trainer.is_global_zero:
            os.makedirs(d, exist_ok=True)
            idx = len([p for p in os.listdir(d) if p.endswith(".log")])
            name[0] = self.log_file_name.format(index=idx, version=time.strftime("%Y%m%d-%H%M%S"))
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.broadcast_object_list(name, src=0)
        rank = trainer.pc.rank if trainer.pc else 0
        fname = os.path.join(d, name[0] + (f".rank{rank}" if rank else "") + ".log")
        os.makedirs(d, exist_ok=True)
        self._orig = (sys.stdout, sys.stderr)
        self._f = open(fname, "a", buffering=1)
        if self.redirect_stdout:
            sys.stdout = _Tee(self._orig[0], self._f)
        if self.redirect_stderr:
            sys.stderr = _Tee(self._orig[1], self._f)
        self._handlers = []
        for h in logging.getLogger("llm_training").handlers:
            if isinstance(h, logging.StreamHandler) and not isinstance(h, logging.FileHandler):
                self._handlers.append((h, h.stream))
                h.setStream(sys.stderr)

    def on_fit_end(self, trainer, lm):
        self.teardown(trainer, lm)

    def teardown(self, trainer=None, lm=None):
        """Undo the redirection (also after a failed fit): streams, logging handlers, the log file."""
        if self._f:
            sys.stdout, sys.stderr = self._orig
            for h, old in getattr(self, "_handlers", []):
                h.setStream(old)
            self._handlers = []
            self._f.close()
            self._f = None


class TQDMProgressBar(Callback):
    def __init__(self, refresh_rate: int = 1, **kw):
        self.refresh_rate = refresh_rate
        self.bar = None

    def on_fit_start(self, trainer, lm):
        if not trainer.is_global_zero:
            return
        try:
            from tqdm.auto import tqdm
        except ImportError:
            return
        total = trainer.estimated_stepping_batches()
        # restarts begin at the resumed step (reference tqdm_progress.py:6-11)
        self.bar = tqdm(total=total, initial=trainer.global_step, dynamic_ncols=True)

    def on_train_batch_end(self, trainer, lm, outputs, batch, batch_idx):
        if self.bar is not None:
            self.bar.update(1)
            if trainer.last_metrics:
                loss = trainer.last_metrics.get("Loss/Train/Step")
                if loss is not None:
                    self.bar.set_postfix(loss=f"{loss:.4f}")

    def on_fit_end(self, trainer, lm):
        if self.bar is not None:
            self.bar.close()


class TrainingTimeEstimator(Callback):
    """Time steps [num_warmup_steps, num_test_steps), stop, print steps/s, tokens/s and ETA."""

    def __init__(self, num_test_steps: int, num_warmup_steps: int = 2, enable_checkpointing: bool = False):
        self.num_test_steps, self.num_warmup_steps = num_test_steps, num_warmup_steps
        self.enable_checkpointing = enable_checkpointing
        self.t0 = None
        self.result: dict | None = None

    def setup(self, trainer, lm, stage):
        if not self.enable_checkpointing:
            trainer.callbacks = [c for c in trainer.callbacks if not isinstance(c, ModelCheckpoint)]

    def on_train_batch_end(self, trainer, lm, outputs, batch, batch_idx):
        step = trainer.global_step
        if step == self.num_warmup_steps:
            if trainer.device.type == "cuda":
                torch.cuda.synchronize()
            self.t0 = time.perf_counter()
            self.tok0 = trainer.state.consumed.get("Consumed Tokens", 0)
        if step == self.num_test_steps:
            if trainer.device.type == "cuda":
                torch.cuda.synchronize()
            el = time.perf_counter() - self.t0
            n = self.num_test_steps - self.num_warmup_steps
            total = trainer.estimated_stepping_batches()
            sps = n / el
            self.result = {"steps_per_sec": sps, "sec_per_step": el / n,
                           "eta_hours": (total - step) / sps / 3600, "total_steps": total}
            if trainer.is_global_zero:
                logger.info("TrainingTimeEstimator: %s", json.dumps(self.result))
            trainer.should_stop = True


class ExtraConfig(Callback):
    """``float32_matmul_precision`` and ``logging_level`` (reference extra_config.py:27-38)."""

    def __init__(self, float32_matmul_precision: str | None = None, logging_level: str | int = "INFO"):
        self.fp32 = float32_matmul_precision
        self.level = logging_level
        self.apply()

    def apply(self):
        if self.fp32:
            torch.set_float32_matmul_precision(self.fp32)
        lvl = self.level if isinstance(self.level, int) else getattr(logging, str(self.level).upper(), logging.INFO)
        logging.getLogger("llm_training").setLevel(lvl)
