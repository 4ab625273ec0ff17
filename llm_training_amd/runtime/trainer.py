"""The training loop (replaces Lightning's Trainer for this framework).

Reference behaviour reproduced: Lightning ``Trainer.fit`` as driven by the reference CLI
(src/llm_training/lightning/cli/cli.py, trainer.py:4-11), gradient accumulation with loss averaging
(SURVEY Q13), ``gradient_clip_val`` (norm clipping, every example sets 1.0), step-interval LR
schedulers with auto-injected ``num_total_steps`` (base_lm.py:269-288), validation every
``val_check_interval``, checkpoint callbacks, resume from ``ckpt_path`` with the data loader skipping
consumed batches (data/resumable_dataloader.py) and grad-norm logging (base_lm.py:290-300).

MI355X-specific choices: one process per GPU, weights built directly on the device in bf16 (TP-aware),
one fused-AdamW launch per FSDP unit, device-side clipping (no host sync), metrics kept on device and
read only every ``log_every_n_steps``.
"""
from __future__ import annotations

import logging
import math
import os
import time
from typing import Any

import torch
import torch.distributed as dist

from ..ops.native import check_kernel_errors
from ..optim import resolve_optimizer
from ..parallel import debug as collective_debug
from ..parallel.context import ParallelContext, init_distributed
from ..parallel.engine import DataParallelEngine, freeze_modules
from .monitor import (StallWatchdog, StepProfiler, ThroughputMeter, find_last_checkpoint, model_flops_per_token,
                      trace_range,
                      record_failure)
from .strategies import Strategy, resolve_strategy

logger = logging.getLogger("llm_training")
_log = logger  # for Trainer.__init__, whose `logger` argument shadows the module logger

# precision -> (parameter / compute dtype, gradient accumulation + reduction dtype)
#  * bf16-true : bf16 params, bf16 gradients, fp32 master weights + Adam state (reference bf16-true with
#                use_master_weights, fsdp2_strategy.py:249-250)
#  * bf16-mixed: bf16 compute copies, fp32 gradients (accumulated and reduced in fp32) on fp32 masters —
#                the numerics of autocast over fp32 parameters (fsdp2_precision.py:55-90,106-117)
#  * 32-true   : fp32 everywhere; on the GPU the torch ops run (the HIP kernels are bf16 MFMA kernels)
#  * 16-true / 16-mixed: fp16 params (fp16 / fp32 gradients) with a dynamic loss scaler (reference
#                FSDP2Precision GradScaler, fsdp2_precision.py:19-21,55-96,129-163, without its Q10 bug):
#                the loss is scaled before backward, gradients are unscaled inside the clip scale, a step
#                whose gradient norm is not finite is skipped and halves the scale, 2000 good steps
#                double it. fp16 tensors run the torch ops (the HIP kernels are bf16 MFMA kernels: bf16
#                runs at the same rate on MI355X with fp32's exponent range and needs no scaler).
PRECISIONS = {"bf16-true": (torch.bfloat16, None), "bf16": (torch.bfloat16, None),
              "bf16-mixed": (torch.bfloat16, torch.float32), "32-true": (torch.float32, None),
              "32": (torch.float32, None), 32: (torch.float32, None), "64-true": None,
              "16-true": (torch.float16, None), "16": (torch.float16, None), 16: (torch.float16, None),
              "16-mixed": (torch.float16, torch.float32), "transformer-engine": None}
FP16 = {"16-true", "16", 16, "16-mixed"}


class LossScaler:
    """Dynamic loss scale for fp16 (torch.amp.GradScaler semantics: init 2**16, x2 every 2000 finite
    steps, x0.5 on an overflow, whose step is skipped)."""

    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000):
        self.scale, self.growth_factor, self.backoff_factor = float(init_scale), growth_factor, backoff_factor
        self.growth_interval, self.good_steps, self.skipped = int(growth_interval), 0, 0

    def update(self, finite: bool) -> bool:
        if finite:
            self.good_steps += 1
            if self.good_steps >= self.growth_interval:
                self.scale *= self.growth_factor
                self.good_steps = 0
        else:
            self.scale *= self.backoff_factor
            self.good_steps = 0
            self.skipped += 1
        return finite

    def state_dict(self):
        return {"scale": self.scale, "good_steps": self.good_steps, "skipped": self.skipped}

    def load_state_dict(self, st):
        self.scale, self.good_steps, self.skipped = float(st["scale"]), int(st["good_steps"]), int(st["skipped"])
# Lightning Trainer arguments that have nothing to act on in this framework, so accepting them is exactly
# Lightning's behaviour here: cuDNN autotuning (no convolutions), BatchNorm sync (none in these models),
# the model-summary printout flag (a summary is logged at setup), inference vs no-grad validation (same
# numbers), dataloader reloading (the loaders are rebuilt every epoch), metric placement, and the
# test / predict loops (not part of `fit`). Everything else Lightning offers is implemented below or
# raises; a misspelled argument raises with a suggestion, as jsonargparse would.
IGNORED_TRAINER_ARGS = {"benchmark", "sync_batchnorm", "reload_dataloaders_every_n_epochs", "enable_model_summary",
                        "inference_mode", "limit_test_batches", "limit_predict_batches", "move_metrics_to_cpu"}


def parse_max_time(v: Any) -> float | None:
    """Lightning's ``max_time``: "DD:HH:MM:SS", a dict of timedelta fields, or a timedelta -> seconds."""
    import datetime
    if v is None:
        return None
    if isinstance(v, datetime.timedelta):
        return v.total_seconds()
    if isinstance(v, dict):
        return datetime.timedelta(**v).total_seconds()
    if isinstance(v, str):
        parts = v.split(":")
        if len(parts) != 4:
            raise ValueError(f"max_time {v!r}: expected DD:HH:MM:SS")
        d, h, m, sec = (float(x) for x in parts)
        return datetime.timedelta(days=d, hours=h, minutes=m, seconds=sec).total_seconds()
    raise TypeError(f"max_time must be a DD:HH:MM:SS string, a dict or a timedelta, got {type(v).__name__}")


class TrainerState:
    def __init__(self):
        self.global_step = 0
        self.epoch = 0
        self.batch_idx = 0  # batches consumed in the current epoch
        self.consumed: dict[str, float] = {}

    def state_dict(self):
        return {"global_step": self.global_step, "epoch": self.epoch, "batch_idx": self.batch_idx,
                "consumed": {k: float(v) for k, v in self.consumed.items()}}

    def load_state_dict(self, st):
        self.global_step = int(st["global_step"])
        self.epoch = int(st["epoch"])
        self.batch_idx = int(st["batch_idx"])
        self.consumed = dict(st.get("consumed", {}))


class Trainer:
    def __init__(self, strategy: Any = None, precision: Any = "bf16-true", logger: Any = None,
                 callbacks: list | None = None, max_epochs: int | None = None, max_steps: int = -1,
                 accumulate_grad_batches: int = 1, gradient_clip_val: float | None = None,
                 gradient_clip_algorithm: str = "norm", val_check_interval: Any = None,
                 check_val_every_n_epoch: int | None = 1, log_every_n_steps: int = 10, num_nodes: int = 1,
                 devices: Any = "auto", accelerator: Any = "auto", limit_train_batches: Any = None,
                 limit_val_batches: Any = None, enable_checkpointing: bool = True, enable_progress_bar: bool = True,
                 default_root_dir: str = "logs", num_sanity_val_steps: int = 2, seed: int | None = None,
                 deterministic: bool = False, benchmark: Any = None, gemm_tuning: str | None = None,
                 max_time: Any = None, fast_dev_run: Any = False, overfit_batches: Any = 0.0,
                 min_epochs: int | None = None, min_steps: int | None = None, profiler: Any = None,
                 detect_anomaly: bool = False, barebones: bool = False, plugins: Any = None,
                 use_distributed_sampler: bool = True, enable_model_summary: bool = True, **unused):
        self.strategy: Strategy = resolve_strategy(strategy)
        # devices / num_nodes decide how many ranks llm_training_amd.launch starts; inside a rank the
        # accelerator picks the device type (cpu -> gloo ranks)
        self.devices, self.accelerator = devices, accelerator
        self.gemm_tuning = gemm_tuning  # runtime/gemm_tuning.py modes; applied in setup()
        self.deterministic = bool(deterministic)
        self.precision = precision
        self.loggers = [] if logger in (None, False) else (list(logger) if isinstance(logger, list) else [logger])
        self.callbacks = list(callbacks or [])
        self.max_epochs = max_epochs
        self.max_steps = max_steps if max_steps is not None else -1
        self.accumulate_grad_batches = int(accumulate_grad_batches)
        self.gradient_clip_val = gradient_clip_val
        if gradient_clip_algorithm != "norm":
            raise ValueError("only norm clipping is supported")
        self.val_check_interval = val_check_interval
        self.check_val_every_n_epoch = check_val_every_n_epoch
        self.max_time = parse_max_time(max_time)  # seconds of fit time (Lightning Timer), None = unlimited
        self._fit_t0 = 0.0
        self.log_every_n_steps = max(1, int(log_every_n_steps))
        self.num_nodes = num_nodes
        self.limit_train_batches = limit_train_batches
        self.limit_val_batches = limit_val_batches
        self.num_sanity_val_steps = int(num_sanity_val_steps)  # Lightning: -1 = the whole validation set
        self.enable_checkpointing = enable_checkpointing
        self.enable_progress_bar = enable_progress_bar
        self.default_root_dir = default_root_dir
        self.seed = seed
        self.state = TrainerState()
        self.should_stop = False
        self.unused = unused
        bad = sorted(k for k in unused if k not in IGNORED_TRAINER_ARGS)
        if bad:
            import difflib
            import inspect
            known = sorted(set(inspect.signature(Trainer.__init__).parameters) - {"self", "unused"}
                           | IGNORED_TRAINER_ARGS)
            hint = {k: difflib.get_close_matches(k, known, n=1) for k in bad}
            raise TypeError("Trainer got unknown argument(s): " + ", ".join(
                f"{k!r}" + (f" (did you mean {h[0]!r}?)" if h else "") for k, h in hint.items()))
        if unused:
            _log.info("Trainer: arguments with nothing to act on in this framework: %s", sorted(unused))
        if plugins:
            raise ValueError("Trainer(plugins=...) is not supported: precision and cluster environments are "
                             "built in (precision=..., the launcher / torchrun / srun environment)")
        self.min_epochs = int(min_epochs) if min_epochs is not None else None
        self.min_steps = int(min_steps) if min_steps is not None else None
        self.detect_anomaly = bool(detect_anomaly)
        self.use_distributed_sampler = bool(use_distributed_sampler)
        self.enable_model_summary = bool(enable_model_summary) and not barebones
        self.fit_profiler = make_fit_profiler(profiler)
        # Lightning debugging flags (trainer/connectors: _init_debugging_flags)
        if fast_dev_run is True:
            fast_dev_run = 1
        self.fast_dev_run = int(fast_dev_run or 0)
        if self.fast_dev_run < 0:
            raise ValueError(f"fast_dev_run must be a bool or a non-negative int, got {fast_dev_run!r}")
        self.overfit_batches = overfit_batches if overfit_batches else 0
        if self.fast_dev_run:
            # N training batches, then N validation batches; no sanity check, loggers, checkpoints or time limit
            n = self.fast_dev_run
            self.max_steps, self.max_epochs, self.max_time = n, 1, None
            self.limit_train_batches, self.limit_val_batches = n * self.accumulate_grad_batches, n
            self.val_check_interval, self.check_val_every_n_epoch, self.num_sanity_val_steps = 1.0, 1, 0
            self.loggers, self.enable_checkpointing = [], False
            _log.info("fast_dev_run=%d: %d training + %d validation batch(es); loggers and checkpoints off", n, n, n)
        elif self.overfit_batches:
            # the same first batches every epoch (no shuffling), validation limited alike
            self.limit_train_batches = self.overfit_batches
            self.limit_val_batches = self.overfit_batches
        if barebones:
            # Lightning barebones: no logging, progress bar, checkpointing, summary or profiler
            if self.fit_profiler is not None:
                raise ValueError("barebones=True cannot be combined with a profiler")
            self.loggers, self.enable_checkpointing, self.enable_progress_bar = [], False, False
        if precision not in PRECISIONS:
            raise ValueError(f"unknown precision {precision!r}; use one of bf16-true, bf16-mixed, 32-true")
        if PRECISIONS[precision] is None:
            raise ValueError(f"precision {precision!r} is not supported; use bf16-true, bf16-mixed, 16-true, "
                             "16-mixed or 32-true")
        self.scaler = LossScaler() if precision in FP16 else None
        self.pc: ParallelContext | None = None
        self.engine: DataParallelEngine | None = None
        self.lm = None
        self.datamodule = None
        self.scheduler = None
        self.last_lr = float("nan")
        self.config_dict: dict | None = None
        self._log_buffer: list[tuple[int, dict]] = []
        self.last_metrics: dict[str, float] = {}
        self.step_times: list[float] = []
        self.meter: ThroughputMeter | None = None
        self.profiler: StepProfiler | None = None
        self.watchdog: StallWatchdog | None = None
        self.collectives = None
        self._fpt: dict[int, float] = {}

    # ------------------------------------------------------------------ properties used by callbacks
    @property
    def global_step(self):
        return self.state.global_step

    @property
    def is_global_zero(self):
        return self.pc is None or self.pc.rank == 0

    @property
    def world_size(self):
        return self.pc.world_size if self.pc else 1

    @property
    def log_dir(self) -> str:
        for lg in self.loggers:
            d = getattr(lg, "log_dir", None)
            if d:
                return d
        return self.default_root_dir

    @property
    def param_dtype(self):
        pd = getattr(self.strategy, "param_dtype", None)  # FSDP2 mp_policy.param_dtype wins
        return getattr(torch, pd) if pd else PRECISIONS[self.precision][0]

    @property
    def grad_dtype(self):
        pd = getattr(self.strategy, "param_dtype", None)
        if pd and PRECISIONS[self.precision][0] != getattr(torch, pd):
            return None  # gradients in the parameter dtype (reduce dtype from mp_policy.reduce_dtype)
        return PRECISIONS[self.precision][1]

    # ------------------------------------------------------------------ setup
    def setup(self, lm, datamodule, ckpt_path: str | None = None):
        st = self.strategy
        rank, local, world, device = init_distributed(st.process_group_backend, st.timeout_minutes,
                                                      device_type="cpu" if self.accelerator == "cpu" else None)
        self.device = device
        self.run_meta = self.compute_path_meta(device)
        if self.gemm_tuning is not None:
            from .gemm_tuning import setup_gemm_tuning
            setup_gemm_tuning(self.gemm_tuning)
        self.pc = ParallelContext.create(st.data_parallel_size, st.tensor_parallel_size, device)
        seed = self.seed if self.seed is not None else 42
        if self.deterministic:
            # bitwise-reproducible steps: sort-based embedding backward (models/modules.py); every HIP
            # kernel already reduces in a fixed order (no float atomics in the backward)
            torch.use_deterministic_algorithms(True, warn_only=True)
            os.environ["LLMT_DETERMINISTIC"] = "1"
        # one generator stream per (dp, tp) rank: under TP + SP every random op (dropout masks, NEFTune
        # noise, attention-dropout seeds) acts on a sequence / head shard of its own, so the TP ranks of a
        # DP group must not share masks (tp 1 keeps seed + dp_rank)
        torch.manual_seed(seed + self.pc.dp_rank + 1_000_003 * self.pc.tp_rank)
        if ckpt_path == "last":
            ckpt_path = self.resolve_last_checkpoint()
        if not self.enable_checkpointing:
            from .callbacks import ModelCheckpoint
            dropped = [cb for cb in self.callbacks if isinstance(cb, ModelCheckpoint)]
            if dropped:
                logger.info("checkpointing off (%s): %d ModelCheckpoint callback(s) inactive",
                            "fast_dev_run" if self.fast_dev_run else "enable_checkpointing=False", len(dropped))
                self.callbacks = [cb for cb in self.callbacks if not isinstance(cb, ModelCheckpoint)]
        self.lm, self.datamodule = lm, datamodule
        for cb in self.callbacks:
            _call(cb, "setup", self, lm, "fit")
        self._prepare_data(datamodule, rank, local)
        datamodule.setup("fit")
        resuming = ckpt_path is not None
        lm.configure_model(self.pc, device, self.param_dtype, seed=seed, resuming=resuming)
        frozen = freeze_modules(lm.model, getattr(lm.config, "frozen_modules", None))
        if frozen:
            logger.info("frozen %d parameters", len(frozen))
        ospec = lm.optimizer_spec()
        hp = resolve_optimizer(ospec["name"], ospec["kwargs"])
        self.optimizer_name = str(ospec["name"]).rsplit(".", 1)[-1]
        self.base_lr = hp["lr"]
        rd = getattr(st, "grad_reduce_dtype", None)
        factory = None
        if hp["kind"] == "generic":
            cls, okw = hp["cls"], hp["kwargs"]
            factory = lambda params: cls(params, **okw)  # noqa: E731
            logger.info("optimizer %s runs generically over the flat fp32 master shards", hp["name"])
        self.engine = DataParallelEngine(lm.model, self.pc, st.zero_stage, lr=hp["lr"], betas=hp["betas"],
                                         eps=hp["eps"], weight_decay=hp["weight_decay"], optimizer_factory=factory,
                                         grad_dtype=self.grad_dtype,
                                         reduce_dtype=getattr(torch, rd) if rd else self.grad_dtype,
                                         reshard_after_forward=st.reshard_after_forward,
                                         overlap_comm=st.overlap_comm, **st.engine_kwargs())
        _call(lm, "on_engine_ready", self.engine)  # e.g. DPO shards its frozen reference model (ZeRO-3)
        if self.enable_model_summary and self.pc.rank == 0:
            log_model_summary(lm.model)
        self.scheduler = lm.build_lr_scheduler(self.base_lr, self.estimated_stepping_batches())
        if ckpt_path:
            from ..ckpt.checkpoint import load_checkpoint
            load_checkpoint(self, ckpt_path)
        for lg in self.loggers:
            _call(lg, "setup", self)
            if self.pc.rank == 0:
                _call(lg, "log_hyperparams", {"run_meta": dict(self.run_meta)})
        self.meter = ThroughputMeter(self.pc.dp_size, device=device)
        self.profiler = StepProfiler(out_dir=self.log_dir, rank=self.pc.rank)
        self.watchdog = StallWatchdog(path=os.path.join(self.log_dir, f"stall_rank{self.pc.rank}.txt"))
        self.collectives = collective_debug.maybe_enable_from_env()

    def compute_path_meta(self, device: torch.device) -> dict:
        """Run metadata on the kernel path this precision takes on ``device``. The HIP kernels are bf16 MFMA
        kernels: ``precision: 32-true`` / ``16-*`` on a GPU runs the torch reference ops for every fused op
        (reference FSDP2Precision runs fp32 / fp16 through the same Liger / flash-attn kernels instead,
        fsdp2_precision.py:19-21,92-96), which is announced here once rather than left silent."""
        from ..ops.native import DIAG, check_probe_env, compute_path, llmt_env
        # wrong-result diagnostic probes are refused for training runs (unless the diagnostic library is
        # loaded on purpose), and every kernel / layout knob the run sees is recorded with it
        check_probe_env()
        path = compute_path(device.type, self.param_dtype)
        meta = {"device": device.type, "precision": str(self.precision), "compute_kernels": path,
                "llmt_env": llmt_env(), "native_lib": "diag" if DIAG else "production"}
        if device.type == "cuda" and path != "hip":
            logger.warning("precision %r on the GPU: the fused ops (attention, RMSNorm, SwiGLU, RoPE, loss, "
                           "AdamW) run the torch reference ops, not the bf16 HIP kernels (run_meta "
                           "compute_kernels=%s); use bf16-true or bf16-mixed for the kernel path",
                           self.precision, path)
        return meta

    @staticmethod
    def _prepare_data(datamodule, rank: int, local_rank: int):
        """Run ``prepare_data`` (download / tokenize into the cache) on one rank — local rank 0 of each
        node with ``prepare_data_per_node`` (node-local caches), else global rank 0 (shared file system)
        — while the others wait, so ``num_proc`` workers of one rank fill the cache instead of every
        rank mapping concurrently into the same files (reference: Lightning's prepare_data contract)."""
        per_node = bool(getattr(datamodule.config, "prepare_data_per_node", False))
        if (local_rank if per_node else rank) == 0:
            datamodule.prepare_data()
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.barrier()

    def resolve_last_checkpoint(self) -> str | None:
        """``ckpt_path: last``: newest complete checkpoint under the checkpoint directories (or None)."""
        from .callbacks import ModelCheckpoint
        roots = [cb.dirpath for cb in self.callbacks if isinstance(cb, ModelCheckpoint) and cb.dirpath]
        roots.append(self.default_root_dir)
        found = [c for c in (find_last_checkpoint(r) for r in roots) if c]
        if not found:
            logger.info("ckpt_path=last: no complete checkpoint under %s; starting from scratch", roots)
            return None
        from .monitor import checkpoint_step
        best = max(found, key=checkpoint_step)
        logger.info("ckpt_path=last: resuming from %s", best)
        return best

    def _dp(self) -> tuple[int, int]:
        """(rank, size) the loaders shard over: the data-parallel group, or (0, 1) with
        use_distributed_sampler=False (every rank iterates the whole dataset, as in Lightning)."""
        return (self.pc.dp_rank, self.pc.dp_size) if self.use_distributed_sampler else (0, 1)

    def train_loader(self):
        kw = {"shuffle": False} if self.overfit_batches else {}
        return self.datamodule.train_dataloader(*self._dp(), seed=(self.seed if self.seed is not None else 42),
                                                skip_batches=self.state.batch_idx, epoch=self.state.epoch, **kw)

    def num_batches_per_epoch(self) -> int:
        n = len(self.datamodule.train_dataloader(*self._dp()).batch_sampler)
        lim = self.limit_train_batches
        if lim is not None:
            n = min(n, int(lim) if (isinstance(lim, int) or float(lim) > 1) else int(n * float(lim)))
        return n

    def estimated_stepping_batches(self) -> int:
        per_epoch = max(1, self.num_batches_per_epoch() // self.accumulate_grad_batches)
        if self.max_steps is not None and self.max_steps > 0:
            return self.max_steps
        epochs = self.max_epochs if self.max_epochs is not None else 1
        return per_epoch * epochs

    # ------------------------------------------------------------------ loop
    def fit(self, lm, datamodule=None, ckpt_path: str | None = None):
        try:
            if self.fit_profiler is not None:
                with self.fit_profiler.session(self):
                    return self._fit(lm, datamodule, ckpt_path)
            return self._fit(lm, datamodule, ckpt_path)
        except Exception as e:
            rank = self.pc.rank if self.pc is not None else int(os.environ.get("RANK", "0"))
            record_failure(e, rank, self.log_dir)
            raise
        finally:
            if self.watchdog is not None:
                self.watchdog.close()
            for cb in self.callbacks:
                _call(cb, "teardown", self, lm)

    def _fit(self, lm, datamodule=None, ckpt_path: str | None = None):
        self._fit_t0 = time.monotonic()
        self.setup(lm, datamodule, ckpt_path)
        for cb in self.callbacks:
            _call(cb, "on_fit_start", self, lm)
        if self.num_sanity_val_steps != 0 and self.limit_val_batches not in (0, 0.0):
            # Lightning's sanity check: a few validation batches before the first training step, so a
            # broken validation path fails at once rather than after the first val_check_interval;
            # nothing is logged or kept
            self.validate(sanity=True)
        max_epochs = self.max_epochs if self.max_epochs is not None else (1 if self.max_steps <= 0 else 10 ** 9)
        if self.min_epochs is not None and self.max_epochs is None:
            max_epochs = max(max_epochs, self.min_epochs)
        lm.train()
        nbe = self.num_batches_per_epoch()
        self._hard_stop = False
        while self.state.epoch < max_epochs and not self._stopping():
            loader = self.train_loader()
            it = iter(loader)
            accum = self.accumulate_grad_batches
            while self.state.batch_idx + accum <= nbe and not self._stopping():
                with self._prof("get_train_batch"):
                    batches = [next(it) for _ in range(accum)]
                self.train_step(batches)  # advances batch_idx before the batch-end callbacks run
                if self.max_steps > 0 and self.state.global_step >= self.max_steps:
                    self.should_stop = self._hard_stop = True
                if self.max_time is not None and self._time_is_up():
                    self.should_stop = True
                if self._should_validate(nbe):
                    with self._prof("validation"):
                        self.validate()
            epoch_done = self.state.batch_idx + accum > nbe
            if epoch_done or self._stopping():
                # Lightning ends the epoch loop also when max_steps / max_time stop it early, so the
                # epoch-end hooks (ModelCheckpoint(save_on_train_epoch_end) among them) run; the counters
                # only advance for a completed epoch, so a resume continues mid-epoch
                for cb in self.callbacks:
                    _call(cb, "on_train_epoch_end", self, lm)
            if epoch_done:
                self.state.epoch += 1
                self.state.batch_idx = 0
        self._flush_logs(force=True)
        from ..ckpt.checkpoint import wait_for_pending_saves
        wait_for_pending_saves()
        for cb in self.callbacks:
            _call(cb, "on_fit_end", self, lm)
        for lg in self.loggers:
            _call(lg, "finalize", "success")
        return self

    def _stopping(self) -> bool:
        """max_steps ends the run at once; any other stop request (max_time, EarlyStopping, a callback
        setting ``should_stop``) waits until ``min_steps`` / ``min_epochs`` are met (Lightning's
        ``_can_stop_early``)."""
        if not self.should_stop:
            return False
        if self._hard_stop:
            return True
        ok = ((self.min_steps is None or self.state.global_step >= self.min_steps)
              and (self.min_epochs is None or self.state.epoch >= self.min_epochs))
        if not ok and not getattr(self, "_min_note", False):
            self._min_note = True
            logger.info("stop requested at step %d but min_steps=%s / min_epochs=%s not met: training continues",
                        self.state.global_step, self.min_steps, self.min_epochs)
        return ok

    def _prof(self, action: str):
        p = self.fit_profiler
        return p.profile(action) if p is not None else _NULLCTX

    def _time_is_up(self) -> bool:
        """max_time reached? Rank 0's clock decides for every rank (Lightning's Timer broadcasts its
        decision), so all ranks leave the loop after the same step."""
        up = time.monotonic() - self._fit_t0 >= self.max_time
        if self.pc is not None and self.pc.world_size > 1:
            t = torch.tensor([1.0 if up else 0.0], device=self.device)
            dist.broadcast(t, src=0)
            up = bool(t.item())
        return up

    def _should_validate(self, nbe: int) -> bool:
        """Lightning's validation schedule, checked after each optimizer step: an int val_check_interval
        counts training batches (micro-batches, so accumulation does not stretch it); a float — 1.0 when
        unset, i.e. at the end of every epoch — is a fraction of the batches an epoch steps through,
        gated by check_val_every_n_epoch."""
        if self.datamodule.datasets.get("validation") is None:
            return False
        v = 1.0 if self.val_check_interval is None else self.val_check_interval
        accum = self.accumulate_grad_batches
        if isinstance(v, float):
            if not 0.0 < v <= 1.0:
                raise ValueError(f"val_check_interval as a float must be in (0, 1], got {v}")
            n = self.check_val_every_n_epoch
            if n is None or (self.state.epoch + 1) % int(n) != 0:
                return False
            every = max(1, int((nbe // accum) * accum * v))
        else:
            every = max(1, int(v))
        done = self.state.batch_idx  # batches of this epoch stepped through, this step included
        return done // every > (done - accum) // every

    def to_device(self, batch: dict) -> dict:
        out = {}
        for k, v in batch.items():
            out[k] = v.to(self.device, non_blocking=True) if isinstance(v, torch.Tensor) else v
        return out

    def train_step(self, batches: list[dict]):
        eng, lm = self.engine, self.lm
        t0 = time.perf_counter()
        if self.meter is not None and self.meter.t0 is None:
            self.meter.start()  # the first logged rate covers the first step's own time
        self.profiler.before_step(self.state.global_step + 1)
        if self.fit_profiler is not None:
            self.fit_profiler.before_step(self, self.state.global_step + 1)
        self.watchdog.arm()
        for cb in self.callbacks:
            _call(cb, "on_train_batch_start", self, lm, batches[0], self.state.batch_idx)
        eng.begin_step(len(batches))
        eng.zero_grad()
        metrics_acc: dict[str, torch.Tensor] = {}
        counters: dict[str, Any] = {}
        anomaly = torch.autograd.detect_anomaly(check_nan=True) if self.detect_anomaly else _NULLCTX
        for i, b in enumerate(batches):
            eng.begin_micro(i)
            b = self.to_device(b)
            with anomaly:
                with trace_range("forward"), self._prof("training_step"):
                    loss, metrics, cnt = lm.training_step(b, self.state.batch_idx + i)
                with trace_range("backward"), self._prof("backward"):
                    (loss * self.scaler.scale if self.scaler is not None else loss).backward()
            for k, v in metrics.items():
                metrics_acc[k] = metrics_acc.get(k, 0) + v.detach().float().to(self.device) / len(batches)
            for k, v in cnt.items():
                counters[k] = counters.get(k, 0) + v
        with trace_range("optimizer"), self._prof("optimizer_step"):
            eng.finish_backward()
            if self.scaler is None:
                eng.clip_and_scale(self.gradient_clip_val)
                lr = self.scheduler.get_lr()
                eng.step(lr)
            else:  # fp16: unscale inside the clip scale; an overflowed step is skipped (one host sync)
                eng.clip_and_scale(self.gradient_clip_val, loss_scale=self.scaler.scale)
                finite = bool(torch.isfinite(eng.grad_norm).all().item())
                lr = self.scheduler.get_lr()
                if self.scaler.update(finite):
                    eng.step(lr)
                else:
                    logger.warning("fp16 gradient overflow at step %d: step skipped, loss scale -> %g",
                                   self.state.global_step + 1, self.scaler.scale)
        self.last_lr = lr
        self.scheduler.step()
        self.state.global_step += 1
        for k, v in counters.items():
            self.state.consumed[k] = self.state.consumed.get(k, 0) + v
        metrics_acc["lr"] = torch.tensor(lr)
        if self.scaler is not None:  # reference: DeepSpeed fp16 skipped steps on the progress bar
            metrics_acc["Loss Scale"] = torch.tensor(self.scaler.scale)
            metrics_acc["Skipped Steps"] = torch.tensor(float(self.scaler.skipped))
        if getattr(lm.config, "log_grad_norm", True) and eng.grad_norm is not None:
            metrics_acc["Gradient Norm"] = eng.grad_norm.reshape(())
        self.state.batch_idx += len(batches)
        self._log_buffer.append((self.state.global_step, metrics_acc))
        self.step_times.append(time.perf_counter() - t0)
        self._count_tokens(batches)
        self.profiler.after_step(self.state.global_step)
        if self.fit_profiler is not None:
            self.fit_profiler.after_step(self, self.state.global_step)
        self.watchdog.disarm()
        if self.collectives is not None and self.state.global_step % collective_debug.check_every() == 0:
            self.collectives.verify()
        for cb in self.callbacks:  # metric contributions for this step's log row (before it is flushed)
            _call(cb, "on_step_metrics", self, lm)
        self._flush_logs()
        for cb in self.callbacks:
            _call(cb, "on_train_batch_end", self, lm, None, batches[-1], self.state.batch_idx)

    def _count_tokens(self, batches: list[dict]):
        # input_ids, or chosen_input_ids + rejected_input_ids of the preference objectives
        ids = [v for b in batches if isinstance(b, dict) for k, v in b.items()
               if k.endswith("input_ids") and isinstance(v, torch.Tensor)]
        if not ids:
            return
        S = int(ids[0].shape[-1])
        if S not in self._fpt:
            fpt = model_flops_per_token(getattr(self.lm.model, "config", None), S)
            if getattr(self.lm, "ref_model", None) is not None:
                fpt *= 4.0 / 3.0  # DPO: the frozen reference model's forward (1/3 of forward + backward)
            self._fpt[S] = fpt
        self.meter.fpt = self._fpt[S]
        self.meter.update(sum(t.numel() for t in ids))

    def add_step_metrics(self, values: dict[str, float]):
        """Extra scalar metrics (host floats) for the most recent optimizer step's log row."""
        vals = {k: torch.tensor(float(v)) for k, v in values.items()}
        if self._log_buffer and self._log_buffer[-1][0] == self.state.global_step:
            self._log_buffer[-1][1].update(vals)
        else:  # the step's row was already written (e.g. an epoch-end value): a row of its own
            self._log_buffer.append((self.state.global_step, vals))

    def _flush_logs(self, force: bool = False):
        if not self._log_buffer:
            return
        if not force and self.state.global_step % self.log_every_n_steps != 0:
            return
        # one host sync per logging interval; DP-average the scalar metrics
        keys = sorted({k for _, m in self._log_buffer for k in m})
        rows = []
        for step, m in self._log_buffer:
            vec = torch.stack([torch.as_tensor(m.get(k, float("nan")), device=self.device).float().reshape(())
                               for k in keys])
            rows.append((step, vec))
        mat = torch.stack([r[1] for r in rows])
        if self.pc.dp and self.pc.world_size > 1:
            dist.all_reduce(mat, group=self.pc.dp_group)
            mat = mat / self.pc.dp_size
        mat = mat.cpu().tolist()
        # device-side index checks of the HIP kernels (RoPE positions, CE labels): the host already
        # synchronised above, so reading the error words costs one small copy per logging interval
        check_kernel_errors(self.device)
        consumed = dict(self.state.consumed)
        if self.pc.dp and consumed:
            t = torch.tensor([float(consumed[k]) for k in sorted(consumed)], device=self.device)
            dist.all_reduce(t, group=self.pc.dp_group)
            consumed = dict(zip(sorted(consumed), t.cpu().tolist()))
        rates = self.meter.metrics() if self.meter is not None else {}
        for i, ((step, _), vals) in enumerate(zip(rows, mat)):
            d = dict(zip(keys, vals))
            d.update({k: float(v) for k, v in consumed.items()})
            if i == len(rows) - 1:
                d.update(rates)
            # the latest value of every metric (Lightning's callback_metrics): a validation loss logged
            # at an earlier step stays visible to ModelCheckpoint(monitor=...) after later train rows
            self.last_metrics.update(d)
            if self.is_global_zero:
                for lg in self.loggers:
                    _call(lg, "log_metrics", d, step)
        if self.is_global_zero and self.enable_progress_bar:
            d = self.last_metrics
            loss = d.get("Loss/Train/Step", next((d[k] for k in d if k.startswith("Loss/Train")), float("nan")))
            logger.info("step %d | loss %.4f | lr %.3e | grad_norm %.3f | %.0f tok/s | %.1f TFLOP/s/gpu",
                        self.state.global_step, loss, d.get("lr", float("nan")), d.get("Gradient Norm", float("nan")),
                        d.get("Throughput/tokens_per_sec", float("nan")),
                        d.get("Throughput/tflops_per_gpu", float("nan")))
        self._log_buffer.clear()

    @torch.no_grad()
    def _val_batch_limit(self, dl, sanity: bool) -> int | None:
        """Batches to run (None = all): Lightning's limit_val_batches (an int count or a float fraction of
        the loader), or num_sanity_val_steps (-1 = all) for the sanity check."""
        if sanity:
            return None if self.num_sanity_val_steps < 0 else self.num_sanity_val_steps
        lim = self.limit_val_batches
        if lim is None or (isinstance(lim, float) and lim >= 1.0):
            return None
        if isinstance(lim, float):
            try:
                return int(len(dl) * lim)
            except TypeError:  # a loader without a length: a fraction cannot be applied
                return None
        return int(lim)

    def validate(self, sanity: bool = False):
        if self.datamodule.datasets.get("validation") is None:
            return {}
        dl = self.datamodule.val_dataloader(*self._dp())
        if dl is None:
            return {}
        limit = self._val_batch_limit(dl, sanity)
        self.lm.eval()
        sums: dict[str, torch.Tensor] = {}
        n = 0
        for i, b in enumerate(dl):
            if limit is not None and i >= limit:
                break
            m = self.lm.validation_step(self.to_device(b), i)
            for k, v in m.items():
                sums[k] = sums.get(k, 0) + v.float()
            n += 1
        self.lm.train()
        if n == 0:
            return {}
        keys = sorted(sums)
        vec = torch.stack([sums[k].reshape(()) / n for k in keys])
        if self.pc.world_size > 1:
            dist.all_reduce(vec)
            vec = vec / self.pc.world_size
        out = dict(zip(keys, vec.cpu().tolist()))
        if "Loss/Val" in out and "Perplexity/Val" in out:
            out["Perplexity/Val"] = math.exp(out["Loss/Val"])
        if sanity:
            logger.info("validation sanity check (%d batches): %s", n, out)
            return out
        self.last_metrics.update(out)  # visible to ModelCheckpoint(monitor="Loss/Val")
        if self.is_global_zero:
            for lg in self.loggers:
                _call(lg, "log_metrics", out, self.state.global_step)
            logger.info("validation @ step %d: %s", self.state.global_step, out)
        for cb in self.callbacks:
            _call(cb, "on_validation_end", self, self.lm, out)
        return out

    # ------------------------------------------------------------------ checkpoint helpers for callbacks
    def save_checkpoint(self, path: str, async_write: bool = False):
        from ..ckpt.checkpoint import save_checkpoint
        save_checkpoint(self, path, async_write=async_write)


def _call(obj, name, *args):
    fn = getattr(obj, name, None)
    if fn is not None:
        return fn(*args)
    return None


class _NullCtx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


_NULLCTX = _NullCtx()


def log_model_summary(model) -> None:
    """Lightning's model summary, condensed: parameters per top-level module (this rank's shard under TP)."""
    rows, total, trainable = [], 0, 0
    for name, mod in model.named_children():
        n = sum(p.numel() for p in mod.parameters())
        rows.append(f"  {name:<24} {type(mod).__name__:<28} {n / 1e6:>10.2f} M")
        total += n
        trainable += sum(p.numel() for p in mod.parameters() if p.requires_grad)
    total += sum(p.numel() for p in model.parameters(recurse=False))
    logger.info("model summary (%s):\n%s\n  total %.2f M parameters, %.2f M trainable", type(model).__name__,
                "\n".join(rows), total / 1e6, trainable / 1e6)


def make_fit_profiler(spec):
    """Lightning ``Trainer(profiler=...)``: "simple", "advanced", "pytorch", a profiler object, or a
    ``class_path`` dict naming Lightning's SimpleProfiler / AdvancedProfiler / PyTorchProfiler."""
    from .profilers import AdvancedProfiler, PyTorchProfiler, SimpleProfiler
    if spec in (None, False, "", "none"):
        return None
    if isinstance(spec, str):
        table = {"simple": SimpleProfiler, "advanced": AdvancedProfiler, "pytorch": PyTorchProfiler}
        if spec.lower() not in table:
            raise ValueError(f"profiler {spec!r}: use 'simple', 'advanced' or 'pytorch'")
        return table[spec.lower()]()
    if isinstance(spec, dict) and "class_path" in spec:
        name = spec["class_path"].rsplit(".", 1)[-1]
        table = {"SimpleProfiler": SimpleProfiler, "AdvancedProfiler": AdvancedProfiler,
                 "PyTorchProfiler": PyTorchProfiler}
        if name not in table:
            raise ValueError(f"profiler class {spec['class_path']!r} is not supported")
        return table[name](**(spec.get("init_args") or {}))
    if hasattr(spec, "profile") and hasattr(spec, "session"):
        return spec
    raise TypeError(f"unsupported profiler {spec!r}")
