"""Observability and failure handling for the training loop.

The reference has no in-tree profiler integration, no stall detection and resumes only by hand
(`L/lightning/callbacks/training_time_estimator.py:38-83` is its only timing tool;
`scripts/train.sh:14,21` its only recovery path). This module adds, MI355X-first:

* :class:`ThroughputMeter` — tokens/s, model TFLOP/s per GPU, MFU against the 2.5 PF/s dense bf16
  MFMA peak and peak HBM use, computed from host clocks at logging boundaries only (the loop never
  synchronises with the device for them: the logging flush already does one host sync).
* :class:`StepProfiler` — a torch.profiler window over a step range (``LLMT_PROFILE_STEPS=a-b``), the
  chrome trace per rank lands in the log directory; :func:`trace_range` emits roctx ranges
  (``LLMT_ROCTX=1``) that ``rocprofv3 --marker-trace`` shows around layers and collectives.
* :class:`StallWatchdog` — faulthandler-based: when one step takes longer than
  ``LLMT_STALL_TIMEOUT`` seconds every thread's Python stack is dumped (a hung collective or a
  kernel that never finishes shows up with its call site instead of a silent 30-minute PG timeout).
* :func:`find_last_checkpoint` — ``--ckpt_path last`` auto-resume: the newest COMPLETE checkpoint
  (meta.json and every tensor-parallel shard present) under the checkpoint root.
* :func:`record_failure` — every rank writes its exception to ``<log_dir>/failure_rank<r>.txt`` and
  logs it with its rank before re-raising, so the first failing rank is identifiable.
"""
from __future__ import annotations

import contextlib
import faulthandler
import json
import logging
import os
import re
import sys
import threading
import time
import traceback
from pathlib import Path

import torch

logger = logging.getLogger("llm_training")

PEAK_BF16_FLOPS = 2.5e15  # MI355X dense bf16 MFMA peak (no sparsity)


def model_flops_per_token(config, seq_len: int) -> float:
    """Training FLOPs per token (fwd + bwd = 6 x matmul params + causal attention scores/values)."""
    h = getattr(config, "hidden_size", None)
    L = getattr(config, "num_hidden_layers", None)
    if h is None or L is None:
        return 0.0
    hq = getattr(config, "num_attention_heads", 1)
    hkv = getattr(config, "num_key_value_heads", None) or hq
    d = getattr(config, "head_dim", None) or h // hq
    inter = getattr(config, "intermediate_size", 4 * h)
    V = getattr(config, "vocab_size", 0)
    n_matmul = L * (h * (hq + 2 * hkv) * d + hq * d * h + 3 * h * inter) + V * h
    attn = 6 * L * seq_len * hq * d  # causal: 2 matmuls x 2 flops x S/2 keys, x3 for fwd + bwd
    return 6.0 * n_matmul + attn


class ThroughputMeter:
    """Accumulates tokens between logging flushes; reports whole-job and per-GPU rates."""

    def __init__(self, world_size: int = 1, flops_per_token: float = 0.0, device: torch.device | None = None,
                 peak_flops: float = PEAK_BF16_FLOPS):
        self.world = max(1, int(world_size))
        self.fpt = float(flops_per_token)
        self.peak = peak_flops
        self.device = device
        self.tokens = 0
        self.steps = 0
        self.t0: float | None = None

    def start(self):
        self.t0 = time.perf_counter()
        self.tokens = 0
        self.steps = 0

    def update(self, local_tokens: int):
        if self.t0 is None:
            self.start()
        self.tokens += int(local_tokens)
        self.steps += 1

    def metrics(self) -> dict[str, float]:
        """Rates since the last call (call after a host sync so device work is accounted)."""
        if self.t0 is None or self.steps == 0:
            return {}
        el = max(time.perf_counter() - self.t0, 1e-9)
        tps_gpu = self.tokens / el
        out = {"Throughput/tokens_per_sec": tps_gpu * self.world, "Throughput/tokens_per_sec_per_gpu": tps_gpu,
               "Throughput/sec_per_step": el / self.steps}
        if self.fpt > 0:
            out["Throughput/tflops_per_gpu"] = tps_gpu * self.fpt / 1e12
            out["Throughput/mfu"] = tps_gpu * self.fpt / self.peak
        if self.device is not None and self.device.type == "cuda":
            out["Memory/peak_allocated_gib"] = torch.cuda.max_memory_allocated(self.device) / 2 ** 30
        self.start()
        return out


def _parse_range(spec: str | None) -> tuple[int, int] | None:
    if not spec:
        return None
    m = re.fullmatch(r"\s*(\d+)\s*(?:-\s*(\d+))?\s*", spec)
    if not m:
        raise ValueError(f"profile step range must look like '10-12', got {spec!r}")
    a = int(m.group(1))
    b = int(m.group(2)) if m.group(2) else a
    return a, b


class StepProfiler:
    """torch.profiler over global steps [a, b] (inclusive); trace written on the last step."""

    def __init__(self, steps: str | None = None, out_dir: str = "logs", rank: int = 0):
        self.range = _parse_range(steps if steps is not None else os.environ.get("LLMT_PROFILE_STEPS"))
        self.out_dir = out_dir
        self.rank = rank
        self.prof = None
        self.trace_path: str | None = None

    @property
    def enabled(self) -> bool:
        return self.range is not None

    def before_step(self, step: int):
        """``step`` is the global step about to run (1-based, as logged)."""
        if self.range is None or self.prof is not None or step != self.range[0]:
            return
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        self.prof = torch.profiler.profile(activities=acts, record_shapes=True, with_stack=False)
        self.prof.__enter__()

    def after_step(self, step: int):
        if self.prof is None or step < self.range[1]:
            return
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.prof.__exit__(None, None, None)
        os.makedirs(self.out_dir, exist_ok=True)
        self.trace_path = os.path.join(self.out_dir, f"profile_steps{self.range[0]}-{self.range[1]}_rank{self.rank}.json")
        self.prof.export_chrome_trace(self.trace_path)
        if self.rank == 0:
            logger.info("profiler trace: %s\n%s", self.trace_path,
                        self.prof.key_averages().table(sort_by="self_device_time_total" if torch.cuda.is_available()
                                                       else "self_cpu_time_total", row_limit=25))
        self.prof = None
        self.range = None


_ROCTX = os.environ.get("LLMT_ROCTX", "0") == "1"


@contextlib.contextmanager
def trace_range(name: str):
    """roctx range (LLMT_ROCTX=1, seen by rocprofv3 --marker-trace) + torch.profiler record_function."""
    pushed = False
    if _ROCTX and torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)  # routed to roctx by the ROCm build of PyTorch
            pushed = True
        except Exception:  # noqa: BLE001 - tracing must never break training
            pushed = False
    try:
        with torch.autograd.profiler.record_function(name):
            yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


class StallWatchdog:
    """Dump every thread's stack if a step does not finish within ``timeout`` seconds."""

    def __init__(self, timeout: float | None = None, path: str | None = None):
        t = timeout if timeout is not None else float(os.environ.get("LLMT_STALL_TIMEOUT", "0") or 0)
        self.timeout = float(t)
        self.path = path
        self._f = None

    @property
    def enabled(self) -> bool:
        return self.timeout > 0

    def arm(self):
        if not self.enabled:
            return
        if self._f is None and self.path:
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            self._f = open(self.path, "a")
        faulthandler.dump_traceback_later(self.timeout, repeat=True, file=self._f or sys.stderr, exit=False)

    def disarm(self):
        if self.enabled:
            faulthandler.cancel_dump_traceback_later()

    def close(self):
        self.disarm()
        if self._f is not None:
            self._f.close()
            self._f = None


class StepWatchdog:
    """Fail fast instead of hanging: if the phase armed by ``arm(label)`` does not end (next ``arm`` or
    ``disarm``) within its time limit, write ``[rank r] watchdog: <label> exceeded T s`` and every
    thread's stack to stderr and end the process with ``exit_code`` (``os._exit``: a rank blocked in a
    collective cannot unwind). The launcher (``launch.py``) then stops the other ranks and returns that
    code, so a stuck RCCL collective ends a multi-GPU run in seconds with every rank's stacks instead of
    running into the job's outer time limit. A Python timer thread does the labelled dump; a
    ``faulthandler`` timer 30 s later is the backstop for a rank whose interpreter lock is held.
    Reference: Lightning / NCCL rely on the 30-minute process-group timeout
    (src/llm_training/lightning/strategy/fsdp2/fsdp2_strategy.py:411-420)."""

    def __init__(self, rank: int = 0, timeout: float = 120.0, exit_code: int = 3, stream=None):
        self.rank = rank
        self.timeout = float(timeout)
        self.exit_code = exit_code
        self.stream = stream if stream is not None else sys.stderr
        self._gen = 0
        self._lock = threading.Lock()

    def arm(self, label: str, timeout: float | None = None):
        t = self.timeout if timeout is None else float(timeout)
        with self._lock:
            self._gen += 1
            gen = self._gen
        faulthandler.cancel_dump_traceback_later()
        if t <= 0:
            return
        faulthandler.dump_traceback_later(t + 30.0, repeat=False, file=self.stream, exit=True)
        th = threading.Thread(target=self._watch, args=(gen, label, t), daemon=True, name="llmt-step-watchdog")
        th.start()

    def disarm(self):
        with self._lock:
            self._gen += 1
        faulthandler.cancel_dump_traceback_later()

    def _watch(self, gen: int, label: str, t: float):
        deadline = time.monotonic() + t
        while True:
            left = deadline - time.monotonic()
            if left <= 0:
                break
            time.sleep(min(left, 0.5))
            with self._lock:
                if self._gen != gen:
                    return
        with self._lock:
            if self._gen != gen:
                return
        try:
            self.stream.write(f"[rank {self.rank}] watchdog: {label} exceeded {t:.0f} s; stacks of every thread:\n")
            self.stream.flush()
            faulthandler.dump_traceback(file=self.stream, all_threads=True)
            self.stream.flush()
        finally:
            os._exit(self.exit_code)


_STEP_RE = re.compile(r"step=(\d+)")


def is_complete_checkpoint(path: str | os.PathLike) -> bool:
    from ..ckpt.checkpoint import is_complete
    return is_complete(path)


def checkpoint_step(path: str | os.PathLike) -> int:
    p = Path(path)
    try:
        if p.is_file():
            from ..ckpt.checkpoint import read_meta
            return int(read_meta(str(p))["trainer"]["global_step"])
        return int(json.loads((p / "meta.json").read_text())["trainer"]["global_step"])
    except Exception:  # noqa: BLE001 - fall back to the step in the name
        m = _STEP_RE.search(p.name)
        return int(m.group(1)) if m else -1


def find_last_checkpoint(root: str | os.PathLike) -> str | None:
    """Newest complete checkpoint directory under ``root`` (searched recursively), by global step."""
    root = Path(root)
    if not root.exists():
        return None
    cands = [m.parent for m in root.rglob("meta.json") if is_complete_checkpoint(m.parent)]
    # consolidated single-file checkpoints (save_distributed_checkpoint: false)
    cands += [f for f in root.rglob("*.ckpt") if f.is_file() and not f.is_symlink() and is_complete_checkpoint(f)]
    if not cands:
        return None
    best = max(cands, key=lambda p: (checkpoint_step(p), p.stat().st_mtime))
    return str(best)


def record_failure(exc: BaseException, rank: int, log_dir: str) -> str | None:
    """Log and persist a rank's exception (returns the file written, if any)."""
    tb = "".join(traceback.format_exception(type(exc), exc, exc.__traceback__))
    logger.error("rank %d failed: %s", rank, tb)
    try:
        os.makedirs(log_dir, exist_ok=True)
        path = os.path.join(log_dir, f"failure_rank{rank}.txt")
        with open(path, "w") as f:
            f.write(f"time: {time.strftime('%Y-%m-%d %H:%M:%S')}\nrank: {rank}\n\n{tb}")
        return path
    except OSError:
        return None
