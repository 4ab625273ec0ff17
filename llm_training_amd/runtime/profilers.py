"""Lightning's ``Trainer(profiler=...)`` for this trainer: ``simple``, ``advanced`` and ``pytorch``.

The reference gets these from Lightning (src/llm_training/lightning/cli/trainer.py:1-11 subclasses
Lightning's Trainer, whose ``profiler`` argument accepts the three names). Same surface here:

* :class:`SimpleProfiler` — host wall time per trainer action (``get_train_batch``, ``training_step``,
  ``backward``, ``optimizer_step``, ``validation``), a table at the end of ``fit`` logged by rank 0 and
  written to ``<log_dir>/fit-profile-rank<r>.txt``. Like Lightning's, it times the host: device work is
  asynchronous, so a kernel-bound step shows up where the host waits (the logging flush, a full queue),
  not where the kernels were enqueued — use ``pytorch`` or rocprofv3 for device time.
* :class:`AdvancedProfiler` — cProfile over the whole ``fit`` (function-level host profile), the top
  functions by cumulative time in the same file.
* :class:`PyTorchProfiler` — ``torch.profiler`` (CPU + GPU activities, HIP kernels included) over a
  window of optimizer steps (default 2-4: after the first step's one-time setup), a chrome trace per
  rank and the top kernels by device time.
"""
from __future__ import annotations

import contextlib
import io
import logging
import os
import time
from collections import defaultdict

import torch

logger = logging.getLogger("llm_training")


class _Base:
    def __init__(self, dirpath: str | None = None, filename: str | None = None):
        self.dirpath, self.filename = dirpath, filename

    @contextlib.contextmanager
    def profile(self, action: str):
        yield

    def before_step(self, trainer, step: int):
        pass

    def after_step(self, trainer, step: int):
        pass

    def _path(self, trainer, suffix: str = "txt") -> str:
        d = self.dirpath or trainer.log_dir
        os.makedirs(d, exist_ok=True)
        rank = trainer.pc.rank if trainer.pc is not None else 0
        return os.path.join(d, f"{self.filename or 'fit-profile'}-rank{rank}.{suffix}")

    def _emit(self, trainer, text: str):
        with open(self._path(trainer), "w") as f:
            f.write(text)
        if trainer.pc is None or trainer.pc.rank == 0:
            logger.info("%s\n%s", type(self).__name__, text)


class SimpleProfiler(_Base):
    def __init__(self, dirpath: str | None = None, filename: str | None = None, extended: bool = True):
        super().__init__(dirpath, filename)
        self.extended = extended
        self.durations: dict[str, list[float]] = defaultdict(list)
        self._t0 = 0.0

    @contextlib.contextmanager
    def profile(self, action: str):
        t = time.perf_counter()
        try:
            yield
        finally:
            self.durations[action].append(time.perf_counter() - t)

    @contextlib.contextmanager
    def session(self, trainer):
        self._t0 = time.perf_counter()
        try:
            yield
        finally:
            self._emit(trainer, self.summary(time.perf_counter() - self._t0))

    def summary(self, total: float) -> str:
        lines = [f"{'action':<20} {'mean (s)':>12} {'calls':>8} {'total (s)':>12} {'% of fit':>9}"]
        for a, ds in sorted(self.durations.items(), key=lambda kv: -sum(kv[1])):
            tot = sum(ds)
            lines.append(f"{a:<20} {tot / len(ds):>12.6f} {len(ds):>8d} {tot:>12.4f} {100 * tot / max(total, 1e-9):>8.2f}%")
        lines.append(f"{'fit (wall)':<20} {'':>12} {'':>8} {total:>12.4f} {100.0:>8.2f}%")
        return "\n".join(lines)


class AdvancedProfiler(_Base):
    def __init__(self, dirpath: str | None = None, filename: str | None = None, line_count_restriction: float = 40):
        super().__init__(dirpath, filename)
        self.restrict = line_count_restriction

    @contextlib.contextmanager
    def session(self, trainer):
        import cProfile
        import pstats
        prof = cProfile.Profile()
        prof.enable()
        try:
            yield
        finally:
            prof.disable()
            out = io.StringIO()
            pstats.Stats(prof, stream=out).sort_stats("cumulative").print_stats(self.restrict)
            self._emit(trainer, out.getvalue())


class PyTorchProfiler(_Base):
    def __init__(self, dirpath: str | None = None, filename: str | None = None, steps: str = "2-4",
                 record_shapes: bool = True, with_stack: bool = False, row_limit: int = 25, **kw):
        super().__init__(dirpath, filename)
        a, _, b = str(steps).partition("-")
        self.first, self.last = int(a), int(b or a)
        self.record_shapes, self.with_stack, self.row_limit = record_shapes, with_stack, row_limit
        self.prof = None
        self.trace_path: str | None = None

    @contextlib.contextmanager
    def session(self, trainer):
        try:
            yield
        finally:
            if self.prof is not None:  # the run ended inside the window
                self._finish(trainer)

    def before_step(self, trainer, step: int):
        if self.prof is not None or step != self.first:
            return
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        self.prof = torch.profiler.profile(activities=acts, record_shapes=self.record_shapes,
                                           with_stack=self.with_stack)
        self.prof.__enter__()

    def after_step(self, trainer, step: int):
        if self.prof is not None and step >= self.last:
            self._finish(trainer)

    def _finish(self, trainer):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.prof.__exit__(None, None, None)
        self.trace_path = self._path(trainer, "json")
        self.prof.export_chrome_trace(self.trace_path)
        key = "self_device_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
        table = self.prof.key_averages().table(sort_by=key, row_limit=self.row_limit)
        self.prof = None
        with open(self._path(trainer), "w") as f:
            f.write(table)
        if trainer.pc is None or trainer.pc.rank == 0:
            logger.info("PyTorchProfiler steps %d-%d: trace %s\n%s", self.first, self.last, self.trace_path, table)
