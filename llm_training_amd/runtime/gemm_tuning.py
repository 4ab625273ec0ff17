"""GEMM algorithm selection for the plain library GEMMs (hipBLASLt / rocBLAS through PyTorch).

The projections and the lm_head are plain GEMMs, so they go to the vendor library rather than to
hand-written kernels; what the framework controls is WHICH library solution runs. hipBLASLt's
default heuristic picks a DepthU-32 tile for the forward ``x @ W^T`` layout of every Llama-3-8B
projection that runs at ~40 % of the MFMA roof while the backward layouts run at 55-60 % (profiles/
r1_llama8b_1gpu_v2_kernel_stats.md), so the framework ships a TunableOp results file measured on
MI355X (gfx950, this ROCm image) and loads it read-only at start-up: every GEMM shape listed there
dispatches the measured-fastest solution, shapes not listed fall back to the default heuristic.

Modes (``LLMT_GEMM_TUNING`` env var or ``Trainer(gemm_tuning=...)``):
  * ``use``  — load the shipped results file if it exists, never tune.
  * ``tune`` — benchmark every new GEMM shape's candidate solutions and write the file.
  * ``off``  (default) — library default heuristic.

Measured on the bench (6 steps, 1x MI355X): ``use`` 16,474 tok/s vs ``off`` 16,521 tok/s — the shipped
partial results (TunableOp times its candidates on constant data, which reads high; random-data
timings in gpurun benchmarks/bench_gemm_layouts.py put every projection at 1.2-1.3 PF/s for fwd+dgrad+
wgrad whatever the weight layout) do not move the end-to-end number, so the default stays ``off``.
"""
from __future__ import annotations

import logging
import os
from pathlib import Path

import torch

logger = logging.getLogger("llm_training")

DEFAULT_RESULTS = Path(__file__).resolve().parents[1] / "tuning" / "tunableop_gfx950.csv"
_state = {"mode": None}


def setup_gemm_tuning(mode: str | None = None, results: str | os.PathLike | None = None) -> str:
    """Configure TunableOp once per process; returns the active mode."""
    mode = (mode or os.environ.get("LLMT_GEMM_TUNING", "off")).lower()
    if _state["mode"] is not None:
        return _state["mode"]
    if mode not in ("use", "tune", "off"):
        raise ValueError(f"gemm tuning mode must be use|tune|off, got {mode!r}")
    if not torch.cuda.is_available() or torch.version.hip is None or mode == "off":
        _state["mode"] = "off"
        return "off"
    import torch.cuda.tunable as tunable
    path = Path(results or os.environ.get("LLMT_GEMM_TUNING_FILE", DEFAULT_RESULTS))
    if mode == "use" and not path.exists():
        _state["mode"] = "off"
        return "off"
    tunable.enable(True)
    tunable.set_filename(str(path), insert_device_ordinal=False)
    if mode == "tune":
        tunable.tuning_enable(True)
        tunable.set_max_tuning_duration(int(os.environ.get("LLMT_GEMM_TUNING_MS", "200")))
        tunable.set_max_tuning_iterations(int(os.environ.get("LLMT_GEMM_TUNING_ITERS", "50")))
        if path.exists():
            tunable.read_file(str(path))
    else:
        tunable.tuning_enable(False)
        tunable.read_file(str(path))
    logger.info("gemm tuning: %s (%s)", mode, path)
    _state["mode"] = mode
    return mode


def write_results() -> None:
    """Flush tuned results (tune mode) — also happens at interpreter exit."""
    if _state["mode"] == "tune":
        import torch.cuda.tunable as tunable
        if hasattr(tunable, "write_file"):
            tunable.write_file()
