"""Loader for the in-tree gfx950 extension (``llm_training_amd/_C.so``).

The HIP kernels are the ONLY implementation used for GPU tensors: if the library is missing or
fails to load on a machine with a GPU, :func:`lib` raises instead of silently falling back to
PyTorch. CPU tensors use the torch reference ops in :mod:`llm_training_amd.ops.reference`.
"""
from __future__ import annotations

import logging
import os
import threading
from pathlib import Path

import torch

_LOCK = threading.Lock()
_LOADED: bool | None = None
_ERR: Exception | None = None
# LLMT_NATIVE_DIAG=1 loads the diagnostic build (_C_diag.so: the wrong-result probes of benchmarks/probes/
# compiled in, `python -m llm_training_amd._build --diag`) instead of the production library
DIAG = os.environ.get("LLMT_NATIVE_DIAG", "0") == "1"
LIB_PATH = Path(__file__).resolve().parent.parent / ("_C_diag.so" if DIAG else "_C.so")
# environment variables that make kernels compute wrong results on purpose (diagnostic probes); only the
# diagnostic library reads them, and a production run refuses to start while one is set
PROBE_VARS = ("LLMT_FA_PROBE", "LLMT_FA_D6_PROBE")


def check_probe_env(environ=None) -> None:
    """Raise if a diagnostic probe variable is set for a production (non-diagnostic) run."""
    env = os.environ if environ is None else environ
    bad = [k for k in PROBE_VARS if env.get(k, "") not in ("", "0")]
    if bad and not DIAG:
        raise RuntimeError(
            f"{', '.join(bad)} select wrong-result diagnostic probes; they are only honoured by the diagnostic "
            "library (LLMT_NATIVE_DIAG=1, built by `python -m llm_training_amd._build --diag`). Unset them for "
            "training runs.")


def llmt_env(environ=None) -> dict:
    """Every LLMT_* variable of the environment (kernel / layout / schedule knobs): recorded with each run
    (bench JSON ``llmt_env``, trainer run metadata) so a result can be traced to the knobs it ran with."""
    env = os.environ if environ is None else environ
    return {k: env[k] for k in sorted(env) if k.startswith("LLMT_")}


def _load() -> bool:
    global _LOADED, _ERR
    with _LOCK:
        if _LOADED is not None:
            return _LOADED
        try:
            check_probe_env()
            if not LIB_PATH.exists() and os.environ.get("LLMT_AUTOBUILD", "1") == "1":
                from .. import _build

                _build.build(diag=DIAG)
            torch.ops.load_library(str(LIB_PATH))
            _LOADED = True
        except RuntimeError as e:
            if "diagnostic probes" in str(e):
                raise
            _ERR = e
            _LOADED = False
        except Exception as e:  # pragma: no cover - exercised on broken installs only
            _ERR = e
            _LOADED = False
        return _LOADED


def available() -> bool:
    return _load()


def lib():
    """Return ``torch.ops.llmt``; raise loudly if the native extension is unavailable."""
    if not _load():
        raise RuntimeError(
            f"llm_training_amd native extension could not be loaded from {LIB_PATH}: {_ERR!r}. "
            "Build it with `python -m llm_training_amd._build` (hipcc, gfx950)."
        )
    return torch.ops.llmt


# GPU dtypes that ran the torch reference ops instead of the HIP kernels in this process (-> op count):
# read by the trainer / bench into their run metadata, warned about once per dtype
REFERENCE_ON_GPU: dict[str, int] = {}


def compute_path(device_type: str, dtype: torch.dtype) -> str:
    """Which implementation the fused ops (attention, norms, SwiGLU, RoPE, CE, AdamW) of a model whose
    activations have ``dtype`` run on ``device_type``: ``"hip"`` (the gfx950 kernels) or
    ``"torch-reference"`` (the kernels are bf16 MFMA kernels: fp32 / fp16 GPU runs and CPU runs use the
    torch ops of :mod:`llm_training_amd.ops.reference`)."""
    return "hip" if device_type == "cuda" and dtype == torch.bfloat16 else "torch-reference"


def use_native(t: torch.Tensor) -> bool:
    """bf16 GPU tensors always go to the HIP kernels (no silent fallback: a missing library raises).

    The kernels are bf16 MFMA kernels; fp32 / fp16 GPU tensors (``precision: 32-true`` / ``16-*``) and
    CPU tensors run the torch reference ops of :mod:`llm_training_amd.ops.reference`. On the GPU that
    switch is announced once per dtype (a warning) and counted in ``REFERENCE_ON_GPU``."""
    if t.device.type == "cuda":
        lib()
        if t.dtype == torch.bfloat16:
            return True
        key = str(t.dtype).replace("torch.", "")
        if key not in REFERENCE_ON_GPU:
            logging.getLogger("llm_training").warning(
                "%s GPU tensors run the torch reference ops, not the HIP kernels (bf16 only): expect a much "
                "slower step; use precision bf16-true / bf16-mixed for the kernel path", key)
        REFERENCE_ON_GPU[key] = REFERENCE_ON_GPU.get(key, 0) + 1
        return False
    return False


_KERNEL_ERRORS = {
    0: "a position id outside the RoPE cos/sin table (max_position_embeddings too small for the data?)",
    1: "a label that is neither ignore_index nor a vocabulary id",
}


def check_kernel_errors(device: torch.device | None = None, raise_error: bool = True) -> list[str]:
    """Read (one host sync) and clear the device-side index-check words the HIP kernels set when a
    data-dependent index is out of range (csrc/bindings.cpp ``kernel_errors``: the kernels clamp / skip,
    so memory stays safe, and the condition is reported here). Raises ``RuntimeError`` when any is set
    unless ``raise_error`` is False; returns the messages."""
    if device is not None and device.type != "cuda":
        return []
    if not torch.cuda.is_available() or not _load():
        return []
    with torch.cuda.device(device if device is not None else torch.cuda.current_device()):
        words = torch.ops.llmt.kernel_errors()
        host = words.tolist()
        if not any(host):
            return []
        words.zero_()
    msgs = [_KERNEL_ERRORS.get(i, f"kernel error word {i}") for i, v in enumerate(host) if v]
    if raise_error:
        raise RuntimeError("HIP kernel index check failed: " + "; ".join(msgs))
    return msgs
