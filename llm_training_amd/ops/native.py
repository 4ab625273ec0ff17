"""Loader for the in-tree gfx950 extension (``llm_training_amd/_C.so``).

The HIP kernels are the ONLY implementation used for GPU tensors: if the library is missing or
fails to load on a machine with a GPU, :func:`lib` raises instead of silently falling back to
PyTorch. CPU tensors use the torch reference ops in :mod:`llm_training_amd.ops.reference`.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

_LOCK = threading.Lock()
_LOADED: bool | None = None
_ERR: Exception | None = None
LIB_PATH = Path(__file__).resolve().parent.parent / "_C.so"


def _load() -> bool:
    global _LOADED, _ERR
    with _LOCK:
        if _LOADED is not None:
            return _LOADED
        try:
            if not LIB_PATH.exists() and os.environ.get("LLMT_AUTOBUILD", "1") == "1":
                from .. import _build

                _build.build()
            torch.ops.load_library(str(LIB_PATH))
            _LOADED = True
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


def use_native(t: torch.Tensor) -> bool:
    """bf16 GPU tensors always go to the HIP kernels (no silent fallback: a missing library raises).

    The kernels are bf16 MFMA kernels; fp32 GPU tensors (``precision: 32-true``) and CPU tensors run
    the torch reference ops of :mod:`llm_training_amd.ops.reference`."""
    if t.device.type == "cuda":
        lib()
        return t.dtype == torch.bfloat16
    return False
