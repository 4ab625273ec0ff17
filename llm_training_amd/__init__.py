"""llm_training_amd — an MI355X-native (gfx950, ROCm) LLM training framework.

Same capabilities and YAML surface as cchou0519/LLM-Training (``llm-training fit --config cfg.yaml``),
re-designed for CDNA4: hand-written HIP kernels for the hot ops, a flat-buffer ZeRO engine and
tensor/sequence parallelism over RCCL/xGMI, one process per GPU.
"""
import logging
import os

# RCCL on MI355X hosts needs dmabuf IPC (legacy IPC handles are rejected by the host driver); set
# before anything initialises HIP, for torchrun / srun launches too (see llm_training_amd/launch.py)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

__version__ = "0.1.0"

logger = logging.getLogger("llm_training")
if not logger.handlers:
    _h = logging.StreamHandler()
    _h.setFormatter(logging.Formatter("[%(asctime)s] [%(levelname)s] %(message)s", "%Y-%m-%d %H:%M:%S"))
    logger.addHandler(_h)
    logger.setLevel(os.environ.get("LLMT_LOG_LEVEL", "INFO").upper())  # e.g. DEBUG: GEMM layout choices
    logger.propagate = False
