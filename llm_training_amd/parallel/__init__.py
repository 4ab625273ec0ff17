from .context import ParallelContext, init_distributed, resolve_mesh_sizes
from .engine import DataParallelEngine, freeze_modules

__all__ = ["ParallelContext", "init_distributed", "resolve_mesh_sizes", "DataParallelEngine", "freeze_modules"]
