"""Process bootstrap and the 2-D (data x tensor) parallel layout.

Reference: FSDP2Strategy mesh sizing and DeviceMesh('data_parallel', 'tensor_parallel')
(src/llm_training/lightning/strategy/fsdp2/fsdp2_strategy.py:105-133,181-199) and process-group init
(:411-420). Here one process drives one GPU (torchrun / srun / env), the backend is ``nccl`` (= RCCL
on ROCm: rings/trees over xGMI) for GPUs and ``gloo`` for CPU, and TP groups are the INNER,
contiguous ranks (same node, directly linked by xGMI), DP groups the outer ones.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist


def env_rank_info() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from torchrun / SLURM / defaults."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        rank = int(os.environ["RANK"])
        world = int(os.environ["WORLD_SIZE"])
        local = int(os.environ.get("LOCAL_RANK", rank))
        return rank, local, world
    if "SLURM_PROCID" in os.environ and int(os.environ.get("SLURM_NTASKS", "1")) > 1:
        rank = int(os.environ["SLURM_PROCID"])
        world = int(os.environ["SLURM_NTASKS"])
        local = int(os.environ.get("SLURM_LOCALID", 0))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        os.environ.setdefault("LOCAL_RANK", str(local))
        host = first_slurm_host(os.environ.get("SLURM_JOB_NODELIST", os.environ.get("SLURM_NODELIST", "")))
        if host:
            os.environ.setdefault("MASTER_ADDR", host)
        jid = os.environ.get("SLURM_JOB_ID")
        if jid and jid.isdigit():
            os.environ.setdefault("MASTER_PORT", str(20000 + int(jid) % 20000))
        return rank, local, world
    return 0, 0, 1


def first_slurm_host(nodelist: str) -> str | None:
    """First host of a SLURM node list ("gpu[03-05,9],cpu1" -> "gpu03") without calling scontrol."""
    nodelist = nodelist.strip()
    if not nodelist:
        return None
    head, depth = [], 0
    for ch in nodelist:  # first top-level comma-separated item
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        elif ch == "," and depth == 0:
            break
        head.append(ch)
    item = "".join(head)
    if "[" not in item:
        return item
    prefix, rng = item.split("[", 1)
    first = rng.rstrip("]").split(",")[0].split("-")[0]
    return prefix + first


def init_distributed(backend: str | None = None, timeout_minutes: float = 30.0, device_type: str | None = None):
    """Initialise torch.distributed once (no-op for world size 1). Returns (rank, local_rank, world, device)."""
    rank, local, world = env_rank_info()
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    # test knobs: LLMT_DIST_BACKEND overrides the backend, LLMT_SHARED_DEVICE=1 puts every rank on GPU 0
    # (several ranks on one GPU need gloo: RCCL refuses two ranks on one device)
    backend = os.environ.get("LLMT_DIST_BACKEND") or backend
    if os.environ.get("LLMT_SHARED_DEVICE") == "1":
        local = 0
    if device_type == "cuda":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        be = backend or ("nccl" if device_type == "cuda" else "gloo")
        kw = {}
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(be, rank=rank, world_size=world,
                                timeout=datetime.timedelta(minutes=timeout_minutes), **kw)
    return rank, local, world, device


@dataclass
class ParallelContext:
    """Ranks and groups of a (dp x tp) layout; tp is the inner (contiguous-rank) dimension."""

    world_size: int = 1
    rank: int = 0
    dp_size: int = 1
    tp_size: int = 1
    dp_rank: int = 0
    tp_rank: int = 0
    dp_group: object = None
    tp_group: object = None
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    sequence_parallel: bool = True

    @property
    def tp(self) -> bool:
        return self.tp_size > 1

    @property
    def dp(self) -> bool:
        return self.dp_size > 1

    @classmethod
    def single(cls, device=None) -> "ParallelContext":
        return cls(device=torch.device(device) if device is not None else torch.device("cpu"))

    @classmethod
    def create(cls, data_parallel_size="auto", tensor_parallel_size=1, device=None) -> "ParallelContext":
        world = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        dp, tp = resolve_mesh_sizes(world, data_parallel_size, tensor_parallel_size)
        pc = cls(world_size=world, rank=rank, dp_size=dp, tp_size=tp, device=torch.device(device or "cpu"))
        pc.tp_rank = rank % tp
        pc.dp_rank = rank // tp
        if world > 1:
            # every rank must create every group in the same order
            for d in range(dp):
                ranks = list(range(d * tp, (d + 1) * tp))
                g = dist.new_group(ranks) if tp > 1 else None
                if rank in ranks:
                    pc.tp_group = g
            for t in range(tp):
                ranks = list(range(t, world, tp))
                g = dist.new_group(ranks) if dp > 1 else None
                if rank in ranks:
                    pc.dp_group = g
            if tp == 1:
                pc.dp_group = dist.group.WORLD
            if dp == 1:
                pc.tp_group = dist.group.WORLD
        return pc


def resolve_mesh_sizes(world: int, dp="auto", tp=1, num_nodes: int = 1) -> tuple[int, int]:
    """Mesh sizing rules of the reference (fsdp2_strategy.py:181-191)."""
    if dp == "auto" and tp == "auto":
        dp = num_nodes
        tp = world // num_nodes
    elif dp == "auto":
        tp = int(tp)
        dp = world // tp
    elif tp == "auto":
        dp = int(dp)
        tp = world // dp
    dp, tp = int(dp), int(tp)
    if dp * tp != world:
        raise ValueError(f"data_parallel_size ({dp}) x tensor_parallel_size ({tp}) != world size ({world})")
    return dp, tp
