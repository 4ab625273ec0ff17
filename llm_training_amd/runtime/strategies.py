"""Distributed strategies (YAML ``trainer.strategy``), all executed by the flat-buffer engine.

Reference strategy surfaces: FSDP2Strategy (src/llm_training/lightning/strategy/fsdp2/
fsdp2_strategy.py:49-78), DeepSpeedStrategy (lightning/strategy/deepspeed/deepspeed_strategy.py:17-72)
and Lightning's ddp / single-device. The knobs keep their names; the ones that only make sense for
DeepSpeed's engine (bucket sizes, ZeRO++ quantisation) are accepted and recorded but the
engine's own choices apply (per-layer units; see parallel/engine.py for why no extra bucketing is
needed on xGMI).
"""
from __future__ import annotations

import datetime
import logging
from dataclasses import dataclass, field
from typing import Any

logger = logging.getLogger("llm_training")


@dataclass
class Strategy:
    zero_stage: int = 0
    data_parallel_size: Any = "auto"
    tensor_parallel_size: Any = 1
    process_group_backend: str | None = None
    timeout: Any = datetime.timedelta(minutes=30)
    reshard_after_forward: bool = True
    grad_reduce_dtype: str | None = None
    overlap_comm: bool = True
    save_distributed_checkpoint: bool = True
    offload_optimizer: bool = False
    offload_parameters: bool = False
    offload_optimizer_device: str = "cpu"
    nvme_path: str | None = None
    zero_hpz_partition_size: int = 1
    zero_quantized_weights: bool = False
    zero_quantized_gradients: bool = False
    param_dtype: str | None = None  # FSDP2 MixedPrecisionPolicy.param_dtype (overrides the precision's)
    extra: dict = field(default_factory=dict)

    def engine_kwargs(self) -> dict:
        """Keyword arguments of :class:`DataParallelEngine` this strategy selects."""
        return {"offload_optimizer": self.offload_optimizer, "offload_params": self.offload_parameters,
                "offload_device": self.offload_optimizer_device, "nvme_path": self.nvme_path,
                "hpz_partition_size": self.zero_hpz_partition_size,
                "quantized_weights": self.zero_quantized_weights,
                "quantized_gradients": self.zero_quantized_gradients}

    @property
    def timeout_minutes(self) -> float:
        t = self.timeout
        if isinstance(t, datetime.timedelta):
            return t.total_seconds() / 60
        return float(t)


class SingleDeviceStrategy(Strategy):
    def __init__(self, **kw):
        super().__init__(zero_stage=0, data_parallel_size=1, tensor_parallel_size=1)
        self.extra = kw


class DDPStrategy(Strategy):
    def __init__(self, process_group_backend=None, timeout=datetime.timedelta(minutes=30), **kw):
        super().__init__(zero_stage=0, process_group_backend=process_group_backend, timeout=timeout)
        self.extra = kw


class FSDP2Strategy(Strategy):
    """ZeRO-3 (parameters, gradients and optimizer state sharded over the data-parallel group) x TP."""

    def __init__(self, data_parallel_size="auto", tensor_parallel_size=1, save_distributed_checkpoint=True,
                 process_group_backend=None, timeout=datetime.timedelta(minutes=30), reshard_after_forward=True,
                 mp_policy=None, offload_policy=None, use_master_weights=True, zero_stage: int | None = None, **kw):
        stage = 3 if zero_stage is None else int(zero_stage)
        hpz = 1
        if not isinstance(reshard_after_forward, bool):
            # FSDP2: an int is the world size to reshard to after forward (a non-trivial divisor of the
            # shard group) = a secondary partition over that many ranks, kept for the backward re-gather:
            # the engine's hpZ partition (ZeRO++), sized to one node's xGMI-connected GPUs
            hpz = int(reshard_after_forward)
            if hpz < 1:
                raise ValueError(f"reshard_after_forward must be a bool or a positive int, got {reshard_after_forward!r}")
            reshard_after_forward = True
        if zero_stage is None and reshard_after_forward is False:
            # reference TP examples set reshard_after_forward=false: params stay gathered across the
            # step; with 288 GB of HBM that is exactly ZeRO-2 (sharded grads + optimizer state)
            stage = 2
        super().__init__(zero_stage=stage, data_parallel_size=data_parallel_size,
                         tensor_parallel_size=tensor_parallel_size, process_group_backend=process_group_backend,
                         timeout=timeout, reshard_after_forward=bool(reshard_after_forward),
                         save_distributed_checkpoint=save_distributed_checkpoint)
        # FSDP2 OffloadPolicy (CPUOffloadPolicy / {"class_path": ...CPUOffloadPolicy} / True): the fp32
        # master and Adam moments move to pinned host memory, updated by the native host AdamW, and
        # (ZeRO-3) the bf16 parameter shards too (CPUOffloadPolicy offloads parameters, fsdp2_strategy.py:58)
        self.offload_optimizer = _wants_offload(offload_policy)
        self.offload_parameters = self.offload_optimizer and stage >= 3
        self.zero_hpz_partition_size = hpz
        # FSDP2 MixedPrecisionPolicy (object, dict or {class_path, init_args}): param_dtype = the dtype
        # parameters are gathered / computed in, reduce_dtype = the gradient reduce-scatter dtype
        pd, rd = _mp_policy_dtypes(mp_policy)
        self.param_dtype, self.grad_reduce_dtype = pd, rd
        _check_kwargs("FSDP2Strategy", kw, FSDP2_PASSIVE)
        self.extra = {"mp_policy": mp_policy, "use_master_weights": use_master_weights, **kw}


class DeepSpeedStrategy(Strategy):
    """ZeRO stage 1/2/3 with DeepSpeed's argument names (stage=2 default, as in the reference)."""

    def __init__(self, stage: int = 2, offload_optimizer: bool = False, offload_parameters: bool = False,
                 offload_optimizer_device: str = "cpu", nvme_path: str = "/local_nvme", overlap_comm: bool = True,
                 process_group_backend=None, timeout=datetime.timedelta(minutes=30), zero_hpz_partition_size: int = 1,
                 zero_quantized_weights: bool = False, zero_quantized_gradients: bool = False, **kw):
        super().__init__(zero_stage=int(stage), process_group_backend=process_group_backend, timeout=timeout,
                         overlap_comm=overlap_comm)
        if offload_optimizer_device not in ("cpu", "nvme"):
            raise ValueError(f"offload_optimizer_device must be cpu or nvme, got {offload_optimizer_device!r}")
        self.offload_optimizer = bool(offload_optimizer) or offload_optimizer_device == "nvme"
        self.offload_optimizer_device = offload_optimizer_device
        self.nvme_path = nvme_path
        if offload_parameters and int(stage) < 3:
            raise ValueError("DeepSpeedStrategy: offload_parameters needs stage 3 (as in DeepSpeed)")
        self.offload_parameters = bool(offload_parameters)
        self.zero_hpz_partition_size = int(zero_hpz_partition_size)
        self.zero_quantized_weights = bool(zero_quantized_weights)
        self.zero_quantized_gradients = bool(zero_quantized_gradients)
        _check_kwargs("DeepSpeedStrategy", kw, DEEPSPEED_PASSIVE)
        self.extra = dict(kw)


# upstream DeepSpeedStrategy / Lightning arguments (deepspeed_strategy.py:17-72) that the engine takes no
# action on (buffer / bucket / aio tuning of DeepSpeed's own engine, fp16 loss scaling): accepted so
# reference configs load, recorded in ``extra``; any other name is a typo and raises
DEEPSPEED_PASSIVE = {
    "accelerator", "zero_optimization", "remote_device", "offload_params_device", "params_buffer_count",
    "params_buffer_size", "max_in_cpu", "optimizer_buffer_count", "block_size", "queue_depth", "single_submit",
    "overlap_events", "thread_count", "pin_memory", "sub_group_size", "contiguous_gradients",
    "allgather_partitions", "reduce_scatter", "allgather_bucket_size", "reduce_bucket_size",
    "zero_allow_untested_optimizer", "logging_batch_size_per_gpu", "config", "logging_level", "parallel_devices",
    "cluster_environment", "loss_scale", "initial_scale_power", "loss_scale_window", "hysteresis",
    "min_loss_scale", "partition_activations", "cpu_checkpointing", "contiguous_memory_optimization",
    "synchronize_checkpoint_boundary", "load_full_weights", "precision_plugin", "exclude_frozen_parameters",
    "raise_error_at_min_scale", "zero3_leaf_modules", "stage3_max_live_parameters", "stage3_max_reuse_distance",
    "stage3_prefetch_bucket_size", "stage3_param_persistence_threshold"}
FSDP2_PASSIVE = {"accelerator", "parallel_devices", "cluster_environment", "checkpoint_io", "precision_plugin",
                 "precision", "use_master_weights"}


def _dtype_name(d) -> str | None:
    if d is None:
        return None
    import torch
    if isinstance(d, torch.dtype):
        return str(d).replace("torch.", "")
    name = str(d).replace("torch.", "")
    name = {"bf16": "bfloat16", "fp32": "float32", "fp16": "float16", "half": "float16", "float": "float32"}.get(
        name, name)
    if not isinstance(getattr(torch, name, None), torch.dtype):
        raise ValueError(f"not a dtype: {d!r}")
    return name


def _mp_policy_dtypes(mp) -> tuple[str | None, str | None]:
    """(param_dtype, reduce_dtype) names of an FSDP2 MixedPrecisionPolicy given as the torch object, a
    plain dict or a {class_path, init_args} dict; output_dtype / cast_forward_inputs have no separate
    meaning here (activations are in the parameter dtype)."""
    if mp is None:
        return None, None
    if isinstance(mp, dict):
        args = mp.get("init_args", mp) if "class_path" in mp else mp
        pd, rd = args.get("param_dtype"), args.get("reduce_dtype")
    else:
        pd, rd = getattr(mp, "param_dtype", None), getattr(mp, "reduce_dtype", None)
    pd, rd = _dtype_name(pd), _dtype_name(rd)
    if pd is not None and pd not in ("bfloat16", "float32"):
        raise ValueError(f"mp_policy.param_dtype {pd}: the MI355X kernels run bf16 (or fp32 via torch ops)")
    return pd, rd


def _check_kwargs(cls_name: str, kw: dict, allowed: set):
    bad = sorted(k for k in kw if k not in allowed)
    if bad:
        import difflib
        hint = {k: difflib.get_close_matches(k, sorted(allowed), n=1) for k in bad}
        raise TypeError(f"{cls_name} got unknown argument(s): " + ", ".join(
            f"{k!r}" + (f" (did you mean {h[0]!r}?)" if h else "") for k, h in hint.items()))


def _wants_offload(policy) -> bool:
    if policy is None or policy is False or policy == {}:
        return False
    if policy is True:
        return True
    if isinstance(policy, dict):  # jsonargparse form: {"class_path": "torch.distributed.fsdp.CPUOffloadPolicy"}
        return "CPUOffload" in str(policy.get("class_path", "")) or bool(policy.get("offload", False))
    return "CPUOffload" in type(policy).__name__  # the base OffloadPolicy means "no offload"


STRATEGY_NAMES = {"ddp": DDPStrategy, "auto": DDPStrategy, "single_device": SingleDeviceStrategy,
                  "fsdp": FSDP2Strategy, "fsdp2": FSDP2Strategy, "deepspeed": DeepSpeedStrategy,
                  "deepspeed_stage_1": lambda: DeepSpeedStrategy(stage=1),
                  "deepspeed_stage_2": lambda: DeepSpeedStrategy(stage=2),
                  "deepspeed_stage_3": lambda: DeepSpeedStrategy(stage=3)}


def resolve_strategy(s) -> Strategy:
    if s is None:
        return DDPStrategy()
    if isinstance(s, Strategy):
        return s
    if isinstance(s, str):
        return STRATEGY_NAMES[s]()
    raise TypeError(f"unknown strategy {s!r}")
