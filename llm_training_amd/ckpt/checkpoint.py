"""Sharded, resumable, reshard-able training checkpoints: one file per rank, no full gather.

Reference behaviour: Lightning checkpoint dict with state_dict / optimizer / lr scheduler / loop
progress / config (src/llm_training/lightning/strategy/fsdp2/fsdp2_strategy.py:315-409 —
FSDP2 writes DCP shards per rank; callbacks/save_config_callback.py:42-44) and the resumable data
loader (data/resumable_dataloader.py).

Layout of ``<dir>/``:
- ``meta.json``                      step / epoch / batch_idx / consumed counters / scheduler / parallel
                                     layout / the resolved YAML config (so ``convert-to-hf`` can rebuild
                                     the model). Written last by rank 0 — its presence plus every rank's
                                     ``.done`` marker means the checkpoint is complete.
- ``shard-tp{t}-dp{d}.safetensors``  what rank (t, d) owns: for every trainable parameter the slice of
                                     its flattened ``master`` / ``exp_avg`` / ``exp_avg_sq`` (fp32) that
                                     falls in this rank's range of the unit's flat buffer (its ZeRO shard;
                                     at stage 0 the DP ranks split the replicated state so every rank
                                     writes 1/dp), and ``model.<name>`` in full for frozen parameters.
- ``shard-tp{t}-dp{d}.json``         index: key -> [start, end, full shape] in flattened-parameter
                                     elements.
- ``shard-tp{t}-dp{d}.done``         written after the rank's files are closed.
- ``rng-tp{t}-dp{d}.safetensors``    the rank's CPU / GPU generator states (NEFTune noise, dropout
                                     masks and attention-dropout seeds continue exactly on resume with
                                     the same layout).

``save_distributed_checkpoint: false`` (FSDP2Strategy, reference fsdp2_strategy.py:391-393) writes ONE
file instead: ``<name>.ckpt`` is a safetensors file holding every parameter's full (TP-unsharded)
master / exp_avg / exp_avg_sq, the frozen parameters, every rank's RNG state and the meta JSON (file
metadata). The ranks write their shards to a scratch directory first; rank 0 assembles the file from it.
Format ``llm_training_amd/v1`` checkpoints (one ``tp{t}.safetensors`` per TP rank keyed by parameter
name, full tensors) are still readable.

Each rank moves only its own shard to the host (12 B/param / dp) and the files are written on a
background thread (``save_checkpoint(..., async_write=True)``; the next save or ``wait_for_pending_saves``
joins it). Loading reads, for every local parameter range of the NEW layout, only the overlapping
pieces (safetensors ``get_slice``), so any (dp, ZeRO stage) saved layout loads into any other; a
tensor-parallel size change assembles one full parameter at a time and re-shards it with the model's
own TP rules. bf16 parameters are re-derived from the fp32 masters (the fused AdamW writes them from
the master in the first place).
"""
from __future__ import annotations

import json
import logging
import os
import threading
from pathlib import Path

import torch
import torch.distributed as dist
from safetensors import safe_open
from safetensors.torch import save_file

logger = logging.getLogger("llm_training")

FORMAT = "llm_training_amd/v2"
FORMAT_V1 = "llm_training_amd/v1"
KINDS = ("master", "exp_avg", "exp_avg_sq")
_pending: list[threading.Thread] = []
_errors: list[BaseException] = []  # exceptions of background writers, re-raised by wait_for_pending_saves


def shard_name(tp: int, dp: int) -> str:
    return f"shard-tp{tp}-dp{dp}"


def rng_name(tp: int, dp: int) -> str:
    return f"rng-tp{tp}-dp{dp}.safetensors"


def wait_for_pending_saves():
    """Join the background shard writers; a failed write raises here (disk full, I/O error) instead of
    leaving an incomplete checkpoint behind silently."""
    while _pending:
        _pending.pop(0).join()
    if _errors:
        errs = list(_errors)
        _errors.clear()
        raise RuntimeError(f"checkpoint write failed on a background thread: {errs[0]!r}") from errs[0]


def rng_state() -> dict[str, torch.Tensor]:
    """This rank's generator states (CPU, and the current GPU's when it is in use)."""
    st = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st: dict[str, torch.Tensor]):
    if "cpu" in st:
        torch.set_rng_state(st["cpu"].to(torch.uint8))
    if "cuda" in st and torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.set_rng_state(st["cuda"].to(torch.uint8))


def _write_range(engine, u) -> tuple[int, int]:
    """Flat range of unit ``u`` that this rank writes: its ZeRO shard, or its 1/dp part of replicated
    state (stage 0), or everything on dp rank 0 (TP-replicated units)."""
    dp = u.dp
    r = engine.pc.dp_rank if dp > 1 else 0
    sn = u.numel // dp
    if u.replicated and engine.pc.dp_rank != 0:
        return 0, 0
    return r * sn, (r + 1) * sn


def collect_shard(trainer) -> tuple[dict[str, torch.Tensor], dict[str, list]]:
    """This rank's pieces (CPU tensors) and their index."""
    eng = trainer.engine
    model = trainer.lm.model
    names = {id(p): n for n, p in model.named_parameters()}
    eng.wait_params()
    tensors: dict[str, torch.Tensor] = {}
    index: dict[str, list] = {}
    for u in eng.units:
        a, b = _write_range(eng, u)
        if b <= a:
            continue
        sa, _ = eng.shard_range(u)  # where the locally held optimizer state starts in flat coords
        # u.shapes, not p.shape: a ZeRO-3 unit's parameters are empty views while it is not gathered
        for pi, (p, o, shp) in enumerate(zip(u.params, u.offsets, u.shapes)):
            s, e = max(o, a), min(o + shp.numel(), b)
            if e <= s:
                continue
            n = names[id(p)]
            for kind in eng.state_kinds():
                src = eng.unit_state(u, kind)
                has = eng.state_params(u, kind)
                if src is None or (has is not None and pi not in has):
                    continue
                piece = src[s - sa:e - sa]
                tensors[f"{kind}.{n}"] = piece.detach().to("cpu", copy=True)
                index[f"{kind}.{n}"] = [s - o, e - o, list(shp)]
    if eng.pc.dp_rank == 0:  # frozen parameters are not engine units: always resident in full
        for n, p in model.named_parameters():
            if not p.requires_grad:
                tensors["model." + n] = p.detach().reshape(-1).to("cpu", copy=True)
                index["model." + n] = [0, p.numel(), list(p.shape)]
    return tensors, index


def _write_files(path: str, base: str, tensors: dict, index: dict):
    save_file({k: v.contiguous() for k, v in tensors.items()}, os.path.join(path, base + ".safetensors"))
    with open(os.path.join(path, base + ".json"), "w") as f:
        json.dump(index, f)
    Path(path, base + ".done").touch()


def _write_files_bg(path: str, base: str, tensors: dict, index: dict):
    try:
        _write_files(path, base, tensors, index)
    except BaseException as e:  # noqa: BLE001 - surfaced by wait_for_pending_saves
        logger.error("background checkpoint write of %s/%s failed: %r", path, base, e)
        _errors.append(e)


def _meta(trainer) -> dict:
    pc, eng = trainer.pc, trainer.engine
    return {
        "format": FORMAT,
        "trainer": trainer.state.state_dict(),
        "scheduler": trainer.scheduler.state_dict() if trainer.scheduler else None,
        "optimizer_step": eng.step_count,
        "tp_size": pc.tp_size, "dp_size": pc.dp_size, "zero_stage": eng.stage,
        "param_dtype": str(eng.param_dtype).replace("torch.", ""),
        "optimizer_kinds": eng.state_kinds(),
        "loss_scaler": trainer.scaler.state_dict() if getattr(trainer, "scaler", None) is not None else None,
        # stateful callbacks (EarlyStopping counters), keyed by class name as Lightning's state_key
        "callbacks": {type(cb).__name__: cb.state_dict() for cb in getattr(trainer, "callbacks", [])
                      if hasattr(cb, "state_dict") and hasattr(cb, "load_state_dict")},
        "config": trainer.config_dict,
        "model_class": f"{type(trainer.lm.model).__module__}.{type(trainer.lm.model).__qualname__}",
        "model_config": trainer.lm.model.config.model_dump(mode="json"),
    }


def save_checkpoint(trainer, path: str, async_write: bool = False, consolidated: bool | None = None):
    pc = trainer.pc
    if consolidated is None:
        consolidated = not getattr(getattr(trainer, "strategy", None), "save_distributed_checkpoint", True)
    wait_for_pending_saves()
    if consolidated:
        _save_consolidated(trainer, path)
        return
    tensors, index = collect_shard(trainer)
    os.makedirs(path, exist_ok=True)
    base = shard_name(pc.tp_rank, pc.dp_rank)
    # the rank's generator states (+ a generic optimizer's non-element-wise state: step counters, factored
    # statistics) in one small file; restored when the layout is unchanged
    extra = {f"opt.{k}": v for k, v in trainer.engine.optimizer_extra_state().items()}
    save_file({**rng_state(), **extra}, os.path.join(path, rng_name(pc.tp_rank, pc.dp_rank)))
    if async_write:
        t = threading.Thread(target=_write_files_bg, args=(path, base, tensors, index), daemon=False)
        t.start()
        _pending.append(t)
    else:
        _write_files(path, base, tensors, index)
    if pc.rank == 0:
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(_meta(trainer), f, indent=1, default=str)
    if dist.is_initialized():
        dist.barrier()
    if pc.rank == 0:
        logger.info("saved checkpoint %s%s", path, " (files written in the background)" if async_write else "")


def _save_consolidated(trainer, path: str):
    """One safetensors file with full, TP-unsharded tensors (see the module docstring)."""
    import shutil
    pc = trainer.pc
    scratch = path + ".parts"
    save_checkpoint(trainer, scratch, async_write=False, consolidated=False)
    if pc.rank == 0:
        reader = ShardReader(scratch)
        model = trainer.lm.model
        out: dict[str, torch.Tensor] = {}
        for key in reader.pieces[0]:
            kind, name = key.split(".", 1)
            parts = [reader.full(t, key) for t in range(reader.tp)]
            out[key] = _tp_unshard(model, name, parts).contiguous()
        for t in range(reader.tp):
            for d in range(reader.dp):
                rf = os.path.join(scratch, rng_name(t, d))
                if os.path.exists(rf):
                    with safe_open(rf, framework="pt") as f:
                        for k in f.keys():
                            out[f"rng.tp{t}.dp{d}.{k}"] = f.get_tensor(k)
        meta = dict(reader.meta, consolidated=True)
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        save_file(out, tmp, metadata={"format": FORMAT, "meta": json.dumps(meta, default=str)})
        os.replace(tmp, path)  # the file appears complete or not at all
        shutil.rmtree(scratch, ignore_errors=True)
        logger.info("saved consolidated checkpoint %s", path)
    if dist.is_initialized():
        dist.barrier()


def read_meta(path: str) -> dict:
    if os.path.isfile(path):  # consolidated single-file checkpoint: the meta rides in the file metadata
        with safe_open(path, framework="pt") as f:
            return json.loads(f.metadata()["meta"])
    with open(os.path.join(path, "meta.json")) as f:
        return json.load(f)


def is_complete(path: str | os.PathLike) -> bool:
    p = Path(path)
    if p.is_file():  # written to a temporary name and renamed: present means complete
        try:
            read_meta(str(p))
            return True
        except Exception:  # noqa: BLE001 - not one of our checkpoint files
            return False
    if not (p / "meta.json").is_file():
        return False
    try:
        meta = json.loads((p / "meta.json").read_text())
    except (ValueError, OSError):
        return False
    tp, dp = int(meta.get("tp_size", 1)), int(meta.get("dp_size", 1))
    if meta.get("format") == FORMAT_V1:
        return all((p / f"tp{t}.safetensors").is_file() for t in range(tp))
    return all((p / (shard_name(t, d) + ".done")).is_file() for t in range(tp) for d in range(dp))


class ShardReader:
    """Reads element ranges of flattened parameters from the per-rank pieces of a checkpoint (v2 shard
    directories, consolidated single files, and v1 per-TP-rank files of full tensors)."""

    def __init__(self, path: str):
        self.path = path
        self.meta = read_meta(path)
        dt = self.meta.get("param_dtype", "bfloat16")
        self.param_dtype = getattr(torch, dt) if isinstance(dt, str) else torch.bfloat16
        self._files: dict[str, object] = {}
        self._flat: dict[tuple[str, str], torch.Tensor] = {}
        if os.path.isfile(path):  # consolidated: full tensors of a tp=1 / dp=1 layout
            self.tp = self.dp = 1
            self.pieces = [{}]
            f = self._file(path)
            for k in f.keys():
                if not k.startswith("rng."):
                    shape = tuple(f.get_slice(k).get_shape())
                    self.pieces[0][k] = [(0, _numel(shape), shape, path)]
            return
        self.tp = int(self.meta.get("tp_size", 1))
        self.dp = int(self.meta.get("dp_size", 1))
        # per tp rank: key -> [(start, end, shape, file)]
        self.pieces: list[dict[str, list]] = [dict() for _ in range(self.tp)]
        if self.meta.get("format") == FORMAT_V1:
            for t in range(self.tp):
                fn = os.path.join(path, f"tp{t}.safetensors")
                f = self._file(fn)
                for k in f.keys():
                    shape = tuple(f.get_slice(k).get_shape())
                    self.pieces[t][k] = [(0, _numel(shape), shape, fn)]
            return
        for t in range(self.tp):
            for d in range(self.dp):
                base = shard_name(t, d)
                with open(os.path.join(path, base + ".json")) as f:
                    idx = json.load(f)
                fn = os.path.join(path, base + ".safetensors")
                for k, (s, e, shape) in idx.items():
                    self.pieces[t].setdefault(k, []).append((s, e, tuple(shape), fn))

    def _file(self, fn):
        f = self._files.get(fn)
        if f is None:
            f = safe_open(fn, framework="pt", device="cpu")
            self._files[fn] = f
        return f

    def has(self, t: int, key: str) -> bool:
        return key in self.pieces[t]

    def shape(self, t: int, key: str) -> tuple:
        return self.pieces[t][key][0][2]

    def _slice(self, fn: str, key: str, a: int, b: int) -> torch.Tensor:
        sl = self._file(fn).get_slice(key)
        if len(sl.get_shape()) <= 1:
            return sl[a:b]
        # full multi-dimensional tensors (v1 / consolidated): flatten once, then slice
        ck = (fn, key)
        flat = self._flat.get(ck)
        if flat is None:
            self._flat.clear()  # one tensor cached at a time
            flat = self._file(fn).get_tensor(key).reshape(-1)
            self._flat[ck] = flat
        return flat[a:b]

    def read(self, t: int, key: str, s: int, e: int) -> torch.Tensor:
        """Elements [s, e) of the flattened tensor ``key`` of saved TP rank ``t``."""
        out = None
        covered = 0
        for ps, pe, _, fn in self.pieces[t][key]:
            a, b = max(s, ps), min(e, pe)
            if b <= a:
                continue
            sl = self._slice(fn, key, a - ps, b - ps)
            if out is None:
                out = torch.empty(e - s, dtype=sl.dtype)
            out[a - s:b - s] = sl
            covered += b - a
        if covered != e - s:
            raise KeyError(f"checkpoint {self.path}: {key}[{s}:{e}] not fully covered ({covered} of {e - s})")
        return out

    def full(self, t: int, key: str) -> torch.Tensor:
        shape = self.shape(t, key)
        return self.read(t, key, 0, _numel(shape)).view(shape)

    def rng(self, tp_rank: int, dp_rank: int) -> dict[str, torch.Tensor] | None:
        """The saved generator states of rank (tp_rank, dp_rank), if the checkpoint has them."""
        if os.path.isfile(self.path):
            f = self._file(self.path)
            pre = f"rng.tp{tp_rank}.dp{dp_rank}."
            st = {k[len(pre):]: f.get_tensor(k) for k in f.keys() if k.startswith(pre)}
            return st or None
        fn = os.path.join(self.path, rng_name(tp_rank, dp_rank))
        if not os.path.exists(fn):
            return None
        with safe_open(fn, framework="pt") as f:
            return {k: f.get_tensor(k) for k in f.keys()}


def _numel(shape) -> int:
    n = 1
    for x in shape:
        n *= int(x)
    return n


def _tp_unshard(model, name: str, parts: list[torch.Tensor]) -> torch.Tensor:
    from ..parallel import tensor_parallel as tpl
    kind, sizes = model._tp_rule(name) if hasattr(model, "_tp_rule") else ("rep", None)
    if len(parts) == 1 or kind == "rep":
        return parts[0]
    if kind == "fused":
        return tpl.unshard_fused_rows(parts, sizes)
    if kind == "cols":
        return torch.cat(parts, 1)
    return torch.cat(parts, 0)[: model.config.vocab_size]


class _LocalParamSource:
    """Element ranges of this rank's (TP-local) parameters, resharding across TP sizes if needed."""

    def __init__(self, reader: ShardReader, model, tp_rank: int, tp_size: int):
        self.r, self.model, self.tp_rank, self.tp_size = reader, model, tp_rank, tp_size
        self.same_tp = reader.tp == tp_size
        self._cache: tuple[str, torch.Tensor] | None = None

    def has(self, key: str) -> bool:
        return self.r.has(0, key)

    def read(self, key: str, s: int, e: int) -> torch.Tensor:
        if self.same_tp:
            return self.r.read(self.tp_rank, key, s, e)
        if self._cache is None or self._cache[0] != key:
            name = key.split(".", 1)[1]
            full = _tp_unshard(self.model, name, [self.r.full(t, key) for t in range(self.r.tp)])
            local = (self.model.shard_full_state_dict({name: full})[name] if self.tp_size > 1 else full)
            self._cache = (key, local.reshape(-1).contiguous())
        return self._cache[1][s:e]


@torch.no_grad()
def load_checkpoint(trainer, path: str, load_optimizer: bool = True):
    if os.path.islink(path):
        path = os.path.join(os.path.dirname(path), os.readlink(path))
    pc, eng = trainer.pc, trainer.engine
    model = trainer.lm.model
    reader = ShardReader(path)
    meta = reader.meta
    if meta.get("format") not in (FORMAT, FORMAT_V1):
        raise ValueError(f"{path}: unsupported checkpoint format {meta.get('format')!r} (expected {FORMAT})")
    src = _LocalParamSource(reader, model, pc.tp_rank, pc.tp_size)
    names = {id(p): n for n, p in model.named_parameters()}
    eng.wait_params()
    # frozen parameters: full tensors
    for n, p in model.named_parameters():
        if not p.requires_grad and src.has("model." + n):
            p.data.copy_(src.read("model." + n, 0, p.numel()).view(p.shape).to(p.device, p.dtype))
    # trainable: this rank's range of every unit, for each optimizer-state kind
    generic = eng.optimizer_factory is not None
    kinds = ["master"] + [k for k in meta.get("optimizer_kinds", KINDS) if k != "master"]
    if not generic and load_optimizer and any(k.startswith("opt:") for k in kinds):
        raise ValueError(f"{path} holds the state of a generic optimizer; resume it with the same optimizer_class")
    gstate: list[dict[str, torch.Tensor]] = [dict() for _ in eng.units]
    gpresent: list[dict[str, set]] = [dict() for _ in eng.units]
    for ui, u in enumerate(eng.units):
        a, b = eng.shard_range(u)
        for kind in kinds:
            if kind != "master" and not load_optimizer:
                continue
            if generic and kind.startswith("opt:"):
                tgt = gstate[ui].setdefault(kind, torch.zeros(u.master.numel(), dtype=torch.float32,
                                                              device=u.master.device))
            elif generic and kind != "master":
                continue  # fused-AdamW moments do not map onto another optimizer's state
            else:
                tgt = getattr(u, kind)
            for pi, (p, o, shp) in enumerate(zip(u.params, u.offsets, u.shapes)):
                s, e = max(o, a), min(o + shp.numel(), b)
                if e <= s:
                    continue
                key = f"{kind}.{names[id(p)]}"
                if not src.has(key):
                    if kind.startswith("opt:"):
                        continue  # this parameter has no such state (e.g. Adafactor's 1-D-only variance)
                    raise KeyError(f"checkpoint {path} has no {key}")
                if kind.startswith("opt:"):
                    gpresent[ui].setdefault(kind, set()).add(pi)
                tgt[s - a:e - a].copy_(src.read(key, s - o, e - o).to(torch.float32))
    same = int(meta.get("tp_size", 1)) == pc.tp_size and int(meta.get("dp_size", 1)) == pc.dp_size
    side = (reader.rng(pc.tp_rank, pc.dp_rank) if same else None) or {}
    if generic and load_optimizer:
        eng.step_count = int(meta.get("optimizer_step", 0))
        eng.load_unit_states(gstate, {k[4:]: v for k, v in side.items() if k.startswith("opt.")}, gpresent)
    eng.sync_params_from_master()
    if load_optimizer:
        eng.step_count = int(meta.get("optimizer_step", 0))
        trainer.state.load_state_dict(meta["trainer"])
        if trainer.scheduler is not None and meta.get("scheduler"):
            trainer.scheduler.load_state_dict(meta["scheduler"])
        if getattr(trainer, "scaler", None) is not None and meta.get("loss_scaler"):
            trainer.scaler.load_state_dict(meta["loss_scaler"])
        for cb in getattr(trainer, "callbacks", []):
            st_cb = (meta.get("callbacks") or {}).get(type(cb).__name__)
            if st_cb is not None and hasattr(cb, "load_state_dict"):
                cb.load_state_dict(st_cb)
        # generator states: exact continuation of NEFTune noise / dropout when the layout is unchanged
        st = {k: v for k, v in side.items() if k in ("cpu", "cuda")}
        if st:
            set_rng_state(st)
        elif pc.rank == 0:
            logger.info("checkpoint %s: random generator states not restored (%s)", path,
                        "layout changed" if not same else "not saved")
    if pc.rank == 0:
        logger.info("resumed from %s (step %d)", path, trainer.state.global_step)


def load_model_state_for_export(path: str) -> tuple[dict, list[dict[str, torch.Tensor]]]:
    """(meta, per-TP-rank model state dicts) from a checkpoint dir, without any process group.

    Trainable parameters come from the fp32 masters cast to the training dtype (exactly what the
    fused AdamW wrote into the bf16 parameters), frozen ones from their stored copy."""
    reader = ShardReader(path)
    parts = []
    for t in range(reader.tp):
        sd = {}
        for key in reader.pieces[t]:
            if "." not in key:
                continue
            kind, name = key.split(".", 1)
            if kind == "model":
                sd[name] = reader.full(t, key)
            elif kind == "master":
                sd[name] = reader.full(t, key).to(reader.param_dtype)
        parts.append(sd)
    return reader.meta, parts
