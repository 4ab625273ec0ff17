"""YAML config loader with the reference's LightningCLI / jsonargparse surface, without those libraries.

Reference surface (src/llm_training/lightning/cli/cli.py:17-83, docs/config.md:7-58):
- top-level keys ``seed_everything``, ``float32_matmul_precision``, ``logging_level``, ``trainer``,
  ``model``, ``data``, ``ckpt_path``, ``output_redirection``, ``tqdm_progress``;
- objects as ``class_path`` + ``init_args`` (recursively), short class names, ``llm_training.*`` paths;
- dotted keys (``init_args.config:`` == ``init_args: {config: ...}``);
- ``${a.b.c}`` interpolation (omegaconf mode, the subset that references other keys);
- CLI overrides ``--a.b.c value`` / ``--a.b.c=value`` and multiple ``--config`` files merged in order;
- numeric strings such as ``1e-5`` (YAML 1.1 parses them as strings) become floats.
"""
from __future__ import annotations

import copy
import inspect
import re
from pathlib import Path
from typing import Any

import yaml

from ..utils.imports import import_object

_FLOAT_RE = re.compile(r"^[+-]?(\d+(\.\d*)?|\.\d+)([eE][+-]?\d+)$")
_INTERP_RE = re.compile(r"\$\{([^}]+)\}")


def _coerce_scalars(x):
    if isinstance(x, dict):
        return {k: _coerce_scalars(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_coerce_scalars(v) for v in x]
    if isinstance(x, str) and _FLOAT_RE.match(x.strip()):
        return float(x)
    return x


def expand_dotted(d: Any) -> Any:
    """{'init_args.config': {...}} -> {'init_args': {'config': {...}}} (recursively, merging)."""
    if isinstance(d, list):
        return [expand_dotted(v) for v in d]
    if not isinstance(d, dict):
        return d
    out: dict = {}
    for k, v in d.items():
        v = expand_dotted(v)
        if isinstance(k, str) and "." in k and not k.startswith("$"):
            head, rest = k.split(".", 1)
            sub = out.setdefault(head, {})
            if not isinstance(sub, dict):
                raise ValueError(f"key {head!r} is both a value and a mapping")
            deep_merge(sub, expand_dotted({rest: v}))
        else:
            if k in out and isinstance(out[k], dict) and isinstance(v, dict):
                deep_merge(out[k], v)
            else:
                out[k] = v
    return out


def deep_merge(dst: dict, src: dict) -> dict:
    for k, v in src.items():
        if k in dst and isinstance(dst[k], dict) and isinstance(v, dict):
            # a new class_path replaces the old object entirely
            if "class_path" in v and v.get("class_path") != dst[k].get("class_path"):
                dst[k] = copy.deepcopy(v)
            else:
                deep_merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _get_path(root: dict, path: str):
    cur: Any = root
    for p in path.split("."):
        if isinstance(cur, dict):
            cur = cur[p]
        elif isinstance(cur, list):
            cur = cur[int(p)]
        else:
            raise KeyError(path)
    return cur


def resolve_interpolations(cfg: dict) -> dict:
    def res(x, depth=0):
        if depth > 20:
            raise ValueError("interpolation cycle")
        if isinstance(x, dict):
            return {k: res(v, depth) for k, v in x.items()}
        if isinstance(x, list):
            return [res(v, depth) for v in x]
        if isinstance(x, str):
            m = _INTERP_RE.fullmatch(x.strip())
            if m:
                return res(_get_path(cfg, m.group(1)), depth + 1)
            return _INTERP_RE.sub(lambda mm: str(res(_get_path(cfg, mm.group(1)), depth + 1)), x)
        return x

    return res(cfg)


def parse_value(s: str):
    try:
        v = yaml.safe_load(s)
    except yaml.YAMLError:
        return s
    return _coerce_scalars(v)


def set_path(cfg: dict, dotted: str, value):
    parts = dotted.split(".")
    cur = cfg
    for p in parts[:-1]:
        if p not in cur or not isinstance(cur[p], dict):
            cur[p] = {}
        cur = cur[p]
    cur[parts[-1]] = value


def load_config(paths: list[str | Path] | str | Path, overrides: list[str] | None = None) -> dict:
    if isinstance(paths, (str, Path)):
        paths = [paths]
    cfg: dict = {}
    for p in paths:
        with open(p) as f:
            d = yaml.safe_load(f) or {}
        deep_merge(cfg, expand_dotted(d))
    for ov in overrides or []:
        k, v = ov.split("=", 1)
        k = k.lstrip("-")
        set_path(cfg, k, parse_value(v))
        cfg = expand_dotted(cfg)
    cfg = resolve_interpolations(cfg)
    return _coerce_scalars(cfg)


def instantiate(spec: Any, _recurse_lists: bool = True):
    """Build objects from ``{class_path, init_args}`` (recursively). Other values pass through."""
    if isinstance(spec, list):
        return [instantiate(v) for v in spec]
    if not isinstance(spec, dict):
        return spec
    if "class_path" not in spec:
        return {k: instantiate(v) for k, v in spec.items()} if _recurse_lists else spec
    cls = import_object(spec["class_path"])
    kwargs = dict(spec.get("init_args") or {})
    for k, v in list(kwargs.items()):
        if isinstance(v, (dict, list)):
            kwargs[k] = instantiate(v)
    if "dict_kwargs" in spec:
        kwargs.update(spec["dict_kwargs"])
    try:
        return cls(**kwargs)
    except TypeError as e:
        sig = None
        try:
            sig = inspect.signature(cls)
        except (TypeError, ValueError):
            pass
        raise TypeError(f"cannot instantiate {spec['class_path']} with {sorted(kwargs)}: {e} (signature {sig})") from e
