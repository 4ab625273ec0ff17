"""Autograd front-ends of the fused hot ops.

GPU tensors run the hand-written gfx950 kernels of ``csrc/`` (loaded by :mod:`.native`); CPU tensors
run :mod:`.reference`. Weight gradients support *gradient-buffer views*: when a parameter carries a
``main_grad`` tensor (a view into the flat per-unit gradient buffer owned by
:class:`llm_training_amd.parallel.engine.DataParallelEngine`), the backward writes (first micro-batch)
or accumulates (later micro-batches) the weight gradient straight into it and returns ``None`` to
autograd — the same trick as fusing gradient accumulation into the weight-gradient GEMM, so there
is no separate ``param.grad`` tensor, no ``grad += new`` pass and the ZeRO engine can reduce-scatter
the flat buffer as soon as a unit's backward is done.

The parameter itself is kept on ``ctx`` (not only in ``save_for_backward``): under non-reentrant
activation checkpointing the saved tensors are recomputed and unpacked as DETACHED aliases, which
carry no ``main_grad`` — the gradient would silently bypass the flat buffer.

Reference parity: these replace the Liger wrappers of src/llm_training/ops/liger_kernel/*.py and
flash-attn calls of src/llm_training/ops/attention_op.py.
"""
from __future__ import annotations

import logging
import math
import os

import torch
from torch.autograd import Function

from . import reference as ref
from .native import available as native_available, lib, use_native

log = logging.getLogger("llm_training.ops")

# ----------------------------------------------------------------------------- GEMM dispatch
# The three GEMMs of a linear layer (fwd x @ W^T, dgrad dy @ W, wgrad dy^T @ x) go to one of:
#  * "lt"   — hipBLASLt through csrc/blaslt.cpp with the solution measured per problem on the device
#             (the library's default heuristic is 1.1 PF/s on the forward layout vs 1.3-1.5 backward);
#  * "blas" — hipBLASLt / rocBLAS through torch.matmul (library default heuristic);
#  * "hip"  — the hand-written gfx950 kernel (csrc/gemm.hip).
# ``LLMT_GEMM`` picks one for all layouts, or per layout as "fwd=lt,dgrad=blas,wgrad=hip". Shapes a path
# cannot take (unaligned / strided operands, K % 32 for "hip") fall back to torch.matmul.
_GEMM_DEFAULT = "lt"


def _gemm_modes() -> dict:
    env = os.environ.get("LLMT_GEMM", _GEMM_DEFAULT).strip().lower()
    if "=" not in env:
        return {k: env for k in ("fwd", "dgrad", "wgrad")}
    modes = {k: _GEMM_DEFAULT for k in ("fwd", "dgrad", "wgrad")}
    for part in env.split(","):
        k, v = part.split("=")
        modes[k.strip()] = v.strip()
    return modes


GEMM_MODES = _gemm_modes()
# Stream-K hipBLASLt solutions spin on partner workgroups and stall when another kernel holds CUs
# (csrc/blaslt.cpp): the engine turns them off whenever collectives or the optimizer overlap compute.
# LLMT_GEMM_STREAMK=0/1 forces the choice.
_SK_ENV = os.environ.get("LLMT_GEMM_STREAMK", "auto").strip().lower()
ALLOW_STREAMK = [_SK_ENV not in ("0", "false", "off")]


def set_streamk(allowed: bool) -> None:
    """Allow stream-K GEMM solutions unless LLMT_GEMM_STREAMK pins the choice."""
    if _SK_ENV == "auto":
        ALLOW_STREAMK[0] = bool(allowed)


def _gemm_operand_ok(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1
            and (t.size(0) <= 1 or t.stride(0) % 8 == 0) and t.data_ptr() % 16 == 0)


def _ld(t: torch.Tensor) -> int:
    return t.stride(0) if t.size(0) > 1 else max(8, (t.size(1) + 7) // 8 * 8)


# Backward layouts through materialised transposes (csrc/elementwise.hip transpose, ~4.7 TB/s).
# hipBLASLt is fastest when both operands are contraction-contiguous (TN, the forward's layout); the
# backward GEMMs of a linear layer are NN (dgrad) and NT (wgrad: the contraction runs over tokens, the
# strided dimension of both token-major operands). Measured at M = 32768 (transposes included,
# profiles/r2_gemm_transposed_layouts*.jsonl):
#   Llama-3-8B dgrad  NN -> TN with W^T   qkv 1.41->1.27  o 0.89->0.73  gate_up 5.50->5.08  down 2.92->2.47 ms
#              wgrad  NT -> NN with dy^T  qkv 1.64->1.45  o 0.95->0.89  down 3.82->3.61;  TT with x^T gate_up 6.31->5.52
#   Phi-3-mini wgrad  o (3072 x 3072): NT 0.61, NN 1.05, TT 1.02 — the best layout is shape-specific
# so each (kind, shape) is decided once by timing its candidate layouts on the live operands (the first
# non-accumulating call; 3 runs each, transposes included) and cached; deterministic mode and
# LLMT_GEMM_LAYOUT_TUNE=0 use the static rule below instead. LLMT_GEMM_TRANSPOSE=0 keeps the direct
# layouts. The weight transpose costs N*K regardless of M, so the dgrad form needs a large token count.
TRANSPOSE_LAYOUTS = [os.environ.get("LLMT_GEMM_TRANSPOSE", "1").strip().lower() not in ("0", "false", "off")]
_LAYOUT_TUNE = os.environ.get("LLMT_GEMM_LAYOUT_TUNE", "1").strip().lower() not in ("0", "false", "off")
_TR_DGRAD_MIN_M = 16384
_TR_WGRAD_MIN_M = 4096
_LAYOUT_CACHE: dict[tuple, str] = {}
# Where each cached choice came from, and how every rank ends up with the same one:
#  * "table": the shipped shape-keyed table (tuning/gemm_layouts_gfx950.json, measured on MI355X by timed
#    runs of the BASELINE workloads): no timing at all, the same choice on every rank and every box;
#  * "timed": measured on this rank's first sight of the problem (shapes the table does not list);
#  * "rank0": adopted from rank 0 by agree_layouts(), which the ZeRO engine calls once after its first
#    optimizer step, so every rank runs rank 0's algorithms from the second step on (a rank whose
#    timings were disturbed by its own collectives cannot pick a different, slower layout);
#  * "static": the rule below (LLMT_DETERMINISTIC=1, LLMT_GEMM_LAYOUT_TUNE=0, graph capture).
# LLMT_GEMM_LAYOUTS=table (default) | timed (ignore the table) | static; LLMT_GEMM_LAYOUT_TABLE=path: another table.
_LAYOUT_SOURCE: dict[tuple, str] = {}
_LAYOUT_MODE = os.environ.get("LLMT_GEMM_LAYOUTS", "table").strip().lower()
_LAYOUT_TABLE_PATH = os.environ.get("LLMT_GEMM_LAYOUT_TABLE") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "gemm_layouts_gfx950.json")
_LAYOUT_TABLE: list = [None]
_AGREED: dict[str, str] = {}  # rank 0's choices for problems this rank has not met yet


def layout_key_str(key: tuple) -> str:
    return "|".join(str(x).replace("torch.", "") for x in key)


def _device_arch() -> str | None:
    try:
        return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]
    except Exception:  # no GPU / no HIP device properties
        return None


def _layout_table() -> dict:
    """The shipped layout table, only on the architecture it was measured on (its ``arch`` field, default
    gfx950): on another GPU the timed first-sight choice is used instead of choices tuned elsewhere."""
    if _LAYOUT_TABLE[0] is None:
        tbl = {}
        if _LAYOUT_MODE == "table" and os.path.exists(_LAYOUT_TABLE_PATH):
            import json
            with open(_LAYOUT_TABLE_PATH) as f:
                doc = json.load(f)
            arch = _device_arch()
            if arch is None or arch == doc.get("arch", "gfx950"):
                tbl = doc.get("layouts", {})
            else:
                log.info("GEMM layout table measured on %s, device is %s: timing layouts instead",
                         doc.get("arch", "gfx950"), arch)
        _LAYOUT_TABLE[0] = tbl
    return _LAYOUT_TABLE[0]


# interleaved timing rounds per layout decision (LLMT_GEMM_LAYOUT_ROUNDS; more rounds time the candidates
# under a longer, more sustained load, as the step runs them)
_LAYOUT_ROUNDS = max(1, int(os.environ.get("LLMT_GEMM_LAYOUT_ROUNDS", "2")))


def _time_variants(variants: dict) -> dict:
    """Milliseconds per call of each variant on the current stream (host-synchronising)."""
    for fn in variants.values():
        fn()  # warm-up (and hipBLASLt's own solution choice for the problem)
    # interleaved rounds of 2 runs per variant, the faster round kept: a clock or power swing during one
    # variant's window cannot decide the choice on its own
    times = {name: float("inf") for name in variants}
    for _ in range(_LAYOUT_ROUNDS):
        for name, fn in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(2):
                fn()
            e1.record()
            e1.synchronize()
            times[name] = min(times[name], e0.elapsed_time(e1) / 2)
    return times


def agree_layouts(group=None) -> int:
    """Make every rank use rank 0's GEMM layout choices: one ``broadcast_object_list`` of rank 0's table
    (called by the engine after its first optimizer step, a point every rank reaches in the same order);
    choices this rank made differently are replaced, problems it has not met yet take rank 0's choice on
    first sight. Returns the number of local choices that changed."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) <= 1:
        return 0
    # rank 0's hipBLASLt solution choices travel with its layouts: a rank that timed a problem's candidates
    # (LLMT_GEMM_TUNE / LLMT_GEMM_NOSK_TIME / LLMT_GEMM_GSU), under its own collectives, could keep a different
    # kernel for the same problem (csrc/blaslt.cpp gemm_lt_adopt)
    lt = native_available() and torch.cuda.is_available()
    mine = {layout_key_str(k): v for k, v in _LAYOUT_CACHE.items()}
    obj = [(mine, lib().gemm_lt_export() if lt else "") if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    theirs, lt_text = obj[0] or ({}, "")
    if lt and lt_text and dist.get_rank() != 0:
        n = lib().gemm_lt_adopt(lt_text)
        if n:
            log.info("hipBLASLt: %d solution choice(s) replaced by rank 0's", n)
    changed = 0
    for k in list(_LAYOUT_CACHE):
        c = theirs.get(layout_key_str(k))
        if c is not None and c != _LAYOUT_CACHE[k]:
            _LAYOUT_CACHE[k] = c
            changed += 1
        if c is not None and _LAYOUT_SOURCE.get(k) == "timed" and dist.get_rank() != 0:
            _LAYOUT_SOURCE[k] = "rank0"
    _AGREED.update(theirs)
    if changed:
        log.info("GEMM layouts: %d choice(s) replaced by rank 0's", changed)
    return changed


def layout_summary() -> dict:
    """{source: how the cached choices were made, n, hash} for run records (bench.py's JSON line)."""
    import hashlib
    from collections import Counter
    items = sorted((layout_key_str(k), v) for k, v in _LAYOUT_CACHE.items())
    srcs = Counter(_LAYOUT_SOURCE.get(k, "timed") for k in _LAYOUT_CACHE)
    src = next(iter(srcs)) if len(srcs) == 1 else ("+".join(sorted(srcs)) if srcs else "static")
    h = hashlib.sha256(repr(items).encode()).hexdigest()[:16]
    return {"source": src, "n": len(items), "hash": h, "mode": _LAYOUT_MODE, "sources": dict(srcs)}


def dump_layouts(path: str) -> None:
    """Write the choices of this process as a table in the shipped format (tuning/gemm_layouts_gfx950.json)."""
    import json
    with open(path, "w") as f:
        json.dump({"arch": _device_arch() or "gfx950",
                   "layouts": {layout_key_str(k): v for k, v in sorted(_LAYOUT_CACHE.items(), key=lambda kv:
                                                                       layout_key_str(kv[0]))}}, f, indent=1)


# largest weight-gradient output (elements) offered the split-K candidates (fp32 slabs: 8 bytes / element)
_SPLITK_MAX_OUT = int(os.environ.get("LLMT_WGRAD_SPLITK_MAX", str(1 << 26)))
_SPLITK = (2, 4)  # contraction splits offered (slabs: n_split x N x K fp32)
# offer the both-operands-transposed (TN) weight-gradient layouts among the timed candidates
_WGRAD_TN = os.environ.get("LLMT_WGRAD_TN", "1").strip().lower() not in ("0", "false", "off")
# offer the hand-written GEMM (direct and split-K) among the timed weight-gradient candidates
_OWN_WGRAD = os.environ.get("LLMT_GEMM_OWN", "1").strip().lower() not in ("0", "false", "off")


def _tr_ok(*ts: torch.Tensor) -> bool:
    return all(t.size(0) % 64 == 0 and t.size(1) % 64 == 0 for t in ts)


def transpose(x: torch.Tensor) -> torch.Tensor:
    """[R, C] -> contiguous [C, R] (bf16 GPU tensors with R, C multiples of 64: the HIP kernel)."""
    out = torch.empty(x.shape[1], x.shape[0], device=x.device, dtype=x.dtype)
    lib().transpose_(x, out)
    return out


def _layout(key: tuple, variants: dict, default: str, can_time: bool) -> str:
    """Cached layout for ``key``: the shipped table's choice, rank 0's (after :func:`agree_layouts`), or, on
    first sight (and when the call may overwrite its output), the fastest of ``variants`` (name ->
    zero-argument launcher producing the same result) timed on the current stream. Otherwise ``default``."""
    hit = _LAYOUT_CACHE.get(key)
    if hit is not None:
        return hit
    det = os.environ.get("LLMT_DETERMINISTIC") == "1" or _LAYOUT_MODE == "static"
    if not det:
        ks = layout_key_str(key)
        for src, tbl in (("rank0", _AGREED), ("table", _layout_table())):
            c = tbl.get(ks)
            if c in variants:
                _LAYOUT_CACHE[key], _LAYOUT_SOURCE[key] = c, src
                return c
    if not (can_time and _LAYOUT_TUNE and len(variants) > 1) or det or torch.cuda.is_current_stream_capturing():
        return default
    times = _time_variants(variants)
    best = min(times, key=times.get)
    _LAYOUT_CACHE[key], _LAYOUT_SOURCE[key] = best, "timed"
    log.debug("GEMM layout %s -> %s (%s)", key, best, ", ".join(f"{k} {v:.3f}" for k, v in sorted(times.items(),
                                                                                         key=lambda kv: kv[1])))
    return best


def _sk_pairs(fns: dict) -> dict:
    """Layout launchers taking the stream-K flag -> zero-argument launchers for :func:`_layout`. With stream-K
    solutions allowed each layout also gets a ``/nosk`` twin restricted to the non-stream-K solutions: which
    of the two is faster is a property of the problem (Llama-3-8B at 32768 tokens: the qkv forward 1.263 vs
    1.128 ms, the o weight gradient 1.036 vs 0.881, the lm_head weight gradient 6.60 vs 7.00;
    profiles/r5_gemm_streamk_ab.md), so it is timed / tabled with the layout."""
    out = {}
    for name, fn in fns.items():
        if ALLOW_STREAMK[0]:
            out[name] = (lambda f: lambda: f(True))(fn)
            out[name + "/nosk"] = (lambda f: lambda: f(False))(fn)
        else:
            out[name] = (lambda f: lambda: f(False))(fn)
    return out


def _path(layout: str, k: int, ncols: int, *ts: torch.Tensor) -> str:
    mode = GEMM_MODES.get(layout, "blas")
    if mode == "blas" or not all(_gemm_operand_ok(t) for t in ts) or not use_native(ts[0]):
        return "blas"
    if mode == "hip" and (k % 32 or k == 0 or ncols % 4):
        return "blas"
    return mode


def mm_nt(x2: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None,
          bias: torch.Tensor | None = None) -> torch.Tensor:
    """x2 [M, K] @ w[N, K]^T (+ bias[N]) -> [M, N] (forward of a linear layer); ``out``: contiguous [M, N]
    target. On the hipBLASLt path the bias is the GEMM's BIAS epilogue (no separate pass over y)."""
    path = _path("fwd", x2.shape[1], w.shape[0], x2, w)
    if out is not None and path != "blas" and not _gemm_operand_ok(out):
        path = "blas"
    if path == "blas":
        y = torch.matmul(x2, w.t()) if out is None else torch.matmul(x2, w.t(), out=out)
        return y if bias is None else y.add_(bias)
    M, K = x2.shape
    N = w.shape[0]
    y = out if out is not None else torch.empty(M, N, device=x2.device, dtype=x2.dtype)
    if path == "lt":  # column-major: y^T (N x M) = w^T (from K x N) . x^T (K x M)
        epi = bias is not None and bias.is_contiguous() and bias.dtype in (torch.bfloat16, torch.float32)

        def nt(s):
            if epi:
                lib().gemm_lt_bias(w, x2, y, bias, True, False, N, M, K, _ld(w), _ld(x2), N, s)
            else:
                lib().gemm_lt(w, x2, y, True, False, N, M, K, _ld(w), _ld(x2), N, False, s)

        sk = ALLOW_STREAMK[0]
        if sk:
            v = _sk_pairs({"nt": nt})
            v[_layout(("fwd", M, N, K, _ld(w), _ld(x2), epi, sk), v, "nt", True)]()
        else:
            nt(False)
        if epi:
            return y
    else:
        lib().gemm_(x2, w, y, False, False, False)
    return y if bias is None else y.add_(bias)


def weight_t(w: torch.Tensor, rows: int) -> torch.Tensor | None:
    """w^T for the TN input-gradient GEMM when ``rows`` tokens in total will be multiplied by ``w``
    (chunked callers such as the fused lm_head + CE transpose once for all chunks); None otherwise."""
    if not TRANSPOSE_LAYOUTS[0] or rows < _TR_DGRAD_MIN_M or not _tr_ok(w):
        return None
    if _path("dgrad", w.shape[0], w.shape[1], w) != "lt":
        return None
    return transpose(w)


def mm_nn(dy2: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None,
          wt: torch.Tensor | None = None) -> torch.Tensor:
    """dy2 [M, N] @ w [N, K] -> [M, K] (input gradient of a linear layer); ``wt``: w^T from
    :func:`weight_t`, shared by the chunks of one product."""
    path = _path("dgrad", dy2.shape[1], w.shape[1], dy2, w)
    if out is not None and path != "blas" and not _gemm_operand_ok(out):
        path = "blas"
    if path == "blas":
        if out is None:
            return torch.matmul(dy2, w)
        return torch.matmul(dy2, w, out=out)
    M, N = dy2.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dy2.device, dtype=dy2.dtype)
    if path == "lt" and (wt is not None or (TRANSPOSE_LAYOUTS[0] and M >= _TR_DGRAD_MIN_M and _tr_ok(dy2, w))):
        sk = ALLOW_STREAMK[0]

        def tn(s):  # dx^T (K x M) = (w^T stored [K, N])^T-op . dy^T, both operands N-contiguous
            lib().gemm_lt(wt if wt is not None else transpose(w), dy2, out, True, False, K, M, N, N,
                          _ld(dy2), _ld(out), False, s)

        def nn(s):
            lib().gemm_lt(w, dy2, out, False, False, K, M, N, _ld(w), _ld(dy2), _ld(out), False, s)

        if wt is not None:  # transposed once for several chunks: TN
            v = _sk_pairs({"tn": tn})
            v[_layout(("dgrad_wt", M, N, K, _ld(dy2), _ld(out), sk), v, "tn", True)]()
        else:
            v = _sk_pairs({"tn": tn, "nn": nn})
            v[_layout(("dgrad", M, N, K, _ld(dy2), _ld(out), sk), v, "tn", True)]()
    elif path == "lt":  # column-major: dx^T (K x M) = w^T (K x N) . dy^T (N x M)
        lib().gemm_lt(w, dy2, out, False, False, K, M, N, _ld(w), _ld(dy2), _ld(out), False, ALLOW_STREAMK[0])
    else:
        lib().gemm_(dy2, w, out, False, True, False)
    return out


def wgrad_into(out: torch.Tensor, dy: torch.Tensor, x: torch.Tensor, accumulate: bool) -> bool:
    """out [N, K] (+)= dy[M, N]^T @ x[M, K] on the selected GEMM path; False if only torch can do it."""
    dy_t = _DY_T.pop(dy.data_ptr(), None) if _DY_T else None
    if dy_t is not None and (tuple(dy_t.shape) != (dy.shape[1], dy.shape[0]) or not dy.is_contiguous()):
        dy_t = None
    if not (out.is_contiguous() and out.dtype in (torch.bfloat16, torch.float32)):
        return False
    path = _path("wgrad", dy.shape[0], x.shape[1], dy, x)
    M, N = dy.shape
    K = x.shape[1]
    if path == "lt" and TRANSPOSE_LAYOUTS[0] and M >= _TR_WGRAD_MIN_M and _tr_ok(dy, x):
        sk, o2 = ALLOW_STREAMK[0], out.view(N, K)
        if dy_t is not None:
            # dy^T came with dy (the SwiGLU backward wrote both): TN, both operands token-contiguous
            def tnd(s):
                lib().gemm_lt(transpose(x), dy_t, o2, True, False, K, N, M, M, M, K, accumulate, s)
            v = _sk_pairs({"tn": tnd})
            v[_layout(("wgrad_dyt", M, N, K, _ld(x), out.dtype, sk), v, "tn", not accumulate)]()
            return True

        def nt(s):  # dW^T (K x N) = x^T (K x M) . dy (M x N), straight from the token-major operands
            lib().gemm_lt(x, dy, o2, False, True, K, N, M, _ld(x), _ld(dy), K, accumulate, s)

        def tt(s):  # x^T materialised
            lib().gemm_lt(transpose(x), dy, o2, True, True, K, N, M, M, _ld(dy), K, accumulate, s)

        def nn(s):  # dy^T materialised
            lib().gemm_lt(x, transpose(dy), o2, False, False, K, N, M, _ld(x), M, K, accumulate, s)

        def tn(s):  # both transposed: token-contiguous operands (the layout hipBLASLt runs fastest)
            lib().gemm_lt(transpose(x), transpose(dy), o2, True, False, K, N, M, M, M, K, accumulate, s)

        lt = {"nt": nt, "tt": tt, "nn": nn}
        if _WGRAD_TN:
            lt["tn"] = tn
        if N * K <= _SPLITK_MAX_OUT and M % 256 == 0:
            # split-K along the token (contraction) dimension into 2 or 4 slices, run as one strided-batch
            # GEMM into fp32 slabs + one reduction pass: 2-4x the output tiles for outputs that fill the
            # 256 CUs in 1.5 / 3.5 waves of 256x256 tiles (qkv, down)
            def _split(a, b, ta, tb, lda, ldb, n_split):
                def run(s):
                    slabs = torch.empty(n_split, N, K, device=out.device, dtype=torch.float32)
                    lib().gemm_lt_splitk(a() if callable(a) else a, b() if callable(b) else b, slabs, ta, tb,
                                         K, N, M, lda, ldb, n_split, s)
                    lib().splitk_reduce_(slabs, o2, accumulate)
                return run

            for ns in _SPLITK:
                lt[f"nt{ns}"] = _split(x, dy, False, True, _ld(x), _ld(dy), ns)
                lt[f"tt{ns}"] = _split(lambda: transpose(x), dy, True, True, M, _ld(dy), ns)
                lt[f"nn{ns}"] = _split(x, lambda: transpose(dy), False, False, _ld(x), M, ns)
                if _WGRAD_TN:
                    lt[f"tn{ns}"] = _split(lambda: transpose(x), lambda: transpose(dy), True, False, M, M, ns)
        variants = _sk_pairs(lt)
        if _OWN_WGRAD and M % 32 == 0 and N % 4 == 0:
            # the hand-written ping-pong GEMM (csrc/gemm.hip) reads both token-major operands directly
            # (transposed LDS reads, no materialised transposes); split into 2 / 4 contraction slices for
            # outputs that fill the chip in few 256 x 256 tiles
            variants["hip"] = lambda: lib().gemm_(dy, x, o2, True, True, accumulate)
            for ns in _SPLITK:
                if N * K <= _SPLITK_MAX_OUT and M % (32 * ns) == 0:
                    def _own_split(ns=ns):
                        slabs = torch.empty(ns, N, K, device=out.device, dtype=torch.float32)
                        lib().gemm_splitk_(dy, x, slabs, True, True)
                        lib().splitk_reduce_(slabs, o2, accumulate)
                    variants[f"hip{ns}"] = _own_split
        # static rule: wide outputs (gate_up, lm_head) transpose the smaller operand x, the rest dy
        default = "tt" if N >= 4 * K else "nn"
        key = ("wgrad", M, N, K, _ld(x), _ld(dy), out.dtype, sk)
        variants[_layout(key, variants, default, not accumulate)]()
        return True
    if path == "lt":  # column-major: dW^T (K x N) = x^T (K x M) . dy (M x N)
        lib().gemm_lt(x, dy, out.view(N, K), False, True, K, N, M, _ld(x), _ld(dy), K, accumulate, ALLOW_STREAMK[0])
        return True
    if path == "hip":
        lib().gemm_(dy, x, out.view(N, K), True, True, accumulate)
        return True
    return False


def _wgrad_mm(w: torch.Tensor, a_t: torch.Tensor, b: torch.Tensor):
    """dW = a_t @ b. Writes into ``w.main_grad`` if present (returns None), else returns dW.

    ``a_t`` is the transpose view of dy [T, N]; on the native paths both operands are read token-major
    straight from dy and x and the output is stored / accumulated in the buffer's dtype.
    """
    mg = getattr(w, "main_grad", None)
    a = a_t.t()
    if mg is None:
        out = torch.empty(a.shape[1], b.shape[1], device=a.device, dtype=w.dtype)
        if wgrad_into(out, a, b, False):
            return out
        return (a_t @ b).to(w.dtype)
    added = bool(getattr(w, "grad_added", False))
    if wgrad_into(mg, a, b, added):
        w.grad_added = True
        return None
    mg2 = mg.view(a_t.shape[0], b.shape[1])
    if mg.dtype == a_t.dtype:
        if added:
            mg2.addmm_(a_t, b)
        else:
            torch.mm(a_t, b, out=mg2)
    else:  # fp32 gradient buffer with bf16 operands
        part = torch.mm(a_t, b, out_dtype=mg.dtype) if a_t.is_cuda else (a_t.float() @ b.float())
        if added:
            mg2.add_(part)
        else:
            mg2.copy_(part)
    w.grad_added = True
    return None


def _wgrad_vec(w: torch.Tensor, g: torch.Tensor):
    mg = getattr(w, "main_grad", None)
    if mg is None:
        return g.to(w.dtype)
    if getattr(w, "grad_added", False):
        mg.add_(g.view_as(mg))
    else:
        mg.copy_(g.view_as(mg))
    w.grad_added = True
    return None


# ----------------------------------------------------------------------------- linear


class _LinearFn(Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x)
        ctx.w = w
        ctx.has_bias = b is not None
        # the bias rides in the GEMM's epilogue on the hipBLASLt path (mm_nt)
        return mm_nt(x.reshape(-1, x.shape[-1]), w, bias=b).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w = ctx.w
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = mm_nn(dy2 if dy2.stride(-1) == 1 else dy2.contiguous(), w).view(*dy.shape[:-1], w.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _wgrad_mm(w, dy2.t(), x.reshape(-1, x.shape[-1]))
        _DY_T.clear()  # consumed above, or not needed (frozen weight)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy2.sum(0)
        return dx, dw, db


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    return _LinearFn.apply(x, w, b)


# ----------------------------------------------------------------------------- RMSNorm


class _RMSNormFn(Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        L = lib()
        x = x.contiguous()
        y, _, rstd = L.rmsnorm_fwd(x, None, w, eps)
        ctx.save_for_backward(x, rstd)
        ctx.w = w
        return y

    @staticmethod
    def backward(ctx, dy):
        x, rstd = ctx.saved_tensors
        w = ctx.w
        L = lib()
        need_w = ctx.needs_input_grad[1]
        mg = getattr(w, "main_grad", None) if need_w else None
        dx, dw = L.rmsnorm_bwd(dy.contiguous(), x, w, rstd, None, mg, bool(getattr(w, "grad_added", False)),
                               need_w)
        if need_w:
            if mg is not None:
                w.grad_added = True
                dw = None
            else:
                dw = dw.to(w.dtype)
        else:
            dw = None
        return dx, dw, None


class _AddRMSNormFn(Function):
    """s = x + residual; y = rmsnorm(s) * w  ->  (y, s). One kernel each way."""

    @staticmethod
    def forward(ctx, x, res, w, eps):
        L = lib()
        y, s, rstd = L.rmsnorm_fwd(x.contiguous(), res.contiguous(), w, eps)
        ctx.save_for_backward(s, rstd)
        ctx.w = w
        return y, s

    @staticmethod
    def backward(ctx, dy, ds):
        s, rstd = ctx.saved_tensors
        w = ctx.w
        L = lib()
        need_w = ctx.needs_input_grad[2]
        mg = getattr(w, "main_grad", None) if need_w else None
        if dy is None:
            dy = torch.zeros_like(s)
        dres = ds.contiguous() if ds is not None else None
        dx, dw = L.rmsnorm_bwd(dy.contiguous(), s, w, rstd, dres, mg, bool(getattr(w, "grad_added", False)), need_w)
        if need_w:
            if mg is not None:
                w.grad_added = True
                dw = None
            else:
                dw = dw.to(w.dtype)
        else:
            dw = None
        return dx, dx, dw, None


class _RefRMSNormFn(Function):
    """CPU path with main_grad support (plain torch math)."""

    @staticmethod
    def forward(ctx, x, w, eps):
        ctx.save_for_backward(x)
        ctx.w = w
        ctx.eps = eps
        return ref.rms_norm(x, w, eps)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w = ctx.w
        with torch.enable_grad():
            xd = x.detach().requires_grad_(True)
            wd = w.detach().requires_grad_(True)
            y = ref.rms_norm(xd, wd, ctx.eps)
            dx, dw = torch.autograd.grad(y, (xd, wd), dy)
        return dx, (_wgrad_vec(w, dw) if ctx.needs_input_grad[1] else None), None


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None):
    """RMSNorm; with ``residual`` returns ``(rmsnorm(x + residual), x + residual)``."""
    if use_native(x):
        if residual is None:
            return _RMSNormFn.apply(x, w, eps)
        return _AddRMSNormFn.apply(x, residual, w, eps)
    if residual is None:
        return _RefRMSNormFn.apply(x, w, eps)
    s = x + residual
    return _RefRMSNormFn.apply(s, w, eps), s


# ----------------------------------------------------------------------------- SwiGLU


# Token-contiguous transposes of input gradients, produced by the kernel that wrote the gradient (the
# SwiGLU backward) for the weight gradient of the layer that consumes it next (gate_up): data_ptr -> dy^T.
# At most one entry lives at a time; the consuming linear backward pops it.
_DY_T: dict[int, torch.Tensor] = {}
# The TN weight gradient it enables (4.8 vs 5.6 ms for gate_up) against the extra transposed write:
# on for wide MLPs (intermediate >= 12288): Llama-3-8B (I = 14336) same-box step pairs on / off 1476.0 /
# 1481.9, 1475.9 / 1479.6, 1474.9 / 1477.1 ms, packed PT 1263.3 / 1267.7 ms; Phi-3-mini (I = 8192)
# 684.7 / 681.8, 682.4 / 682.6 ms (neutral to slower), DPO 899.6 / 900.1 ms (profiles/r3_workloads_1gpu.jsonl).
# LLMT_SWIGLU_DY_T=1 / 0 forces it; None = by width.
_DY_T_ENV = os.environ.get("LLMT_SWIGLU_DY_T")
FUSED_DY_T = [None if _DY_T_ENV is None else _DY_T_ENV == "1"]
DY_T_MIN_I = 12288


def drop_dy_t():
    _DY_T.clear()


class _SwiGLUFn(Function):
    @staticmethod
    def forward(ctx, gu, dy_t_consumer):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        ctx.dy_t_consumer = dy_t_consumer
        return lib().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dc):
        (gu,) = ctx.saved_tensors
        dc = dc.contiguous()
        _DY_T.clear()
        I2 = gu.shape[-1]
        T = gu.numel() // I2
        on = FUSED_DY_T[0] if FUSED_DY_T[0] is not None else I2 // 2 >= DY_T_MIN_I
        # only when the caller guarantees that gate_up's weight gradient runs through _LinearFn, which
        # pops the transposed copy (HF modules / torch linears would leave a T x 2I buffer behind)
        if (on and ctx.dy_t_consumer and TRANSPOSE_LAYOUTS[0] and T % 64 == 0 and (I2 // 2) % 64 == 0
                and T >= _TR_WGRAD_MIN_M and GEMM_MODES.get("wgrad") == "lt"):
            # dgu plus dgu^T in one pass: the gate_up weight gradient then runs hipBLASLt's TN kernel
            dgu, dgu_t = lib().swiglu_bwd_tr(gu, dc)
            _DY_T[dgu.data_ptr()] = dgu_t
            return dgu, None
        return lib().swiglu_bwd(gu, dc), None


# The down projection's input gradient with the SwiGLU backward in its epilogue (csrc/gemm.hip SwiArgs, the
# hand-written ping-pong GEMM): dc = dy @ W_down is never written; the epilogue reads gate / up of its tile and
# writes dgu (and dgu^T for the TN gate_up weight gradient). Opt-in (LLMT_SWIGLU_GEMM=1): in alternating
# same-box step runs it LOST to hipBLASLt + the separate swiglu_bwd_tr pass — Llama-3-8B PT 1511.3 / 1509.9 /
# 1512.0 vs 1509.6 / 1508.9 / 1509.7 ms, Phi-3-mini IT 1342.7 / 1343.9 vs 1332.2 / 1338.1 ms
# (profiles/r6_swiglu_gemm.md): the own GEMM is 0.58 ms behind hipBLASLt on this problem, more than the
# dc round trip it saves, and the epilogue's 5.6 GB move at HBM rate with every CU in its epilogue at once.
SWIGLU_GEMM = [os.environ.get("LLMT_SWIGLU_GEMM", "0").strip().lower() in ("1", "true", "on")]


class _SwiGLUDownFn(Function):
    """y = swiglu(gu) @ W_down^T (+ b): the SwiGLU forward and the down projection, with the backward's input
    gradient GEMM and SwiGLU backward fused (one kernel)."""

    @staticmethod
    def forward(ctx, gu, w, b, dy_t_consumer):
        gu = gu.contiguous()
        c = lib().swiglu_fwd(gu)
        ctx.save_for_backward(gu, c)
        ctx.w, ctx.has_bias, ctx.dy_t_consumer = w, b is not None, dy_t_consumer
        return mm_nt(c.reshape(-1, c.shape[-1]), w, bias=b).view(*c.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        gu, c = ctx.saved_tensors
        w = ctx.w
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.stride(-1) != 1 or (dy2.size(0) > 1 and dy2.stride(0) % 8):
            dy2 = dy2.contiguous()
        I2 = gu.shape[-1]
        T = gu.numel() // I2
        _DY_T.clear()
        dgu = dw = db = None
        if ctx.needs_input_grad[0]:
            on = FUSED_DY_T[0] if FUSED_DY_T[0] is not None else I2 // 2 >= DY_T_MIN_I
            tr = (on and ctx.dy_t_consumer and TRANSPOSE_LAYOUTS[0] and T >= _TR_WGRAD_MIN_M
                  and GEMM_MODES.get("wgrad") == "lt")
            outs = lib().gemm_swiglu_bwd(dy2, w, gu.view(T, I2), tr)
            dgu = outs[0].view(gu.shape)
            if tr:
                _DY_T[dgu.data_ptr()] = outs[1]
        if ctx.needs_input_grad[1]:
            dw = _wgrad_mm(w, dy2.t(), c.reshape(-1, c.shape[-1]))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy2.sum(0)
        return dgu, dw, db, None


def swiglu_down(gate_up: torch.Tensor, w_down: torch.Tensor, b_down: torch.Tensor | None = None,
                dy_t_consumer: bool = False) -> torch.Tensor:
    """down_proj(silu(gate) * up) for a fused [..., 2I] gate_up buffer: on bf16 GPU tensors of fitting shapes
    (tokens and I multiples of 64, H of 32) one autograd node whose backward runs the fused GEMM + SwiGLU
    backward kernel; otherwise ``linear(swiglu(gate_up), w_down, b_down)``."""
    I2 = gate_up.shape[-1]
    T = gate_up.numel() // max(1, I2)
    if (SWIGLU_GEMM[0] and use_native(gate_up) and GEMM_MODES.get("dgrad") != "blas" and T % 64 == 0 and T > 0
            and (I2 // 2) % 64 == 0 and w_down.shape[1] == I2 // 2 and w_down.shape[0] % 32 == 0
            and _gemm_operand_ok(w_down)):
        return _SwiGLUDownFn.apply(gate_up, w_down, b_down, bool(dy_t_consumer))
    return linear(swiglu(gate_up, dy_t_consumer), w_down, b_down)


def swiglu(gate_up: torch.Tensor, dy_t_consumer: bool = False) -> torch.Tensor:
    """silu(gate) * up for a fused [..., 2I] buffer laid out [gate | up]. ``dy_t_consumer``: gate_up came
    from this module's ``linear`` (so its backward can take the transposed input gradient the SwiGLU
    backward writes for wide MLPs)."""
    if use_native(gate_up):
        return _SwiGLUFn.apply(gate_up, bool(dy_t_consumer))
    return ref.swiglu_fused(gate_up)


# ----------------------------------------------------------------------------- RoPE + flash attention

# RoPE inside the attention kernels (see _RopeFlashAttnFn), LLMT_ROPE_FUSED:
#   "bwd"  the forward rotates q / k in place by the standalone kernel; the dQ / dK epilogues apply the
#          inverse rotation (no pass over dq / dk);
#   "full" only k is rotated by the standalone kernel; the forward / dQ kernels rotate their q rows on load
#          (the dQ kernel hands the rotated rows to the dK/dV kernel), the epilogues as "bwd";
#   "auto" (default) = "bwd": the Llama-3-8B step runs 1455.8 / 1458.6 / 1460.3 ms/step with bwd / full / off
#          (alternating bench runs on one box, profiles/r5_rope_fused.md) — in the step the on-load rotation of
#          "full" costs the forward and dQ kernels 8 ms/step (their per-row table reads miss L2 between the
#          GEMMs), more than the q pass it replaces; isolated, full was ahead on the Llama shape;
#   "off"  the standalone passes over q / k and dq / dk (A/B reference).
_RF = os.environ.get("LLMT_ROPE_FUSED", "auto").strip().lower()
ROPE_FUSED = ["off" if _RF in ("0", "false", "off") else (_RF if _RF in ("full", "bwd") else "auto")]


def _rope_mode(D: int) -> str:
    m = ROPE_FUSED[0]
    return "bwd" if m == "auto" else m


class _RopeFlashAttnFn(Function):
    """qkv [B, S, Hq+2Hkv, D] (fused QKV GEMM output) -> attention output [B, S, Hq, D].

    RoPE (reference ``ops/rope_op.py:10-20``, applied at ``models/llama/llama_model.py:553``) is fused into
    the attention kernels (``ROPE_FUSED``): by default ("bwd") the forward rotates q / k in place with the
    standalone kernel and the dQ / dK epilogues apply the inverse rotation; with "full":
      * the k heads are rotated IN PLACE by the standalone kernel (the buffer has no other consumer: the QKV
        GEMM's backward needs its input, not its output) — the forward and dQ kernels stage K through
        LDS-DMA, so K must sit rotated in memory;
      * the q heads stay unrotated in ``qkv``: the forward kernel rotates its rows as it loads them, the dQ
        kernel does the same and writes the rotated rows to a scratch buffer for the dK/dV kernel;
      * the dQ and dK epilogues apply the inverse rotation, so the backward writes the gradient of the QKV
        GEMM output directly (no inverse pass over dQKV).
    "full" leaves ``qkv`` consistent under selective recompute (the saved buffer never depends on whether the
    attention forward ran), but its on-load rotation costs the forward / dQ kernels about what the q pass
    costs (per-WG table reads of 2x the Q bytes), so "bwd" is the default
    (profiles/r5_rope_fused.md).
    """

    # Activations are sequence-major: qkv is [S, B, Htot, D] contiguous, positions [S, B]. The flash
    # kernels see [B, S, H, D] strided views (transpose(0, 1)) and return O in the same seq-major memory
    # order, so the output projection consumes it without a copy.
    # bm=True: a batch-major buffer [B, S, Htot, D] (transformers' layout), positions [B * S] in the same
    # token order; O comes back batch-major [B, S, Hq, D]
    @staticmethod
    def forward(ctx, qkv, pos, cos, sin, seg, nq, nkv, causal, window, scale, dropout_p=0.0, seed=0, bm=False,
                tok=None):
        # tok: per-token tables (ct, st, sb, ss) whose row b * sb + s * ss is token (b, s)'s cos / sin (see
        # rope_token_tables); None -> the kernels index cos / sin through pos
        L = lib()
        mode = _rope_mode(qkv.shape[-1])
        if mode == "full":
            L.rope_(qkv[..., nq:nq + nkv, :], pos, cos, sin, nkv, False)  # the k heads only
        else:
            L.rope_(qkv, pos, cos, sin, nq + nkv, False)
        x = qkv if bm else qkv.transpose(0, 1)
        q, k, v = x[:, :, :nq], x[:, :, nq:nq + nkv], x[:, :, nq + nkv:]
        if mode != "off":
            if tok is None:  # positions of token (b, s): pos[b * S + s] (batch-major) or pos[s * B + b] (seq-major)
                B, S = q.shape[0], q.shape[1]
                rp, rc, rs, (sb, ss) = pos, cos, sin, ((S, 1) if bm else (1, B))
            else:
                rp, (rc, rs, sb, ss) = None, tok
            ctx.rope = (rp, rc, rs, sb, ss)
        if mode == "full":
            o, lse = L.flash_attn_fwd(q, k, v, seg, scale, causal, window, dropout_p, seed, *ctx.rope)
        else:
            o, lse = L.flash_attn_fwd(q, k, v, seg, scale, causal, window, dropout_p, seed)
        ctx.save_for_backward(qkv, o, lse, pos, cos, sin, seg)
        ctx.cfg = (nq, nkv, causal, window, scale, dropout_p, seed, bm, mode)
        return o if bm else o.transpose(0, 1)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, pos, cos, sin, seg = ctx.saved_tensors
        nq, nkv, causal, window, scale, dropout_p, seed, bm, mode = ctx.cfg
        L = lib()
        if not bm:
            do = do.transpose(0, 1)
        if not _same_layout(do, o):
            do = torch.empty_like(o).copy_(do)
        elif do.stride() != o.stride():
            do = do.as_strided(o.shape, o.stride())  # differs only in the strides of size-1 dims
        dqkv = torch.empty_like(qkv)
        x, dx = (qkv, dqkv) if bm else (qkv.transpose(0, 1), dqkv.transpose(0, 1))
        args = (x[:, :, :nq], x[:, :, nq:nq + nkv], x[:, :, nq + nkv:], o, do, lse, seg, dx[:, :, :nq],
                dx[:, :, nq:nq + nkv], dx[:, :, nq + nkv:], scale, causal, window, dropout_p, seed)
        if mode != "off":  # q unrotated ("full") or both rotated in memory ("bwd")
            L.flash_attn_bwd(*args, *ctx.rope, mode == "bwd")
        else:
            L.flash_attn_bwd(*args)
            L.rope_(dqkv, pos, cos, sin, nq + nkv, True)
        return dqkv, None, None, None, None, None, None, None, None, None, None, None, None, None


def _same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same shape and the same element -> memory mapping (strides of size-1 dims do not matter)."""
    if a.shape != b.shape:
        return False
    return all(n == 1 or sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()))


class _FlashAttnFn(Function):
    """Plain flash attention on separate q/k/v [B, S, H, D] tensors."""

    @staticmethod
    def forward(ctx, q, k, v, seg, causal, window, scale, dropout_p=0.0, seed=0):
        o, lse = lib().flash_attn_fwd(q, k, v, seg, scale, causal, window, dropout_p, seed)
        ctx.save_for_backward(q, k, v, o, lse, seg)
        ctx.cfg = (causal, window, scale, dropout_p, seed)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, seg = ctx.saved_tensors
        causal, window, scale, dropout_p, seed = ctx.cfg
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        if not _same_layout(do, o):
            do = torch.empty_like(o).copy_(do)
        elif do.stride() != o.stride():
            do = do.as_strided(o.shape, o.stride())
        lib().flash_attn_bwd(q, k, v, o, do, lse, seg, dq, dk, dv, scale, causal, window, dropout_p, seed)
        return dq, dk, dv, None, None, None, None, None, None


def segment_info(segment_ids: torch.Tensor, doc_major: bool = False) -> torch.Tensor:
    """Run layout of packed rows for the flash kernels, int32, flat: [3, B, S] (segment id, first and last
    index of the contiguous run of equal ids containing each token) followed by two work orders of the
    B x ceil(S / 128) (row, 128-token block) pairs — query blocks by their key tiles, key blocks by their
    query tiles under the causal mask, heaviest first — so the kernels start long blocks first as they do
    on dense rows. Computed once per forward (a handful of scans and two small sorts, on device, no host
    sync) and shared by every layer; lets a query block skip all key tiles outside its runs.

    ``doc_major``: the blocks of one document back to back instead (heaviest first inside it, longest
    documents first), for attention without grouped K / V heads, where co-running workgroups share K / V only
    through blocks of the same document: Phi-3 D=96 MHA, 8 random documents per 4096 row, B8: forward 0.522 ->
    0.424 ms, forward + backward 2.327 -> 2.145 ms; Llama GQA (4 query heads per K / V head) loses 1 %
    (profiles/r5_seg_order_ab.jsonl). LLMT_SEG_ORDER = 0 (index order) / 1 / 2 overrides."""
    seg = segment_ids.to(torch.int32)
    B, S = seg.shape
    idx = torch.arange(S, device=seg.device, dtype=torch.int32).expand(B, S)
    start = torch.ones_like(seg, dtype=torch.bool)
    start[:, 1:] = seg[:, 1:] != seg[:, :-1]
    end = torch.ones_like(seg, dtype=torch.bool)
    end[:, :-1] = start[:, 1:]
    rs = torch.cummax(torch.where(start, idx, torch.zeros_like(idx)), dim=1).values
    re = torch.where(end, idx, torch.full_like(idx, S)).flip(1).cummin(dim=1).values.flip(1)
    runs = torch.stack([seg, rs.to(torch.int32), re.to(torch.int32)])
    order = os.environ.get("LLMT_SEG_ORDER", "2" if doc_major else "1")
    if order == "0":  # A/B: the [3, B, S] layout alone (index-order blocks)
        return runs.contiguous()
    nb = (S + 127) // 128
    starts = torch.arange(nb, device=seg.device, dtype=torch.int64) * 128
    # query block: 64-key tiles from its first query's run start to the diagonal
    tq = (torch.clamp(starts + 128, max=S) - (rs[:, starts].long() // 64) * 64 + 63) // 64
    # key block: 32-row query tiles from the block to its last key's run end
    tk = (re[:, torch.clamp(starts + 127, max=S - 1)].long() + 1 - starts + 31) // 32
    if order == "2":
        # document-major: the blocks of one document (by the run of the block's last token) back to back,
        # heaviest first inside it, longest documents first: co-running workgroups share the document's K / V
        # (or Q / dO) in L2, as consecutive blocks of one dense row do
        last = torch.clamp(starts + 127, max=S - 1)
        d0 = rs[:, last].long()
        dlen = torch.clamp(re[:, last].long() - d0 + 1, max=(1 << 18) - 1)
        doc = torch.arange(B, device=seg.device, dtype=torch.int64)[:, None] * S + d0
        base = (((1 << 18) - 1 - dlen) << 43) | (doc << 12)
        qord = torch.argsort((base | (4095 - torch.clamp(tq, max=4095))).reshape(-1)).to(torch.int32)
        kord = torch.argsort((base | (4095 - torch.clamp(tk, max=4095))).reshape(-1)).to(torch.int32)
    else:
        qord = torch.argsort(-tq.reshape(-1), stable=True).to(torch.int32)
        kord = torch.argsort(-tk.reshape(-1), stable=True).to(torch.int32)
    return torch.cat([runs.reshape(-1), qord, kord])


def _native_seg(segment_ids, seg_info):
    if segment_ids is None:
        return None
    if seg_info is not None:
        return seg_info
    if segment_ids.dim() == 3:  # already [3, B, S]
        return segment_ids.to(torch.int32).contiguous()
    return segment_info(segment_ids)


def dropout_seed() -> int:
    """Seed of one attention call's dropout mask (from torch's CPU generator: reproducible under
    torch.manual_seed, no device sync); the backward regenerates the mask from it."""
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item())


def flash_attention(q, k, v, causal: bool = True, segment_ids=None, window: int = -1, scale: float | None = None,
                    seg_info=None, dropout_p: float = 0.0, seed: int | None = None):
    """q: [B, S, Hq, D]; k/v: [B, S, Hkv, D]; segment_ids: optional int [B, S] — tokens attend within
    their contiguous run of equal ids (packed documents; 0 = padding). ``dropout_p``: attention
    dropout on the probabilities, in the kernels (mask from a counter hash of (seed, b, h, q, k))."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if use_native(q):
        seg = _native_seg(segment_ids, seg_info)
        if dropout_p > 0 and seed is None:
            seed = dropout_seed()
        return _FlashAttnFn.apply(q, k, v, seg, causal, -1 if window is None else int(window), scale,
                                  float(dropout_p), int(seed or 0))
    if dropout_p > 0:
        return ref.attention_dropout(q, k, v, causal, segment_ids, -1 if window is None else window, scale,
                                     dropout_p, dropout_seed() if seed is None else seed)
    return ref.attention(q, k, v, causal, segment_ids, -1 if window is None else window, scale)


def rope_tables_to_full(cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor):
    """Half-width fp32 tables [P, D/2] gathered at positions -> full-width HF-style [.., D] cos/sin."""
    c = cos[pos]
    s = sin[pos]
    return torch.cat([c, c], -1), torch.cat([s, s], -1)


def rope_token_tables(positions: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor):
    """Per-token rows of the half-width tables for the attention kernels' fused RoPE: (cos[pos], sin[pos],
    sb, ss) in the seq-major token order of the fused QKV buffer (row s * B + b). Computed once per forward
    (the model's runtime dict) and shared by every layer, so the kernels read a token's table row directly
    instead of through its position id."""
    B, S = positions.shape
    p = positions.t().reshape(-1).clamp(0, cos.shape[0] - 1)
    return cos.index_select(0, p), sin.index_select(0, p), 1, B


def rope_attention(qkv, positions, cos, sin, n_q: int, n_kv: int, causal: bool = True, segment_ids=None,
                   window: int = -1, scale: float | None = None, impl: str = "flash", seg_info=None,
                   dropout_p: float = 0.0, rope_tok=None):
    """Fused RoPE + attention on the SEQ-MAJOR fused QKV buffer [S, B, n_q + 2 n_kv, D] -> [S, B, n_q, D].

    ``cos``/``sin``: fp32 half-width tables [max_pos, D/2]; ``positions``: [B, S] int;
    ``segment_ids``: optional [B, S] (tokens attend only within their contiguous run of equal ids);
    ``seg_info``: its precomputed :func:`segment_info` (shared across layers); ``rope_tok``: the
    precomputed :func:`rope_token_tables` (shared across layers); ``dropout_p``: attention
    dropout on the probabilities (reference ``attention_dropout``, llama_model.py:593-621 — FA2 / SDPA
    ``dropout_p``): in the HIP kernels on the GPU (the generic forward / backward kernels, which carry the
    keep-mask hash), SDPA with dropout on the CPU / SDPA paths.
    """
    D = qkv.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    win = -1 if window is None else int(window)
    if use_native(qkv) and impl in ("flash", "flash_attention_2", "hip"):
        qkv = qkv.contiguous()
        pos = positions.t().contiguous().reshape(-1)
        seg = _native_seg(segment_ids, seg_info)
        seed = dropout_seed() if dropout_p > 0 else 0
        return _RopeFlashAttnFn.apply(qkv, pos, cos, sin, seg, n_q, n_kv, causal, win, scale, float(dropout_p), seed,
                                      False, rope_tok)
    if dropout_p > 0:
        return _ref_rope_attention(qkv.transpose(0, 1), positions, cos, sin, n_q, n_kv, causal, segment_ids, win,
                                   scale, "sdpa", dropout_p).transpose(0, 1)
    return _ref_rope_attention(qkv.transpose(0, 1), positions, cos, sin, n_q, n_kv, causal, segment_ids, win, scale,
                               impl).transpose(0, 1)


# transformers-style rotary tables (full-width cos / sin [B or 1, S, D], rotate-half convention, computed once
# per forward by the model and handed to every layer) as the per-token half-width fp32 tables the RoPE
# kernel indexes: one conversion per forward (the last pair is cached by identity)
_HF_ROPE = [None]


def _token_tables(cos: torch.Tensor, sin: torch.Tensor, B: int, S: int):
    hit = _HF_ROPE[0]
    if hit is not None and hit[0] is cos and hit[1] is sin:
        return hit[2]
    Bc, Sc, D = cos.shape
    if Sc != S or Bc not in (1, B):
        raise ValueError(f"rotary tables {tuple(cos.shape)} for a [{B}, {S}] batch")
    h = D // 2
    ct = cos[..., :h].float().reshape(Bc * S, h).contiguous()
    st = sin[..., :h].float().reshape(Bc * S, h).contiguous()
    pos = torch.arange(Bc * S, device=cos.device).view(Bc, S).expand(B, S)
    _HF_ROPE[0] = (cos, sin, (ct, st, pos))
    return ct, st, pos


def rope_attention_bm(qkv, cos, sin, n_q: int, n_kv: int, segment_ids=None, window: int | None = None,
                      scale: float | None = None, dropout_p: float = 0.0):
    """Causal fused RoPE + attention on a BATCH-MAJOR fused QKV buffer [B, S, n_q + 2 n_kv, D] (the HF
    decoder layer's layout) with transformers' rotary tables ``cos`` / ``sin`` [B or 1, S, D] -> [B, S, n_q, D].
    The same kernels as :func:`rope_attention` (RoPE fused into the flash kernels on strided views of the
    buffer, see _RopeFlashAttnFn), fed per-token tables so any rope_type / scaling the model's rotary
    embedding computed applies unchanged."""
    B, S, _, D = qkv.shape
    ct, st, pos = _token_tables(cos, sin, B, S)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    win = -1 if window is None else int(window)
    if use_native(qkv):
        qkv = qkv.contiguous()
        seg = _native_seg(segment_ids, None)
        seed = dropout_seed() if dropout_p > 0 else 0
        # ct / st are already per-token rows (row b * S + s, or s when the tables are shared by the batch)
        tok = (ct, st, S if ct.shape[0] == B * S and B > 1 else 0, 1)
        return _RopeFlashAttnFn.apply(qkv, pos.reshape(-1).contiguous(), ct, st, seg, n_q, n_kv, True, win, scale,
                                      float(dropout_p), seed, True, tok)
    return _ref_rope_attention(qkv, pos, ct, st, n_q, n_kv, True, segment_ids, win, scale, "sdpa", dropout_p)


def _ref_rope_attention(qkv, positions, cos, sin, n_q, n_kv, causal, segment_ids, win, scale, impl,
                        dropout_p: float = 0.0):
    q, k, v = qkv[:, :, :n_q], qkv[:, :, n_q:n_q + n_kv], qkv[:, :, n_q + n_kv:]
    cf, sf = rope_tables_to_full(cos, sin, positions)
    q, k = ref.apply_rope(q, k, cf.to(q.dtype) if q.dtype != torch.float32 else cf,
                          sf.to(q.dtype) if q.dtype != torch.float32 else sf)
    if impl == "sdpa" and segment_ids is None and win < 0:
        rep = n_q // n_kv
        qh, kh, vh = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        if rep > 1:
            kh = kh.repeat_interleave(rep, dim=1)
            vh = vh.repeat_interleave(rep, dim=1)
        o = torch.nn.functional.scaled_dot_product_attention(qh, kh, vh, is_causal=causal, scale=scale,
                                                             dropout_p=dropout_p)
        return o.transpose(1, 2)
    if impl == "sdpa":
        mask = ref.visibility_mask(q.shape[1], q.device, causal, segment_ids, win, q.shape[0])
        rep = n_q // n_kv
        qh, kh, vh = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        if rep > 1:
            kh = kh.repeat_interleave(rep, dim=1)
            vh = vh.repeat_interleave(rep, dim=1)
        o = torch.nn.functional.scaled_dot_product_attention(qh, kh, vh, attn_mask=mask[:, None], scale=scale,
                                                             dropout_p=dropout_p)
        return o.transpose(1, 2)
    return ref.attention(q, k, v, causal, segment_ids, win, scale)


# ----------------------------------------------------------------------------- cross entropy


def _apply_weight_grad(w: torch.Tensor, dw: torch.Tensor, g: torch.Tensor):
    """Add g * dw (g: 0-dim device scalar) into ``w.main_grad`` (returns None), or return it."""
    mg = getattr(w, "main_grad", None)
    gs = g.to(dw.dtype)
    if mg is None:
        return (dw * gs).to(w.dtype)
    mg2 = mg.view(dw.shape)
    # mixed dtypes (fp32 dw into a bf16 buffer or back) are computed in fp32 and rounded once, with
    # no [V, H]-sized temporary
    if getattr(w, "grad_added", False):
        mg2.addcmul_(dw, gs)
    else:
        torch.mul(dw, gs, out=mg2)
    w.grad_added = True
    return None


def dw_accumulator(w: torch.Tensor, n_rows: int, chunk: int) -> torch.Tensor:
    """Weight-gradient accumulator of a row-chunked loss head: fp32 whenever several chunks add into it
    or the weight's gradient buffer is fp32 (bf16-mixed), so the sum over chunks is not rounded to bf16
    per chunk; a single chunk's GEMM already accumulates in fp32 and rounds once."""
    mg = getattr(w, "main_grad", None)
    fp32 = n_rows > chunk or (mg is not None and mg.dtype == torch.float32)
    return torch.empty(w.shape, device=w.device, dtype=torch.float32 if fp32 else w.dtype)


def dw_add_chunk(dw: torch.Tensor, lg: torch.Tensor, h: torch.Tensor, first: bool):
    """dw (+)= lg^T @ h on the native GEMM path (fp32 or bf16 output), else in torch."""
    if wgrad_into(dw, lg, h, not first):
        return
    if dw.dtype == lg.dtype:
        if first:
            torch.mm(lg.t(), h, out=dw)
        else:
            dw.addmm_(lg.t(), h)
    else:
        part = torch.mm(lg.t(), h, out_dtype=dw.dtype) if lg.is_cuda else lg.t().to(dw.dtype) @ h.to(dw.dtype)
        if first:
            dw.copy_(part)
        else:
            dw.add_(part)


class _FusedLinearCEFn(Function):
    """loss = mean_{valid rows} CE(h @ W^T, labels), memory bounded by ONE logits chunk.

    Forward, per row chunk (Liger-style gradient-in-forward): one GEMM for the bf16
    logits, the HIP CE kernel computes the loss rows AND overwrites the logits with d loss / d logits
    (scaled by 1/n_valid read from device memory — no host sync), then the same chunk's dh rows and its
    dW contribution are computed right away and the chunk's logits are dropped. Only dh [N, H] and dW
    [V, H] survive to the backward, which scales them by the incoming gradient (1 for a plain loss)
    and accumulates dW into the weight's flat gradient buffer.
    """

    @staticmethod
    def forward(ctx, h, w, labels, ignore_index, chunk):
        L = lib()
        N = h.shape[0]
        valid = (labels != ignore_index).sum()
        inv_n = (1.0 / valid.clamp(min=1).float()).reshape(1)
        loss_rows = torch.empty(N, device=h.device, dtype=torch.float32)
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dh = torch.empty_like(h) if need_h else None
        dw = dw_accumulator(w, N, chunk) if need_w else None
        wt = weight_t(w, N) if need_h and N > chunk else None
        for s0 in range(0, N, chunk):
            s1 = min(N, s0 + chunk)
            lg = mm_nt(h[s0:s1], w)
            _, _, lr = L.cross_entropy_(lg, labels[s0:s1], 0, ignore_index, None, None, inv_n, True)
            loss_rows[s0:s1] = lr
            if need_h:
                mm_nn(lg, w, out=dh[s0:s1], wt=wt)
            if need_w:
                dw_add_chunk(dw, lg, h[s0:s1], s0 == 0)
            del lg
        ctx.save_for_backward(*(t for t in (dh, dw) if t is not None))
        ctx.has = (need_h, need_w)
        ctx.w = w
        return loss_rows.sum() * inv_n[0]

    @staticmethod
    def backward(ctx, g):
        saved = list(ctx.saved_tensors)
        need_h, need_w = ctx.has
        dh = saved.pop(0) if need_h else None
        dw = saved.pop(0) if need_w else None
        if dh is not None:
            dh = dh * g.to(dh.dtype)
        dwr = _apply_weight_grad(ctx.w, dw, g) if dw is not None else None
        return dh, dwr, None, None, None


def fused_linear_cross_entropy(h, w, labels, ignore_index: int = -100, chunk_size: int = 8192):
    """Mean token CE of ``h @ w.T`` against ``labels`` (already shifted). h: [N, H], labels: [N]."""
    h = h.reshape(-1, h.shape[-1])
    labels = labels.reshape(-1)
    if use_native(h):
        return _FusedLinearCEFn.apply(h.contiguous(), w, labels.contiguous(), ignore_index, chunk_size)
    logits = linear(h, w)
    return ref.cross_entropy(logits, labels, ignore_index)


class _CEFn(Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        L = lib()
        lg = logits.reshape(-1, logits.shape[-1]).contiguous().clone()
        lab = labels.reshape(-1).contiguous()
        inv_n = (1.0 / (lab != ignore_index).sum().clamp(min=1).float()).reshape(1)
        _, _, lr = L.cross_entropy_(lg, lab, 0, ignore_index, None, None, inv_n, True)
        ctx.save_for_backward(lg)
        ctx.shape = logits.shape
        return lr.sum() * inv_n[0]

    @staticmethod
    def backward(ctx, g):
        (lg,) = ctx.saved_tensors
        return (lg * g.to(lg.dtype)).view(ctx.shape), None, None


def cross_entropy(logits, labels, ignore_index: int = -100):
    """Mean CE over non-ignored tokens (bf16 logits on GPU, in-place-gradient kernel)."""
    if use_native(logits) and logits.dtype == torch.bfloat16:
        return _CEFn.apply(logits, labels, ignore_index)
    return ref.cross_entropy(logits, labels, ignore_index)


class _LinearLogpsFn(Function):
    """Per-token log p(label) of h @ W^T without materialising log_softmax (DPO / ORPO heads).

    Backward recomputes each logits chunk (one extra GEMM) instead of keeping [N, V] alive, and the
    HIP kernel writes g_t * (onehot - softmax) in place (coef_row = -g).
    """

    @staticmethod
    def forward(ctx, h, w, labels, ignore_index, chunk):
        L = lib()
        N = h.shape[0]
        out = torch.empty(N, device=h.device, dtype=torch.float32)
        rowsum = torch.empty(N, device=h.device, dtype=torch.float32)  # sum of each row's logits (metrics)
        for s0 in range(0, N, chunk):
            s1 = min(N, s0 + chunk)
            lg = mm_nt(h[s0:s1], w)
            _, _, lr = L.cross_entropy_(lg, labels[s0:s1], 0, ignore_index, None, None, None, False, -1,
                                        rowsum[s0:s1])
            out[s0:s1] = -lr
        ctx.save_for_backward(h, labels)
        ctx.w = w
        ctx.cfg = (ignore_index, chunk)
        ctx.mark_non_differentiable(rowsum)
        return out, rowsum

    @staticmethod
    def backward(ctx, g, _g_rowsum=None):
        h, labels = ctx.saved_tensors
        w = ctx.w
        ignore_index, chunk = ctx.cfg
        L = lib()
        N = h.shape[0]
        dh = torch.empty_like(h)
        coef = (-g).float().contiguous()
        need_w = ctx.needs_input_grad[1]
        dw = dw_accumulator(w, N, chunk) if need_w else None
        wt = weight_t(w, N) if N > chunk else None
        for s0 in range(0, N, chunk):
            s1 = min(N, s0 + chunk)
            lg = mm_nt(h[s0:s1], w)
            L.cross_entropy_(lg, labels[s0:s1], 0, ignore_index, None, coef[s0:s1], None, True)
            mm_nn(lg, w, out=dh[s0:s1], wt=wt)
            if need_w:
                dw_add_chunk(dw, lg, h[s0:s1], s0 == 0)
        dwr = None
        if need_w:
            dwr = _apply_weight_grad(w, dw, torch.ones((), device=dw.device, dtype=torch.float32))
        return dh, dwr, None, None, None


def linear_token_logps(h, w, labels, ignore_index: int = -100, chunk_size: int = 8192,
                       logit_sums: bool = False):
    """log p(labels) per token for logits = h @ w.T; zeros where label == ignore_index. h: [N, H].
    ``logit_sums``: also return each row's sum of logits (fp32, no gradient; the CE kernel's side output)
    for the reference's ORPO "Chosen / Rejected Logits" metrics without materialising the logits."""
    h2 = h.reshape(-1, h.shape[-1])
    lab = labels.reshape(-1)
    if use_native(h2):
        out, rs = _LinearLogpsFn.apply(h2.contiguous(), w, lab.contiguous(), ignore_index, chunk_size)
    else:
        logits = linear(h2, w)
        out = ref.token_logps(logits, lab, ignore_index)
        rs = logits.detach().float().sum(-1)
    out = out.view(labels.shape)
    return (out, rs.view(labels.shape)) if logit_sums else out


def token_logps(logits, labels, ignore_index: int = -100):
    return ref.token_logps(logits, labels, ignore_index)
