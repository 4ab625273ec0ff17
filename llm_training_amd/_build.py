"""In-tree builder for the gfx950 HIP extension (``llm_training_amd/_C.so``).

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into an object; the torch
operator registrations in ``csrc/bindings.cpp`` are compiled host-only (they include torch headers,
which have no device code); everything is linked into one shared library that
``llm_training_amd.ops.native`` loads with ``torch.ops.load_library``. No hipify step, no CUDA
sources, no JIT cache: the ``.so`` lives in the source tree so it travels with the repository
snapshot to the GPU box.

Run ``python -m llm_training_amd._build`` (or ``__graft_entry__.build()``). Rebuilds are incremental
(object newer than its source and every header).

``python -m llm_training_amd._build --diag`` builds the DIAGNOSTIC library ``_C_diag.so`` (``-DLLMT_DIAG``,
objects under ``csrc/build_diag``): the same kernels with the wrong-result probes of
``benchmarks/probes/`` (``LLMT_FA_PROBE``) compiled in. The production ``_C.so`` has no probe code;
``ops.native`` loads the diagnostic library only when ``LLMT_NATIVE_DIAG=1`` and refuses probe variables
against the production one.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG / "csrc" / "build"
LIB = PKG / "_C.so"
BUILD_DIAG = PKG / "csrc" / "build_diag"
LIB_DIAG = PKG / "_C_diag.so"
ARCH = os.environ.get("LLMT_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _hipcc() -> str:
    p = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    return p


def _clangxx() -> str:
    p = ROCM / "lib" / "llvm" / "bin" / "clang++"
    return str(p) if p.exists() else (shutil.which("clang++") or "g++")


def _torch_dirs():
    import torch

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    return inc, root / "lib", int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _stale(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(verbose: bool = False, debug: bool = False, diag: bool = False) -> Path:
    build_dir, lib = (BUILD_DIAG, LIB_DIAG) if diag else (BUILD, LIB)
    build_dir.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.h"))
    hips = sorted(CSRC.glob("*.hip"))
    inc, tlib, abi = _torch_dirs()
    opt = (["-O1", "-g"] if debug else ["-O3"]) + (["-DLLMT_DIAG=1"] if diag else [])
    jobs = []
    objs = []
    for src in hips:
        obj = build_dir / (src.stem + ".o")
        objs.append(obj)
        if _stale(obj, [src, *headers]):
            jobs.append([_hipcc(), f"--offload-arch={ARCH}", *opt, "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
                         f"-I{CSRC}", "-c", str(src), "-o", str(obj)])
    # host-only C++ (torch op registrations, CPU data-pipeline code): compiled without device passes
    for bsrc in sorted(CSRC.glob("*.cpp")):
        bobj = build_dir / (bsrc.stem + ".o")
        objs.append(bobj)
        if _stale(bobj, [bsrc, *headers]):
            jobs.append([_clangxx(), "-x", "c++", *opt, "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1",
                         "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", *[f"-I{p}" for p in inc],
                         f"-I{ROCM / 'include'}", f"-I{sysconfig.get_paths()['include']}", "-c", str(bsrc), "-o",
                         str(bobj)])
    if jobs:
        workers = min(len(jobs), int(os.environ.get("MAX_JOBS", "8")))
        with cf.ThreadPoolExecutor(workers) as ex:
            for cmd, _ in zip(jobs, ex.map(_run, jobs)):
                if verbose:
                    print(" ".join(cmd))
    if jobs or _stale(lib, objs):
        tmp = lib.with_suffix(".so.tmp")
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *[str(o) for o in objs], "-o", str(tmp),
              f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip",
              # torch's own hipBLASLt build (same soname as /opt/rocm's): one copy in the process
              "-lhipblaslt", f"-Wl,-rpath,{tlib}"])
        os.replace(tmp, lib)
        if verbose:
            print(f"linked {lib}")
    return lib


if __name__ == "__main__":
    p = build(verbose=True, debug="--debug" in sys.argv, diag="--diag" in sys.argv)
    print(p)
