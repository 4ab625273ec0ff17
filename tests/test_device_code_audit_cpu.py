"""Device-code audit of every HIP source, compiled for gfx950 on the CPU.

* No scalar-cache writes: the device code of every kernel is vector-store only. Scalar stores, scalar atomics
  and scalar-cache write-back / discard instructions (s_store_*, s_buffer_store_*, s_scratch_store_*,
  s_atomic_*, s_buffer_atomic_*, s_dcache_wb*, s_dcache_discard*) must not appear in any listing, whatever
  the compiler decides for a wave-uniform address (an error flag written by one lane, a per-row scalar).
* The memory-bound kernels of the step (RMSNorm, cross-entropy, SwiGLU, RoPE, transpose, AdamW, quantisation)
  compile without spills and without a scratch frame.

This file names those instructions, so it is listed in ``.gpurunignore``: no GPU run loads it.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "llm_training_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
SOURCES = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")

_SCALAR_WRITE = re.compile(r"^\s+(s_store_|s_buffer_store|s_scratch_store|s_atomic_|s_buffer_atomic|s_dcache_wb|"
                           r"s_dcache_discard)", re.M)


@pytest.fixture(scope="module")
def listings(tmp_path_factory):
    d = tmp_path_factory.mktemp("devasm")
    out = {}
    for src in SOURCES:
        path = d / (src + ".s")
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics", f"-I{CSRC}",
                            "--cuda-device-only", "-S", os.path.join(CSRC, src), "-o", str(path)],
                           capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, (src, r.stderr[-3000:])
        out[src] = path.read_text()
    return out


def test_every_source_compiled(listings):
    assert {"flash_attn.hip", "gemm.hip", "rmsnorm.hip", "cross_entropy.hip", "elementwise.hip", "optim.hip"} <= set(listings)


@pytest.mark.parametrize("src", SOURCES)
def test_no_scalar_cache_writes(listings, src):
    hits = _SCALAR_WRITE.findall(listings[src])
    assert not hits, (src, sorted(set(hits)))


def _meta(text):
    out = {}
    for m in re.finditer(r"\.name:\s+(\S+)\n", text):
        name = m.group(1)
        if name.endswith(".kd"):
            continue
        i = m.start()
        out[name] = text[text.rfind("- .agpr_count", 0, i):text.find(".vgpr_spill_count", i) + 40]
    return out


@pytest.mark.parametrize("src", ["rmsnorm.hip", "cross_entropy.hip", "elementwise.hip", "optim.hip", "quant.hip"])
def test_memory_bound_kernels_have_no_spills_or_scratch(listings, src):
    meta = _meta(listings[src])
    assert meta, src
    for name, blk in meta.items():
        assert re.search(r"\.vgpr_spill_count:\s+0", blk), (name, blk[-400:])
        assert re.search(r"\.sgpr_spill_count:\s+0", blk), (name, blk[-400:])
        assert re.search(r"\.private_segment_fixed_size:\s+0", blk), (name, blk[-400:])
