"""Register / memory audit of the production attention and GEMM kernels, compiled for gfx950 on the CPU.

The hot kernels pin operands with inline asm ("a"-constrained MFMA operands in the dK/dV loop, asm LDS-DMA
statements that own M0); a change that pushes one of them over its register budget shows up as a spill or a
scratch (private segment) allocation, which costs a silent slowdown rather than a failure (cdna guide §5.7).
Every default-path kernel of ``flash_attn.hip`` and ``gemm.hip`` must compile without spills and without
scratch.

The production build also must not contain the wrong-result diagnostic probes (``LLMT_FA_PROBE``): the probe
reads compile only under ``-DLLMT_DIAG`` (the ``_C_diag.so`` library), so the production and diagnostic
assembly of the default kernels differ, and the production code of the forward kernel is the same with and
without a probe-free source (checked by the kernel text being probe-independent: no ``probe`` field load)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "llm_training_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


def _asm(tmp_path_factory, src, *defs):
    out = tmp_path_factory.mktemp("asm") / (os.path.basename(src) + "".join(d.strip("-D=") for d in defs) + ".s")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{CSRC}", "--cuda-device-only", "-S",
                        *defs, os.path.join(CSRC, src), "-o", str(out)], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    return out.read_text()


@pytest.fixture(scope="module")
def fa_asm(tmp_path_factory):
    return _asm(tmp_path_factory, "flash_attn.hip")


@pytest.fixture(scope="module")
def gemm_asm(tmp_path_factory):
    return _asm(tmp_path_factory, "gemm.hip")


def _kernel_meta(text):
    """{kernel symbol: metadata block} from the amdhsa metadata of an assembly listing."""
    out = {}
    for m in re.finditer(r"\.name:\s+(\S+)\n", text):
        name = m.group(1)
        if name.endswith(".kd"):
            continue
        i = m.start()
        blk = text[text.rfind("- .agpr_count", 0, i):text.find(".vgpr_spill_count", i) + 40]
        out[name] = blk
    return out


# the kernels of the default training path: range-masked forward / dQ / dK/dV (D 64 / 96 / 128) and the GEMM.
# (The per-element-mask forms for segment ids without run bounds and the generic dropout kernels carry SGPR
# spills into VGPR lanes, and the generic D=128 forward a small scratch frame: off the hot path.)
_HOT = re.compile(r"fa_fwd3_kernelILi\d+ELi2ELi1E|fa_bwd_dq3_kernelILi\d+ELb1ELb1ELi4ELb0E|fa_bwd_dkdv5_kernelILi\d+ELb0E|"
                  r"gemm_pp_kernel")


@pytest.mark.parametrize("which", ["fa", "gemm"])
def test_kernels_have_no_spills_or_scratch(which, fa_asm, gemm_asm):
    text = fa_asm if which == "fa" else gemm_asm
    meta = {k: v for k, v in _kernel_meta(text).items() if _HOT.search(k)}
    assert len(meta) >= (9 if which == "fa" else 4), sorted(_kernel_meta(text))
    for name, blk in meta.items():
        assert re.search(r"\.vgpr_spill_count:\s+0", blk), (name, blk[-400:])
        assert re.search(r"\.sgpr_spill_count:\s+0", blk), (name, blk[-400:])
        assert re.search(r"\.private_segment_fixed_size:\s+0", blk), (name, blk[-400:])


def test_default_attention_kernels_present(fa_asm):
    """The one-kernel-per-pass dispatch (forward fwd3, dQ dq3, dK/dV dkdv5, generic fallbacks) and nothing of
    the removed variants (fwd4 / fwd3c / dkdv6 / dkdv128 / separate prep pass)."""
    names = set(_kernel_meta(fa_asm))
    for k in ("fa_fwd3_kernel", "fa_bwd_dq3_kernel", "fa_bwd_dkdv5_kernel", "fa_fwd_kernel", "fa_bwd_dq_kernel",
              "fa_bwd_dkdv_kernel"):
        assert any(k in n for n in names), k
    for k in ("fa_fwd4_kernel", "fa_fwd3c_kernel", "fa_bwd_dkdv6_kernel", "fa_bwd_dkdv128_kernel",
              "fa_bwd_prep128_kernel"):
        assert not any(k in n for n in names), k


def test_probes_only_in_diagnostic_build(tmp_path_factory, fa_asm):
    """The diagnostic build (-DLLMT_DIAG) reads AttnArgs::probe in the forward kernel; the production build's
    forward kernel is identical to one compiled with the probe bits forced off, i.e. it has no probe code."""
    diag = _asm(tmp_path_factory, "flash_attn.hip", "-DLLMT_DIAG=1")

    def body(text, pat):
        m = re.search(rf"^(_ZN4llmt14fa_fwd3_kernel{pat}\S*):(.*?)^\.Lfunc_end", text, re.S | re.M)
        assert m, pat
        return [ln.split(";")[0].strip() for ln in m.group(2).splitlines() if ln.strip() and not ln.strip().startswith(";")]

    prod = body(fa_asm, "ILi128ELi2ELi1E")
    dg = body(diag, "ILi128ELi2ELi1E")
    assert prod != dg, "the diagnostic build should differ from production (probe reads compiled in)"
    assert len(prod) < len(dg)
