"""Register-ownership audit of the hand-allocated attention kernels (cdna guide §5.7 item 4).

``fa_fwd4_kernel`` (O^T, Q and the K tile) and ``fa_bwd_dkdv6_kernel`` (dV^T and dK^T of 64 keys) name the
accumulator registers a[0:255] literally in their inline asm; hipcc does not know they are in use, so any compiler-placed ``v_accvgpr_*`` outside the
asm statements, a VGPR spill or a scratch access would silently overwrite them (the first build of the
kernel parked addresses in a0..a12 and faulted on the GPU). This compiles the kernel for gfx950 on the CPU
and checks the emitted code: no compiler accumulator traffic, no spills, no scratch, all 256 accumulator
registers claimed in the kernel descriptor."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "llm_training_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def fa_asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("asm") / "fa.s"
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{CSRC}", "--cuda-device-only", "-S",
                        os.path.join(CSRC, "flash_attn.hip"), "-o", str(out)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return out.read_text()


# fa_fwd4 (O^T / Q / K in a[0:255]) and fa_bwd_dkdv6 (dV^T / dK^T of 64 keys in a[0:255])
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("name", ["_ZN4llmt14fa_fwd4_kernelILi128EEEvNS_8AttnArgsE",
                                  "_ZN4llmt19fa_bwd_dkdv6_kernelILi128ELi3ELi0ELb0EEEvNS_8AttnArgsEPKf"])
def test_accumulator_registers_are_asm_owned(fa_asm, name):
    text = fa_asm
    body = re.search(rf"^{name}:(.*?)^\.Lfunc_end", text, re.S | re.M).group(1)
    inasm, bad = False, []
    for line in body.splitlines():
        if ";;#ASMSTART" in line:
            inasm = True
        elif ";;#ASMEND" in line:
            inasm = False
        elif not inasm and re.search(r"v_accvgpr|[\s,]a\[?\d", line.split(";")[0]):
            bad.append(line.strip())
    assert not bad, f"compiler-placed accumulator traffic in {name}: {bad[:5]}"
    assert "scratch_" not in body
    i = text.index(f".name:           {name}")
    meta = text[text.rfind("- .agpr_count", 0, i):text.index(".vgpr_spill_count", i) + 40]
    assert re.search(r"\.agpr_count:\s+256", meta), meta
    assert re.search(r"\.vgpr_spill_count:\s+0", meta) and re.search(r"\.sgpr_spill_count:\s+0", meta), meta
    assert re.search(r"\.private_segment_fixed_size:\s+0", meta), meta
