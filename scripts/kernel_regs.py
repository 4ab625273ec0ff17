"""Register / LDS / spill table of every kernel in a HIP source, compiled for gfx950 on the CPU:
    python scripts/kernel_regs.py llm_training_amd/csrc/flash_attn.hip [filter]"""
import os
import re
import subprocess
import sys
import tempfile

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "llm_training_amd", "csrc")
with tempfile.TemporaryDirectory() as d:
    out = os.path.join(d, "k.s")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{csrc}", "--cuda-device-only", "-S", src,
                    "-o", out], check=True)
    text = open(out).read()
for m in re.finditer(r"^\s+\.name:\s+(\S+)$", text, re.M):
    name = m.group(1)
    if flt not in name or name.endswith(".kd"):
        continue
    blk = text[text.rfind("- .agpr_count", 0, m.start()):m.start() + 2000]

    def f(key):
        mm = re.search(rf"\.{key}:\s+(\d+)", blk)
        return int(mm.group(1)) if mm else -1
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    print(f"{dem[:90]:90s} v{f('vgpr_count'):4d} a{f('agpr_count'):4d} s{f('sgpr_count'):4d} "
          f"vsp{f('vgpr_spill_count')} ssp{f('sgpr_spill_count')} lds{f('group_segment_fixed_size')} "
          f"priv{f('private_segment_fixed_size')}")
