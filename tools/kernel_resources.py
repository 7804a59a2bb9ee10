"""Registers, spills, scratch and LDS of the gfx950 kernels in a built object (from its code-object notes).
usage: python tools/kernel_resources.py noparama_amd/lib/np8_kernels.o [name-regex]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
obj, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else ".")
with tempfile.TemporaryDirectory() as d:
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "o")], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--input={fat}", f"--output={co}", "--unbundle"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
blocks = re.split(r"\n\s+- \.agpr_count:", notes)
for b in blocks[1:]:
    f = dict(re.findall(r"\n\s+\.(\w+):\s+(\S+)", "\n.agpr_count: " + b))
    name = f.get("name", "?")
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    if re.search(pat, dem):
        print(f"{dem[:90]:90s} vgpr {f.get('vgpr_count')} agpr {b.split()[0]} spill {f.get('vgpr_spill_count')} "
              f"sgpr_spill {f.get('sgpr_spill_count')} scratch {f.get('private_segment_fixed_size')} "
              f"lds {f.get('group_segment_fixed_size')}")
