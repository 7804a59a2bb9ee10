"""Register / scratch budget of the kernels in a built object whose names match a pattern (run here, on the CPU):
    python tools/kres.py noparama_amd/lib/np8_kernels.o 'np8_assign_fastILi8ELi3'"""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"
obj, pat = sys.argv[1], sys.argv[2]
with tempfile.TemporaryDirectory() as t:
    subprocess.run([f"{B}/llvm-objcopy", "--dump-section", f".hip_fatbin={t}/fat.bin", obj, f"{t}/junk.o"], check=True)
    subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={t}/fat.bin",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t}/k.co"], check=True)
    notes = subprocess.run([f"{B}/llvm-readelf", "--notes", f"{t}/k.co"], capture_output=True, text=True).stdout
for b in re.split(r"\n\s*- \.agpr_count", notes)[1:]:
    n = re.search(r"\.name:\s+(\S+)", b)
    if not n or not re.search(pat, n.group(1)):
        continue

    def g(k):
        m = re.search(r"\." + k + r":\s+(\d+)", b)
        return m.group(1) if m else "-"

    print(f"{n.group(1)[:88]:88s} vgpr {g('vgpr_count')} vspill {g('vgpr_spill_count')} sgpr {g('sgpr_count')} "
          f"sspill {g('sgpr_spill_count')} scratch {g('private_segment_fixed_size')}")
