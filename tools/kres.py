"""Kernel resources (VGPR/SGPR/scratch/LDS) of a hipcc object or device bundle.
usage: python tools/kres.py file.o [name_substring]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
f, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
with tempfile.TemporaryDirectory() as d:
    src = f
    fat = os.path.join(d, "fat.bin")
    if subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", f, os.path.join(d, "x")],
                      capture_output=True).returncode == 0:
        src = fat
    co = os.path.join(d, "k.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={src}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    t = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
for b in t.split(".agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", b)
    if not name or pat not in name.group(1):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", b) or [None, "?"])[1]
    print(f"{name.group(1)[:80]:80s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} "
          f"scratch {g('private_segment_fixed_size'):>5} lds {g('group_segment_fixed_size'):>6}")
