"""Register / LDS / spill usage of the gfx950 kernels in one built object (build-time check).
python tools/kernel_resources.py render_bwd [regex]"""
import os
import re
import subprocess
import sys
import tempfile

import yaml

LLVM = "/opt/rocm/lib/llvm/bin"
obj = os.path.join(os.environ.get("R3DG_OBJ_DIR") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "relightable3dgaussian_amd", "build", "obj"),
                   sys.argv[1] + ".o")
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
with tempfile.TemporaryDirectory() as d:
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={d}/fb.bin", obj], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={d}/fb.bin",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={d}/k.co"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f"{d}/k.co"], check=True, capture_output=True,
                           text=True).stdout
text = notes[notes.index("---"):notes.rindex("...") + 3]
meta = yaml.safe_load(text)
for k in meta["amdhsa.kernels"]:
    name = subprocess.run(["c++filt", k[".name"]], capture_output=True, text=True).stdout.strip()
    if not pat.search(name):
        continue
    print(f"{name}: vgpr {k['.vgpr_count']} agpr {k.get('.agpr_count', 0)} sgpr {k['.sgpr_count']} "
          f"lds {k['.group_segment_fixed_size']} scratch {k['.private_segment_fixed_size']} "
          f"spill v{k.get('.vgpr_spill_count', 0)}/s{k.get('.sgpr_spill_count', 0)}")
