"""Per-kernel VGPR/AGPR/spill/occupancy from hipcc -Rpass-analysis=kernel-resource-usage.
usage: python tools/kernel_regs.py file.hip [name-substring ...]"""
import re
import subprocess
import sys

src, pats = sys.argv[1], sys.argv[2:]
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                      "-c", src, "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for name, r in rows.items():
    if pats and not any(p in name for p in pats):
        continue
    print(f"{name[:70]:70s} vgpr {r.get('VGPRs', '?'):>3} agpr {r.get('AGPRs', '?'):>3} "
          f"vspill {r.get('VGPRs Spill', '?'):>3} sspill {r.get('SGPRs Spill', '?'):>3} "
          f"occ {r.get('Occupancy [waves/SIMD]', '?')} lds {r.get('LDS Size [bytes/block]', '?')}")
for line in out.splitlines():
    if "error" in line:
        print(line)
