"""Resource usage (VGPR / AGPR / scratch / LDS / occupancy) per kernel of one .hip file:
python tools/kres.py csrc/FILE.hip [name-substring ...]"""
import re
import subprocess
import sys

src = sys.argv[1]
keys = sys.argv[2:]
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I",
                    "ikea-recommender-system_amd/csrc", "-c", src, "-o", "/tmp/kres.o",
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
if r.returncode:
    print(r.stderr[-3000:])
    sys.exit(1)
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).split(" ")[0], m.group(2)
    if k == "Function":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for n, d in rows.items():
    if keys and not any(k in n for k in keys):
        continue
    print(f"{n[:70]:70s} V {d.get('VGPRs')} A {d.get('AGPRs')} scr {d.get('ScratchSize')} "
          f"occ {d.get('Occupancy')} lds {d.get('LDS')}")
