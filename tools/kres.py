"""Per-kernel resource usage (VGPRs, spills, LDS, occupancy) of one HIP source for gfx950, from
hipcc -Rpass-analysis=kernel-resource-usage. usage: kres.py file.hip [name-filter]"""
import re
import subprocess
import sys
from pathlib import Path

root = Path(__file__).resolve().parents[1]
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src,
                      f"-I{root}/transplat_amd/csrc", f"-I{root}/include", "-o", "/tmp/_kres.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|Name|VGPRs|AGPRs|VGPRs Spill|LDS Size \[bytes/block\]|"
                  r"Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k in ("Function Name", "Name"):
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    if flt in name:
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        print(f"v{r.get('VGPRs', '?'):>4s} a{r.get('AGPRs', '?'):>4s} spill {r.get('VGPRs Spill', '?'):>3s} "
              f"lds {r.get('LDS Size [bytes/block]', '?'):>7s} occ {r.get('Occupancy [waves/SIMD]', '?')}  {dm[:110]}")
