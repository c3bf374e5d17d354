"""Per-kernel VGPR / scratch / occupancy table from `make resource` output.

  make -s -C raytraceheattransfer.jl_amd/csrc resource 2>&1 | python tools/resource_usage.py [substring]
"""
import re
import subprocess
import sys

sub = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"(VGPRs|AGPRs|SGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split(" [")[0]] = int(m.group(2))
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except Exception:
    dem = names
for r, d in zip(rows, dem):
    if sub and sub not in d:
        continue
    d = re.sub(r"\(rthx::DevDomain.*", "", d)
    print(f"{d:80s} vgpr {r.get('VGPRs', 0):3d} sgpr {r.get('SGPRs', 0):3d} scratch {r.get('ScratchSize', 0):4d} "
          f"occ {r.get('Occupancy', 0)} spill s{r.get('SGPRs Spill', 0)}/v{r.get('VGPRs Spill', 0)}")
