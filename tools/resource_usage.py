"""Per-kernel VGPR / AGPR / spill / occupancy table from a hipcc -Rpass-analysis=kernel-resource-usage
log on stdin.  usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python3 tools/resource_usage.py [name-filter]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
names = [r["name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
for r, d in zip(rows, dem):
    if flt in d:
        print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>4} a  spill {r.get('VGPRs Spill', '?'):>3}  occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  "
              f"lds {r.get('LDS Size [bytes/block]', '?'):>6}  {d[:110]}")
