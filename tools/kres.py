"""Kernel resource summary from hipcc -Rpass-analysis=kernel-resource-usage output:
python tools/kres.py remarks.txt [name-regex]  ->  kernel  VGPRs  spills  occupancy"""
import re
import sys

cur, rows = None, []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = int(m.group(2))
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
for r in rows:
    m = re.search(r"(pass_kernel|fin_kernel|pair_\w+kernel)ILi(\d+)E(\w+?)E", r["name"])
    if not m:
        continue
    short = "%s<%s,%s>" % (m.group(1), m.group(2), m.group(3).replace("Li", "").replace("Lb", "b"))
    if pat.search(short):
        print("%-24s VGPR %3d  spill %3d  occ %d" % (short, r.get("VGPRs", -1), r.get("VGPRs Spill", -1),
                                                   r.get("Occupancy [waves/SIMD]", -1)))
