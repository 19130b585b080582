"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (stdin) as one line per kernel:
name, VGPRs, AGPRs, scratch bytes/lane, occupancy (waves/SIMD), LDS bytes/block."""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except OSError:
    dem = names
for r, d in zip(rows, dem):
    if flt and flt not in d:
        continue
    print(f"v{r.get('vgpr', '?'):>3} a{r.get('agpr', '?'):>3} scr{r.get('scratch', '?'):>4} occ{r.get('occ', '?')} "
          f"lds{r.get('lds', '?'):>6}  {d}")
