"""Kernel resource usage of one engine source, compiled for gfx950 (CPU only, no GPU needed):
one line per kernel -- VGPRs, AGPRs, spills, scratch bytes per lane, waves per SIMD.

usage: python tools/diag/kres.py kad_refresh.hip [-D...] [--grep k_kad_refresh]"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
args = sys.argv[1:]
pat = None
if "--grep" in args:
    i = args.index("--grep")
    pat = args[i + 1]
    del args[i:i + 2]
src, defs = args[0], args[1:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
       "-Rpass-analysis=kernel-resource-usage", *defs, "-x", "hip", "-c", str(ROOT / "oversim_amd" / "csrc" / src),
       "-I", str(ROOT / "include"), "-o", "/tmp/kres.o"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs Spill): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" [")[0]] = v
for r in rows:
    if pat and pat not in r["name"]:
        continue
    print(f"v{r.get('VGPRs', '?'):>4} a{r.get('AGPRs', '?'):>3} vsp{r.get('VGPRs Spill', '?'):>4} "
          f"ssp{r.get('SGPRs Spill', '?'):>4} scr{r.get('ScratchSize', '?'):>5} occ{r.get('Occupancy', '?'):>2}  {r['name'][:150]}")
