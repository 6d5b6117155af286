#!/usr/bin/env python3
"""Per-kernel VGPRs / LDS / occupancy of cgx_kernels.hip (hipcc
-Rpass-analysis=kernel-resource-usage), one line per kernel.
Usage: python3 tools/kres.py [regex]"""
import re, subprocess, sys
from pathlib import Path
root = Path(__file__).resolve().parent.parent / "conjugate-gradient_amd"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-I../include", "-Icsrc", "-c", "csrc/cgx_kernels.hip", "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, cwd=root, capture_output=True, text=True).stderr
pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
dm = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.split("\n")
for (k, v), d in zip(rows.items(), dm):
    d = re.sub(r"cgx::\(anonymous namespace\)::", "", d)
    d = re.sub(r"\(cgx::SpmvArgs<[a-z]+>\)", "", d)
    if pat and not pat.search(d):
        continue
    print(f"{d[:70]:70s} vgpr {v.get('VGPRs','?'):>4} lds {v.get('LDS','?'):>6} occ {v.get('Occupancy','?'):>2} scratch {v.get('ScratchSize','?')}")
