#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of lib/libdpe_mvs.so's three translation units
(hipcc -Rpass-analysis=kernel-resource-usage, each with the Makefile's flags: the default scheduler
for csrc/dpe_mvs.hip (SLP vectorizer off) and csrc/tap_launch.hip, iterative-maxocc for
csrc/tap_f32.hip).
Usage: python tools/ru.py [extra hipcc flags...]"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
        "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/tmp/dpe_ru.o"]
out = subprocess.run(base + ["-fno-slp-vectorize", ROOT + "/dpe-mvs_amd/csrc/dpe_mvs.hip"] + sys.argv[1:],
                     capture_output=True, text=True).stderr
out += subprocess.run(base + [ROOT + "/dpe-mvs_amd/csrc/tap_launch.hip"] + sys.argv[1:],
                      capture_output=True, text=True).stderr
out += subprocess.run(base + ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc", ROOT + "/dpe-mvs_amd/csrc/tap_f32.hip"]
                      + sys.argv[1:], capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = ("Spill" if m.group(1) == "VGPRs Spill" else m.group(1).split()[0]), m.group(2)
    if k == "Function":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    n = re.sub(r"\(.*", "", r["name"]).replace("dpe::", "")
    print(f"{n:40s} vgpr {r.get('VGPRs','?'):>4} scratch {r.get('ScratchSize','?'):>5} spill {r.get('Spill','?'):>4} occ {r.get('Occupancy','?'):>2} lds {r.get('LDS','?')}")
