#!/usr/bin/env python
"""Per-kernel VGPR / AGPR / scratch / occupancy of one .hip file (compile-only, gfx950)."""
import re
import subprocess
import sys

import os
src = os.path.abspath(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang++", "--offload-arch=gfx950", "-O3",
                      "-std=c++17", "-fPIC", "-c", "-x", "hip", src, "-o", "/tmp/_ru.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True,
                     cwd="/tmp").stderr
cur = {}
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+([^:]+): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    if flt and not re.search(flt, r["name"]):
        continue
    print(f"{r.get('VGPRs','?'):>4} v {r.get('AGPRs','?'):>3} a  scratch {r.get('ScratchSize [bytes/lane]','?'):>4}"
          f"  occ {r.get('Occupancy [waves/SIMD]','?'):>2}  lds {r.get('LDS Size [bytes/block]','?'):>6}  {r['name'][:110]}")
