#!/bin/bash
# Register / spill / LDS usage per kernel of one csrc source (gfx950 device compile, no GPU needed).
# usage: tools/kres.sh k_irw.hip [name-filter]
cd "$(dirname "$0")/.."
C=spacecraft-pose-estimation-framework_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans -fno-slp-vectorize \
  -I include -I $C -x hip -c $C/$1 --offload-device-only -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c '
import re, sys
flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip(); d = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1); d[k.strip()] = v.strip()
        if k.strip() == "LDS Size [bytes/block]":
            if flt in cur:
                g = d.get; print("%4s vgpr %3s spill %2s occ  %s" % (g("VGPRs","?"), g("VGPRs Spill","?"), g("Occupancy [waves/SIMD]","?"), cur[:110]))
' "${2:-}"
