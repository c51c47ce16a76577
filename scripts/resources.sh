#!/bin/bash
# Per-kernel register / spill / occupancy summary of a HIP source (compile only).
#   scripts/resources.sh chiaroscuro-raytracer_amd/csrc/wavefront.hip  (built objects: scripts/kernel_regs.py)
set -e
src=${1:-chiaroscuro-raytracer_amd/csrc/wavefront.hip}
dir=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -fPIC -ffp-contract=off \
    -I"$dir/chiaroscuro-raytracer_amd/csrc" -I"$dir/include" -c "$src" -o /tmp/resources.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 |
    awk '/Function Name:/ {if (n) print line; n=1; sub(/.*Function Name: /,""); sub(/ \[.*/,""); line=$0}
         /VGPRs:|SGPRs:|Spill:|Occupancy/ {s=$0; sub(/.*remark: +/,"",s); sub(/ \[.*/,"",s); line=line " | " s}
         END {if (n) print line}'
