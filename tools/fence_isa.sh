#!/bin/bash
# Device assembly of tools/fence_isa.hip for gfx950: the instruction
# sequences of HIP's system-scope release / acquire fences next to the
# fence-free slot hand-off.  CPU only (hipcc -S).
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S tools/fence_isa.hip -o $T/f.s 2>/dev/null
echo "# hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S tools/fence_isa.hip ($(/opt/rocm/bin/hipcc --version 2>/dev/null | grep -m1 -o 'HIP version: [^ ]*'))"
awk '/^[a-z_]+:/ {p=1} p && !/^\s*\./ && !/^\s*;/ && NF {print} /s_endpgm/ {p=0; print ""}' $T/f.s
rm -rf $T
