#!/bin/bash
# A/B variant libraries for tools/stream_bench.py / tools/gpu_ab.sh:
#   tools/build_ab.sh NAME [-DDEFINE ...]      current source
#   BASE=/path/to/tree tools/build_ab.sh NAME   another source tree (e.g. git archive HEAD)
set -e
name=$1; shift
root=${BASE:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$(dirname "$0")/probe/ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -Wno-unused-result "$@" \
  -o "$(dirname "$0")/probe/ab/$name.so" "$root/mcaq_yolo_amd/csrc/mcaq_kernels.hip"
echo "$(dirname "$0")/probe/ab/$name.so"
