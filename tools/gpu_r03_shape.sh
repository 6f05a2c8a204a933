#!/bin/bash
# r03: HBM access-shape probe (pass-1 / pass-2 unit shapes vs flat kernels, x cold)
set -o pipefail
mkdir -p gpurun_out/r03_shape
timeout -k 10 120 ./tools/probe/shape_probe > gpurun_out/r03_shape/shape_probe.txt 2>&1; rc=$?; cat gpurun_out/r03_shape/shape_probe.txt; exit $rc
