#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_qoff
timeout -k 10 120 ./tools/probe/shape_probe > gpurun_out/r03_qoff/shape_probe.txt 2>&1; rc=$?; head -4 gpurun_out/r03_qoff/shape_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/quant_offsets.py > gpurun_out/r03_qoff/qoff.json 2> gpurun_out/r03_qoff/qoff.err; rc=$?; cat gpurun_out/r03_qoff/qoff.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03_qoff/qoff.err; exit $rc; }
timeout -k 10 200 python tools/quant_offsets.py > gpurun_out/r03_qoff/qoff2.json 2>> gpurun_out/r03_qoff/qoff.err; cat gpurun_out/r03_qoff/qoff2.json
