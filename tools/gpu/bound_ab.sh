#!/bin/bash
# bound_probe.py (full / stream_only / morph_only / pass A / pass B per step)
# for the built library and variant libraries tools/probe/ab/$v.so.  Tag $1, variants $2...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=$1; shift
mkdir -p $R/gpurun_out/$T
cd $R
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
for v in base "$@"; do
  if [ $v = base ]; then cp /tmp/base.so $L; else cp tools/probe/ab/$v.so $L; fi
  echo "== $v"
  timeout -k 10 200 python tools/probe/bound_probe.py > gpurun_out/$T/bound_$v.txt 2> gpurun_out/$T/bound_$v.err || { cp /tmp/base.so $L; tail -5 gpurun_out/$T/bound_$v.err; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T/bound_$v.txt
done
cp /tmp/base.so $L
