#!/bin/bash
# end-to-end leg variants: Conv+BN fusion, bf16 network, channels_last
set -o pipefail
mkdir -p gpurun_out/e2e
export TMPDIR=/tmp
for v in "nofuse:--no-fuse" "fuse:" "fuse_amp:--amp" "fuse_cl:--channels-last" "fuse_amp_cl:--amp --channels-last"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 python bench.py --e2e --steps 20 --warmup 3 $a > gpurun_out/e2e/$n.json 2> gpurun_out/e2e/$n.err || { tail -8 gpurun_out/e2e/$n.err; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/e2e/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    c = d["config"]
    print("%-16s %8.0f img/s  step %6.3f ms  net %6.3f ms  hooks+nms %6.3f ms  det/img %.1f" % (f.split("/")[-1], d["value"], d["ms_per_step"], c["network_only_ms_per_step"], c["mcaq_hooks_and_nms_ms_per_step"], c["detections_per_image"]))
PY
