set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_dist_qat_gpu.py tests/test_train_fused_gpu.py tests/test_qat_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_ddp.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" gpurun_out/r04_ddp.log | tail -12
[ $rc -eq 0 ] || exit $rc
cp mcaq_yolo_amd/lib/libmcaq_hip.so /tmp/b0.so && cp tools/probe/ab/tb32.so mcaq_yolo_amd/lib/libmcaq_hip.so && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "batch_tile or golden" --timeout 200 --timeout-method thread 2>&1 | tail -2 && cp /tmp/b0.so mcaq_yolo_amd/lib/libmcaq_hip.so && bash tools/gpu/bound_ab.sh r04_tb32 tb32 notb
