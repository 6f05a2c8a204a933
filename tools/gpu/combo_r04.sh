set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_dist_qat_gpu.py tests/test_train_fused_gpu.py tests/test_qat_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_ddp.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" gpurun_out/r04_ddp.log | tail -12
for d in 2 3 4; do
  timeout -k 10 150 python bench.py --no-cpu --no-e2e --steps 200 --schedule prefetch --pipeline $d > gpurun_out/r04_pf_p$d.json 2> gpurun_out/r04_pf_p$d.err || { tail -5 gpurun_out/r04_pf_p$d.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r04_pf_p$d.json')); print('prefetch p$d', round(d['value']), round(d['ms_per_step']*1e3,1), d['path_roofline']['frac'])"
done
timeout -k 10 150 python bench.py --no-cpu --no-e2e --steps 200 > gpurun_out/r04_pf_streams.json 2> gpurun_out/r04_pf_streams.err && python -c "
import json; d=json.load(open('gpurun_out/r04_pf_streams.json')); print('streams p3', round(d['value']), round(d['ms_per_step']*1e3,1), d['path_roofline']['frac'])"
exit $rc
