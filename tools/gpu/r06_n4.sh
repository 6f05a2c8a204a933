set -o pipefail
mkdir -p gpurun_out/r06_n4
timeout -k 10 400 python -u -m pytest tests/test_dist_qat_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r06_n4/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r06_n4/pytest.log; [ $rc -eq 0 ] || exit $rc
MCAQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --no-cpu --no-e2e --steps 20 --warmup 4 > gpurun_out/r06_n4/bench_gloo_n4.json 2> gpurun_out/r06_n4/bench_gloo_n4.err || { tail -5 gpurun_out/r06_n4/bench_gloo_n4.err; exit 1; }
MCAQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --config 5 --no-cpu --steps 10 --warmup 3 > gpurun_out/r06_n4/bench_gloo_n4_c5.json 2> gpurun_out/r06_n4/bench_gloo_n4_c5.err || { tail -5 gpurun_out/r06_n4/bench_gloo_n4_c5.err; exit 1; }
grep -h "^{" gpurun_out/r06_n4/bench_gloo_n4*.json | cut -c1-300
