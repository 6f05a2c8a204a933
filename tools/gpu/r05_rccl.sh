#!/bin/bash
# Round 5: RCCL collectives inside the step graphs (world-1 nccl tests + benches),
# the drop-in module, the frozen-mapper QAT fix, and the gloo N=2 rehearsal.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_rccl
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dataset_gpu.py tests/test_rccl_graph_gpu.py tests/test_dropin_gpu.py tests/test_optim_gpu.py "tests/test_train_multi_gpu.py::test_frozen_mapper_in_training_hooks_takes_per_scale_path" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
b() {  # name, env..., -- args
  local n=$1; shift
  timeout -k 10 300 env "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { echo "FAIL $n"; tail -15 $OUT/b_$n.err; exit 1; }
  tail -c 700 $OUT/b_$n.json; echo
}
b c2 python -u bench.py --no-cpu --no-e2e --steps 120
b c2_sharded MCAQ_BENCH_SHARDED=1 python -u bench.py --no-cpu --no-e2e --steps 120
b c5 python -u bench.py --config 5 --no-cpu --steps 100
b c5_torchopt python -u bench.py --config 5 --no-cpu --steps 100 --torch-optim
b score python -u bench.py --score --steps 10 --warmup 2
b c5_sharded MCAQ_BENCH_SHARDED=1 python -u bench.py --config 5 --no-cpu --steps 100
for c in 2 5; do
  MCAQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + c)) bench.py --gpus 2 --config $c --steps 10 --warmup 4 --no-cpu --no-e2e > $OUT/gloo_n2_config$c.json 2> $OUT/gloo_n2_config$c.err || { tail -20 $OUT/gloo_n2_config$c.err; exit 1; }
  tail -c 600 $OUT/gloo_n2_config$c.json; echo
done
