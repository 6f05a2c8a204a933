#!/bin/bash
# Round 6: the data-parallel QAT fast path, ClipAdamW fixes and the
# self-launching bench.  Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r06_dp}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_amp_gpu.py tests/test_core_gpu.py tests/test_optim_gpu.py tests/test_rccl_graph_gpu.py tests/test_dist_qat_gpu.py tests/test_train_multi_gpu.py tests/test_qat_gpu.py -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|error" $OUT/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --config 5 > $OUT/b_c5.json 2> $OUT/b_c5.err || { tail -5 $OUT/b_c5.err; exit 1; }
MCAQ_BENCH_SHARDED=1 timeout -k 10 300 python bench.py --config 5 > $OUT/b_c5_sharded.json 2> $OUT/b_c5_sharded.err || { tail -5 $OUT/b_c5_sharded.err; exit 1; }
MCAQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu --steps 20 --warmup 4 > $OUT/b_gloo_n2.json 2> $OUT/b_gloo_n2.err || { tail -5 $OUT/b_gloo_n2.err; exit 1; }
python3 - <<PY
import json
for k in ("b_c5", "b_c5_sharded", "b_gloo_n2"):
    ls = [l for l in open("$OUT/%s.json" % k).read().splitlines() if l.startswith("{")]
    d = json.loads(ls[-1])
    print(k, d["n_gpus"], d["value"], d["ms_per_step"], (d.get("step_roofline") or d.get("path_roofline") or {}).get("frac"), (d.get("e2e") or {}).get("value"), d["config"].get("rccl_in_graph"))
PY
