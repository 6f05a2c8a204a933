#!/bin/bash
# Round 6: pass A at 768 threads vs 1024 (base), 4 interleaved rounds at the
# default schedule, then 2 rounds at 4 launch sets in flight.
ROUNDS=4 bash tools/gpu/ab.sh r06_ab_t768 t768 &&
ROUNDS=2 BENCH_ARGS="--pipeline 4" bash tools/gpu/ab.sh r06_ab_t768_p4 t768
