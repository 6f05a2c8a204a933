#!/bin/bash
# Round 6: pipelined persistent pass 2 at 3 workgroups per CU vs base -
# 4 rounds at config 2, 2 rounds each at configs 3 and 4.
ROUNDS=4 bash tools/gpu/ab.sh r06_ab_pipe3_c2 pipe3 &&
ROUNDS=2 BENCH_ARGS="--config 3" bash tools/gpu/ab.sh r06_ab_pipe3_c3 pipe3 &&
ROUNDS=2 BENCH_ARGS="--config 4" bash tools/gpu/ab.sh r06_ab_pipe3_c4 pipe3
