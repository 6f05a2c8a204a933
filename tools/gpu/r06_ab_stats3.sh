#!/bin/bash
# Round 6: pass-1 occupancy - fewer floats per lane in flight (LANE_FLOATS 32 / 16)
# at 6 / 8 waves per SIMD (MINW), and MINW 6 alone; configs 2 and 3.
ROUNDS=2 bash tools/gpu/ab.sh r06_ab_stats3_c2 lf32m6 lf32m8 m6 lf16m8 &&
ROUNDS=2 BENCH_ARGS="--config 3 --launch-batches 1" bash tools/gpu/ab.sh r06_ab_stats3_c3 lf32m6 lf32m8 m6 lf16m8
