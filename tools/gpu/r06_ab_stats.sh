#!/bin/bash
# Round 6: pass-1 pixels-per-lane variants (MCAQ_STATS_PPL_R4, LANE_FLOATS,
# MINW) at config 3 (k = 1) and config 2 (default), interleaved A/B.
ROUNDS=2 BENCH_ARGS="--config 3 --launch-batches 1" bash tools/gpu/ab.sh r06_ab_stats_c3 r4p2 r4p4 r4p2lf128 r4p4lf128 &&
ROUNDS=2 bash tools/gpu/ab.sh r06_ab_stats_c2 r4p2 r4p4 r4p2lf128 r4p4lf128
