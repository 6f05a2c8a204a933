#!/bin/bash
# Round 6: pass 2 as a persistent kernel with a 2-deep register pipeline
# (MCAQ_QUANT_PIPE workgroups per CU) vs one workgroup per unit - config 2
# default and config 4.
ROUNDS=2 bash tools/gpu/ab.sh r06_ab_pipe_c2 pipe1 pipe2 pipe3 pipe4 &&
ROUNDS=2 BENCH_ARGS="--config 4" bash tools/gpu/ab.sh r06_ab_pipe_c4 pipe2 pipe4
