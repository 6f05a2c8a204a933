#!/bin/bash
# Round 6: pass A at 768 / 512 threads per workgroup (3 / 2 waves per SIMD at
# 128 VGPRs: a CU running pass A keeps VGPRs for streaming waves) with and
# without capped streaming passes - config 2 default.
ROUNDS=2 bash tools/gpu/ab.sh r06_ab_threads t768 t768cap1 t512 t512cap2
