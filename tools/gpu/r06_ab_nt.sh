#!/bin/bash
# Round 6: cache policy of the streaming passes at config 2 (k = 2, depth 3)
# and config 4: pass-2 x loads nontemporal too (qnt3), no nontemporal at all
# in pass 2 (qnt0), pass-1 x loads plain (s1plain) - against the default
# (pass 1 nt loads; pass 2 nt stores, plain loads below 256 MB per launch).
ROUNDS=2 bash tools/gpu/ab.sh r06_ab_nt_c2 qnt3 qnt0 s1plain &&
ROUNDS=2 BENCH_ARGS="--config 4" bash tools/gpu/ab.sh r06_ab_nt_c4 qnt3 qnt0 s1plain
