bash tools/gpu/r06_dp.sh r06_dp; echo "dp rc=$?"
ROUNDS=2 bash tools/gpu/ab.sh r06_ab1 cap1 cap2 cap4 minw5 cap2m5 cap1m5 cap4m5
