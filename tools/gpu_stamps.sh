cd $GRAFT_REPO_ROOT && timeout -k 10 120 python tools/prof_morph_stamps.py 2 > gpurun_out/stamps.log 2>&1; head -24 gpurun_out/stamps.log
