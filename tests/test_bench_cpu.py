"""bench.py's self-launch: `python bench.py --gpus N` with no
WORLD_SIZE in the environment starts N rank processes of itself (the env
torch.distributed.run would set) before anything touches a GPU, and passes
rank 0's one JSON line through.  Checked with the launcher rehearsal
(--launch-check: gloo rendezvous + all-reduce, no GPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_spawns_its_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--launch-check"],
                       env=env, capture_output=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    # (gloo itself prints a "[Gloo] Rank 0 is connected" line on stdout)
    lines = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["rank_sum"] == 3.0
