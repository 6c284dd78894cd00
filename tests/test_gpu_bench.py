"""bench.py --gpus N starts its own N ranks (no external launcher), as the driver's scaling runs invoke it.

Two ranks share the one card of the test box over gloo (CTR_DIST_BACKEND=gloo: the collective sequence RCCL runs at
N > 1, host-staged); the timings are not performance numbers.  The parent process must not touch the GPU before it
starts the ranks (bench.launch_ranks), each rank checks WORLD_SIZE against --gpus, and rank 0's JSON line reaches
the parent's stdout."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra, timeout=420):
    env = dict(os.environ, **env_extra)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    p = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


@pytest.mark.gpu
@pytest.mark.timeout(480)
def test_bench_gpus2_spawns_its_own_ranks():
    p, lines = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--kernel-events", "none"],
                      {"CTR_DIST_BACKEND": "gloo"})
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    assert len(lines) == 1, p.stdout[-2000:]          # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2, rec
    assert rec["config"]["parallelism"] == "dp2, tables row-sharded", rec["config"]
    assert rec["config"]["global_batch"] == 2 * 4096
    assert rec["steps"] == 2 and rec["value"] > 0 and rec["scaling"] == "weak"


@pytest.mark.timeout(240)
def test_bench_rank_count_mismatch_fails():
    """A rank launched with WORLD_SIZE != --gpus exits non-zero instead of reporting the wrong n_gpus (checked before
    anything touches the GPU: runs on CPU)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                        "0", "--no-cpu-baseline"], cwd=REPO, env=env, capture_output=True, text=True, timeout=200)
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stdout + p.stderr)
