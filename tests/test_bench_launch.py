"""bench.py's own rank launcher: `bench.py --gpus N`
without an outside launcher starts N ranks itself (torch.distributed.run as a
child process, never exec) and every rank sees a world of N.  --launch-check stops
after the process group is up, so this runs on the CPU (gloo)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args],
                         capture_output=True, text=True, env=env, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_spawns_world_2():
    rec = _run("--gpus", "2", "--launch-check")
    assert rec["nranks_seen"] == 2 and rec["spawned_by_bench"]
    assert sorted(r["rank"] for r in rec["ranks"]) == [0, 1]
    assert len({r["pid"] for r in rec["ranks"]}) == 2


def test_bench_gpus_1_stays_in_process():
    rec = _run("--gpus", "1", "--launch-check")
    assert rec["nranks_seen"] == 1 and not rec["spawned_by_bench"]
