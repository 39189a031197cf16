"""bench.py's launch contract on CPU (gloo): `--gpus N` without torchrun spawns N local ranks that
rendezvous on 127.0.0.1 and form one process group of N ranks; a process group whose size differs
from --gpus fails the run (no silent 1-GPU measurement)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", NCN_DIST_BACKEND="gloo", **kw)
    return env


def test_spawns_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-selftest"], env=_env(), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout  # one JSON line, from rank 0 only
    out = json.loads(line[0])
    assert out == {"world": 2, "backend": "gloo", "rank_sum": 1.0}


def test_world_mismatch_fails():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # a single-rank "torchrun" environment while --gpus asks for 2: must not report a 1-GPU result
    env = _env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-selftest"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "--gpus 2" in r.stderr


def test_crashed_rank_ends_the_launch():
    """A rank that exits non-zero ends the others (blocked in the all-reduce) and the parent returns
    its status instead of hanging (spawn_ranks polls every rank)."""
    import time
    t = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-selftest"],
                       env=_env(NCN_SELFTEST_CRASH_RANK="0", NCN_SELFTEST_HANG_RANK="1"), capture_output=True,
                       text=True, timeout=200)
    assert r.returncode == 7, (r.returncode, r.stderr[-2000:])
    assert time.time() - t < 150
