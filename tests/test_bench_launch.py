"""bench.py's multi-rank launch contract on the CPU (gloo): `--gpus N` starts N ranks itself when
torchrun's environment is absent and reports n_gpus = N; a world size other than N exits non-zero
(--gpus was parsed and ignored)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", **kw)
    return env


def _run(args, env):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=240)


def test_gpus_2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--plumbing", "--steps", "3", "--warmup", "1"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["steps"] == 3 and rec["value"] > 0


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "2", "--plumbing", "--steps", "1", "--warmup", "0"],
             _env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0", MASTER_PORT="29533"))
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr


def test_gpus_1_runs_in_process():
    r = _run(["--gpus", "1", "--plumbing", "--steps", "2", "--warmup", "0"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 1
