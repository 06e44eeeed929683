"""bench.py's multi-GPU launcher on CPU: `bench.py --gpus N` with no WORLD_SIZE spawns
N worker processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1),
before any GPU call, and relays rank 0's single JSON line; `--dry-run` stops after
the gloo rendezvous. A failing worker makes the whole run fail."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=REPO)


def test_self_spawn_dry_run_two_workers():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout  # exactly one JSON line on stdout
    out = json.loads(lines[0])
    assert out["dry_run"] and out["n_gpus"] == 2
    assert sorted(d["rank"] for d in out["ranks"]) == [0, 1]
    assert sorted(d["local_rank"] for d in out["ranks"]) == [0, 1]
    assert len({d["pid"] for d in out["ranks"]}) == 2


def test_single_gpu_dry_run_needs_no_spawn():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip())["n_gpus"] == 1


def test_launcher_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
