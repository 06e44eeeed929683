"""The N > 1 bench path on a one-GPU box: `bench.py --gpus 2` self-spawns two workers
(RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* on 127.0.0.1), and with LLMI_BENCH_ONE_DEVICE=1 both
ranks build their TP = 2 shard of Llama-2-7B on device 0, map each other's inbox over
IPC and run the timed decode loop with the one-shot peer exchange as the TP reduction --
as its own launches or fused into the producing launches, whichever the timing picks
(RCCL refuses two ranks on one device, so it is left out). Checks that the whole flow --
spawn, rendezvous, exchange open + cross-rank token check, graphs with exchange kernels,
max-over-ranks timing, rank 0's JSON line -- completes with consistent tokens. The
throughput of two ranks sharing one GPU is not a scaling number."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_one_device_oneshot():
    env = dict(os.environ, LLMI_BENCH_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--max-seq", "128", "--steps", "1",
           "--warmup", "0", "--no-side", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    print(json.dumps({k: out[k] for k in ("value", "n_gpus", "ms_per_step", "tp_tokens_consistent")}))
    print(json.dumps(out.get("tp_exchange")))
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert out["tp_tokens_consistent"] is True
    # the exchange form is picked by timing (one launch per exchange vs fused into the producers)
    assert out["tp_exchange"]["mode"] in ("oneshot", "fused") and out["tp_exchange"]["one_device_rehearsal"] is True
    assert len(out["tp_exchange"]["us_per_forward_oneshot_vs_fused"]) == 2
