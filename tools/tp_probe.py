#!/usr/bin/env python3
"""Run a tensor-parallel greedy decode with W ranks as W processes (one engine
each, RCCL). On a multi-GPU node each rank gets its own device; with
--same-device every rank uses device 0 (only if RCCL accepts it).
Prints rank 0's tokens and the fixture comparison as JSON."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))


def worker(rank, world, port, same_device, preset, fixture, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch.distributed as dist
    from llmi.engine import Engine, preset as P, tp_unique_id
    import llmi
    dist.init_process_group("gloo", rank=rank, world_size=world)
    obj = [tp_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    f = np.load(fixture)
    cfg = P(preset, tp_rank=rank, tp_world=world)
    cfg.kv_dtype = llmi.F32
    if preset == "llama2-7b":
        cfg.layers, cfg.max_seq = 2, 64
    with Engine(cfg, device=0 if same_device else rank, tp_id=obj[0]) as e:
        e.load_synthetic(int(f["seed"]))
        toks = e.generate(f["prompt"], len(f["tokens"]))
        logits = e.logits()
    gathered = [None] * world
    dist.all_gather_object(gathered, logits.tolist())
    if rank == 0:
        full = np.concatenate([np.array(g, np.float32) for g in gathered])
        rel = float(np.linalg.norm(full - f["last_logits"]) / np.linalg.norm(f["last_logits"]))
        q.put({"world": world, "tokens_equal": bool((toks == f["tokens"]).all()), "logits_rel": rel,
               "tokens": toks.tolist()})
    dist.barrier()
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--preset", default="tiny")
    ap.add_argument("--fixture", default=os.path.join(REPO, "tests", "golden", "tiny.npz"))
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 300
    ps = [ctx.Process(target=worker, args=(r, a.world, port, a.same_device, a.preset, a.fixture, q))
          for r in range(a.world)]
    for p in ps:
        p.start()
    import queue
    import time
    res, t_end = None, time.time() + 240
    while res is None and time.time() < t_end:
        try:
            res = q.get(timeout=2)
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in ps):  # a rank failed: the others would wait forever
                break
    if res is None:
        res = {"world": a.world, "tokens_equal": False, "logits_rel": float("inf"), "error": "a rank failed"}
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.terminate()
            p.join(timeout=10)
    res["exitcodes"] = [p.exitcode for p in ps]
    print(json.dumps(res))
    sys.exit(0 if res["tokens_equal"] and res["logits_rel"] < 1e-3 else 1)


if __name__ == "__main__":
    main()
