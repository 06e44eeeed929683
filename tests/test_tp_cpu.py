"""Tensor-parallel decode math on CPU (no GPU): the Megatron split the engine
uses -- column-parallel q/k/v/gate/up, row-parallel o/down with
a sum all-reduce, vocab-parallel lm_head with a max-reduce of the argmax keys --
run as world-size-2 gloo processes with oracle arithmetic, checked against the
TP=1 reference fixture; and the oracle's 8-way shards against the reference's
own `pretraining_tp = 8` run (modeling_llama.py:251-266,368-383,443-446,1196-1199)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import llama_ref as R
from oracle import prng

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TINY = R.LlamaConfig(hidden=512, heads=4, kv_heads=4, inter=1024, layers=2, vocab=32000, max_seq=64)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def argmax_key(v: float, idx: int) -> int:
    """The engine's order-preserving (value, index) key (csrc/common.h argmax_key)."""
    b = int(np.float32(v).view(np.uint32))
    b = (~b & 0xFFFFFFFF) if b & 0x80000000 else (b | 0x80000000)
    return (b << 32) | (0xFFFFFFFF - idx)


class ShardedDecoder:
    """One rank's view: its weight shards + its slice of the KV cache."""

    def __init__(self, cfg, seed, rank, world):
        self.cfg, self.rank, self.world = cfg, rank, world
        w = R.make_model_weights(cfg, seed, tp_rank=rank, tp_world=world)
        self.embed = w.embed
        self.lm = w.lm_head.astype(np.float32)
        self.vn = cfg.vocab // world
        self.fnorm = w.final_norm.astype(np.float32)
        self.layers = [dict(qkv=l.qkv.astype(np.float32), o=l.o.astype(np.float32),
                            gate_up=l.gate_up.astype(np.float32), down=l.down.astype(np.float32),
                            attn_norm=l.attn_norm.astype(np.float32), ffn_norm=l.ffn_norm.astype(np.float32))
                       for l in w.layers]
        kvl = cfg.kv_heads // world
        self.kc = np.zeros((cfg.layers, kvl, cfg.max_seq, cfg.head_dim), np.float32)
        self.vc = np.zeros_like(self.kc)

    def forward(self, token, pos, allreduce_sum, allreduce_max):
        c = self.cfg
        x = self.embed[token].astype(np.float32)
        for l, W in enumerate(self.layers):
            o_part, mlp = R.tp_layer_partials(c, W, x, self.kc[l], self.vc[l], pos, self.world)
            # rank 0 carries the residual into the all-reduce (engine: attention seeds xacc)
            x = allreduce_sum((x if self.rank == 0 else np.zeros_like(x)) + o_part)
            x = allreduce_sum((x if self.rank == 0 else np.zeros_like(x)) + mlp(x))
        logits = R.linear(R.rmsnorm(x, self.fnorm, c.rms_eps), self.lm)
        best = max(argmax_key(v, self.rank * self.vn + i) for i, v in enumerate(logits))
        best = allreduce_max(best)
        return 0xFFFFFFFF - (best & 0xFFFFFFFF), logits


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    f = np.load(os.path.join(G, "tiny.npz"))

    def ar_sum(v):
        t = torch.from_numpy(np.ascontiguousarray(v, np.float32))
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.numpy()

    def ar_max(k):
        t = torch.tensor([k >> 1], dtype=torch.int64)  # keys are 64-bit unsigned; halve into int64 range
        lo = torch.tensor([k & 1], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        mine = (k >> 1) == int(t.item())
        lo = lo if mine else torch.tensor([-1], dtype=torch.int64)
        dist.all_reduce(lo, op=dist.ReduceOp.MAX)
        return (int(t.item()) << 1) | int(lo.item())

    d = ShardedDecoder(TINY, int(f["seed"]), rank, world)
    toks, pos, logits = [], 0, None
    for t in f["prompt"]:
        nxt, logits = d.forward(int(t), pos, ar_sum, ar_max)
        pos += 1
    for i in range(len(f["tokens"])):
        toks.append(nxt)
        if i + 1 < len(f["tokens"]):
            nxt, logits = d.forward(nxt, pos, ar_sum, ar_max)
            pos += 1
    gathered = [None] * world
    dist.all_gather_object(gathered, logits.tolist())
    if rank == 0:
        q.put((toks, np.concatenate([np.array(g, np.float32) for g in gathered])))
    dist.destroy_process_group()


def test_tp2_gloo_decode_matches_reference_fixture():
    f = np.load(os.path.join(G, "tiny.npz"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    toks, logits = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(np.array(toks), f["tokens"])
    assert rel(logits, f["last_logits"]) < 1e-5


def test_argmax_key_order_and_ties():
    ks = [argmax_key(v, i) for i, v in enumerate([1.0, -2.0, 3.0, 3.0, -0.0, 0.0])]
    assert max(range(6), key=lambda i: ks[i]) == 2          # tie 3.0 at 2 and 3 -> lowest index
    assert argmax_key(-1.0, 0) < argmax_key(-0.5, 0) < argmax_key(0.0, 0) < argmax_key(1e-30, 0)


@pytest.mark.slow
def test_oracle_tp8_shards_match_reference_pretraining_tp8():
    """Sum of 8 oracle shards == the reference's pretraining_tp=8 run (F4), token-exact."""
    f = np.load(os.path.join(G, "f4_tp8.npz"))
    cfg = R.LlamaConfig(layers=2, max_seq=64)
    world = 8
    shards = [ShardedDecoder(cfg, int(f["seed"]), r, world) for r in range(world)]
    state = {"x": None}

    def forward(token, pos):
        xs = [s.embed[token].astype(np.float32) for s in shards]
        x = xs[0]
        for l in range(cfg.layers):
            parts = [R.tp_layer_partials(cfg, s.layers[l], x, s.kc[l], s.vc[l], pos, world) for s in shards]
            x = x + sum(p[0] for p in parts)
            x = x + sum(p[1](x) for p in parts)
        logits = np.concatenate([R.linear(R.rmsnorm(x, s.fnorm, cfg.rms_eps), s.lm) for s in shards])
        return logits

    logits, pos = None, 0
    for t in f["prompt"]:
        logits = forward(int(t), pos)
        pos += 1
    toks = []
    for i in range(len(f["tokens"])):
        toks.append(int(np.argmax(logits)))
        if i + 1 < len(f["tokens"]):
            logits = forward(toks[-1], pos)
            pos += 1
    np.testing.assert_array_equal(np.array(toks), f["tokens"])
    assert rel(logits, f["last_logits"]) < 1e-5
    f3 = np.load(os.path.join(G, "f3_decode.npz"))
    np.testing.assert_array_equal(f3["tokens"], f["tokens"])  # TP=8 and TP=1 agree in the reference too
