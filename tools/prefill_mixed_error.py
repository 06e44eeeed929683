#!/usr/bin/env python3
"""Error budget of the prefill GEMM input precision, per GEMM site (oracle study, CPU).

The engine's prefill feeds each GEMM its fp32 A operand either as two fp16 planes
(hi + lo: fp32-faithful, 2x the MFMA work) or as one (hi = fp16(a)). This runs the
oracle's batched prefill (oracle/llama_ref.py: LlamaOracle.prefill, the same math)
layer by layer over Llama-2-7B (32 layers, PRNG weights, 512 rows) with every
combination of sites rounded to fp16 and reports the last row's logits rel-L2 against
the unrounded run -- the north-star bar is 1e-3.

    python tools/prefill_mixed_error.py [--layers 32] [--rows 512]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import llama_ref as R  # noqa: E402
from oracle import prng  # noqa: E402

SITES = ("qkv", "o", "gate_up", "down")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--rows", type=int, default=512)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    c = R.LlamaConfig(layers=a.layers, max_seq=a.rows)
    f16 = lambda t: t.astype(np.float16).astype(np.float32)  # noqa: E731
    ident = lambda t: t  # noqa: E731
    combos = [(), ("qkv",), ("gate_up",), ("o", "down"), ("qkv", "gate_up"), ("qkv", "gate_up", "o"),
              ("qkv", "gate_up", "down"), SITES]
    ids = prng.prompt_ids(a.seed, a.rows, c.vocab) if hasattr(prng, "prompt_ids") else \
        np.random.default_rng(a.seed).integers(0, c.vocab, a.rows)
    embed = prng.embedding_fp16(a.seed, c.vocab, c.hidden) if hasattr(prng, "embedding_fp16") else None
    if embed is None:
        w = R.make_model_weights(R.LlamaConfig(layers=0, max_seq=a.rows), a.seed)
        embed, lm_head, final_norm = w.embed, w.lm_head.astype(np.float32), w.final_norm.astype(np.float32)
    X0 = embed[ids].astype(np.float32)
    X = {cb: X0.copy() for cb in combos}
    m = a.rows
    cos, sin = R.rope_cos_sin(np.arange(m), c.head_dim, c.rope_base)
    cos, sin = cos[:, None, :], sin[:, None, :]
    for l in range(c.layers):
        lw = R.make_layer_weights(c, a.seed, l)
        W = dict(qkv=lw.qkv.astype(np.float32), o=lw.o.astype(np.float32), gate_up=lw.gate_up.astype(np.float32),
                 down=lw.down.astype(np.float32), attn_norm=lw.attn_norm.astype(np.float32),
                 ffn_norm=lw.ffn_norm.astype(np.float32))
        for cb in combos:
            ra = {s: (f16 if s in cb else ident) for s in SITES}
            x = X[cb]
            qkv = R.linear(ra["qkv"](R.rmsnorm(x, W["attn_norm"], c.rms_eps)), W["qkv"])
            q = qkv[:, :c.q_rows].reshape(m, c.heads, c.head_dim)
            k = qkv[:, c.q_rows:c.q_rows + c.kv_rows].reshape(m, c.kv_heads, c.head_dim)
            v = qkv[:, c.q_rows + c.kv_rows:].reshape(m, c.kv_heads, c.head_dim)
            q, k = R.apply_rope(q, cos, sin), R.apply_rope(k, cos, sin)
            kc = k.transpose(1, 0, 2).astype(np.float16).astype(np.float32)  # the bench's fp16 cache
            vc = v.transpose(1, 0, 2).astype(np.float16).astype(np.float32)
            attn = R.attention_prefill(q, kc, vc, 0).reshape(m, -1)
            x = x + R.linear(ra["o"](attn), W["o"])
            gu = R.linear(ra["gate_up"](R.rmsnorm(x, W["ffn_norm"], c.rms_eps)), W["gate_up"])
            X[cb] = (x + R.linear(ra["down"](R.silu(gu[:, :c.inter]) * gu[:, c.inter:]), W["down"])).astype(np.float32)
        print(f"layer {l} done", file=sys.stderr, flush=True)
    logits = {cb: R.linear(R.rmsnorm(X[cb][-1], final_norm, c.rms_eps), lm_head) for cb in combos}
    ref = logits[()]
    out = {"layers": c.layers, "rows": m, "seed": a.seed, "bar": 1e-3, "rel_l2_vs_fp32": {}}
    for cb in combos[1:]:
        e = float(np.linalg.norm(logits[cb] - ref) / np.linalg.norm(ref))
        out["rel_l2_vs_fp32"]["+".join(cb)] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
