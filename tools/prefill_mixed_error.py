#!/usr/bin/env python3
"""Error budget of the prefill GEMM input precision, per GEMM site (oracle study, CPU).

The engine's prefill feeds each GEMM its fp32 A operand either as two fp16 planes
(hi + lo: fp32-faithful, 2x the MFMA work) or as one (hi = fp16(a)). This runs the
oracle's batched prefill (oracle/llama_ref.py: LlamaOracle.prefill, the same math)
layer by layer over Llama-2-7B (32 layers, PRNG weights, 512 rows) with every
combination of sites rounded to fp16 and reports the last row's logits rel-L2 against
the unrounded run -- the north-star bar is 1e-3.

    python tools/prefill_mixed_error.py [--layers 32] [--rows 512] [--fp8lo]

--fp8lo: instead, every site as the engine's split mode 3 runs it (llmi_engine_prefill
exact = 2): hi = fp16(a) exact, plus e4m3(lo * 2^12) / 2^12 against e4m3(W * 2^e) / 2^e
(e per tensor from max |W|, as w8_prepare), beside all four sites at fp16 (the fast mode).
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


def e4m3(x):
    """OCP e4m3 round-to-nearest-even, saturated to +-448 (3 mantissa bits; subnormal step 2^-9)."""
    x = np.clip(x.astype(np.float64), -448.0, 448.0)
    _, e = np.frexp(x)  # x = m 2^e, 0.5 <= |m| < 1
    step = np.ldexp(1.0, np.maximum(e, -5) - 4)
    return (np.round(x / step) * step).astype(np.float32)


def w8_exp(w):
    amax = float(np.max(np.abs(w)))
    e = int(np.floor(np.log2(448.0 / amax)))
    while amax * 2.0 ** e > 448.0:
        e -= 1
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--rows", type=int, default=512)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--fp8lo", action="store_true")
    a = ap.parse_args()
    c = R.LlamaConfig(layers=a.layers, max_seq=a.rows)
    f16 = lambda t: t.astype(np.float16).astype(np.float32)  # noqa: E731
    ident = lambda t: t  # noqa: E731
    combos = [(), ("qkv",), ("gate_up",), ("o", "down"), ("qkv", "gate_up"), ("qkv", "gate_up", "o"),
              ("qkv", "gate_up", "down"), SITES]
    if a.fp8lo:  # exact, all four sites fp16 (fast mode), all four sites fp16 hi + e4m3 lo (mode 3)
        combos = [(), SITES, ("fp8lo",)]
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
        W8 = {}
        if a.fp8lo:
            for s_ in SITES:
                e = w8_exp(W[s_])
                W8[s_] = e4m3(W[s_] * np.float32(2.0 ** e)) * np.float32(2.0 ** -e)

        def gemm(site, t, cb):
            if cb == ("fp8lo",):
                hi = f16(t)
                lo8 = e4m3((t - hi) * np.float32(4096.0)) * np.float32(1.0 / 4096.0)
                return R.linear(hi, W[site]) + R.linear(lo8, W8[site])
            return R.linear(f16(t) if site in cb else t, W[site])

        for cb in combos:
            x = X[cb]
            qkv = gemm("qkv", R.rmsnorm(x, W["attn_norm"], c.rms_eps), cb)
            q = qkv[:, :c.q_rows].reshape(m, c.heads, c.head_dim)
            k = qkv[:, c.q_rows:c.q_rows + c.kv_rows].reshape(m, c.kv_heads, c.head_dim)
            v = qkv[:, c.q_rows + c.kv_rows:].reshape(m, c.kv_heads, c.head_dim)
            q, k = R.apply_rope(q, cos, sin), R.apply_rope(k, cos, sin)
            kc = k.transpose(1, 0, 2).astype(np.float16).astype(np.float32)  # the bench's fp16 cache
            vc = v.transpose(1, 0, 2).astype(np.float16).astype(np.float32)
            attn = R.attention_prefill(q, kc, vc, 0).reshape(m, -1)
            x = x + gemm("o", attn, cb)
            gu = gemm("gate_up", R.rmsnorm(x, W["ffn_norm"], c.rms_eps), cb)
            X[cb] = (x + gemm("down", R.silu(gu[:, :c.inter]) * gu[:, c.inter:], cb)).astype(np.float32)
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
