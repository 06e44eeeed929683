#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE's own modeling_llama.py.

Runs only in the build container (where /root/reference exists); the GPU box
never executes this file. It imports /root/reference/modeling_llama.py in
memory with the three shims of SURVEY.md Appendix B (the file targets
transformers ~4.36; this image has transformers 5.x), fills the reference
modules with the portable PRNG weights of oracle/prng.py (fp16 values held
as fp32, i.e. the reference's fp32 CPU path), and records inputs + outputs:

  f1_ops.npz      per-op vectors at 7B width: RMSNorm, RoPE at positions
                  {0,1,127,128,2047}, SiLU*mul (LlamaMLP act), q_proj rows
  f2_layer.npz    config 1: one LlamaDecoderLayer, hidden 4096, seq 8, fp32
  f3_decode.npz   2-layer 7B-width model: 8-token prompt, 16 greedy steps,
                  token ids, logits of the first and last step, layer-0 K/V
  f4_tp8.npz      f3 with pretraining_tp = 8 (sharded-linear semantics)
  f5_int8.npz     13B-width 1-layer W8A16 model (dequantised weights)
  f6_prefill.npz  7B-width 1 layer, prefill seq 512, last-token logits
  f7_longctx.npz  2-layer 7B width, max_seq 2048: batched 2040-token prompt, then
                  greedy steps to ctx 2048 (+ the oracle's fp16-KV emulation)
  f8_ctx_history_{tiny,7b}.npz  ragged context batch with history: 3 sequences, histories
                  {0, 5, 17}, chunks {8, 4, 11}; history K/V, chunk logits + written K/V
  f9_7b_32layers.npz  the bench model itself: Llama-2-7B shape, all 32 layers, fp32,
                  8-token prompt, 16 greedy cached steps (tokens, first/last logits)
  tiny.npz        test_llama_run.py-like tiny model (hidden 512, 2 layers)
  manifest.json   versions + what each fixture holds

Weights are NOT stored (they are regenerated from the seed); only ids,
activations and outputs are. Usage: python tests/golden/gen_golden.py [f.npz ...]
(all fixtures, or the named ones; --skip name.npz leaves one out); --check regenerates
everything into a temporary directory and compares the arrays with the committed fixtures
(F9 alone takes ~10 minutes of the check: the 32-layer reference run and the oracle's).
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import prng  # noqa: E402
from oracle.llama_ref import LlamaConfig, make_model_weights  # noqa: E402

REF = "/root/reference/modeling_llama.py"
OUT = os.path.dirname(os.path.abspath(__file__))


def load_reference():
    """SURVEY.md Appendix B recipe: our harness code around the reference file."""
    import transformers.utils.import_utils as iu
    iu.is_torch_fx_available = getattr(iu, "is_torch_fx_available", lambda: False)
    import transformers.models.llama  # noqa: F401  parent package for relative imports
    name = "transformers.models.llama.ref_modeling_llama"
    spec = importlib.util.spec_from_file_location(name, REF)
    ref = importlib.util.module_from_spec(spec)
    sys.modules[name] = ref
    spec.loader.exec_module(ref)

    class KV:  # stands in for the v4.36 DynamicCache API (modeling_llama.py:402,408,1016-1017)
        def __init__(s):
            s.k, s.v = [], []

        def get_usable_length(s, n, i=0):
            return s.k[i].shape[-2] if i < len(s.k) else 0

        def update(s, k, v, i, kw=None):
            if i == len(s.k):
                s.k.append(k)
                s.v.append(v)
            else:
                s.k[i] = torch.cat([s.k[i], k], -2)
                s.v[i] = torch.cat([s.v[i], v], -2)
            return s.k[i], s.v[i]

    ref.Cache = KV
    return ref, KV


def ref_config(ref, c: LlamaConfig, tp: int = 1):
    cfg = ref.LlamaConfig(hidden_size=c.hidden, intermediate_size=c.inter,
                          num_hidden_layers=c.layers, num_attention_heads=c.heads,
                          num_key_value_heads=c.kv_heads, vocab_size=c.vocab,
                          rms_norm_eps=c.rms_eps, max_position_embeddings=max(c.max_seq, 2048))
    for k, v in dict(_attn_implementation="eager", rope_theta=c.rope_base, rope_scaling=None,
                     pretraining_tp=tp, attention_bias=False, attention_dropout=0.0,
                     hidden_act="silu").items():
        object.__setattr__(cfg, k, v)
    return cfg


def f32(a):
    return torch.from_numpy(np.ascontiguousarray(a.astype(np.float32)))


def build_model(ref, c: LlamaConfig, seed: int, tp: int = 1, int8: bool = False):
    torch.manual_seed(0)
    m = ref.LlamaForCausalLM(ref_config(ref, c, tp)).eval()
    w = make_model_weights(c, seed, int8=int8)
    from oracle.llama_ref import dequant
    sd = {"model.embed_tokens.weight": f32(w.embed), "lm_head.weight": f32(w.lm_head),
          "model.norm.weight": f32(w.final_norm)}
    q, kv, I = c.q_rows, c.kv_rows, c.inter
    for l, lw in enumerate(w.layers):
        p = f"model.layers.{l}."
        qkv = dequant(lw.qkv, lw.qkv_s)
        gu = dequant(lw.gate_up, lw.gate_up_s)
        sd[p + "self_attn.q_proj.weight"] = f32(qkv[:q])
        sd[p + "self_attn.k_proj.weight"] = f32(qkv[q:q + kv])
        sd[p + "self_attn.v_proj.weight"] = f32(qkv[q + kv:])
        sd[p + "self_attn.o_proj.weight"] = f32(dequant(lw.o, lw.o_s))
        sd[p + "mlp.gate_proj.weight"] = f32(gu[:I])
        sd[p + "mlp.up_proj.weight"] = f32(gu[I:])
        sd[p + "mlp.down_proj.weight"] = f32(dequant(lw.down, lw.down_s))
        sd[p + "input_layernorm.weight"] = f32(lw.attn_norm)
        sd[p + "post_attention_layernorm.weight"] = f32(lw.ffn_norm)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if "rotary_emb" not in k]
    assert not missing and not unexpected, (missing, unexpected)
    return m


@torch.no_grad()
def greedy_ref(ref, KV, m, prompt: np.ndarray, n_new: int, keep_kv_pos=()):
    cache = KV()
    ids = torch.from_numpy(prompt.astype(np.int64))[None]
    out = m(input_ids=ids, past_key_values=cache, use_cache=True)
    logits = out.logits[0, -1].float().numpy()
    first_logits = logits.copy()
    toks, pos = [], len(prompt)
    for i in range(n_new):
        t = int(np.argmax(logits))
        toks.append(t)
        if i + 1 == n_new:
            break
        out = m(input_ids=torch.tensor([[t]]), position_ids=torch.tensor([[pos]]),
                past_key_values=cache, use_cache=True)
        logits = out.logits[0, -1].float().numpy()
        pos += 1
    kv = {}
    for p in keep_kv_pos:
        kv[f"k_l0_p{p}"] = cache.k[0][0, :, p].numpy().astype(np.float32)
        kv[f"v_l0_p{p}"] = cache.v[0][0, :, p].numpy().astype(np.float32)
    return np.array(toks, np.int32), first_logits, logits, kv


@torch.no_grad()
def gen_f1(ref, seed=11):
    c = LlamaConfig(layers=1)
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((4, c.hidden)).astype(np.float32)
    gamma = prng.gamma_fp16(seed, prng.layer_tid(0, prng.KIND_ATTN_NORM), c.hidden)
    norm = ref.LlamaRMSNorm(c.hidden, eps=c.rms_eps)
    norm.weight.data = f32(gamma)
    rms_out = norm(f32(x)).numpy()
    # RoPE on q/k [1, heads, npos, d] at chosen positions
    positions = np.array([0, 1, 127, 128, 2047], np.int64)
    q = rng.standard_normal((1, c.heads, len(positions), c.head_dim)).astype(np.float32)
    k = rng.standard_normal((1, c.kv_heads, len(positions), c.head_dim)).astype(np.float32)
    rot = ref.LlamaRotaryEmbedding(c.head_dim, max_position_embeddings=2048, base=c.rope_base)
    cos, sin = rot(f32(q), seq_len=2048)
    qe, ke = ref.apply_rotary_pos_emb(f32(q), f32(k), cos, sin, torch.from_numpy(positions)[None])
    # SiLU*mul exactly as LlamaMLP forms it (modeling_llama.py:268)
    gu = rng.standard_normal((2, 3 * 512)).astype(np.float32) * 3
    act = ref.ACT2FN["silu"]
    silu_mul = (act(f32(gu[:, :512 * 1])) * f32(gu[:, 512:1024])).numpy()
    # q_proj rows 0..255 of layer 0 (fp16 weights as fp32) applied to x
    wq = prng.linear_fp16(seed, prng.layer_tid(0, prng.KIND_Q), 256, c.hidden)
    lin = torch.nn.functional.linear(f32(x), f32(wq)).numpy()
    np.savez_compressed(os.path.join(OUT, "f1_ops.npz"), seed=seed, x=x, rms_out=rms_out,
                        rope_pos=positions, rope_q=q, rope_k=k, rope_q_out=qe.numpy(),
                        rope_k_out=ke.numpy(), silu_in=gu[:, :1024], silu_mul_out=silu_mul,
                        linear_out=lin)


@torch.no_grad()
def gen_f2(ref, seed=12):
    """Config 1: one decoder layer forward, hidden 4096, seq 8, fp32 (BASELINE.json configs[0])."""
    c = LlamaConfig(layers=1)
    m = build_model(ref, c, seed)
    layer = m.model.layers[0]
    x = np.random.default_rng(seed).standard_normal((1, 8, c.hidden)).astype(np.float32)
    mask = torch.full((8, 8), float("-inf")).triu(1)[None, None]
    pos = torch.arange(8)[None]
    kw = {}
    if hasattr(m.model, "rotary_emb"):
        kw["position_embeddings"] = m.model.rotary_emb(f32(x), pos)
    t0 = time.perf_counter()
    y = layer(f32(x), attention_mask=mask, position_ids=pos, **kw)[0].numpy()
    dt = time.perf_counter() - t0
    np.savez_compressed(os.path.join(OUT, "f2_layer.npz"), seed=seed, x=x, y=y, ref_cpu_s=dt)


def gen_decode(ref, KV, c, seed, tp, fname, n_new=16, int8=False, keep_kv_pos=(0, 7, 22)):
    m = build_model(ref, c, seed, tp=tp, int8=int8)
    prompt = prng.prompt_ids(seed, 8, c.vocab)
    t0 = time.perf_counter()
    toks, first, last, kv = greedy_ref(ref, KV, m, prompt, n_new, keep_kv_pos)
    dt = time.perf_counter() - t0
    np.savez_compressed(os.path.join(OUT, fname), seed=seed, prompt=prompt, tokens=toks,
                        first_logits=first, last_logits=last, ref_cpu_s=dt, **kv)
    return toks


@torch.no_grad()
def gen_f6(ref, seed=16, seq=512):
    c = LlamaConfig(layers=1)
    m = build_model(ref, c, seed)
    ids = prng.prompt_ids(seed + 1, seq, c.vocab)
    out = m(input_ids=torch.from_numpy(ids.astype(np.int64))[None], use_cache=False)
    np.savez_compressed(os.path.join(OUT, "f6_prefill.npz"), seed=seed, ids=ids,
                        last_logits=out.logits[0, -1].float().numpy(),
                        logits_rows=out.logits[0, [0, 1, 255, 511]].float().numpy())


@torch.no_grad()
def gen_f7(ref, KV, seed=17, prompt_len=2040, n_new=9):
    """The bench shape end to end at full context: 2 layers at 7B width, max_seq 2048.
    The reference runs ONE batched forward over a 2040-token prompt (its cached path,
    modeling_llama.py:351-454), then greedy steps until a forward at position 2047
    (ctx 2048). Also recorded: the same run of the numpy oracle with an fp16 KV cache
    (oracle/llama_ref.py, kv_dtype=float16), the emulation of the engine's throughput
    mode, and each step's top-2 logit margin."""
    from oracle.llama_ref import LlamaOracle
    c = LlamaConfig(layers=2, max_seq=2048)
    m = build_model(ref, c, seed)
    prompt = prng.prompt_ids(seed, prompt_len, c.vocab)
    t0 = time.perf_counter()
    toks, first, last, kv = greedy_ref(ref, KV, m, prompt, n_new, keep_kv_pos=())
    dt = time.perf_counter() - t0
    o = LlamaOracle(c, seed=seed, kv_dtype=np.float16)
    logits = o.prefill(prompt)
    o_first, o_toks = logits.copy(), []
    for i in range(n_new):
        t = int(np.argmax(logits))
        o_toks.append(t)
        if i + 1 < n_new:
            logits = o.forward_token(t)
    np.savez_compressed(os.path.join(OUT, "f7_longctx.npz"), seed=seed, prompt=prompt, tokens=toks,
                        first_logits=first, last_logits=last, ref_cpu_s=dt,
                        f16kv_tokens=np.array(o_toks, np.int32), f16kv_first_logits=o_first,
                        f16kv_last_logits=logits)
    return toks


@torch.no_grad()
def gen_f8(ref, KV, c, seed, fname, hist=(0, 5, 17), lens=(8, 4, 11), new_heads=4):
    """Ragged context batch WITH history (LlamaContextDecoder / LLaMAContextAttentionLayer
    with history_length, context_decoder.cpp:61-82, context_attention.cpp:85-174): for each
    sequence b the reference runs its h_b history tokens into a fresh cache, then its
    q_b-row chunk with that cache (positions h_b .. h_b + q_b - 1). Recorded: the ids, the
    history K/V every layer holds before the chunk (the test uploads them into the
    batch's cache), the K/V the chunk writes (last layer, first new_heads kv heads), and
    the logits of the chunk's last row."""
    m = build_model(ref, c, seed)
    out = {"seed": np.int64(seed), "hist": np.array(hist, np.int32), "lens": np.array(lens, np.int32)}
    for b, (h, q) in enumerate(zip(hist, lens)):
        ids = prng.prompt_ids(seed + 100 + b, h + q, c.vocab)
        cache = KV()
        if h > 0:
            m(input_ids=torch.from_numpy(ids[:h].astype(np.int64))[None], past_key_values=cache, use_cache=True)
            out[f"hist_k{b}"] = np.stack([cache.k[l][0].numpy() for l in range(c.layers)]).astype(np.float32)
            out[f"hist_v{b}"] = np.stack([cache.v[l][0].numpy() for l in range(c.layers)]).astype(np.float32)
        res = m(input_ids=torch.from_numpy(ids[h:].astype(np.int64))[None], past_key_values=cache, use_cache=True)
        out[f"ids{b}"] = ids.astype(np.int32)
        out[f"logits{b}"] = res.logits[0, -1].float().numpy()  # the chunk's last row
        # the K/V the chunk writes: the last layer, kv heads [0, new_heads) (size-bounded)
        nh = min(c.kv_heads, new_heads)
        out[f"new_k{b}"] = cache.k[c.layers - 1][0, :nh, h:].numpy().astype(np.float32)
        out[f"new_v{b}"] = cache.v[c.layers - 1][0, :nh, h:].numpy().astype(np.float32)
    np.savez_compressed(os.path.join(OUT, fname), **out)


@torch.no_grad()
def gen_f9(ref, KV, seed=20, n_new=16):
    """Parity at the bench's depth: the reference's LlamaForCausalLM
    (modeling_llama.py:975-1104, 1138-1202) at the full Llama-2-7B shape, 32 layers, fp32,
    the PRNG weights of seed 20; an 8-token prompt through the batched forward, then 15
    greedy cached steps. ~27 GB of fp32 parameters: the module is built once (its own
    random init) and the PRNG weights are copied in layer by layer, so no second full copy
    of the model is ever held (the container has 62 GB)."""
    c = LlamaConfig()
    torch.manual_seed(0)
    m = ref.LlamaForCausalLM(ref_config(ref, c)).eval()
    from oracle.llama_ref import make_layer_weights
    q, kv, I = c.q_rows, c.kv_rows, c.inter

    def put(t, a):
        t.copy_(torch.from_numpy(np.ascontiguousarray(a)).to(torch.float32))

    put(m.model.embed_tokens.weight, prng.embed_fp16(seed, prng.GLOBAL_EMBED, c.vocab, c.hidden))
    put(m.lm_head.weight, prng.linear_fp16(seed, prng.GLOBAL_LM_HEAD, c.vocab, c.hidden, 0, 0, c.hidden))
    put(m.model.norm.weight, prng.gamma_fp16(seed, prng.GLOBAL_FINAL_NORM, c.hidden))
    for l, layer in enumerate(m.model.layers):
        lw = make_layer_weights(c, seed, l)
        a = layer.self_attn
        put(a.q_proj.weight, lw.qkv[:q])
        put(a.k_proj.weight, lw.qkv[q:q + kv])
        put(a.v_proj.weight, lw.qkv[q + kv:])
        put(a.o_proj.weight, lw.o)
        put(layer.mlp.gate_proj.weight, lw.gate_up[:I])
        put(layer.mlp.up_proj.weight, lw.gate_up[I:])
        put(layer.mlp.down_proj.weight, lw.down)
        put(layer.input_layernorm.weight, lw.attn_norm)
        put(layer.post_attention_layernorm.weight, lw.ffn_norm)
        del lw
    prompt = prng.prompt_ids(seed, 8, c.vocab)
    t0 = time.perf_counter()
    toks, first, last, _ = greedy_ref(ref, KV, m, prompt, n_new)
    dt = time.perf_counter() - t0
    del m
    # the bench's fp16 KV cache, emulated by the numpy oracle (same weights, the cache's
    # stores rounded to fp16; token-by-token like the engine's decode): what the fp16-KV
    # engine is held to at this depth, next to its drift from the fp32 reference
    from oracle.llama_ref import LlamaOracle
    import gc
    gc.collect()
    o = LlamaOracle(c, seed=seed, kv_dtype=np.float16)
    o_toks, o_last = o.greedy(prompt, n_new)
    del o
    np.savez_compressed(os.path.join(OUT, "f9_7b_32layers.npz"), seed=seed, prompt=prompt, tokens=toks,
                        first_logits=first, last_logits=last, ref_cpu_s=dt,
                        f16kv_tokens=np.asarray(o_toks, np.int32), f16kv_last_logits=o_last)
    return toks


def check():
    """Regenerate every fixture into a temporary directory and compare its arrays with
    the committed ones (timings excluded): the committed fixtures are what this script
    produces from the reference (zip timestamps make a byte comparison meaningless)."""
    global OUT
    import tempfile
    committed = OUT
    with tempfile.TemporaryDirectory() as tmp:
        OUT = tmp
        main(write_manifest=False)
        bad = []
        for name in sorted(os.listdir(tmp)):
            a = np.load(os.path.join(tmp, name), allow_pickle=False)
            b = np.load(os.path.join(committed, name), allow_pickle=False)  # (skipped fixtures are not regenerated)
            keys = sorted(k for k in a.files if k != "ref_cpu_s")
            if keys != sorted(k for k in b.files if k != "ref_cpu_s"):
                bad.append(f"{name}: keys {keys} vs {sorted(b.files)}")
                continue
            for k in keys:
                if k.startswith("f16kv_") and k != "f16kv_tokens":
                    # the numpy oracle's emulation arrays (not the reference's): BLAS may sum in
                    # another order on another host / thread count -- compared at 1e-5 rel-L2
                    x, y = a[k].astype(np.float64), b[k].astype(np.float64)
                    if np.linalg.norm(x - y) > 1e-5 * np.linalg.norm(y):
                        bad.append(f"{name}:{k}")
                elif not np.array_equal(a[k], b[k]):
                    bad.append(f"{name}:{k}")
        OUT = committed
    print("fixtures reproduce" if not bad else "MISMATCH: " + ", ".join(bad))
    return not bad


def main(write_manifest=True):
    ref, KV = load_reference()
    torch.set_num_threads(os.cpu_count() or 8)
    import transformers
    manifest = {"torch": torch.__version__, "transformers": transformers.__version__,
                "numpy": np.__version__, "reference": REF, "prng": "llmi-prng-v1 (oracle/prng.py)",
                "fixtures": {}}
    steps = [
        ("f1_ops.npz", lambda: gen_f1(ref)),
        ("f2_layer.npz", lambda: gen_f2(ref)),
        ("tiny.npz", lambda: gen_decode(ref, KV, LlamaConfig(hidden=512, heads=4, kv_heads=4,
                                                              inter=1024, layers=2, vocab=32000,
                                                              max_seq=64), 21, 1, "tiny.npz", n_new=24,
                                        keep_kv_pos=(0, 7, 23))),
        ("f3_decode.npz", lambda: gen_decode(ref, KV, LlamaConfig(layers=2), 13, 1, "f3_decode.npz")),
        ("f4_tp8.npz", lambda: gen_decode(ref, KV, LlamaConfig(layers=2), 13, 8, "f4_tp8.npz")),
        ("f5_int8.npz", lambda: gen_decode(ref, KV, LlamaConfig(hidden=5120, heads=40, kv_heads=40,
                                                                 inter=13824, layers=1), 15, 1,
                                            "f5_int8.npz", n_new=8, int8=True,
                                            keep_kv_pos=(0, 7, 14))),
        ("f6_prefill.npz", lambda: gen_f6(ref)),
        ("f7_longctx.npz", lambda: gen_f7(ref, KV)),
        ("f8_ctx_history_tiny.npz", lambda: gen_f8(ref, KV, LlamaConfig(hidden=512, heads=4, kv_heads=4, inter=1024,
                                                                          layers=2, vocab=32000, max_seq=64), 18,
                                                   "f8_ctx_history_tiny.npz")),
        ("f8_ctx_history_7b.npz", lambda: gen_f8(ref, KV, LlamaConfig(layers=2, max_seq=64), 19,
                                                  "f8_ctx_history_7b.npz")),
        ("f9_7b_32layers.npz", lambda: gen_f9(ref, KV)),
    ]
    args = sys.argv[1:]
    skip = set(args[i + 1] for i, a in enumerate(args[:-1]) if a == "--skip")
    only = set(a for i, a in enumerate(args) if a.endswith(".npz") and (i == 0 or args[i - 1] != "--skip"))
    for name, fn in steps:
        if (only and name not in only) or name in skip:
            continue
        t0 = time.time()
        fn()
        print(f"{name}: {time.time() - t0:.1f}s", flush=True)
        manifest["fixtures"][name] = {"generated_s": round(time.time() - t0, 1)}
    if not write_manifest:
        return
    # data fixture copied from the reference (not generated): the tokenizer vocabulary
    import hashlib
    import shutil
    tok_src = os.path.join(os.path.dirname(REF), "llama2-7b-tokenizer.bin")
    tok_dst = os.path.join(OUT, "llama2-7b-tokenizer.bin")
    shutil.copyfile(tok_src, tok_dst)
    manifest["fixtures"]["llama2-7b-tokenizer.bin"] = {
        "source": "copied verbatim from /root/reference/llama2-7b-tokenizer.bin (data file the reference's "
                  "user_entry.cpp:8 loads)",
        "sha256": hashlib.sha256(open(tok_dst, "rb").read()).hexdigest(),
        "known_answer": "src/models/llama/llama.cpp:382 hard-coded ids of 'Hey, are you conscious? Can you "
                        "talk to me?'"}
    mpath = os.path.join(OUT, "manifest.json")
    if os.path.exists(mpath) and only:
        old = json.load(open(mpath))
        old["fixtures"].update(manifest["fixtures"])
        manifest["fixtures"] = old["fixtures"]
    json.dump(manifest, open(mpath, "w"), indent=1)


if __name__ == "__main__":
    if "--check" in sys.argv:
        sys.exit(0 if check() else 1)
    main()
