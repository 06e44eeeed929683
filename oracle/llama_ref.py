"""CPU restatement (numpy, fp32) of the reference's Llama-2 decode path.

TEST INFRASTRUCTURE -- the checker, never the thing measured or shipped.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module. The product path is llm-inference_amd/csrc (HIP) and
fails loudly when its shared library is missing; nothing there falls back
to this file.

What it restates (all citations into /root/reference):
  * RMSNorm                 modeling_llama.py:103-117  (fp32 compute, x*rsqrt(mean(x^2)+eps), then *gamma)
  * rotary embedding        modeling_llama.py:123-156  (inv_freq = 1/base^(2i/d), fp32 cos/sin cache)
  * rotate_half / apply     modeling_llama.py:204-236  (pairs (d, d+64))
  * MLP (SwiGLU)            modeling_llama.py:239-270  (down(silu(gate(x)) * up(x)); tp slicing :251-266)
  * repeat_kv               modeling_llama.py:273-282
  * attention w/ KV cache   modeling_llama.py:351-454  (q/k/v proj, RoPE, cache update, softmax fp32, o_proj;
                                                        tp slicing :368-383, :443-446)
  * decoder layer           modeling_llama.py:764-823  (pre-norm residual)
  * model + lm_head         modeling_llama.py:975-1104, 1138-1202 (final norm, logits.float(); tp :1196-1199)
  * greedy sampling         the reference C++ wires top-K with K = beamwidth = 1 (llama.cpp:59, sampling.cu:99),
                            i.e. argmax; ties -> lowest index (numpy/torch argmax).
Layouts restated from the reference C++ path:
  * fused QKV weight rows [q; k; v]          layer_weights.cc:25, fused_decoder_self_attention.cu:356-358
  * fused gate_up rows [gate; up]            layer_weights.cc:40, act_kernel.cu:17-31
  * KV cache [layers, kv_heads, max_seq, d]  llama.cpp:77-78 (batch 1), concat_past_kv.cu:122
Parity pinning: tests/test_oracle_golden.py checks this module against
fixtures produced by the reference's modeling_llama.py itself
(tests/golden/gen_golden.py).

Weights come from oracle/prng.py (identical fp16 bits to the GPU generator);
they are held as fp32 copies of fp16 values so all arithmetic is fp32, as in
the reference's fp32 CPU path. `kv_dtype=np.float16` emulates an fp16 KV
cache by rounding K/V on write (the GPU throughput mode).
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional

import numpy as np

from . import prng


@dataclasses.dataclass(frozen=True)
class LlamaConfig:
    """Mirror of the dims hard-coded at src/utils/model_utils.h:18-31 and llama.h:24-48."""
    hidden: int = 4096
    heads: int = 32
    kv_heads: int = 32
    head_dim: int = 128
    inter: int = 11008
    layers: int = 32
    vocab: int = 32000
    max_seq: int = 2048
    rms_eps: float = 1e-5
    rope_base: float = 10000.0

    @property
    def q_rows(self) -> int:
        return self.heads * self.head_dim

    @property
    def kv_rows(self) -> int:
        return self.kv_heads * self.head_dim


LLAMA2_7B = LlamaConfig()
LLAMA2_13B = LlamaConfig(hidden=5120, heads=40, kv_heads=40, inter=13824, layers=40)


# --------------------------------------------------------------------------- ops
def rmsnorm(x: np.ndarray, gamma: np.ndarray, eps: float) -> np.ndarray:
    """modeling_llama.py:112-117 (fp32 input: the .to(input_dtype) cast is a no-op)."""
    x = x.astype(np.float32)
    var = np.mean(x * x, axis=-1, keepdims=True, dtype=np.float32)
    return gamma.astype(np.float32) * (x * (np.float32(1.0) / np.sqrt(var + np.float32(eps))))


def rope_inv_freq(head_dim: int, base: float) -> np.ndarray:
    """modeling_llama.py:130: 1.0 / base ** (arange(0, d, 2).float() / d), fp32.

    torch's fp32 pow here is correctly rounded (== pow in double, then rounded);
    np.power in fp32 is not (1-2 ulp off), which moves angles at pos 2047 by 1e-5.
    """
    expo = np.arange(0, head_dim, 2, dtype=np.float32) / np.float32(head_dim)
    p = np.power(np.float64(base), expo.astype(np.float64)).astype(np.float32)
    return (np.float32(1.0) / p).astype(np.float32)


def rope_cos_sin(positions: np.ndarray, head_dim: int, base: float):
    """modeling_llama.py:136-146: freqs = outer(t, inv_freq); emb = cat(freqs, freqs)."""
    inv = rope_inv_freq(head_dim, base)
    freqs = np.outer(np.asarray(positions, dtype=np.float32), inv).astype(np.float32)
    emb = np.concatenate([freqs, freqs], axis=-1)
    e64 = emb.astype(np.float64)   # correctly rounded fp32 cos/sin of the fp32 angle
    return np.cos(e64).astype(np.float32), np.sin(e64).astype(np.float32)


def rotate_half(x: np.ndarray) -> np.ndarray:
    """modeling_llama.py:204-208."""
    h = x.shape[-1] // 2
    return np.concatenate([-x[..., h:], x[..., :h]], axis=-1)


def apply_rope(x: np.ndarray, cos: np.ndarray, sin: np.ndarray) -> np.ndarray:
    """modeling_llama.py:233-235 for one tensor; x [..., heads, d], cos/sin [d]."""
    return (x * cos + rotate_half(x) * sin).astype(np.float32)


def silu(x: np.ndarray) -> np.ndarray:
    """ACT2FN['silu'] used at modeling_llama.py:248,268: x * sigmoid(x)."""
    x = x.astype(np.float32)
    return x / (np.float32(1.0) + np.exp(-x))


def linear(x: np.ndarray, w: np.ndarray) -> np.ndarray:
    """nn.Linear without bias: x @ W^T, W row-major [out, in] (linear.cu:38-99 trans_b)."""
    return (x.astype(np.float32) @ w.astype(np.float32).T).astype(np.float32)


def attention_decode(q: np.ndarray, k_cache: np.ndarray, v_cache: np.ndarray, ctx: int) -> np.ndarray:
    """One query position against ctx cached positions (modeling_llama.py:417-437).

    q [heads, d]; caches [kv_heads, >=ctx, d] (already holding the current k/v).
    """
    heads, d = q.shape
    group = heads // k_cache.shape[0]
    k = np.repeat(k_cache[:, :ctx].astype(np.float32), group, axis=0)   # repeat_kv :273-282
    v = np.repeat(v_cache[:, :ctx].astype(np.float32), group, axis=0)
    s = np.einsum("hd,hjd->hj", q.astype(np.float32), k) / np.float32(math.sqrt(d))
    s = s - s.max(axis=-1, keepdims=True)
    p = np.exp(s)
    p = p / p.sum(axis=-1, keepdims=True)
    return np.einsum("hj,hjd->hd", p.astype(np.float32), v).astype(np.float32)


def attention_prefill(q: np.ndarray, k_cache: np.ndarray, v_cache: np.ndarray, p0: int) -> np.ndarray:
    """Causal attention for M query rows at positions p0..p0+M-1 (modeling_llama.py:417-437
    with the 4-D causal mask of :1043-1046; build_causal_mask.cu:29 semantics).

    q [M, heads, d]; caches [kv_heads, >= p0+M, d] holding this chunk's k/v."""
    m, heads, d = q.shape
    ctx = p0 + m
    group = heads // k_cache.shape[0]
    k = np.repeat(k_cache[:, :ctx].astype(np.float32), group, axis=0)
    v = np.repeat(v_cache[:, :ctx].astype(np.float32), group, axis=0)
    s = np.matmul(q.astype(np.float32).transpose(1, 0, 2), k.transpose(0, 2, 1)) / np.float32(math.sqrt(d))
    allowed = np.arange(ctx)[None, :] <= (p0 + np.arange(m))[:, None]
    s = np.where(allowed[None], s, np.float32(-np.inf))
    s = s - s.max(axis=-1, keepdims=True)
    pr = np.exp(s)
    pr = pr / pr.sum(axis=-1, keepdims=True)
    return np.matmul(pr.astype(np.float32), v).transpose(1, 0, 2).astype(np.float32)


def argmax_first(logits: np.ndarray) -> int:
    return int(np.argmax(logits))


# ----------------------------------------------------------------------- weights
@dataclasses.dataclass
class LayerWeights:
    qkv: np.ndarray          # [q_rows + 2*kv_rows, hidden] fp16
    o: np.ndarray            # [hidden, q_rows]
    gate_up: np.ndarray      # [2*inter, hidden]
    down: np.ndarray         # [hidden, inter]
    attn_norm: np.ndarray    # [hidden]
    ffn_norm: np.ndarray     # [hidden]
    # int8 mode (W8A16): per-row fp16 scales; matrices above then hold int8
    qkv_s: Optional[np.ndarray] = None
    o_s: Optional[np.ndarray] = None
    gate_up_s: Optional[np.ndarray] = None
    down_s: Optional[np.ndarray] = None


def _lin(seed, tid, rows, cols, row0, col0, ld, int8):
    if int8:
        return prng.int8_weight(seed, tid, rows, cols, row0, col0, ld)
    return prng.linear_fp16(seed, tid, rows, cols, row0, col0, ld)


def make_layer_weights(cfg: LlamaConfig, seed: int, layer: int, int8: bool = False,
                       tp_rank: int = 0, tp_world: int = 1) -> LayerWeights:
    """Weights of one layer (or its tensor-parallel shard).

    Column-parallel q/k/v/gate/up take output rows [r*n/tp, (r+1)*n/tp) of each
    of q, k, v (resp. gate, up); row-parallel o/down take the matching input
    columns -- the slicing of modeling_llama.py:251-266, 368-383, 443-446.
    """
    H, I = cfg.hidden, cfg.inter
    qn, kn = cfg.q_rows // tp_world, cfg.kv_rows // tp_world
    In = I // tp_world
    t = lambda k: prng.layer_tid(layer, k)
    q = _lin(seed, t(prng.KIND_Q), qn, H, tp_rank * qn, 0, H, int8)
    k = _lin(seed, t(prng.KIND_K), kn, H, tp_rank * kn, 0, H, int8)
    v = _lin(seed, t(prng.KIND_V), kn, H, tp_rank * kn, 0, H, int8)
    o = _lin(seed, t(prng.KIND_O), H, qn, 0, tp_rank * qn, cfg.q_rows, int8)
    g = _lin(seed, t(prng.KIND_GATE), In, H, tp_rank * In, 0, H, int8)
    u = _lin(seed, t(prng.KIND_UP), In, H, tp_rank * In, 0, H, int8)
    d = _lin(seed, t(prng.KIND_DOWN), H, In, 0, tp_rank * In, I, int8)
    lw = LayerWeights(
        qkv=np.concatenate([q, k, v], axis=0), o=o,
        gate_up=np.concatenate([g, u], axis=0), down=d,
        attn_norm=prng.gamma_fp16(seed, t(prng.KIND_ATTN_NORM), H),
        ffn_norm=prng.gamma_fp16(seed, t(prng.KIND_FFN_NORM), H))
    if int8:
        sc = lambda kind, rows, row0: prng.int8_row_scale(seed, t(kind), rows, row0)
        lw.qkv_s = np.concatenate([sc(prng.KIND_Q, qn, tp_rank * qn), sc(prng.KIND_K, kn, tp_rank * kn),
                                   sc(prng.KIND_V, kn, tp_rank * kn)])
        lw.o_s = sc(prng.KIND_O, H, 0)
        lw.gate_up_s = np.concatenate([sc(prng.KIND_GATE, In, tp_rank * In), sc(prng.KIND_UP, In, tp_rank * In)])
        lw.down_s = sc(prng.KIND_DOWN, H, 0)
    return lw


def dequant(w: np.ndarray, s: Optional[np.ndarray]) -> np.ndarray:
    """W8A16 dequantisation: w_q[r, :] * scale[r] (build-defined)."""
    if s is None:
        return w.astype(np.float32)
    return w.astype(np.float32) * s.astype(np.float32)[:, None]


@dataclasses.dataclass
class ModelWeights:
    embed: np.ndarray        # [vocab, hidden] fp16   (pre_decoder_embedding_weight, llama_weights.cc:28-31)
    lm_head: np.ndarray      # [vocab(/tp), hidden]   (post_decoder_embedding_weight, untied, :32-35)
    final_norm: np.ndarray   # [hidden]
    layers: List[LayerWeights]


# In-process memo of generated weights (test-suite time: a 7B-width PRNG model takes ~30 s
# of numpy): the embedding per (seed, vocab, hidden) -- every TP rank shares it -- and
# whole unsharded models per (config without max_seq, seed, int8), at most two kept.
# The arrays are shared, so they are made read-only.
_EMBED_MEMO: Dict[tuple, np.ndarray] = {}
_MODEL_MEMO: Dict[tuple, "ModelWeights"] = {}


def _readonly(a: np.ndarray) -> np.ndarray:
    a.setflags(write=False)
    return a


def make_model_weights(cfg: LlamaConfig, seed: int, int8: bool = False,
                       tp_rank: int = 0, tp_world: int = 1) -> ModelWeights:
    key = (dataclasses.replace(cfg, max_seq=0), seed, int8)
    if tp_world == 1 and key in _MODEL_MEMO:
        return _MODEL_MEMO[key]
    ek = (seed, cfg.vocab, cfg.hidden)
    if ek not in _EMBED_MEMO:
        _EMBED_MEMO[ek] = _readonly(prng.embed_fp16(seed, prng.GLOBAL_EMBED, cfg.vocab, cfg.hidden))
    vn = cfg.vocab // tp_world
    w = ModelWeights(
        embed=_EMBED_MEMO[ek],
        lm_head=prng.linear_fp16(seed, prng.GLOBAL_LM_HEAD, vn, cfg.hidden, tp_rank * vn, 0, cfg.hidden),
        final_norm=prng.gamma_fp16(seed, prng.GLOBAL_FINAL_NORM, cfg.hidden),
        layers=[make_layer_weights(cfg, seed, l, int8, tp_rank, tp_world) for l in range(cfg.layers)])
    if tp_world == 1:
        for a in (w.lm_head, w.final_norm):
            _readonly(a)
        for lw in w.layers:
            for f in dataclasses.fields(lw):
                a = getattr(lw, f.name)
                if isinstance(a, np.ndarray):
                    _readonly(a)
        if len(_MODEL_MEMO) >= 2:
            _MODEL_MEMO.pop(next(iter(_MODEL_MEMO)))
        _MODEL_MEMO[key] = w
    return w


# ------------------------------------------------------------------------- model
class LlamaOracle:
    """Single-stream greedy decoder: the reference's continueTokenGen loop
    (llama.cpp:318-349, Response :362-457) with HF arithmetic.

    fp32 copies of every weight are made once (the fp16 values are exact in fp32).
    """

    def __init__(self, cfg: LlamaConfig, seed: int = 0, int8: bool = False,
                 kv_dtype=np.float32, weights: Optional[ModelWeights] = None):
        self.cfg = cfg
        self.kv_dtype = kv_dtype
        w = weights or make_model_weights(cfg, seed, int8)
        self.embed = w.embed                                     # gathered rows only: keep fp16
        self.lm_head = w.lm_head.astype(np.float32)
        self.final_norm = w.final_norm.astype(np.float32)
        self.layers = []
        for lw in w.layers:
            self.layers.append(dict(
                qkv=dequant(lw.qkv, lw.qkv_s), o=dequant(lw.o, lw.o_s),
                gate_up=dequant(lw.gate_up, lw.gate_up_s), down=dequant(lw.down, lw.down_s),
                attn_norm=lw.attn_norm.astype(np.float32), ffn_norm=lw.ffn_norm.astype(np.float32)))
        shape = (cfg.layers, cfg.kv_heads, cfg.max_seq, cfg.head_dim)
        self.k_cache = np.zeros(shape, dtype=kv_dtype)
        self.v_cache = np.zeros(shape, dtype=kv_dtype)
        self.pos = 0

    def reset(self):
        self.pos = 0

    def layer_forward(self, l: int, x: np.ndarray, pos: int) -> np.ndarray:
        """modeling_llama.py:764-823 for one token; x [hidden] fp32 residual stream."""
        c, W = self.cfg, self.layers[l]
        h = rmsnorm(x, W["attn_norm"], c.rms_eps)
        qkv = linear(h, W["qkv"])
        q = qkv[:c.q_rows].reshape(c.heads, c.head_dim)
        k = qkv[c.q_rows:c.q_rows + c.kv_rows].reshape(c.kv_heads, c.head_dim)
        v = qkv[c.q_rows + c.kv_rows:].reshape(c.kv_heads, c.head_dim)
        cos, sin = rope_cos_sin([pos], c.head_dim, c.rope_base)
        q = apply_rope(q, cos[0], sin[0])
        k = apply_rope(k, cos[0], sin[0])
        self.k_cache[l, :, pos] = k.astype(self.kv_dtype)            # cache.update :408
        self.v_cache[l, :, pos] = v.astype(self.kv_dtype)
        attn = attention_decode(q, self.k_cache[l], self.v_cache[l], pos + 1).reshape(-1)
        x = x + linear(attn, W["o"])                                 # residual :807
        h = rmsnorm(x, W["ffn_norm"], c.rms_eps)
        gu = linear(h, W["gate_up"])
        act = silu(gu[:c.inter]) * gu[c.inter:]
        return (x + linear(act, W["down"])).astype(np.float32)       # residual :813

    def forward_token(self, token: int, pos: Optional[int] = None) -> np.ndarray:
        """One decode step: embedding -> layers -> final norm -> lm_head -> fp32 logits."""
        pos = self.pos if pos is None else pos
        x = self.embed[token].astype(np.float32)
        for l in range(self.cfg.layers):
            x = self.layer_forward(l, x, pos)
        self.pos = pos + 1
        self.last_hidden = x
        return linear(rmsnorm(x, self.final_norm, self.cfg.rms_eps), self.lm_head)

    def prefill(self, ids: np.ndarray, round_a=None) -> np.ndarray:
        """Llama<T>::firstTokenGen (llama.cpp:273-316): all prompt rows at once through
        LlamaContextDecoder (context_decoder.cpp:47-143) -- causal attention, KV slots
        0..M-1 written -- then final norm + lm_head on the LAST row only (llama.cpp:218-233).
        Returns the last row's fp32 logits; self.last_hidden_rows holds the residual stream.

        round_a (optional) is applied to every GEMM A operand (normed x, attention output,
        SiLU product) -- used to size the error of rounding them to the MFMA input type."""
        c = self.cfg
        ra = (lambda t: t) if round_a is None else round_a
        ids = np.asarray(ids)
        m, p0 = len(ids), self.pos
        X = self.embed[ids].astype(np.float32)
        cos, sin = rope_cos_sin(np.arange(p0, p0 + m), c.head_dim, c.rope_base)
        cos, sin = cos[:, None, :], sin[:, None, :]
        for l in range(c.layers):
            W = self.layers[l]
            qkv = linear(ra(rmsnorm(X, W["attn_norm"], c.rms_eps)), W["qkv"])
            q = qkv[:, :c.q_rows].reshape(m, c.heads, c.head_dim)
            k = qkv[:, c.q_rows:c.q_rows + c.kv_rows].reshape(m, c.kv_heads, c.head_dim)
            v = qkv[:, c.q_rows + c.kv_rows:].reshape(m, c.kv_heads, c.head_dim)
            q, k = apply_rope(q, cos, sin), apply_rope(k, cos, sin)
            self.k_cache[l, :, p0:p0 + m] = k.transpose(1, 0, 2).astype(self.kv_dtype)
            self.v_cache[l, :, p0:p0 + m] = v.transpose(1, 0, 2).astype(self.kv_dtype)
            attn = attention_prefill(q, self.k_cache[l], self.v_cache[l], p0).reshape(m, -1)
            X = X + linear(ra(attn), W["o"])
            gu = linear(ra(rmsnorm(X, W["ffn_norm"], c.rms_eps)), W["gate_up"])
            X = (X + linear(ra(silu(gu[:, :c.inter]) * gu[:, c.inter:]), W["down"])).astype(np.float32)
        self.pos = p0 + m
        self.last_hidden_rows = X
        self.last_hidden = X[-1]
        return linear(rmsnorm(X[-1], self.final_norm, c.rms_eps), self.lm_head)

    def greedy(self, prompt: np.ndarray, n_new: int):
        """Feed the prompt token by token, then n_new greedy tokens.

        Returns (generated ids [n_new], logits of the last forward)."""
        logits = None
        for t in prompt:
            logits = self.forward_token(int(t))
        out = []
        for i in range(n_new):
            nxt = argmax_first(logits)
            out.append(nxt)
            if i + 1 < n_new:
                logits = self.forward_token(nxt)
        return np.array(out, dtype=np.int32), logits


# ---------------------------------------------------------- tensor-parallel emul
def tp_layer_partials(cfg: LlamaConfig, shard: Dict[str, np.ndarray], x: np.ndarray,
                      k_cache: np.ndarray, v_cache: np.ndarray, pos: int, tp_world: int):
    """One rank's share of a decoder layer under Megatron TP.

    Returns (o_partial, fn) where fn(x_after_attn) -> down_partial, mirroring
    the per-slice F.linear calls of modeling_llama.py:368-383,443-446,251-266.
    """
    c = cfg
    hn, kvn = c.heads // tp_world, c.kv_heads // tp_world
    qn, kn, In = hn * c.head_dim, kvn * c.head_dim, c.inter // tp_world
    h = rmsnorm(x, shard["attn_norm"], c.rms_eps)
    qkv = linear(h, shard["qkv"])
    q = qkv[:qn].reshape(hn, c.head_dim)
    k = qkv[qn:qn + kn].reshape(kvn, c.head_dim)
    v = qkv[qn + kn:].reshape(kvn, c.head_dim)
    cos, sin = rope_cos_sin([pos], c.head_dim, c.rope_base)
    q, k = apply_rope(q, cos[0], sin[0]), apply_rope(k, cos[0], sin[0])
    k_cache[:, pos] = k
    v_cache[:, pos] = v
    attn = attention_decode(q, k_cache, v_cache, pos + 1).reshape(-1)
    o_part = linear(attn, shard["o"])

    def mlp_part(x_mid):
        hh = rmsnorm(x_mid, shard["ffn_norm"], c.rms_eps)
        gu = linear(hh, shard["gate_up"])
        return linear(silu(gu[:In]) * gu[In:], shard["down"])
    return o_part, mlp_part
