"""CPU restatement of the reference's Tokenizer (src/models/tokenizer.h) -- TEST
INFRASTRUCTURE: only tests/ may import it; the product is include/llmi/tokenizer.h.

  load():   Tokenizer::Initialize (tokenizer.h:137-167), the fastllm vocabulary file
  encode(): Tokenizer::Encode (tokenizer.h:168-305): blank (U+2581) normalisation,
            shortest-piece initial symbols, BPE merges by piece score (ties to the
            leftmost pair, tokenizer.h:95-97), <0xXX> byte fallback, <FLM_FIX_TOKEN_n>
  decode(): Tokenizer::DecodeTokens (tokenizer.h:313-348)
Restated with the intended trie semantics (only real pieces are tokens); the
reference's value-initialised TrieNode::tokenId makes its own Encode wrong, which is
why llama.cpp:382 hard-codes its prompt ids -- those ids pin this restatement.
"""
from __future__ import annotations

import struct

BLANK = "▁".encode()
FIX = b"<FLM_FIX_TOKEN_"


class Vocab:
    def __init__(self, path: str):
        b = open(path, "rb").read()
        o = 0

        def i32():
            nonlocal o
            v = struct.unpack_from("<i", b, o)[0]
            o += 4
            return v

        def f32():
            nonlocal o
            v = struct.unpack_from("<f", b, o)[0]
            o += 4
            return v

        self.meta = {}
        if i32() >= 1:
            for _ in range(i32()):
                kl = i32(); k = b[o:o + kl]; o += kl
                vl = i32(); v = b[o:o + vl]; o += vl
                self.meta[k.decode()] = v.decode()
        self.id_of, self.piece_of, self.score = {}, {}, {}
        for _ in range(i32()):
            n = i32()
            piece = bytes(i32() & 0xFF for _ in range(n))
            tid = i32()
            self.id_of[piece] = tid
            self.piece_of[tid] = piece
            self.score[tid] = f32()
        self.max_len = max(len(p) for p in self.id_of)

    def encode(self, text: str) -> list:
        ori = text.encode()
        s = b"" if (len(ori) > 15 and ori[:15] == FIX) else BLANK
        for i, ch in enumerate(ori):
            if ch == 0x20:
                if i != 0 and ori[i - 1] != 0x20:
                    s += BLANK
            else:
                s += bytes([ch])
        syms = []  # [pos, len, fix, unknown]
        i = 0
        while i < len(s):
            if s[i:i + 15] == FIX and i + 15 < len(s):
                j, v = i + 15, 0
                while j < len(s) and 0x30 <= s[j] <= 0x39:
                    v = v * 10 + s[j] - 0x30
                    j += 1
                syms.append([j, 0, v, False])
                i = j + 1
                continue
            ln = next((l for l in range(1, self.max_len + 1) if i + l <= len(s) and s[i:i + l] in self.id_of), 0)
            syms.append([i, ln, None, ln == 0])
            i += max(ln, 1)
        alive = list(range(len(syms)))  # indices of the current symbol list (merged-away ones dropped)
        while True:
            best = None
            for a, bb in zip(alive, alive[1:]):
                if syms[a][1] == 0 or syms[bb][1] == 0:
                    continue
                piece = s[syms[a][0]:syms[a][0] + syms[a][1] + syms[bb][1]]
                if piece in self.id_of:
                    sc = self.score[self.id_of[piece]]
                    if best is None or sc > best[0]:
                        best = (sc, a, bb)
            if best is None:
                break
            _, a, bb = best
            syms[a][1] += syms[bb][1]
            syms[bb][1] = 0
            alive.remove(bb)
        out = []
        for pos, ln, fix, unk in syms:
            if ln > 0:
                out.append(self.id_of[s[pos:pos + ln]])
            elif fix is not None:
                out.append(fix)
            elif unk:
                bp = ("<0x%02X>" % s[pos]).encode()
                if bp in self.id_of:
                    out.append(self.id_of[bp])
        return out

    def decode(self, ids) -> str:
        ret = b""
        for t in ids:
            p = self.piece_of.get(int(t), b"")
            if len(p) == 6 and p[:3] == b"<0x" and p[-1:] == b">":
                p = bytes([int(p[3:5], 16)])
            ret += b"\n" if p == b"<n>" else b"\t" if p == b"<|tab|>" else p
        ret = ret.replace(BLANK, b" ")
        if b"<|blank_" in ret and len(ret) > 10:
            return " " * int(ret[8:len(ret) - 2])
        return ret.decode("utf-8", errors="replace")
