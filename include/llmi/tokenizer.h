// The reference's Tokenizer (src/models/tokenizer.h:57-348): the fastllm ".flm"
// vocabulary file (Initialize, :137-167) and SentencePiece-style BPE (Encode,
// :168-305; Decode / DecodeTokens, :307-348), host-side C++.
//
// Same file format, same normalisation (a U+2581 "blank" prefix; a space that
// follows a non-space becomes a blank, other spaces are dropped; <FLM_FIX_TOKEN_n>
// passes id n through), same merge rule (adjacent symbols whose concatenation is
// a vocabulary piece merge, highest piece score first, ties to the leftmost pair),
// same byte fallback (<0xXX>) and the same decode mapping (<0xXX> bytes, "<n>",
// "<|tab|>", blank -> space). One defect is not carried over: the reference's
// trie nodes value-initialise tokenId to 0, so every prefix of a piece counts as
// a token with score 0 and Encode returns wrong ids -- which is why llama.cpp:382
// hard-codes the ids of its prompt. Here only real pieces are tokens, and Encode
// reproduces those hard-coded ids (tests/test_tokenizer.py).
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <queue>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

class Tokenizer {
public:
    // Tokenizer::Initialize(file): version int; (version >= 1) key/value table of
    // length-prefixed strings; vocabulary: count, then per piece {len, len ints
    // (one byte each), id, float score}.
    void Initialize(std::string file) {
        // the file is external data: every count, length and id is range-checked, a short
        // read stops the parse at once, and the FILE* is closed on every path
        std::unique_ptr<std::FILE, int (*)(std::FILE*)> f(std::fopen(file.c_str(), "rb"), &std::fclose);
        if (!f) throw std::runtime_error("[oneLLM][ERROR] Tokenizer: cannot open " + file);
        auto bad = [&](const std::string& why) {
            return std::runtime_error("[oneLLM][ERROR] Tokenizer: " + why + " in " + file);
        };
        Reader r{f.get()};
        auto i32 = [&](const char* what) {
            const int v = r.i32();
            if (!r.ok) throw bad(std::string("truncated file (reading ") + what + ")");
            return v;
        };
        const int version = i32("version");
        if (version >= 1) {
            const int kv = i32("metadata count");
            if (kv < 0 || kv > kMaxCount) throw bad("metadata count out of range");
            for (int i = 0; i < kv; ++i) {
                std::string key = r.str(kMaxPiece), value = r.str(kMaxPiece);
                if (!r.ok) throw bad("truncated or oversized metadata entry");
                meta_[key] = value;
            }
        }
        const int n = i32("vocabulary count");
        if (n <= 0 || n > kMaxCount) throw bad("vocabulary count out of range");
        for (int i = 0; i < n; ++i) {
            const int len = i32("piece length");
            if (len < 0 || len > kMaxPiece) throw bad("piece length out of range");
            std::string piece(len, '\0');
            for (int j = 0; j < len; ++j) piece[j] = (char)(uint8_t)i32("piece byte");
            const int id = i32("piece id");
            if (id < 0 || id >= kMaxCount) throw bad("piece id out of range");
            const float score = r.f32();
            if (!r.ok) throw bad("truncated file (reading piece score)");
            add_piece(piece, id, score);
        }
    }

    std::vector<int> Encode(const std::string& ori) const {
        const std::string blank = "\xe2\x96\x81";
        const std::string fix = "<FLM_FIX_TOKEN_";
        std::string s = blank;
        if (ori.size() > 15 && ori.compare(0, 15, fix) == 0) s.clear();
        for (size_t i = 0; i < ori.size(); ++i) {
            if (ori[i] == ' ') {
                if (i != 0 && ori[i - 1] != ' ') s += blank;
            } else {
                s += ori[i];
            }
        }
        // initial symbols: the shortest piece starting at each position; a byte that
        // starts no piece is an empty symbol (a merge barrier, byte-fallback later)
        std::vector<Sym> sym;
        for (size_t i = 0; i < s.size(); ++i) {
            if (s.compare(i, fix.size(), fix) == 0 && i + 15 < s.size()) {
                size_t j = i + fix.size();
                int id = 0;
                while (j < s.size() && s[j] >= '0' && s[j] <= '9') id = id * 10 + (s[j++] - '0');
                sym.push_back({(int)j, 0, id, false});
                i = j;  // the reference skips the closing '>' with its loop increment
                continue;
            }
            int len = 0;
            for (int l = 1; l <= max_len_ && i + l <= s.size(); ++l)
                if (id_of_.count(s.substr(i, l))) {
                    len = l;
                    break;
                }
            sym.push_back({(int)i, len, kNoFix, len == 0});
            if (len > 0) i += len - 1;
        }
        const int n = (int)sym.size();
        std::vector<int> prev(n), next(n);
        for (int i = 0; i < n; ++i) {
            prev[i] = i - 1;
            next[i] = i + 1 < n ? i + 1 : -1;
        }
        std::priority_queue<Pair> q;
        auto consider = [&](int l, int r) {
            if (l < 0 || r < 0 || sym[l].len == 0 || sym[r].len == 0) return;
            auto it = id_of_.find(s.substr(sym[l].pos, sym[l].len + sym[r].len));
            if (it == id_of_.end()) return;
            q.push({score_[it->second], l, r, sym[l].len + sym[r].len});
        };
        for (int i = 1; i < n; ++i) consider(i - 1, i);
        while (!q.empty()) {
            const Pair t = q.top();
            q.pop();
            if (sym[t.l].len == 0 || sym[t.r].len == 0 || sym[t.l].len + sym[t.r].len != t.size) continue;
            sym[t.l].len += sym[t.r].len;
            sym[t.r].len = 0;
            next[t.l] = next[t.r];
            if (next[t.r] >= 0) prev[next[t.r]] = t.l;
            consider(prev[t.l], t.l);
            consider(t.l, next[t.l]);
        }
        std::vector<int> out;
        for (int i = 0; i < n; ++i) {
            if (sym[i].len > 0) {
                out.push_back(id_of_.at(s.substr(sym[i].pos, sym[i].len)));
            } else if (sym[i].fix != kNoFix) {
                out.push_back(sym[i].fix);
            } else if (sym[i].unk) {  // merged-away symbols (len 0, not unknown) emit nothing
                char b[8];
                std::snprintf(b, sizeof(b), "<0x%02X>", (unsigned)(uint8_t)s[sym[i].pos]);
                auto it = id_of_.find(b);
                if (it != id_of_.end()) out.push_back(it->second);
            }
        }
        return out;
    }

    std::string Decode(std::vector<int> ids) const { return DecodeTokens(ids); }

    std::string DecodeTokens(const std::vector<int>& tokens) const {
        std::string ret;
        for (int id : tokens) {
            auto it = piece_of_.find(id);
            std::string p = it == piece_of_.end() ? std::string() : it->second;
            if (p.size() == 6 && p.compare(0, 3, "<0x") == 0 && p.back() == '>') {
                p = std::string(1, (char)std::strtol(p.substr(3, 2).c_str(), nullptr, 16));
            }
            if (p == "<n>")
                ret += "\n";
            else if (p == "<|tab|>")
                ret += "\t";
            else
                ret += p;
        }
        const std::string blank = "\xe2\x96\x81";
        for (size_t pos; (pos = ret.find(blank)) != std::string::npos;) ret.replace(pos, blank.size(), " ");
        // the reference's "<|blank_N|>" piece (tokenizer.h:340-344): the whole result is N spaces
        if (ret.find("<|blank_") != std::string::npos && ret.size() > 10)
            return std::string(std::atoi(ret.substr(8, ret.size() - 10).c_str()), ' ');
        return ret;
    }

    int vocab_size() const { return (int)piece_of_.size(); }
    const std::string& meta(const std::string& key) const {
        static const std::string none;
        auto it = meta_.find(key);
        return it == meta_.end() ? none : it->second;
    }

private:
    static constexpr int kNoFix = -999999;
    static constexpr int kMaxPiece = 1024;     // bytes per piece / metadata string
    static constexpr int kMaxCount = 1 << 24;  // pieces, metadata entries, ids
    struct Sym {
        int pos, len, fix;
        bool unk;  // a byte that starts no piece: emitted as its <0xXX> byte piece
    };
    struct Pair {
        float score;
        int l, r, size;
        // max-heap: higher score first, then the leftmost pair (tokenizer.h:95-97)
        bool operator<(const Pair& o) const { return score < o.score || (score == o.score && l > o.l); }
    };
    struct Reader {
        std::FILE* f;
        bool ok = true;
        int i32() {
            int v = 0;
            ok = ok && std::fread(&v, 4, 1, f) == 1;
            return v;
        }
        float f32() {
            float v = 0.f;
            ok = ok && std::fread(&v, 4, 1, f) == 1;
            return v;
        }
        std::string str(int max_len) {
            const int len = i32();
            if (!ok || len < 0 || len > max_len) {
                ok = false;
                return std::string();
            }
            std::string s(len, '\0');
            if (len > 0) ok = std::fread(&s[0], 1, len, f) == (size_t)len;
            return s;
        }
    };
    void add_piece(const std::string& piece, int id, float score) {
        id_of_[piece] = id;
        piece_of_[id] = piece;
        if (id >= (int)score_.size()) score_.resize(id + 1, 0.f);
        score_[id] = score;
        if ((int)piece.size() > max_len_) max_len_ = (int)piece.size();
    }
    std::unordered_map<std::string, int> id_of_;
    std::unordered_map<int, std::string> piece_of_;
    std::vector<float> score_;
    std::unordered_map<std::string, std::string> meta_;
    int max_len_ = 0;
};
