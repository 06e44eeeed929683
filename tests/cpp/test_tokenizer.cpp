// Drives include/llmi/tokenizer.h for tests/test_tokenizer.py: argv[1] = the
// vocabulary file; each stdin line is encoded, and the ids are decoded back.
// Prints one JSON object per line: {"ids": [...], "text": "..."}.
#include <cstdio>
#include <iostream>
#include <string>

#include "llmi/tokenizer.h"

static std::string json_escape(const std::string& s) {
    std::string o;
    for (unsigned char c : s) {
        if (c == '"' || c == '\\') {
            o += '\\';
            o += (char)c;
        } else if (c < 0x20) {
            char b[8];
            std::snprintf(b, sizeof(b), "\\u%04x", c);
            o += b;
        } else {
            o += (char)c;
        }
    }
    return o;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    Tokenizer tok;
    try {
        tok.Initialize(argv[1]);
    } catch (const std::exception& e) {  // a malformed vocabulary file is reported, never parsed on
        std::fprintf(stderr, "%s\n", e.what());
        return 3;
    }
    std::string line;
    while (std::getline(std::cin, line)) {
        std::vector<int> ids = tok.Encode(line);
        std::printf("{\"ids\": [");
        for (size_t i = 0; i < ids.size(); ++i) std::printf("%s%d", i ? ", " : "", ids[i]);
        std::printf("], \"text\": \"%s\"}\n", json_escape(tok.Decode(ids)).c_str());
    }
    return 0;
}
