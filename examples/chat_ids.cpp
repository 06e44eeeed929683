// Token-id chat loop over llm::LlamaModel (the id-level twin of user_entry.cpp):
// build a dummy (synthetic-weight) Llama, read a prompt, stream the answer
// through the callback, keep going until "exit". Prompts and answers are
// whitespace-separated token ids (examples/user_entry.cpp is the text version).
//
//   g++ -std=c++17 -I include examples/chat_ids.cpp -L llm-inference_amd/lib -lllmi
//       -Wl,-rpath,$PWD/llm-inference_amd/lib -o chat_ids
//   echo "1 306 4966 29871" | ./chat_ids [preset] [max_new]
#include <cstdio>
#include <iostream>
#include <sstream>
#include <string>

#include "llmi/model.h"

int main(int argc, char** argv) {
    const std::string preset = argc > 1 ? argv[1] : "llama2-7b";
    const int max_new = argc > 2 ? std::atoi(argv[2]) : 256;  // output_token_limit (llama.h:29)
    try {
        auto llm_model = llm::CreateDummyLLMModel(preset);
        while (true) {
            std::printf("please input the question (token ids): ");
            std::fflush(stdout);
            std::string input;
            if (!std::getline(std::cin, input) || input == "exit") break;
            std::istringstream is(input);
            std::vector<int> ids;
            for (int t; is >> t;) ids.push_back(t);
            if (ids.empty()) continue;
            llm_model->Response(ids, max_new, [](int index, int token) {
                if (index == -1) std::printf("\n");
                else std::printf(index == 0 ? ":%d" : " %d", token);
                std::fflush(stdout);
            });
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
