// Text chat on the MI355X engine through the reference's model API
// (basemodel.h / model_utils.h / llama.cpp:149-162,362-457): a synthetic-weight
// Llama (or the reference's .bin weights), its tokenizer file, MakeInput ->
// Response (streamed pieces) -> MakeHistory per round, until "exit".
// The reference's own user_entry.cpp compiles unchanged against include/llmi/model.h
// apart from its two src/ includes (tests/test_dropin_api.py builds it that way).
//
//   g++ -std=c++17 -I include examples/user_entry.cpp -L llm-inference_amd/lib -lllmi
//       -Wl,-rpath,$PWD/llm-inference_amd/lib -o user_entry
//   ./user_entry tests/golden/llama2-7b-tokenizer.bin [weight_dir/]
#include <cstdio>
#include <iostream>
#include <string>

#include "llmi/model.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s tokenizer.bin [weight_path_prefix]\n", argv[0]);
        return 2;
    }
    const std::string tokenizer_path = argv[1];
    try {
        std::unique_ptr<BaseModel> llm_model = argc > 2 ? llm::CreateRealLLMModel<float>(argv[2], tokenizer_path)
                                                        : llm::CreateDummyLLMModel<float>(tokenizer_path);
        const std::string name = llm_model->model_name;
        std::string history;
        for (int round = 0;; ++round) {
            std::printf("please input the question: ");
            std::fflush(stdout);
            std::string input;
            if (!std::getline(std::cin, input) || input == "exit") break;
            const std::string answer =
                llm_model->Response(llm_model->MakeInput(history, round, input), [&name](int index, const char* piece) {
                    if (index == 0) std::printf("%s:%s", name.c_str(), piece);
                    else if (index > 0) std::printf("%s", piece);
                    else std::printf("\n");
                    std::fflush(stdout);
                });
            history = llm_model->MakeHistory(history, round, input, answer);
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
