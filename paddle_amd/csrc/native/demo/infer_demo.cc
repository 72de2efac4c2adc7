// C++ inference demo on the public API (paddle_inference_api.h; reference
// inference/api/demo_ci/simple_on_word2vec.cc + api_impl_tester.cc): create a
// predictor from a saved model directory, run it on inputs read from raw files,
// then run `threads` clones concurrently and check they agree.
//
//   infer_demo <model_dir> <out_file> <threads> <use_gpu> <ir_optim> \
//              <in_file> <dtype:f|l> <d0,d1,...> [<in_file> <dtype> <dims> ...]
//
// Writes every output as raw bytes (concatenated, in fetch order) to out_file and
// prints one line per output: "output <i> <name> <shape...>".
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fstream>
#include <sstream>
#include <thread>
#include <vector>

#include "paddle_inference_api.h"

namespace {
std::vector<int> parse_dims(const char* s) {
  std::vector<int> d;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) d.push_back(atoi(tok.c_str()));
  return d;
}

bool read_file(const std::string& path, paddle::PaddleBuf* buf) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  buf->Resize(s.size());
  memcpy(buf->data(), s.data(), s.size());
  return true;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 9 || (argc - 6) % 3 != 0) {
    fprintf(stderr, "usage: %s model_dir out_file threads use_gpu ir_optim (in_file dtype dims)+\n", argv[0]);
    return 2;
  }
  paddle::AnalysisConfig cfg;
  cfg.model_dir = argv[1];
  const std::string out_file = argv[2];
  const int threads = atoi(argv[3]);
  cfg.use_gpu = atoi(argv[4]) != 0;
  cfg.device = 0;
  cfg.enable_ir_optim = atoi(argv[5]) != 0;

  std::vector<paddle::PaddleTensor> inputs;
  for (int a = 6; a + 2 < argc; a += 3) {
    paddle::PaddleTensor t;
    t.name = "input" + std::to_string(inputs.size());
    if (!read_file(argv[a], &t.data)) {
      fprintf(stderr, "cannot read %s\n", argv[a]);
      return 1;
    }
    t.dtype = argv[a + 1][0] == 'l' ? paddle::INT64 : paddle::FLOAT32;
    t.shape = parse_dims(argv[a + 2]);
    inputs.push_back(std::move(t));
  }

  auto predictor = paddle::CreatePaddlePredictor<paddle::AnalysisConfig, paddle::PaddleEngineKind::kAnalysis>(cfg);
  if (!predictor) {
    fprintf(stderr, "predictor creation failed: %s\n", paddle::LastError().c_str());
    return 1;
  }
  std::vector<paddle::PaddleTensor> outputs;
  if (!predictor->Run(inputs, &outputs)) return 1;

  std::ofstream f(out_file, std::ios::binary);
  for (size_t i = 0; i < outputs.size(); ++i) {
    printf("output %zu %s", i, outputs[i].name.c_str());
    for (int d : outputs[i].shape) printf(" %d", d);
    printf("\n");
    f.write(static_cast<const char*>(outputs[i].data.data()), (std::streamsize)outputs[i].data.length());
  }

  // clones share the parameters; each runs on its own thread
  std::vector<std::unique_ptr<paddle::PaddlePredictor>> clones;
  for (int t = 0; t < threads; ++t) clones.push_back(predictor->Clone());
  std::vector<int> ok(threads, 0);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      std::vector<paddle::PaddleTensor> out;
      for (int rep = 0; rep < 3; ++rep) {
        if (!clones[t]->Run(inputs, &out) || out.size() != outputs.size()) return;
        for (size_t i = 0; i < out.size(); ++i)
          if (out[i].data.length() != outputs[i].data.length() ||
              memcmp(out[i].data.data(), outputs[i].data.data(), out[i].data.length()) != 0)
            return;
      }
      ok[t] = 1;
    });
  for (auto& th : pool) th.join();
  int good = 0;
  for (int v : ok) good += v;
  printf("clones_agree %d/%d\n", good, threads);
  return good == threads ? 0 : 3;
}
