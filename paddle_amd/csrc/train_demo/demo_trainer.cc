// C++ training driver on the native executor (reference
// paddle/fluid/train/demo/demo_trainer.cc): load the serialized startup / main
// ProgramDescs, initialise the parameters, own the input tensors, run the training
// program step by step and report the loss and a per-op time profile.  Links
// libpaddle_amd_native.so only -- no Python interpreter.
//
//   demo_trainer <model_dir> [steps] [params_dir] [device]
//
// params_dir (optional, "-" for none): LoDTensor files overriding the startup
// initialisation (used by the tests to start from the Python executor's weights).
// device >= 0 runs the device kernels on that HIP device.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "framework.h"

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <model_dir> [steps] [params_dir] [device]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int steps = argc > 2 ? atoi(argv[2]) : 10;
  const std::string params = argc > 3 ? argv[3] : "-";
  const int device = argc > 4 ? atoi(argv[4]) : -1;
  try {
    const pa::ProgramDesc startup = pa::ProgramDesc::Load(dir + "/startup_program");
    const pa::ProgramDesc main_prog = pa::ProgramDesc::Load(dir + "/main_program");
    std::string loss_name;
    for (const pa::OpDesc& op : main_prog.Block(0).ops)
      if (op.type == "mean") {
        loss_name = op.Output("Out");
        break;
      }
    if (loss_name.empty()) {
      fprintf(stderr, "demo_trainer: no mean op (loss) in the main program\n");
      return 1;
    }
    // the demo network's ops are host kernels; `device` places the tensors in HBM
    // and runs whatever has a device kernel there
    pa::Executor exe(device);
    pa::Scope scope;
    exe.Run(startup, &scope, 0);
    if (params != "-") pa::load_persistables(main_prog, &scope, params, "", device, exe.context().stream);

    // inputs: x [2, 13] = 0..25, y [2, 1] = 0..1 (as the reference demo)
    pa::Tensor x, y;
    float* xp = x.alloc<float>({2, 13}, -1);
    for (int i = 0; i < 26; ++i) xp[i] = (float)i;
    float* yp = y.alloc<float>({2, 1}, -1);
    for (int i = 0; i < 2; ++i) yp[i] = (float)i;
    scope.Var("x")->tensor = device >= 0 ? x.to(device) : x;
    scope.Var("y")->tensor = device >= 0 ? y.to(device) : y;

    exe.profile = true;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < steps; ++i) {
      exe.Run(main_prog, &scope, 0);
      pa::Tensor loss = scope.Find(loss_name)->tensor;
      if (loss.device >= 0) loss = loss.to(-1, exe.context().stream);
      printf("step: %d loss: %.9g\n", i, loss.data<float>()[0]);
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("run_time_ms = %.3f\n", ms);
    // profiler summary sorted by total time (reference: DisableProfiler(kTotal, ...))
    std::vector<std::pair<std::string, std::pair<int64_t, double>>> rows(exe.op_time_ms.begin(), exe.op_time_ms.end());
    std::sort(rows.begin(), rows.end(), [](auto& a, auto& b) { return a.second.second > b.second.second; });
    printf("%-28s %8s %12s\n", "op", "calls", "total_ms");
    for (auto& r : rows) printf("%-28s %8lld %12.4f\n", r.first.c_str(), (long long)r.second.first, r.second.second);
    fflush(stdout);
  } catch (const std::exception& e) {
    fprintf(stderr, "demo_trainer: %s\n", e.what());
    return 1;
  }
  return 0;
}
