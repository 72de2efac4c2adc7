// C++ training driver (reference paddle/fluid/train/demo/demo_trainer.cc).
//
// Loads serialized startup / main ProgramDescs, initialises the parameters, owns
// the input buffers and runs the training loop from C++.  The executor, the op
// kernels and the gfx950 kernel library are reached through the embedded
// interpreter (paddle_amd.train_demo.DemoTrainer): this framework's executor is
// Python over native kernels, so a C++ host embeds it instead of linking a C++
// executor.
//
//   demo_trainer <model_dir> [steps] [gpu]
#include <Python.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

[[noreturn]] void die(const char* what) {
  std::fprintf(stderr, "demo_trainer: %s\n", what);
  if (PyErr_Occurred()) PyErr_Print();
  std::exit(1);
}

PyObject* call(PyObject* obj, const char* method, PyObject* args) {
  PyObject* fn = PyObject_GetAttrString(obj, method);
  if (!fn) die(method);
  PyObject* r = PyObject_CallObject(fn, args);
  Py_DECREF(fn);
  Py_XDECREF(args);
  if (!r) die(method);
  return r;
}

void set_input(PyObject* trainer, const char* name, const std::vector<float>& buf, long rows, long cols) {
  PyObject* mem = PyMemoryView_FromMemory(reinterpret_cast<char*>(const_cast<float*>(buf.data())),
                                          static_cast<Py_ssize_t>(buf.size() * sizeof(float)), PyBUF_READ);
  PyObject* shape = Py_BuildValue("(ll)", rows, cols);
  PyObject* r = call(trainer, "set_input", Py_BuildValue("(sNN)", name, mem, shape));
  Py_DECREF(r);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <model_dir> [steps] [gpu]\n", argv[0]);
    return 2;
  }
  const std::string model_dir = argv[1];
  const int steps = argc > 2 ? std::atoi(argv[2]) : 10;
  const int use_gpu = argc > 3 ? std::atoi(argv[3]) : 0;

  Py_Initialize();
  PyObject* mod = PyImport_ImportModule("paddle_amd.train_demo");
  if (!mod) die("import paddle_amd.train_demo");
  PyObject* cls = PyObject_GetAttrString(mod, "DemoTrainer");
  if (!cls) die("DemoTrainer");
  PyObject* trainer = PyObject_CallFunction(cls, "si", model_dir.c_str(), use_gpu);
  if (!trainer) die("DemoTrainer(model_dir)");
  Py_DECREF(call(trainer, "run_startup", nullptr));

  // prepare data: x [2, 13] = 0..25, y [2, 1] = 0..1 (as the reference demo)
  std::vector<float> x(2 * 13), y(2);
  for (int i = 0; i < 2 * 13; ++i) x[i] = static_cast<float>(i);
  for (int i = 0; i < 2; ++i) y[i] = static_cast<float>(i);
  set_input(trainer, "x", x, 2, 13);
  set_input(trainer, "y", y, 2, 1);

  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < steps; ++i) {
    PyObject* loss = call(trainer, "step", nullptr);
    std::printf("step: %d loss: %.6f\n", i, PyFloat_AsDouble(loss));
    Py_DECREF(loss);
  }
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::printf("run_time_ms = %.3f\n", ms);
  std::fflush(stdout);
  Py_DECREF(trainer);
  Py_DECREF(cls);
  Py_DECREF(mod);
  return Py_FinalizeEx() < 0 ? 1 : 0;
}
