/* C-API inference demo (reference paddle/legacy/capi/examples/model_inference/dense):
 *   capi_demo MERGED_MODEL PROGRAM PARAM_DIR INPUT.bin BATCH DIM OUTPUT.bin
 * runs one dense batch through a merged-model machine, a program + parameter-dir
 * machine and a shared-parameter clone, checks the three agree, writes the output. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../paddle_capi.h"

#define CHECK(x)                                                                      \
  do {                                                                                \
    paddle_error e_ = (x);                                                            \
    if (e_ != kPD_NO_ERROR) {                                                         \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, paddle_error_string(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

static void* read_file(const char* path, long* n) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(1); }
  fseek(f, 0, SEEK_END);
  *n = ftell(f);
  fseek(f, 0, SEEK_SET);
  void* b = malloc((size_t)*n);
  if (fread(b, 1, (size_t)*n, f) != (size_t)*n) { perror("read"); exit(1); }
  fclose(f);
  return b;
}

static float* run(paddle_gradient_machine m, paddle_matrix in, uint64_t* h, uint64_t* w) {
  paddle_arguments ins = paddle_arguments_create_none(), outs = paddle_arguments_create_none();
  CHECK(paddle_arguments_resize(ins, 1));
  CHECK(paddle_arguments_set_value(ins, 0, in));
  CHECK(paddle_gradient_machine_forward(m, ins, outs, false));
  uint64_t n = 0;
  CHECK(paddle_arguments_get_size(outs, &n));
  if (n < 1) { fprintf(stderr, "no output\n"); exit(1); }
  paddle_matrix prob = paddle_matrix_create_none();
  CHECK(paddle_arguments_get_value(outs, 0, prob));
  CHECK(paddle_matrix_get_shape(prob, h, w));
  float* out = malloc(sizeof(float) * (*h) * (*w));
  CHECK(paddle_matrix_get_value(prob, out));
  paddle_real* row = NULL;
  CHECK(paddle_matrix_get_row(prob, *h - 1, &row));
  if (row[0] != out[(*h - 1) * (*w)]) { fprintf(stderr, "get_row mismatch\n"); exit(1); }
  CHECK(paddle_matrix_destroy(prob));
  CHECK(paddle_arguments_destroy(ins));
  CHECK(paddle_arguments_destroy(outs));
  return out;
}

int main(int argc, char** argv) {
  if (argc != 8) { fprintf(stderr, "usage: %s merged program param_dir in.bin batch dim out.bin\n", argv[0]); return 2; }
  char* flags[] = {"--use_gpu=false"};
  CHECK(paddle_init(1, flags));
  long nm = 0, np = 0, ni = 0;
  void* merged = read_file(argv[1], &nm);
  void* prog = read_file(argv[2], &np);
  float* x = read_file(argv[4], &ni);
  const uint64_t batch = (uint64_t)atoi(argv[5]), dim = (uint64_t)atoi(argv[6]);
  if ((uint64_t)ni != batch * dim * 4) { fprintf(stderr, "input size\n"); return 1; }

  paddle_gradient_machine m1 = NULL, m2 = NULL, m3 = NULL;
  CHECK(paddle_gradient_machine_create_for_inference_with_parameters(&m1, merged, (uint64_t)nm));
  CHECK(paddle_gradient_machine_create_for_inference(&m2, prog, (int)np));
  CHECK(paddle_gradient_machine_load_parameter_from_disk(m2, argv[3]));
  CHECK(paddle_gradient_machine_create_shared_param(m1, prog, (int)np, &m3));
  if (paddle_gradient_machine_forward(m1, NULL, NULL, false) != kPD_NULLPTR) return 1;

  paddle_matrix in = paddle_matrix_create(batch, dim, false);
  CHECK(paddle_matrix_set_value(in, x));
  CHECK(paddle_matrix_set_row(in, 0, x));  /* row API on the same data */
  uint64_t h1, w1, h2, w2, h3, w3;
  float* o1 = run(m1, in, &h1, &w1);
  float* o2 = run(m2, in, &h2, &w2);
  float* o3 = run(m3, in, &h3, &w3);
  if (h1 != h2 || w1 != w2 || h1 != h3 || w1 != w3 || memcmp(o1, o2, h1 * w1 * 4) || memcmp(o1, o3, h1 * w1 * 4)) {
    fprintf(stderr, "machines disagree\n");
    return 1;
  }
  printf("machines_agree %llu x %llu\n", (unsigned long long)h1, (unsigned long long)w1);

  /* ivector + sequence-position bookkeeping */
  int ids[4] = {3, 1, 4, 1}, pos[3] = {0, 1, 4};
  paddle_ivector iv = paddle_ivector_create(ids, 4, true, false), sp = paddle_ivector_create(pos, 3, true, false);
  paddle_arguments a = paddle_arguments_create_none();
  CHECK(paddle_arguments_resize(a, 2));
  CHECK(paddle_arguments_set_ids(a, 1, iv));
  CHECK(paddle_arguments_set_sequence_start_pos(a, 1, 0, sp));
  paddle_ivector back = paddle_ivector_create_none();
  CHECK(paddle_arguments_get_sequence_start_pos(a, 1, 0, back));
  uint64_t bn = 0;
  int* bb = NULL;
  CHECK(paddle_ivector_get_size(back, &bn));
  CHECK(paddle_ivector_get(back, &bb));
  if (bn != 3 || bb[2] != 4) { fprintf(stderr, "seq pos\n"); return 1; }
  if (paddle_arguments_set_value(a, 5, in) != kPD_OUT_OF_RANGE) return 1;
  CHECK(paddle_ivector_destroy(iv));
  CHECK(paddle_ivector_destroy(sp));
  CHECK(paddle_ivector_destroy(back));
  CHECK(paddle_arguments_destroy(a));

  FILE* f = fopen(argv[7], "wb");
  fwrite(o1, 4, h1 * w1, f);
  fclose(f);
  CHECK(paddle_matrix_destroy(in));
  CHECK(paddle_gradient_machine_destroy(m3));
  CHECK(paddle_gradient_machine_destroy(m1));
  CHECK(paddle_gradient_machine_destroy(m2));
  free(o1); free(o2); free(o3); free(merged); free(prog); free(x);
  return 0;
}
