/* C inference API with the function set of the reference's legacy C-API
 * (paddle/legacy/capi: main.h, matrix.h, vector.h, arguments.h, gradient_machine.h),
 * served by the native executor (csrc/native) instead of the GradientMachine.
 *
 * Model inputs are Fluid inference models:
 *   - paddle_gradient_machine_create_for_inference(m, program, size): a serialised
 *     ProgramDesc (the `__model__` file of fluid.io.save_inference_model), then
 *     paddle_gradient_machine_load_parameter_from_disk(m, dir) for its parameters;
 *   - paddle_gradient_machine_create_for_inference_with_parameters(m, merged, size):
 *     a merged model (paddle_amd.utils.merge_model: "PAMERGE1", program, combined
 *     parameter stream) in one buffer.
 * forward() feeds input slot i to the program's i-th feed target (value matrices as
 * float32 [height, width]; ids as int64 [n, 1]; sequence start positions as level-1
 * LoD) and returns each fetch target as a value matrix [dim0, product of the rest].
 * Matrices, vectors and arguments share buffers the way the reference's do
 * (set_value / get_value alias, destroy releases one reference).
 */
#ifndef PADDLE_AMD_CAPI_H_
#define PADDLE_AMD_CAPI_H_

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PD_API __attribute__((visibility("default")))

typedef enum {
  kPD_NO_ERROR = 0,
  kPD_NULLPTR = 1,
  kPD_OUT_OF_RANGE = 2,
  kPD_PROTOBUF_ERROR = 3,
  kPD_NOT_SUPPORTED = 4,
  kPD_UNDEFINED_ERROR = -1,
} paddle_error;

typedef float paddle_real;
typedef void* paddle_matrix;
typedef void* paddle_ivector;
typedef void* paddle_arguments;
typedef void* paddle_gradient_machine;

PD_API const char* paddle_error_string(paddle_error err);
/* flags: --use_gpu=true|false (default false), --gpu_id=N */
PD_API paddle_error paddle_init(int argc, char** argv);
PD_API paddle_error paddle_init_thread();

PD_API paddle_matrix paddle_matrix_create(uint64_t height, uint64_t width, bool useGpu);
PD_API paddle_matrix paddle_matrix_create_none();
PD_API paddle_matrix paddle_matrix_create_sparse(uint64_t height, uint64_t width, uint64_t nnz, bool isBinary,
                                                 bool useGpu);
PD_API paddle_error paddle_matrix_destroy(paddle_matrix mat);
PD_API paddle_error paddle_matrix_set_row(paddle_matrix mat, uint64_t rowID, paddle_real* rowArray);
PD_API paddle_error paddle_matrix_set_value(paddle_matrix mat, paddle_real* value);
PD_API paddle_error paddle_matrix_get_row(paddle_matrix mat, uint64_t rowID, paddle_real** rawRowBuffer);
PD_API paddle_error paddle_matrix_get_value(paddle_matrix mat, paddle_real* result);
PD_API paddle_error paddle_matrix_get_shape(paddle_matrix mat, uint64_t* height, uint64_t* width);
PD_API paddle_error paddle_matrix_sparse_copy_from(paddle_matrix mat, int* rowArray, uint64_t rowSize, int* colArray,
                                                   uint64_t colSize, float* valueArray, uint64_t valueSize);

PD_API paddle_ivector paddle_ivector_create_none();
PD_API paddle_ivector paddle_ivector_create(int* array, uint64_t size, bool copy, bool useGPU);
PD_API paddle_error paddle_ivector_destroy(paddle_ivector ivec);
PD_API paddle_error paddle_ivector_get(paddle_ivector ivec, int** buffer);
PD_API paddle_error paddle_ivector_resize(paddle_ivector ivec, uint64_t size);
PD_API paddle_error paddle_ivector_get_size(paddle_ivector ivec, uint64_t* size);

PD_API paddle_arguments paddle_arguments_create_none();
PD_API paddle_error paddle_arguments_destroy(paddle_arguments args);
PD_API paddle_error paddle_arguments_get_size(paddle_arguments args, uint64_t* size);
PD_API paddle_error paddle_arguments_resize(paddle_arguments args, uint64_t size);
PD_API paddle_error paddle_arguments_set_value(paddle_arguments args, uint64_t ID, paddle_matrix mat);
PD_API paddle_error paddle_arguments_get_value(paddle_arguments args, uint64_t ID, paddle_matrix mat);
PD_API paddle_error paddle_arguments_get_prob(paddle_arguments args, uint64_t ID, paddle_matrix mat);
PD_API paddle_error paddle_arguments_get_ids(paddle_arguments args, uint64_t ID, paddle_ivector ids);
PD_API paddle_error paddle_arguments_set_ids(paddle_arguments args, uint64_t ID, paddle_ivector ids);
PD_API paddle_error paddle_arguments_set_frame_shape(paddle_arguments args, uint64_t ID, uint64_t frameHeight,
                                                     uint64_t frameWidth);
PD_API paddle_error paddle_arguments_set_sequence_start_pos(paddle_arguments args, uint64_t ID, uint32_t nestedLevel,
                                                            paddle_ivector seqPos);
PD_API paddle_error paddle_arguments_get_sequence_start_pos(paddle_arguments args, uint64_t ID, uint32_t nestedLevel,
                                                            paddle_ivector seqPos);

PD_API paddle_error paddle_gradient_machine_create_for_inference(paddle_gradient_machine* machine,
                                                                 void* modelConfigProtobuf, int size);
PD_API paddle_error paddle_gradient_machine_create_for_inference_with_parameters(paddle_gradient_machine* machine,
                                                                                 void* mergedModel, uint64_t size);
PD_API paddle_error paddle_gradient_machine_load_parameter_from_disk(paddle_gradient_machine machine,
                                                                     const char* path);
PD_API paddle_error paddle_gradient_machine_forward(paddle_gradient_machine machine, paddle_arguments inArgs,
                                                    paddle_arguments outArgs, bool isTrain);
PD_API paddle_error paddle_gradient_machine_create_shared_param(paddle_gradient_machine origin,
                                                                void* modelConfigProtobuf, int size,
                                                                paddle_gradient_machine* slave);
PD_API paddle_error paddle_gradient_machine_randomize_param(paddle_gradient_machine machine);
PD_API paddle_error paddle_gradient_machine_destroy(paddle_gradient_machine machine);
PD_API paddle_error paddle_gradient_machine_get_layer_output(paddle_gradient_machine machine, const char* layerName,
                                                             paddle_arguments args);
PD_API paddle_error paddle_gradient_machine_release_layer_output(paddle_gradient_machine machine);

#ifdef __cplusplus
}
#endif

#endif /* PADDLE_AMD_CAPI_H_ */
