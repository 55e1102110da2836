// libsn_core — C ABI over the sparknet_amd engine, the counterpart of SparkNet's
// libccaffe (libccaffe/ccaffe.h, libccaffe/ccaffe.cpp:22-296) for non-Python callers
// (C/C++, or the JVM through JNA as in CaffeLibrary.java:8-76).
//
// Every function returns 0 on success and non-zero on failure (sn_last_error() then
// describes the failure), except where a count / pointer is returned.  Handles are
// thread-compatible: calls may come from any thread, one call at a time per handle.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// java_callback_t (CaffeLibrary.java:12-14): fill `buf` (batch x shape[1..] floats,
// logical NCHW) for the next minibatch.
typedef void (*sn_data_callback_t)(float* buf, int batch, int ndims, const int* shape, void* user);

const char* sn_last_error(void);

void* sn_create_state(void);
void sn_destroy_state(void* state);
int sn_set_device(void* state, int device);  // -1 = CPU reference path
int sn_load_solver_from_protobuf(void* state, const char* bytes, int len);  // serialized SolverParameter
int sn_load_net_from_protobuf(void* state, const char* bytes, int len);     // serialized NetParameter (TEST)
int sn_set_train_data_callback(void* state, int layer_index, sn_data_callback_t cb, void* user);
int sn_set_test_data_callback(void* state, int layer_index, sn_data_callback_t cb, void* user);

int sn_forward(void* state, float* loss);
int sn_backward(void* state);
// On a GPU state the iterations run in a native C++ loop over a captured hipGraph of one
// training iteration (the first call captures it, running 3 iterations through Python);
// SN_NATIVE_STEP=0 keeps every iteration on the Python engine.
int sn_solver_step(void* state, int iters);
long long sn_native_iterations(void* state);  // iterations run by the native loop so far
long long sn_python_entries(void);  // interpreter entries so far (0 growth: the verbs ran natively)
int sn_solver_test(void* state, int iters);  // returns the number of scores (>= 0) or -1
float sn_get_test_score(void* state, int index);

long long sn_num_params(void* state);  // flat fp32 parameter count (incl. alignment padding)
int sn_get_weights(void* state, float* out, long long n);
int sn_set_weights(void* state, const float* in, long long n);
void* sn_weights_device_ptr(void* state);  // flat fp32 master buffer (device memory on GPU)

int sn_save_weights_to_file(void* state, const char* path);  // .caffemodel
int sn_load_weights_from_file(void* state, const char* path);
int sn_restore_solver_from_file(void* state, const char* path);  // .solverstate

int sn_num_layers(void* state);
int sn_layer_name(void* state, int index, char* buf, int buflen);

int sn_parse_net_prototxt(const char* path, char** out, int* len);     // -> serialized bytes
int sn_parse_solver_prototxt(const char* path, char** out, int* len);  // (free with sn_free)
void sn_free(void* p);

// -- process-level helpers (ccaffe.cpp:33-49, 245-259) ---------------------------------------
int sn_init_logging(const char* log_filename, int verbosity);  // verbosity: 0 INFO .. 3 FATAL
int sn_set_basepath(const char* path);                          // chdir, like set_basepath
int sn_get_int_size(void);
int sn_get_dtype_size(void);  // size of the host exchange type (fp32)
typedef void (*sn_error_callback_t)(const char* message);
void sn_set_global_error_callback(sn_error_callback_t cb);  // called with every error message
int sn_set_mode_cpu(void* state);
int sn_set_mode_gpu(void* state);

// -- Datum databases (create_db / write_to_db / commit_db_txn / close_db, ccaffe.cpp:51-81)
int sn_create_db(void* state, const char* db_name, const char* db_type);  // "leveldb" | "lmdb" | "sndb"
int sn_write_to_db(void* state, const char* image, int label, int channels, int height, int width,
                   const char* key);
int sn_commit_db_txn(void* state);
int sn_close_db(void* state);
int sn_save_mean_image(const float* mean, int channels, int height, int width, const char* filename);

// -- blob access (num_layer_weights / get_*_blob / get_data / get_num_axes ..., ccaffe.cpp:142-195)
// Blobs are addressed as (layer, index): layer >= 0 selects parameter blob `index` of that
// layer, layer == -1 selects activation blob `index` of the net.  Device-resident
// blobs are exchanged by copy in logical (Caffe) layout as fp32.
int sn_num_layer_weights(void* state, int layer);
int sn_num_data_blobs(void* state);
int sn_data_blob_name(void* state, int index, char* buf, int buflen);
int sn_num_output_blobs(void* state);
int sn_num_test_scores(void* state);
int sn_blob_num_axes(void* state, int layer, int index);
int sn_blob_axis_shape(void* state, int layer, int index, int axis);
int sn_blob_get(void* state, int layer, int index, int diff, float* out, long long n);
int sn_blob_set(void* state, int layer, int index, int diff, const float* in, long long n);

#ifdef __cplusplus
}
#endif
