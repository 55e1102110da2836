/* C host program driving the engine through libsn_core (the libccaffe verbs SparkNet's
 * CaffeNet wrapper used: src/main/scala/libs/Net.scala:67-251).  Trains a small net on
 * callback-fed data, tests, round-trips the flat weights and a .caffemodel.
 * usage: core_demo <solver.prototxt> <out.caffemodel> [device]   (prints OK on success) */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "sn_core.h"

static int calls = 0;

static void data_cb(float* buf, int batch, int ndims, const int* shape, void* user) {
  long n = 1;
  for (int i = 0; i < ndims; ++i) n *= shape[i];
  for (long i = 0; i < n; ++i) buf[i] = (float)sin(0.37 * (double)(i + 13 * calls));
  (void)batch;
  (void)user;
  ++calls;
}

static void label_cb(float* buf, int batch, int ndims, const int* shape, void* user) {
  for (int i = 0; i < batch; ++i) buf[i] = (float)(i % 3);
  (void)ndims;
  (void)shape;
  (void)user;
}

#define CHECK(x)                                                     \
  do {                                                               \
    if (x) {                                                         \
      fprintf(stderr, "FAILED %s: %s\n", #x, sn_last_error());      \
      return 1;                                                      \
    }                                                                \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  char* sp = NULL;
  int splen = 0;
  CHECK(sn_parse_solver_prototxt(argv[1], &sp, &splen));
  void* st = sn_create_state();
  if (!st) {
    fprintf(stderr, "create: %s\n", sn_last_error());
    return 1;
  }
  CHECK(sn_set_device(st, argc > 3 ? atoi(argv[3]) : -1));
  CHECK(sn_load_solver_from_protobuf(st, sp, splen));
  sn_free(sp);
  CHECK(sn_set_train_data_callback(st, 0, data_cb, NULL));
  CHECK(sn_set_train_data_callback(st, 1, label_cb, NULL));
  CHECK(sn_solver_step(st, 5));
  CHECK(sn_load_net_from_protobuf(st, "\xff\xff\xff", 3) == 0); /* garbage bytes must fail cleanly */
  int nl = sn_num_layers(st);
  char name[64];
  CHECK(sn_layer_name(st, 2, name, sizeof name));
  float loss = 0.f;
  CHECK(sn_forward(st, &loss));
  CHECK(sn_backward(st));
  long long n = sn_num_params(st);
  float* w = (float*)malloc(sizeof(float) * n);
  float* w2 = (float*)malloc(sizeof(float) * n);
  CHECK(sn_get_weights(st, w, n));
  for (long long i = 0; i < n; ++i) w[i] *= 0.5f;
  CHECK(sn_set_weights(st, w, n));
  CHECK(sn_get_weights(st, w2, n));
  for (long long i = 0; i < n; ++i)
    if (w2[i] != w[i]) {
      fprintf(stderr, "weight round trip mismatch at %lld\n", i);
      return 1;
    }
  CHECK(sn_save_weights_to_file(st, argv[2]));
  for (long long i = 0; i < n; ++i) w[i] = 0.f;
  CHECK(sn_set_weights(st, w, n));
  CHECK(sn_load_weights_from_file(st, argv[2]));
  CHECK(sn_get_weights(st, w, n));
  for (long long i = 0; i < n; ++i)
    if (w[i] != w2[i]) {
      fprintf(stderr, "caffemodel round trip mismatch at %lld\n", i);
      return 1;
    }
  printf("layers=%d layer2=%s params=%lld loss=%.4f callbacks=%d\n", nl, name, n, loss, calls);
  sn_destroy_state(st);
  free(w);
  free(w2);
  printf("OK\n");
  return isfinite(loss) ? 0 : 1;
}
