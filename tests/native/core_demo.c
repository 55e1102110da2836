/* C host program driving the engine through libsn_core (the libccaffe verbs SparkNet's
 * CaffeNet wrapper used: src/main/scala/libs/Net.scala:67-251).  Trains a small net on
 * callback-fed data, tests, round-trips the flat weights and a .caffemodel.
 * Also exercises the per-blob verbs and the Datum database verbs (CreateDB.scala).
 * usage: core_demo <solver.prototxt> <out.caffemodel> [device] [db_dir]   (prints OK) */
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
  printf("native=%lld\n", sn_native_iterations(st)); /* > 0 on a GPU: the C++ step loop ran */
  /* steady state: once each verb has run (its first call builds the native plan), step,
   * test, forward, get / set weights and the parameter blob verbs never enter the interpreter
   * on a GPU state */
  CHECK(sn_set_test_data_callback(st, 0, data_cb, NULL));
  CHECK(sn_set_test_data_callback(st, 1, label_cb, NULL));
  CHECK(sn_solver_test(st, 2) != 1);
  float warm = 0.f;
  CHECK(sn_forward(st, &warm));
  long long np = sn_num_params(st);
  float* ws = (float*)malloc(sizeof(float) * np);
  CHECK(sn_get_weights(st, ws, np));
  /* a layer parameter blob through the per-blob verbs (conv1 weights: the internal
   * [K][R][S][C] layout converted to Caffe's [K][C][R][S] natively) */
  long long pc = 1;
  for (int a = 0; a < sn_blob_num_axes(st, 2, 0); ++a) pc *= sn_blob_axis_shape(st, 2, 0, a);
  float* pb = (float*)malloc(sizeof(float) * pc);
  /* backward, activation blobs (data and gradient) and the name / count verbs: their first
   * calls build the native backward plan, blob table and metadata */
  CHECK(sn_backward(st));
  long long ac = 1;
  const int nb_axes = sn_blob_num_axes(st, -1, 2);
  for (int a = 0; a < nb_axes; ++a) ac *= sn_blob_axis_shape(st, -1, 2, a);
  float* ab = (float*)malloc(sizeof(float) * ac);
  CHECK(sn_blob_get(st, -1, 2, 0, ab, ac));
  CHECK(sn_blob_get(st, -1, 2, 1, ab, ac));
  char nm[64];
  CHECK(sn_num_layers(st) <= 0 || sn_layer_name(st, 2, nm, sizeof nm) || sn_num_data_blobs(st) <= 0);
  const long long py0 = sn_python_entries();
  CHECK(sn_solver_step(st, 3));
  CHECK(sn_blob_num_axes(st, 2, 0) != 4);
  CHECK(sn_blob_get(st, 2, 0, 0, pb, pc));
  CHECK(sn_blob_set(st, 2, 0, 0, pb, pc));
  CHECK(sn_blob_get(st, 2, 0, 1, pb, pc));
  CHECK(sn_solver_test(st, 2) != 1);
  const int nscores = sn_num_test_scores(st);
  const float score = sn_get_test_score(st, 0);
  CHECK(sn_get_weights(st, ws, np));
  CHECK(sn_set_weights(st, ws, np));
  CHECK(sn_forward(st, &warm));
  CHECK(sn_backward(st));
  CHECK(sn_blob_num_axes(st, -1, 2) != nb_axes);
  CHECK(sn_blob_get(st, -1, 2, 0, ab, ac));
  CHECK(sn_blob_get(st, -1, 2, 1, ab, ac));
  CHECK(sn_blob_set(st, -1, 2, 1, ab, ac));
  CHECK(sn_num_layers(st) <= 0 || sn_layer_name(st, 2, nm, sizeof nm) || sn_num_data_blobs(st) <= 0 ||
        sn_data_blob_name(st, 0, nm, sizeof nm) || sn_num_output_blobs(st) < 0 || sn_num_layer_weights(st, 2) != 2);
  const long long py = sn_python_entries() - py0;
  free(ws);
  free(pb);
  free(ab);
  printf("steady_py=%lld scores=%d score0=%.4f fwd=%.4f\n", py, nscores, score, warm);
  CHECK(!isfinite(score) || !isfinite(warm) || nscores != 1);
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
  /* per-blob access: parameter blob 0 of layer 2 and activation blob 0 */
  int nw = sn_num_layer_weights(st, 2);
  int axes = sn_blob_num_axes(st, 2, 0);
  long long cnt = 1;
  for (int a = 0; a < axes; ++a) cnt *= sn_blob_axis_shape(st, 2, 0, a);
  float* b = (float*)malloc(sizeof(float) * cnt);
  CHECK(sn_blob_get(st, 2, 0, 0, b, cnt));
  for (long long i = 0; i < cnt; ++i) b[i] = (float)i * 0.25f;
  CHECK(sn_blob_set(st, 2, 0, 0, b, cnt));
  for (long long i = 0; i < cnt; ++i) b[i] = -1.f;
  CHECK(sn_blob_get(st, 2, 0, 0, b, cnt));
  for (long long i = 0; i < cnt; ++i)
    if (b[i] != (float)i * 0.25f) {
      fprintf(stderr, "blob round trip mismatch at %lld\n", i);
      return 1;
    }
  char bname[64];
  CHECK(sn_data_blob_name(st, 0, bname, sizeof bname));
  printf("blobs=%d outputs=%d weights2=%d axes=%d count=%lld blob0=%s\n", sn_num_data_blobs(st),
         sn_num_output_blobs(st), nw, axes, cnt, bname);
  free(b);
  if (argc > 4) { /* CreateDB.makeDBFromPartition through the C verbs */
    unsigned char img[3 * 4 * 4];
    char key[16];
    CHECK(sn_create_db(st, argv[4], "lmdb"));
    for (int i = 0; i < 5; ++i) {
      for (int j = 0; j < 48; ++j) img[j] = (unsigned char)(i * 48 + j);
      snprintf(key, sizeof key, "%d", i);
      CHECK(sn_write_to_db(st, (const char*)img, i, 3, 4, 4, key));
      if (i == 2) CHECK(sn_commit_db_txn(st));
    }
    CHECK(sn_close_db(st));
    float mean[3] = {1.f, 2.f, 3.f};
    char mpath[512];
    snprintf(mpath, sizeof mpath, "%s.mean.binaryproto", argv[4]);
    CHECK(sn_save_mean_image(mean, 3, 1, 1, mpath));
  }
  printf("layers=%d layer2=%s params=%lld loss=%.4f callbacks=%d\n", nl, name, n, loss, calls);
  sn_destroy_state(st);
  free(w);
  free(w2);
  printf("OK\n");
  return isfinite(loss) ? 0 : 1;
}
