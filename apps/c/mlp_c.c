/* C-API example: the reference's mnist_mlp through flexmi_c.h (python/flexflow_c.h parity).
 *
 *   gcc apps/c/mlp_c.c -Icsrc/capi -Lflexmi -lflexmi_c -Wl,-rpath,$PWD/flexmi -o mlp_c
 *   ./mlp_c -b 32 -e 4 --device cpu
 *
 * Synthetic 4-class problem (label = argmax of the first 4 features); prints the final
 * accuracy and the reference's THROUGHPUT line. */
#include <stdio.h>
#include <stdlib.h>

#include "flexmi_c.h"

#define CHECK(x)                                                             \
  do {                                                                       \
    if (!(x)) {                                                              \
      fprintf(stderr, "%s failed: %s\n", #x, flexmi_last_error());           \
      return 1;                                                              \
    }                                                                        \
  } while (0)

int main(int argc, char** argv) {
  CHECK(flexmi_init(argc, argv) == 0);
  flexmi_config_t cfg = flexmi_config_create();
  CHECK(cfg);
  CHECK(flexmi_config_parse_args_default(cfg) == 0);
  const int B = flexmi_config_get_batch_size(cfg), E = flexmi_config_get_epochs(cfg);
  const int F = 16, C = 4, N = 512;

  flexmi_model_t m = flexmi_model_create(cfg);
  CHECK(m);
  int dims[2] = {B, F};
  flexmi_tensor_t x = flexmi_tensor_create(m, 2, dims, 40, 1, "input");
  CHECK(x);
  flexmi_initializer_t glorot = flexmi_glorot_uniform_initializer_create(7);
  flexmi_tensor_t t = flexmi_model_add_dense(m, x, 64, 11, 1, glorot, NULL, "dense1");
  CHECK(t);
  t = flexmi_model_add_dense(m, t, 64, 11, 1, NULL, NULL, "dense2");
  t = flexmi_model_add_dense(m, t, C, 10, 1, NULL, NULL, "dense3");
  t = flexmi_model_add_softmax(m, t, "softmax");
  CHECK(t);
  flexmi_optimizer_t sgd = flexmi_sgd_optimizer_create(m, 0.1, 0.0, 0, 0.0);
  int metrics[2] = {1001, 1004};
  CHECK(flexmi_model_compile(m, sgd, 51, metrics, 2) == 0);
  CHECK(flexmi_model_init_layers(m) == 0);

  float* xs = (float*)malloc(sizeof(float) * N * F);
  int* ys = (int*)malloc(sizeof(int) * N);
  srand(1);
  for (int i = 0; i < N; ++i) {
    int best = 0;
    for (int j = 0; j < F; ++j) {
      xs[i * F + j] = (float)rand() / RAND_MAX;
      if (j < C && xs[i * F + j] > xs[i * F + best]) best = j;
    }
    ys[i] = best;
  }
  flexmi_tensor_t label = flexmi_model_get_label_tensor(m);
  flexmi_dataloader_t dx = flexmi_single_dataloader_create(m, x, xs, N, 40);
  flexmi_dataloader_t dy = flexmi_single_dataloader_create(m, label, ys, N, 42);
  CHECK(dx && dy);

  double t0 = flexmi_get_current_time(cfg);
  for (int e = 0; e < E; ++e) {
    flexmi_dataloader_reset(dx);
    flexmi_dataloader_reset(dy);
    flexmi_model_reset_metrics(m);
    for (int it = 0; it < N / B; ++it) {
      CHECK(flexmi_dataloader_next_batch(dx, m) == 0);
      CHECK(flexmi_dataloader_next_batch(dy, m) == 0);
      CHECK(flexmi_model_forward(m) == 0);
      CHECK(flexmi_model_zero_gradients(m) == 0);
      CHECK(flexmi_model_backward(m) == 0);
      CHECK(flexmi_model_update(m) == 0);
    }
  }
  double t1 = flexmi_get_current_time(cfg);
  flexmi_perf_metrics_t pm = flexmi_model_get_perf_metrics(m);
  CHECK(pm);
  printf("accuracy %.2f loss %.4f\n", flexmi_perf_metrics_get_accuracy(pm), flexmi_perf_metrics_get_loss(pm));

  flexmi_parameter_t w = flexmi_op_get_parameter_by_id(flexmi_model_get_layer_by_id(m, 0), 0);
  CHECK(w);
  printf("dense1 kernel elements %d\n", flexmi_parameter_get_num_elements(w));
  printf("ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s\n", (t1 - t0) * 1e-6, (double)N * E / ((t1 - t0) * 1e-6));

  flexmi_parameter_destroy(w);
  flexmi_perf_metrics_destroy(pm);
  flexmi_dataloader_destroy(dx);
  flexmi_dataloader_destroy(dy);
  flexmi_tensor_destroy(label);
  flexmi_optimizer_destroy(sgd);
  flexmi_initializer_destroy(glorot);
  flexmi_model_destroy(m);
  flexmi_config_destroy(cfg);
  flexmi_finalize();
  free(xs);
  free(ys);
  return 0;
}
