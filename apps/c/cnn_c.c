/* C-API example: a small CNN built from functional ("no in/out") layers and fed by the 4-D input +
 * label loaders -- the reference's cffi flow (python/flexflow_c.h: model_add_*_no_inout,
 * op_init_inout, dataloader_4d_create_v2, tensor_attach_raw_ptr / inline_map).
 *
 *   gcc apps/c/cnn_c.c -Icsrc/capi -Lflexmi -lflexmi_c -Wl,-rpath,$PWD/flexmi -o cnn_c
 *   ./cnn_c -b 16 -e 2 --device cpu
 *
 * Full dataset: host arrays attached zero-copy to host tensors (v2 loader); a second loader uses
 * the random-data mode (dataloader_4d_create).  Prints loss / accuracy and a THROUGHPUT line. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
  CHECK(cfg && flexmi_config_parse_args_default(cfg) == 0);
  const int B = flexmi_config_get_batch_size(cfg), E = flexmi_config_get_epochs(cfg);
  const int C = 3, H = 12, W = 12, K = 4, N = 8 * B;

  flexmi_model_t m = flexmi_model_create(cfg);
  int xd[4] = {B, C, H, W}, yd[2] = {B, 1};
  flexmi_tensor_t x = flexmi_tensor_create(m, 4, xd, 40, 1, "input");
  CHECK(x);
  /* functional layers, connected afterwards */
  flexmi_initializer_t none = flexmi_initializer_create_null();
  flexmi_op_t conv = flexmi_model_add_conv2d_no_inout(m, C, 8, 3, 3, 1, 1, 1, 1, 11, 1, none, none);
  flexmi_op_t pool = flexmi_model_add_pool2d_no_inout(m, 2, 2, 2, 2, 0, 0, 30, 10);
  flexmi_op_t flat = flexmi_model_add_flat_no_inout(m);
  flexmi_op_t fc = flexmi_model_add_dense_no_inout(m, 8 * 6 * 6, K, 10, 1, none, none);
  CHECK(conv && pool && flat && fc);
  flexmi_tensor_t t = flexmi_op_init_inout(conv, m, x);
  t = flexmi_op_init_inout(pool, m, t);
  t = flexmi_op_init_inout(flat, m, t);
  t = flexmi_op_init_inout(fc, m, t);
  CHECK(t);
  t = flexmi_model_add_softmax(m, t, "softmax");
  flexmi_optimizer_t sgd = flexmi_sgd_optimizer_create(m, 0.05, 0.0, 0, 0.0);
  CHECK(flexmi_model_set_sgd_optimizer(m, sgd) == 0);
  int metrics[1] = {1001};
  CHECK(flexmi_model_compile(m, sgd, 51, metrics, 1) == 0);
  flexmi_tensor_t label = flexmi_model_get_label_tensor(m);
  CHECK(label);
  CHECK(flexmi_model_init_layers(m) == 0);
  CHECK(flexmi_op_init(conv, m) == 0);

  /* full dataset in host memory, attached zero-copy: label = channel-0 mean > 0.5 -> class 1, else 0 */
  float* xs = (float*)malloc(sizeof(float) * N * C * H * W);
  int32_t* ys = (int32_t*)malloc(sizeof(int32_t) * N);
  srand(3);
  for (int n = 0; n < N; ++n) {
    double s = 0;
    for (int i = 0; i < C * H * W; ++i) {
      float v = (float)rand() / RAND_MAX;
      xs[n * C * H * W + i] = v;
      if (i < H * W) s += v;
    }
    ys[n] = s / (H * W) > 0.5 ? 1 : 0;
  }
  int fxd[4] = {N, C, H, W}, fyd[2] = {N, 1};
  flexmi_tensor_t fx = flexmi_tensor_create(m, 4, fxd, 40, 0, "full_input");
  flexmi_tensor_t fy = flexmi_tensor_create(m, 2, fyd, 42, 0, "full_label");
  CHECK(fx && fy);
  CHECK(flexmi_tensor_attach_raw_ptr(fx, cfg, xs, 0) == 0 && flexmi_tensor_attach_raw_ptr(fy, cfg, ys, 0) == 0);
  CHECK(flexmi_tensor_is_mapped(fx) == 1);
  flexmi_dataloader_4d_t dl = flexmi_dataloader_4d_create_v2(m, x, label, fx, fy, N);
  CHECK(dl && flexmi_dataloader_4d_get_num_samples(dl) == N);

  double t0 = flexmi_get_current_time(cfg);
  for (int e = 0; e < E; ++e) {
    flexmi_dataloader_4d_reset(dl);
    flexmi_model_reset_metrics(m);
    for (int it = 0; it < N / B; ++it) {
      CHECK(flexmi_dataloader_4d_next_batch(dl, m) == 0);
      CHECK(flexmi_model_forward(m) == 0);
      CHECK(flexmi_model_zero_gradients(m) == 0);
      CHECK(flexmi_model_backward(m) == 0);
      CHECK(flexmi_model_update(m) == 0);
    }
  }
  double t1 = flexmi_get_current_time(cfg);
  flexmi_perf_metrics_t pm = flexmi_model_get_perf_metrics(m);
  printf("loss %.4f accuracy %.2f\n", flexmi_perf_metrics_get_loss(pm), flexmi_per_metrics_get_accuracy(pm));
  flexmi_per_metrics_destroy(pm);

  /* host view of the current input batch through inline_map / raw pointer */
  CHECK(flexmi_tensor_inline_map(x, cfg) == 0);
  float* px = flexmi_tensor_get_raw_ptr_float(x, cfg);
  CHECK(px != NULL);
  printf("mapped input[0] %.4f is_mapped %d\n", px[0], flexmi_tensor_is_mapped(x));
  CHECK(flexmi_tensor_inline_unmap(x, cfg) == 0);
  CHECK(flexmi_op_forward(conv, m) == 0);

  /* random-data mode of the 4-D loader (no --dataset) */
  flexmi_net_config_t nc = flexmi_net_config_create();
  flexmi_dataloader_4d_t rnd = flexmi_dataloader_4d_create(m, nc, x, label);
  CHECK(rnd && flexmi_dataloader_4d_get_num_samples(rnd) == 4 * B);
  CHECK(flexmi_dataloader_4d_next_batch(rnd, m) == 0);
  flexmi_dataloader_4d_destroy(rnd);
  flexmi_net_config_destroy(nc);

  printf("ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s\n", (t1 - t0) * 1e-6, (double)N * E / ((t1 - t0) * 1e-6));
  flexmi_tensor_detach_raw_ptr(fx, cfg);
  flexmi_tensor_detach_raw_ptr(fy, cfg);
  flexmi_dataloader_4d_destroy(dl);
  flexmi_sgd_optimizer_destroy(sgd);
  flexmi_initializer_destroy(none);
  flexmi_model_destroy(m);
  flexmi_config_destroy(cfg);
  free(xs);
  free(ys);
  flexmi_finalize();
  return 0;
}
