/* Trains an MLP through the native C API alone (libflexmi_native_c: C++ plan compiler + engine,
 * no Python anywhere in the process) and records everything a replay needs.
 *
 *   native_mlp <cpu|hip> <out.bin> [steps] [loss 51|52|54] [rank world rendezvous]
 *
 * out.bin (little-endian): int32 nparams, per param int64 numel + float init[numel]; int32 B,
 * int32 F, int32 C, int32 steps, int32 loss; per step float x[B*F] + labels (int32[B] or
 * float[B*C]); per step double loss; per param float final[numel].  The planned step (fused
 * epilogues, flat buffer, buckets) goes to stdout. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flexmi_native_c.h"

#define CHECK(x)                                                              \
  do {                                                                        \
    if ((x) < 0) {                                                            \
      fprintf(stderr, "native_mlp: %s failed: %s\n", #x, fmn_last_error());   \
      return 1;                                                               \
    }                                                                         \
  } while (0)

static uint32_t rng = 12345u;
static float frand(void) {
  rng = rng * 1664525u + 1013904223u;
  return (float)(rng >> 8) / (float)(1u << 24);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: native_mlp <cpu|hip> <out.bin> [steps] [loss] [rank world rendezvous]\n");
    return 2;
  }
  const int device = strcmp(argv[1], "hip") == 0 ? 1 : 0;
  const int steps = argc > 3 ? atoi(argv[3]) : 5;
  const int loss = argc > 4 ? atoi(argv[4]) : 51;
  const int rank = argc > 7 ? atoi(argv[5]) : 0, world = argc > 7 ? atoi(argv[6]) : 1;
  const char* rdv = argc > 7 ? argv[7] : "";
  const int B = 64, F = 24;
  const int C = loss == 51 ? 10 : (loss == 54 ? 1 : 3);
  fmn_model_t m = fmn_model_create(B, device, rank, world, rdv);
  if (!m) {
    fprintf(stderr, "native_mlp: create: %s\n", fmn_last_error());
    return 1;
  }
  int x = fmn_model_input(m, F);
  CHECK(x);
  int h = fmn_model_dense(m, x, 64, 11, 1);
  CHECK(h);
  h = fmn_model_dense(m, h, 32, 13, 1);
  CHECK(h);
  h = fmn_model_dense(m, h, 16, 11, 1);
  CHECK(h);
  h = fmn_model_dense(m, h, C, loss == 54 ? 12 : 10, 1);
  CHECK(h);
  CHECK(fmn_model_compile(m, loss, 0.05f, 0.004));
  CHECK(fmn_model_init_weights(m, 7));
  char desc[4096];
  CHECK(fmn_model_describe(m, desc, sizeof(desc)));
  printf("%s", desc);
  FILE* f = fopen(argv[2], "wb");
  if (!f) return 1;
  const int np = fmn_model_num_params(m);
  fwrite(&np, 4, 1, f);
  for (int i = 0; i < np; ++i) {
    const int64_t n = fmn_model_param_numel(m, i);
    float* w = (float*)malloc(n * 4);
    CHECK(fmn_model_get_param(m, i, w));
    fwrite(&n, 8, 1, f);
    fwrite(w, 4, n, f);
    free(w);
  }
  const int hdr[5] = {B, F, C, steps, loss};
  fwrite(hdr, 4, 5, f);
  float* xs = (float*)malloc((size_t)B * F * 4);
  float* lf = (float*)malloc((size_t)B * C * 4);
  int* li = (int*)malloc((size_t)B * 4);
  double* losses = (double*)malloc(steps * sizeof(double));
  for (int s = 0; s < steps; ++s) {
    for (int i = 0; i < B * F; ++i) xs[i] = frand() * 2.f - 1.f;
    for (int i = 0; i < B; ++i) li[i] = (int)(frand() * C) % C;
    for (int i = 0; i < B * C; ++i) lf[i] = loss == 54 ? (frand() < 0.5f ? 0.f : 1.f) : frand();
    fwrite(xs, 4, (size_t)B * F, f);
    if (loss == 51) fwrite(li, 4, B, f);
    else fwrite(lf, 4, (size_t)B * C, f);
    int64_t correct = 0;
    CHECK(fmn_model_train_step(m, xs, loss == 51 ? (const void*)li : (const void*)lf, &losses[s], &correct));
    printf("step %d loss %.6f correct %lld\n", s, losses[s], (long long)correct);
  }
  fwrite(losses, 8, steps, f);
  for (int i = 0; i < np; ++i) {
    const int64_t n = fmn_model_param_numel(m, i);
    float* w = (float*)malloc(n * 4);
    CHECK(fmn_model_get_param(m, i, w));
    fwrite(w, 4, n, f);
    free(w);
  }
  fclose(f);
  fmn_model_destroy(m);
  printf("native_mlp ok\n");
  return 0;
}
