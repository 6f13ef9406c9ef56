/* Trains a small AlexNet-shaped CNN through the native C API alone (libflexmi_native_c: C++ plan
 * compiler + engine, no Python in the process): image 3x20x20 -> conv 8 5x5/1 pad 2 relu -> max pool
 * 3x3/2 -> conv 16 3x3/1 pad 1 relu -> avg pool 2x2/2 pad 1 -> dense 32 relu -> dense 10 (logits),
 * softmax cross-entropy, SGD, data parallel over `world` rank processes (bucketed all-reduce through
 * the CPU engine's host communicator, or RCCL on the HIP engine).
 *
 *   native_cnn <cpu|hip> <out prefix> <steps> <world> <rendezvous dir> [options]
 *
 * options (comma-separated): bn -- the first convolution has no activation and feeds a batch norm with
 * a fused ReLU (statistics over each rank's samples); mom / nag -- SGD with momentum 0.9 (Nesterov);
 * adam -- Adam (alpha 0.01); wd -- weight decay 0.01; zero -- ZeRO-1 sharded optimizer state.
 *
 * <prefix>.init.bin (rank 0): int32 B, int32 steps, int32 nparams; per param int64 numel + float
 *   init[numel]; per step float x[B*3*20*20], int32 labels[B].
 * <prefix>.r<rank>.bin: int32 rank, int32 nparams; per param float final[numel]; per step double loss. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "flexmi_native_c.h"

#define B 16
#define CIN 3
#define HW 20
#define NCLS 10

#define CHECK(x)                                                                     \
  do {                                                                               \
    if ((x) < 0) {                                                                   \
      fprintf(stderr, "native_cnn r%d: %s failed: %s\n", rank, #x, fmn_last_error()); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

static uint32_t rng = 4242u;
static int g_bn = 0;
static const char* g_opts = "";
static float frand(void) {
  rng = rng * 1664525u + 1013904223u;
  return (float)(rng >> 8) / (float)(1u << 24);
}

static int run_rank(int device, const char* prefix, int steps, int rank, int world, const char* rdv) {
  fmn_model_t m = fmn_model_create(B, device, rank, world, rdv);
  if (!m) {
    fprintf(stderr, "native_cnn r%d: create: %s\n", rank, fmn_last_error());
    return 1;
  }
  int t;
  CHECK(t = fmn_model_input_image(m, CIN, HW, HW));
  if (g_bn) {
    CHECK(t = fmn_model_conv2d(m, t, 8, 5, 5, 1, 1, 2, 2, 10, 1));
    CHECK(t = fmn_model_batch_norm(m, t, 1));
  } else {
    CHECK(t = fmn_model_conv2d(m, t, 8, 5, 5, 1, 1, 2, 2, 11, 1));
  }
  CHECK(t = fmn_model_pool2d(m, t, 3, 3, 2, 2, 0, 0, 1));
  CHECK(t = fmn_model_conv2d(m, t, 16, 3, 3, 1, 1, 1, 1, 11, 1));
  CHECK(t = fmn_model_pool2d(m, t, 2, 2, 2, 2, 1, 1, 0));
  CHECK(t = fmn_model_dense(m, t, 32, 11, 1));
  CHECK(t = fmn_model_dense(m, t, NCLS, 10, 1));
  const int adam = strstr(g_opts, "adam") != NULL, nag = strstr(g_opts, "nag") != NULL;
  const float mom = (strstr(g_opts, "mom") != NULL || nag) ? 0.9f : 0.f, wd = strstr(g_opts, "wd") ? 0.01f : 0.f;
  if (adam || mom > 0.f || wd > 0.f) CHECK(fmn_model_set_optimizer(m, adam, mom, nag, wd, 0.9f, 0.999f, 1e-8f));
  if (strstr(g_opts, "zero")) CHECK(fmn_model_set_zero(m, 1));
  CHECK(fmn_model_compile(m, 51, adam ? 0.01f : 0.05f, 0.002));
  static char desc[8192];
  fmn_model_describe(m, desc, sizeof(desc));
  if (rank == 0) printf("%s", desc);
  const int np = fmn_model_num_params(m);
  float** init = (float**)calloc(np, sizeof(float*));
  int64_t* numel = (int64_t*)calloc(np, sizeof(int64_t));
  for (int i = 0; i < np; ++i) {
    numel[i] = fmn_model_param_numel(m, i);
    init[i] = (float*)malloc(numel[i] * sizeof(float));
    for (int64_t k = 0; k < numel[i]; ++k) init[i][k] = (frand() * 2.f - 1.f) * 0.25f;
    CHECK(fmn_model_set_param(m, i, init[i]));
  }
  const int F = CIN * HW * HW;
  float* x = (float*)malloc(sizeof(float) * B * F * steps);
  int32_t* lab = (int32_t*)malloc(sizeof(int32_t) * B * steps);
  for (int s = 0; s < steps; ++s) {
    for (int k = 0; k < B * F; ++k) x[(int64_t)s * B * F + k] = frand() * 2.f - 1.f;
    for (int b = 0; b < B; ++b) lab[s * B + b] = (int32_t)(frand() * NCLS) % NCLS;
  }
  if (rank == 0) {
    char path[1024];
    snprintf(path, sizeof(path), "%s.init.bin", prefix);
    FILE* f = fopen(path, "wb");
    if (!f) return 1;
    int32_t hdr[3] = {B, steps, np};
    fwrite(hdr, 4, 3, f);
    for (int i = 0; i < np; ++i) {
      fwrite(&numel[i], 8, 1, f);
      fwrite(init[i], 4, numel[i], f);
    }
    for (int s = 0; s < steps; ++s) {
      fwrite(x + (int64_t)s * B * F, 4, B * F, f);
      fwrite(lab + s * B, 4, B, f);
    }
    fclose(f);
  }
  double* losses = (double*)calloc(steps, sizeof(double));
  for (int s = 0; s < steps; ++s) {
    int64_t correct = 0;
    CHECK(fmn_model_train_step(m, x + (int64_t)s * B * F, lab + s * B, &losses[s], &correct));
  }
  char path[1024];
  snprintf(path, sizeof(path), "%s.r%d.bin", prefix, rank);
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  int32_t hdr[2] = {rank, np};
  fwrite(hdr, 4, 2, f);
  for (int i = 0; i < np; ++i) {
    float* w = (float*)malloc(numel[i] * sizeof(float));
    CHECK(fmn_model_get_param(m, i, w));
    fwrite(w, 4, numel[i], f);
    free(w);
  }
  fwrite(losses, 8, steps, f);
  fclose(f);
  fmn_model_destroy(m);
  if (rank == 0) printf("native_cnn ok: %d ranks, %d steps, loss %.5f -> %.5f\n", world, steps, losses[0], losses[steps - 1]);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: native_cnn <cpu|hip> <out prefix> <steps> <world> <rendezvous dir> [options]\n");
    return 2;
  }
  g_opts = argc > 6 ? argv[6] : "";
  g_bn = strstr(g_opts, "bn") != NULL;
  const int device = strcmp(argv[1], "hip") == 0 ? 1 : 0;
  const int steps = atoi(argv[3]), world = atoi(argv[4]);
  if (world < 1 || world > 16 || B % world) return 2;
  fflush(stdout);
  pid_t kids[16];
  for (int r = 1; r < world; ++r) {
    kids[r] = fork();
    if (kids[r] == 0) _exit(run_rank(device, argv[2], steps, r, world, argv[5]));
  }
  int rc = run_rank(device, argv[2], steps, 0, world, argv[5]);
  for (int r = 1; r < world; ++r) {
    int st = 0;
    waitpid(kids[r], &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
  }
  return rc;
}
