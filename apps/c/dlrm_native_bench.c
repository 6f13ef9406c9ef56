/* The DLRM MLPerf-like configuration (BASELINE.json: 13 dense features, 26 Criteo-Terabyte tables of
 * 128 columns, bottom MLP 13-512-256-128, dot interaction, top MLP 479-1024-1024-512-256-1 with a
 * sigmoid, binary cross-entropy, SGD) trained on the NATIVE engine alone: libflexmi_native_c's C++ plan
 * compiler and its HIP engine (flexmi's gfx950 kernels), no Python in the process.  Times `steps`
 * training steps after `warmup` and prints one JSON line.
 *
 *   gcc apps/c/dlrm_native_bench.c -Icsrc/capi -Lflexmi -lflexmi_native_c -Wl,-rpath,$PWD/flexmi -o dlrm_native_bench
 *   ./dlrm_native_bench <cpu|hip> [steps 20] [warmup 5] [batch 8192] [small]
 *
 * Each step feeds the same synthetic batch from host memory (train_step_sparse copies it in, as a
 * data loader would).  The dense layers start from small random weights; the tables stay
 * zero-initialised (host-side initialisation of the 96 GB of MLPerf tables would take minutes; the
 * kernels' work does not depend on the values).  `small` caps every table at 100 000 rows (a
 * CPU-engine smoke run).  Reference: examples/cpp/DLRM/dlrm.cc (model), run_summit/mlperf scripts. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "flexmi_native_c.h"

#define NT 26
#define D 128
#define FEAT 13
#define FEAT_PAD 16   /* the dense input zero-padded to 16 features (as the executor pads it): 16-B rows */
static const int64_t MLPERF_ROWS[NT] = {39884406, 39043,    17289,    7420,     20263,   3,     7120,  1543,   63,
                                        38532951, 2953546,  403346,   10,       2208,    11938, 155,   4,      976,
                                        14,       39979771, 25641295, 39664984, 585935,  12972, 108,   36};

#define CHECK(x)                                                          \
  do {                                                                    \
    if ((x) < 0) {                                                        \
      fprintf(stderr, "dlrm_native_bench: %s failed: %s\n", #x, fmn_last_error()); \
      return 1;                                                           \
    }                                                                     \
  } while (0)

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static uint64_t next_u64(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}
static float frand(void) { return (float)(next_u64() >> 40) / (float)(1u << 24); }

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: dlrm_native_bench <cpu|hip> [steps] [warmup] [batch] [small]\n");
    return 2;
  }
  const int device = strcmp(argv[1], "hip") == 0 ? 1 : 0;
  const int steps = argc > 2 ? atoi(argv[2]) : 20, warmup = argc > 3 ? atoi(argv[3]) : 5;
  const int B = argc > 4 ? atoi(argv[4]) : 8192;
  const int small = argc > 5 && strcmp(argv[5], "small") == 0;
  if (steps < 1 || warmup < 0 || B < 1) return 2;

  fmn_model_t m = fmn_model_create(B, device, 0, 1, "");
  if (!m) {
    fprintf(stderr, "dlrm_native_bench: create: %s\n", fmn_last_error());
    return 1;
  }
  int x, t, emb[NT];
  int64_t rows[NT];
  CHECK(x = fmn_model_input(m, FEAT_PAD));
  CHECK(t = fmn_model_dense(m, x, 512, 11, 1));
  CHECK(t = fmn_model_dense(m, t, 256, 11, 1));
  CHECK(t = fmn_model_dense(m, t, D, 11, 1));
  const int bottom = t;
  for (int i = 0; i < NT; ++i) {
    int sp;
    rows[i] = small && MLPERF_ROWS[i] > 100000 ? 100000 : MLPERF_ROWS[i];
    CHECK(sp = fmn_model_sparse_input(m, 1));
    CHECK(emb[i] = fmn_model_embedding(m, sp, rows[i], D));
  }
  /* 479 interaction features padded to 480 (a zero column, as the executor pads): 16-B rows for the
   * staged interaction kernels and the top GEMM */
  CHECK(t = fmn_model_dot_interaction(m, bottom, NT, emb, 8));
  const int top[5] = {1024, 1024, 512, 256, 1};
  for (int i = 0; i < 5; ++i) CHECK(t = fmn_model_dense(m, t, top[i], i == 4 ? 12 : 11, 1));
  CHECK(fmn_model_compile(m, 54, 0.01f, 64.0));
  static char desc[16384];
  fmn_model_describe(m, desc, sizeof(desc));
  printf("%s", desc);

  /* dense layers: small random weights (tables stay zero).  Parameters in model order: the bottom
   * layers' W, b (6 entries), the 26 tables, the top layers' W, b */
  const int np = fmn_model_num_params(m);
  for (int i = 0; i < np; ++i) {
    if (i >= 6 && i < 6 + NT) continue;
    const int64_t n = fmn_model_param_numel(m, i);
    float* w = (float*)malloc(sizeof(float) * (size_t)n);
    for (int64_t k = 0; k < n; ++k) w[k] = (frand() * 2.f - 1.f) * 0.05f;
    CHECK(fmn_model_set_param(m, i, w));
    free(w);
  }
  float* dense = (float*)calloc((size_t)B * FEAT_PAD, sizeof(float));
  float* lab = (float*)malloc(sizeof(float) * (size_t)B);
  int64_t* idx[NT];
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < FEAT; ++k) dense[(size_t)b * FEAT_PAD + k] = frand();
  for (int b = 0; b < B; ++b) lab[b] = (float)(next_u64() & 1);
  for (int i = 0; i < NT; ++i) {
    idx[i] = (int64_t*)malloc(sizeof(int64_t) * (size_t)B);
    for (int b = 0; b < B; ++b) idx[i][b] = (int64_t)(next_u64() % (uint64_t)rows[i]);
  }
  const int64_t* sparse[NT];
  for (int i = 0; i < NT; ++i) sparse[i] = idx[i];
  double loss = 0.0;
  int64_t correct = 0;
  for (int s = 0; s < warmup; ++s) CHECK(fmn_model_train_step_sparse(m, dense, sparse, lab, &loss, &correct));
  const double t0 = now_s();
  for (int s = 0; s < steps; ++s) CHECK(fmn_model_train_step_sparse(m, dense, sparse, lab, &loss, &correct));
  const double dt = now_s() - t0;   /* every train_step ends with a device sync (loss readback) */
  const double ms = dt * 1e3 / steps;
  printf("{\"engine\": \"native-%s\", \"model\": \"dlrm-mlperf%s\", \"batch\": %d, \"steps\": %d, \"warmup\": %d, "
         "\"ms_per_step\": %.4f, \"samples_per_s\": %.1f, \"loss\": %.5f}\n",
         device ? "hip" : "cpu", small ? "-small" : "", B, steps, warmup, ms, B / (ms * 1e-3), loss);
  fmn_model_destroy(m);
  for (int i = 0; i < NT; ++i) free(idx[i]);
  free(dense);
  free(lab);
  return 0;
}
