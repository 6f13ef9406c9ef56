/* Trains a small DLRM through the native C API alone (libflexmi_native_c: C++ plan compiler +
 * engine, no Python anywhere in the process): bottom MLP 13-32-16, four embedding tables
 * (100 / 50 / 200 / 30 rows x 16) placed TABLE-WISE over the ranks (NATIVE_DLRM_PLAN: colsplit / rowsplit /
 * mixed split some of them by columns or rows over every rank), dot interaction, top MLP
 * -32-1 with a sigmoid, binary cross-entropy, SGD.  With world > 1 the program forks one process
 * per rank; the ranks exchange embeddings (all-to-all) and dense gradients (all-reduce) through
 * the CPU engine's host communicator in the rendezvous directory (or RCCL on the HIP engine).
 *
 *   native_dlrm <cpu|hip> <out prefix> <steps> <world> <rendezvous dir>
 *
 * <prefix>.init.bin (written by rank 0): int32 B, int32 steps, int32 nparams; per param int64
 *   numel + float init[numel]; per step float dense[B*13], int64 idx[4][B], float labels[B].
 * <prefix>.r<rank>.bin: int32 rank, int32 nparams; per param int32 local + (local) float
 *   final[numel]; per step double loss.  The plan goes to stdout. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "flexmi_native_c.h"

#define NT 4
static const int64_t ROWS[NT] = {100, 50, 200, 30};
#define D 16
#define FEAT 13
/* batch: 64, or NATIVE_DLRM_B (the uneven-ownership host-communicator test uses a batch whose
 * per-rank embedding exchange exceeds the 4 MiB staging-slot floor) */
static int B = 64;

#define CHECK(x)                                                                     \
  do {                                                                               \
    if ((x) < 0) {                                                                   \
      fprintf(stderr, "native_dlrm r%d: %s failed: %s\n", rank, #x, fmn_last_error()); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

static uint32_t rng = 777u;
static float frand(void) {
  rng = rng * 1664525u + 1013904223u;
  return (float)(rng >> 8) / (float)(1u << 24);
}

static int run_rank(int device, const char* prefix, int steps, int rank, int world, const char* rdv) {
  fmn_model_t m = fmn_model_create(B, device, rank, world, rdv);
  if (!m) {
    fprintf(stderr, "native_dlrm r%d: create: %s\n", rank, fmn_last_error());
    return 1;
  }
  int x, t, emb[NT], sp[NT];
  CHECK(x = fmn_model_input(m, FEAT));
  CHECK(t = fmn_model_dense(m, x, 32, 11, 1));
  CHECK(t = fmn_model_dense(m, t, D, 11, 1));
  const int bottom = t;
  for (int i = 0; i < NT; ++i) {
    CHECK(sp[i] = fmn_model_sparse_input(m, 1));
    CHECK(emb[i] = fmn_model_embedding(m, sp[i], ROWS[i], D));
  }
  CHECK(t = fmn_model_dot_interaction(m, bottom, NT, emb, 16));
  CHECK(t = fmn_model_dense(m, t, 32, 11, 1));
  CHECK(t = fmn_model_dense(m, t, 1, 12, 1));
  /* a fixed table-wise placement over the ranks (round robin); NATIVE_DLRM_PLAN=colsplit splits
   * tables 0 and 2 by columns over every rank (the bench "table" plan's large tables) */
  const char* plan = getenv("NATIVE_DLRM_PLAN") ? getenv("NATIVE_DLRM_PLAN") : "table";
  /* "mixed": table 0 split by columns, table 1 by rows over every rank, the others whole;
   * "chan": the first bottom layer (13 -> 32) and the first top layer (-> 32) channel-split over
   * every rank, table 0 split by columns; "chanhalf": the top layer over ranks {1, 0} of a larger
   * world (holders in reverse order, other ranks only exchange) */
  const int colsplit = strcmp(plan, "colsplit") == 0, rowsplit = strcmp(plan, "rowsplit") == 0, mixed = strcmp(plan, "mixed") == 0;
  const int chan = strcmp(plan, "chan") == 0, chanhalf = strcmp(plan, "chanhalf") == 0;
  /* "rowsplitrev": tables 1 and 3 split by rows over every rank in DESCENDING rank order (slice j on
   * rank world-1-j: the partial sums arrive in an order other than slice order) */
  const int rowsplitrev = strcmp(plan, "rowsplitrev") == 0;
  int all[16], rev[16];
  for (int r = 0; r < world; ++r) all[r] = r, rev[r] = world - 1 - r;
  for (int i = 0; i < NT; ++i) {
    if ((colsplit && (i == 0 || i == 2)) || ((mixed || chan) && i == 0)) {
      CHECK(fmn_model_set_table_columns(m, i, world, all));
    } else if ((rowsplit && (i == 1 || i == 3)) || (mixed && i == 1)) {
      CHECK(fmn_model_set_table_rows(m, i, world, all));
    } else if (rowsplitrev && (i == 1 || i == 3)) {
      CHECK(fmn_model_set_table_rows(m, i, world, rev));
    } else {
      CHECK(fmn_model_set_table_owner(m, i, i % world));
    }
  }
  if (chan) {
    CHECK(fmn_model_set_dense_channels(m, 0, world, all));
    CHECK(fmn_model_set_dense_channels(m, 2, world, all));
  }
  if (chanhalf) {
    const int two[2] = {1, 0};
    CHECK(fmn_model_set_dense_channels(m, 2, world > 1 ? 2 : 1, world > 1 ? two : all));
  }
  /* NATIVE_DLRM_STRATEGY=<.pb> with NATIVE_DLRM_NAMES="dense0,..,dense3;table0,..,table3": the
   * placement a strategy file gives (e.g. the MCMC search's result) */
  if (getenv("NATIVE_DLRM_STRATEGY")) {
    fmn_strategy_t st = fmn_strategy_load(getenv("NATIVE_DLRM_STRATEGY"));
    if (!st) {
      fprintf(stderr, "native_dlrm r%d: strategy: %s\n", rank, fmn_last_error());
      return 1;
    }
    static char names[2048];
    const char* dn[4] = {0, 0, 0, 0};
    const char* tn[NT];
    for (int i = 0; i < NT; ++i) tn[i] = 0;
    strncpy(names, getenv("NATIVE_DLRM_NAMES") ? getenv("NATIVE_DLRM_NAMES") : "", sizeof(names) - 1);
    int k = 0;
    char* save = 0;
    for (char* tok = strtok_r(names, ",;", &save); tok && k < 4 + NT; tok = strtok_r(0, ",;", &save), ++k) {
      if (k < 4) dn[k] = tok;
      else tn[k - 4] = tok;
    }
    int placed;
    CHECK(placed = fmn_model_apply_strategy(m, st, 4, dn, NT, tn));
    if (rank == 0) printf("strategy: %d ops placed\n", placed);
    fmn_strategy_destroy(st);
  }
  CHECK(fmn_model_compile(m, 54, 0.1f, 0.0005));
  static char desc[8192];
  fmn_model_describe(m, desc, sizeof(desc));
  if (rank == 0) printf("%s", desc);

  /* identical initial weights and batches on every rank (same generator, same order) */
  const int np = fmn_model_num_params(m);
  float** init = (float**)calloc(np, sizeof(float*));
  int64_t* numel = (int64_t*)calloc(np, sizeof(int64_t));
  for (int i = 0; i < np; ++i) {
    numel[i] = fmn_model_param_numel(m, i);
    init[i] = (float*)malloc(numel[i] * sizeof(float));
    for (int64_t k = 0; k < numel[i]; ++k) init[i][k] = (frand() * 2.f - 1.f) * 0.3f;
    if (fmn_model_param_local(m, i) == 1) CHECK(fmn_model_set_param(m, i, init[i]));
  }
  float* dense = (float*)malloc(sizeof(float) * B * FEAT * steps);
  int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * NT * B * steps);
  float* lab = (float*)malloc(sizeof(float) * B * steps);
  for (int s = 0; s < steps; ++s) {
    for (int k = 0; k < B * FEAT; ++k) dense[s * B * FEAT + k] = frand();
    for (int i = 0; i < NT; ++i)
      for (int b = 0; b < B; ++b) {
        /* skewed: half the lookups hit the first 8 rows (duplicates within the batch) */
        const int64_t r = frand() < 0.5f ? (int64_t)(frand() * 8) : (int64_t)(frand() * ROWS[i]);
        idx[((int64_t)s * NT + i) * B + b] = r < ROWS[i] ? r : ROWS[i] - 1;
      }
    for (int b = 0; b < B; ++b) lab[s * B + b] = frand() < 0.5f ? 0.f : 1.f;
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
      fwrite(dense + s * B * FEAT, 4, B * FEAT, f);
      fwrite(idx + (int64_t)s * NT * B, 8, NT * B, f);
      fwrite(lab + s * B, 4, B, f);
    }
    fclose(f);
  }
  double* losses = (double*)calloc(steps, sizeof(double));
  for (int s = 0; s < steps; ++s) {
    const int64_t* sparse[NT];
    for (int i = 0; i < NT; ++i) sparse[i] = idx + ((int64_t)s * NT + i) * B;
    int64_t correct = 0;
    CHECK(fmn_model_train_step_sparse(m, dense + s * B * FEAT, sparse, lab + s * B, &losses[s], &correct));
  }
  char path[1024];
  snprintf(path, sizeof(path), "%s.r%d.bin", prefix, rank);
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  int32_t hdr[2] = {rank, np};
  fwrite(hdr, 4, 2, f);
  for (int i = 0; i < np; ++i) {
    const int32_t local = fmn_model_param_local(m, i) == 1;
    fwrite(&local, 4, 1, f);
    if (local) {
      /* a column-split table fills only this rank's columns: the rest keep the initial values */
      float* w = (float*)malloc(numel[i] * sizeof(float));
      memcpy(w, init[i], numel[i] * sizeof(float));
      CHECK(fmn_model_get_param(m, i, w));
      fwrite(w, 4, numel[i], f);
      free(w);
    }
  }
  fwrite(losses, 8, steps, f);
  fclose(f);
  fmn_model_destroy(m);
  if (rank == 0) printf("native_dlrm ok: %d ranks, %d steps, loss %.5f -> %.5f\n", world, steps, losses[0], losses[steps - 1]);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: native_dlrm <cpu|hip> <out prefix> <steps> <world> <rendezvous dir>\n");
    return 2;
  }
  const int device = strcmp(argv[1], "hip") == 0 ? 1 : 0;
  if (getenv("NATIVE_DLRM_B")) B = atoi(getenv("NATIVE_DLRM_B"));
  const int steps = atoi(argv[3]), world = atoi(argv[4]);
  fflush(stdout);
  int rc = 0;
  pid_t kids[16];
  if (world < 1 || world > 16) return 2;
  for (int r = 1; r < world; ++r) {
    kids[r] = fork();
    if (kids[r] == 0) _exit(run_rank(device, argv[2], steps, r, world, argv[5]));
  }
  rc = run_rank(device, argv[2], steps, 0, world, argv[5]);
  for (int r = 1; r < world; ++r) {
    int st = 0;
    waitpid(kids[r], &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
  }
  return rc;
}
