/* A C program on flexmi's native C API (flexmi_native_c.h) -- no Python in the process.
 *   native_demo <scratch dir> [hdf5 file] [reference .pb]
 * Prints one "ok <area>" line per checked area; exits non-zero on the first failure. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flexmi_native_c.h"

#define CHECK(c, msg)                                                             \
  do {                                                                            \
    if (!(c)) {                                                                   \
      fprintf(stderr, "FAIL %s (%s): %s\n", msg, #c, fmn_last_error());           \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

static int strategies(const char* dir, const char* ref_pb) {
  char path[1024];
  snprintf(path, sizeof path, "%s/s.pb", dir);
  fmn_strategy_t s = fmn_strategy_create();
  int dims[2] = {1, 4}, devs[4] = {0, 1, 2, 3}, one[1] = {1}, dev1[1] = {2};
  CHECK(fmn_strategy_set(s, "linear1", 0, 2, dims, 4, devs) == 0, "set");
  CHECK(fmn_strategy_set(s, "embedding0", 0, 1, one, 1, dev1) == 0, "set");
  CHECK(fmn_strategy_set(s, "bad", 0, 2, dims, 1, devs) < 0, "parts must match devices");
  CHECK(fmn_strategy_save(s, path) == 0, "save");
  fmn_strategy_destroy(s);
  s = fmn_strategy_load(path);
  CHECK(s && fmn_strategy_num_ops(s) == 2, "reload");
  char name[64];
  int dt, nd, d[8], nv, v[64];
  int i = fmn_strategy_find(s, "linear1");
  CHECK(i >= 0 && fmn_strategy_get(s, i, name, sizeof name, &dt, &nd, d, 8, &nv, v, 64) == 4, "get");
  CHECK(!strcmp(name, "linear1") && nd == 2 && d[1] == 4 && nv == 4 && v[3] == 3, "fields");
  fmn_strategy_destroy(s);
  if (ref_pb) {   /* the reference's shipped DLRM strategy: 8 embeddings placed on 8 GPUs */
    s = fmn_strategy_load(ref_pb);
    CHECK(s != NULL && fmn_strategy_num_ops(s) > 8, "reference .pb");
    int placed = 0;
    for (int k = 0; k < fmn_strategy_num_ops(s); ++k) {
      fmn_strategy_get(s, k, name, sizeof name, &dt, &nd, d, 8, &nv, v, 64);
      if (!strncmp(name, "embedding", 9) && nv == 1) ++placed;
    }
    CHECK(placed == 8, "8 table-wise embeddings");
    fmn_strategy_destroy(s);
  }
  printf("ok strategies\n");
  return 0;
}

static int sharding(void) {
  int64_t lo, hi;
  CHECK(fmn_split_extent(10, 3, 2, &lo, &hi) == 0 && lo == 8 && hi == 10, "split_extent (ceil blocks)");
  int64_t shape[2] = {8, 6}, rows[2] = {4, 1}, cols[2] = {1, 2};
  int h4[4] = {0, 1, 2, 3}, h2[2] = {0, 1};
  fmn_layout_t a = fmn_layout_create(2, shape, rows, h4, 0);
  fmn_layout_t b = fmn_layout_create(2, shape, cols, h2, 0);
  CHECK(a && b && fmn_layout_num_parts(a) == 4, "layouts");
  int64_t blo[2], bhi[2];
  CHECK(fmn_layout_part_box(a, 3, blo, bhi) == 0 && blo[0] == 6 && bhi[0] == 8 && bhi[1] == 6, "part box");
  int n = fmn_reshard_transfers(a, b, 0, NULL, NULL, NULL, NULL);
  CHECK(n == 8, "row split -> column split = 4 x 2 pieces");
  int src[8], dst[8];
  int64_t tlo[16], thi[16];
  fmn_reshard_transfers(a, b, 8, src, dst, tlo, thi);
  int64_t vol = 0;
  for (int i = 0; i < n; ++i) vol += (thi[2 * i] - tlo[2 * i]) * (thi[2 * i + 1] - tlo[2 * i + 1]);
  CHECK(vol == 48, "transfers cover the tensor once");
  fmn_layout_destroy(a);
  fmn_layout_destroy(b);
  printf("ok sharding\n");
  return 0;
}

/* two chained linear layers on 2 GPUs: data parallel (2 parts, weight all-reduce) or whole on one GPU */
static int simulator(void) {
  fmn_sim_t s = fmn_sim_create(2, 8, 0, 0);
  int x = fmn_sim_add_tensor(s, 4, -1, 0, 0);
  int h = fmn_sim_add_tensor(s, 4, 0, 0, 1);
  int y = fmn_sim_add_tensor(s, 4, 1, 0, 1);
  const int B = 4096, F = 1024;
  for (int layer = 0; layer < 2; ++layer) {
    int in = layer ? h : x, out = layer ? y : h;
    fmn_sim_add_op(s, layer ? "fc2" : "fc1", 1, &in, 1, &out);
    /* candidate 0: data parallel, half the batch per GPU */
    int dev2[2] = {0, 1};
    double f2[2] = {50, 50}, b2[2] = {100, 100};
    int64_t lo2[4] = {0, 0, B / 2, 0}, hi2[4] = {B / 2, F, B, F};
    fmn_sim_add_candidate(s, 2, dev2, f2, b2, 2, lo2, hi2, lo2, hi2, 4.0 * F * F, 4.0 * F * F, "dp2");
    /* candidate 1: the whole layer on GPU 0 */
    int dev1[1] = {0};
    double f1[1] = {100}, b1[1] = {200};
    int64_t lo1[2] = {0, 0}, hi1[2] = {B, F};
    fmn_sim_add_candidate(s, 1, dev1, f1, b1, 2, lo1, hi1, lo1, hi1, 0, 4.0 * F * F, "gpu0");
  }
  int dp[2] = {0, 0}, one[2] = {1, 1}, best[2];
  double t_dp = fmn_sim_simulate(s, dp), t_one = fmn_sim_simulate(s, one);
  CHECK(t_dp > 0 && t_one > 0, "simulate");
  double t_best = fmn_sim_search(s, one, 400, 0.05, 7, best);   /* low alpha: climbs out of the single-GPU basin */
  CHECK(t_best > 0 && t_best <= t_one + 1e-6 && t_best <= t_dp + 1e-6, "search finds the better plan");
  printf("ok simulator dp=%.1f single=%.1f best=%.1f (%d,%d)\n", t_dp, t_one, t_best, best[0], best[1]);
  fmn_sim_destroy(s);
  return 0;
}

static int hdf5(const char* path) {
  fmn_h5_t h = fmn_h5_open(path);
  CHECK(h != NULL, "open");
  int n = fmn_h5_num_datasets(h), found = 0;
  for (int i = 0; i < n; ++i) {
    char name[64], dt[16];
    int nd;
    int64_t shape[4];
    fmn_h5_dataset_info(h, i, name, sizeof name, dt, sizeof dt, &nd, shape, 4);
    if (!strcmp(name, "X_int")) {
      CHECK(!strcmp(dt, "<f4") && nd == 2 && shape[1] == 13, "X_int info");
      float rows[2 * 13];
      CHECK(fmn_h5_read_rows(h, "X_int", 3, 2, rows, sizeof rows) == 2, "read rows");
      double s = 0;
      for (int k = 0; k < 26; ++k) s += rows[k];
      printf("X_int[3:5] sum %.6f\n", s);
      ++found;
    }
  }
  CHECK(found == 1, "X_int present");
  fmn_h5_close(h);
  printf("ok hdf5\n");
  return 0;
}

static int loader(void) {
  enum { ROWS = 10, COLS = 4, BATCH = 4 };
  float data[ROWS][COLS];
  for (int r = 0; r < ROWS; ++r)
    for (int c = 0; c < COLS; ++c) data[r][c] = (float)(r * 100 + c);
  fmn_loader_t l = fmn_loader_create(BATCH, 8, 2, 2, 1, 11);
  CHECK(l != NULL, "create");
  /* this "rank" holds rows 1..3 of each batch and columns 1..2 */
  CHECK(fmn_loader_add_source(l, data, ROWS, COLS * 4, 4, 8, 1, 3, -1) == 0, "source");
  static float slots[2][2][2];
  for (int s = 0; s < 2; ++s) fmn_loader_set_slot(l, 0, s, slots[s]);
  CHECK(fmn_loader_start(l) == 0 && fmn_loader_batches_per_epoch(l) == 2, "start");
  for (int b = 0; b < 4; ++b) {
    int slot = fmn_loader_acquire(l);
    int64_t ids[BATCH];
    CHECK(fmn_loader_batch_ids(l, b, ids, BATCH) == BATCH, "ids");
    for (int r = 0; r < 2; ++r)
      for (int c = 0; c < 2; ++c) CHECK(slots[slot][r][c] == data[ids[1 + r]][1 + c], "gathered rows / columns");
    fmn_loader_release(l, slot);
  }
  fmn_loader_destroy(l);
  printf("ok loader\n");
  return 0;
}

static int embedding(void) {
  enum { R = 50, D = 37, B = 33, BAG = 3 };
  static float W[R * D], out[B * D], G[R * D], dy[B * D];
  int64_t idx[B * BAG];
  for (int i = 0; i < R * D; ++i) W[i] = (float)((i * 7919) % 1000) / 1000.f - 0.5f;
  for (int i = 0; i < B * BAG; ++i) idx[i] = (i * 31) % 70;     /* some outside the shard */
  for (int i = 0; i < B * D; ++i) dy[i] = (float)((i * 104729) % 997) / 997.f;
  const int64_t lo = 10;                                      /* shard holds rows 10..59 */
  CHECK(fmn_embedding_bag_forward(W, R, D, idx, B, BAG, lo, 0.5f, out, D) == 0, "forward");
  double err = 0;
  for (int b = 0; b < B; ++b)
    for (int d = 0; d < D; ++d) {
      double s = 0;
      for (int j = 0; j < BAG; ++j) {
        int64_t r = idx[b * BAG + j] - lo;
        if (r >= 0 && r < R) s += W[r * D + d];
      }
      err = fmax(err, fabs(0.5 * s - out[b * D + d]));
    }
  CHECK(err < 1e-5, "forward values");
  memset(G, 0, sizeof G);
  CHECK(fmn_embedding_bag_backward(G, R, D, idx, B, BAG, lo, dy, D, 2.0f) == 0, "backward");
  err = 0;
  for (int r = 0; r < R; ++r)
    for (int d = 0; d < D; ++d) {
      double s = 0;
      for (int i = 0; i < B * BAG; ++i)
        if (idx[i] - lo == r) s += 2.0 * dy[(i / BAG) * D + d];
      err = fmax(err, fabs(s - G[r * D + d]));
    }
  CHECK(err < 1e-4, "backward values");
  printf("ok embedding\n");
  return 0;
}

/* graph planner: dense chain d1 -> d2 and an embedding chain e0 -> e1 whose output crosses ranks
 * into the join j; the remote producer and its ancestor are scheduled first */
static int planner(void) {
  fmn_plan_t p = fmn_plan_create();
  CHECK(p != NULL, "plan create");
  int64_t o;
  o = 11; fmn_plan_add_op(p, 1, 1, &o); fmn_plan_add_input(p, 100, -1, 0, 0, 3);
  o = 12; fmn_plan_add_op(p, 2, 1, &o); fmn_plan_add_input(p, 11, 1, 0, 0, 3);
  o = 13; fmn_plan_add_op(p, 3, 1, &o); fmn_plan_add_input(p, 101, -1, 0, 0, 3);
  o = 14; fmn_plan_add_op(p, 4, 1, &o); fmn_plan_add_input(p, 13, 3, 0, 0, 3);
  o = 15; fmn_plan_add_op(p, 5, 1, &o);
  fmn_plan_add_input(p, 12, 2, 0, 0, 3);
  fmn_plan_add_input(p, 14, 4, 0, 7, 1 | 2 | 4 | 8);   /* float, grad, reshard, remote */
  CHECK(fmn_plan_run(p, 2, 0) == 0, "plan run");
  int64_t order[8];
  CHECK(fmn_plan_order(p, order, 8) == 5, "order size");
  CHECK(order[0] == 3 && order[1] == 4 && order[2] == 1 && order[3] == 2 && order[4] == 5, "comm-first order");
  int kind[16], nin[16], ins[16];
  int64_t op[16];
  const int64_t nf = fmn_plan_steps(p, 0, kind, op, nin, ins, 16, 16);
  CHECK(nf == 6 && kind[4] == 1 && op[4] == 5 && nin[4] == 1 && ins[0] == 1, "forward reshard step");
  const int64_t nb = fmn_plan_steps(p, 1, kind, op, nin, ins, 16, 16);
  CHECK(nb == 6 && kind[0] == 0 && op[0] == 5 && kind[1] == 1, "backward gradient reduce after the join");
  int64_t live[8];
  CHECK(fmn_plan_bwd_live(p, live, 8) == 5, "all ops live");
  fmn_plan_destroy(p);
  printf("ok planner\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <scratch dir> [hdf5] [reference .pb]\n", argv[0]);
    return 2;
  }
  printf("%s\n", fmn_version());
  if (strategies(argv[1], argc > 3 ? argv[3] : NULL)) return 1;
  if (sharding()) return 1;
  if (simulator()) return 1;
  if (argc > 2 && hdf5(argv[2])) return 1;
  if (loader()) return 1;
  if (embedding()) return 1;
  if (planner()) return 1;
  printf("ALL OK\n");
  return 0;
}
