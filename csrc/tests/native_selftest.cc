// Host self-test of flexmi's native runtime, built under sanitizers by tests/test_native_sanitizers.py
// (the reference had no race detection; flexmi runs its C++ runtime under
// ASan+UBSan and ThreadSanitizer on the CPU box):
//   * strategy .pb codec: encode/decode round trips, truncated and corrupted inputs must fail cleanly;
//   * sharding algebra: random layout pairs, every destination element delivered once per holder;
//   * data-loader ring: worker threads gather shuffled batches into the staging slots while the
//     consumer acquires/releases them in order, across epochs and a stop()/start() cycle.
// Exit code 0 = all checks passed; messages name the failing check.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "loader.h"
#include "shard.h"
#include "strategy_pb.h"

namespace {

int g_fail = 0;
#define CHECK(c, msg)                                                      \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, msg, #c); \
      ++g_fail;                                                            \
    }                                                                      \
  } while (0)

void test_codec(std::mt19937& rng) {
  for (int trial = 0; trial < 200; ++trial) {
    std::vector<flexmi::OpStrategy> ops(rng() % 12);
    for (auto& o : ops) {
      o.name = "op" + std::to_string(rng() % 100000);
      o.device_type = rng() % 2;
      int nd = 1 + rng() % 4, parts = 1;
      for (int i = 0; i < nd; ++i) {
        int d = 1 + rng() % 4;
        o.dims.push_back(d);
        parts *= d;
      }
      for (int p = 0; p < parts; ++p) o.device_ids.push_back(rng() % 64);
      if (rng() % 3 == 0) o.memory_types.push_back(rng() % 2);
    }
    const std::string enc = flexmi::encode_strategy(ops);
    std::vector<flexmi::OpStrategy> dec;
    std::string err;
    CHECK(flexmi::decode_strategy(enc, dec, err), "round trip decodes");
    CHECK(dec.size() == ops.size(), "round trip op count");
    for (size_t i = 0; i < dec.size() && i < ops.size(); ++i) {
      CHECK(dec[i].name == ops[i].name && dec[i].dims == ops[i].dims && dec[i].device_ids == ops[i].device_ids,
            "round trip fields");
    }
    // every truncation and a random corruption must be rejected or decode without touching
    // memory out of bounds (ASan checks the latter)
    for (size_t cut = 0; cut < enc.size(); cut += 1 + enc.size() / 17) {
      std::vector<flexmi::OpStrategy> tmp;
      flexmi::decode_strategy(enc.substr(0, cut), tmp, err);
    }
    if (!enc.empty()) {
      std::string bad = enc;
      bad[rng() % bad.size()] = (char)(rng() & 0xFF);
      std::vector<flexmi::OpStrategy> tmp;
      flexmi::decode_strategy(bad, tmp, err);
    }
  }
}

flexmi::ShardLayout rand_layout(std::mt19937& rng, const std::vector<int64_t>& shape, int world) {
  flexmi::ShardLayout l;
  l.shape = shape;
  int64_t parts = 1;
  for (auto n : shape) {
    int64_t d = 1 + rng() % std::min<int64_t>(4, n);
    l.degrees.push_back(d);
    parts *= d;
  }
  for (int64_t p = 0; p < parts; ++p) {
    std::vector<int> h{(int)(rng() % world)};
    if (world > 1 && rng() % 3 == 0) h.push_back((h[0] + 1) % world);
    l.holders.push_back(h);
  }
  return l;
}

void test_shard(std::mt19937& rng) {
  for (int trial = 0; trial < 300; ++trial) {
    const int world = 1 + rng() % 8;
    std::vector<int64_t> shape;
    for (int i = 0, nd = 1 + rng() % 4; i < nd; ++i) shape.push_back(1 + rng() % 13);
    auto src = rand_layout(rng, shape, world);
    auto dst = rand_layout(rng, shape, world);
    const auto tr = flexmi::reshard_transfers(src, dst);
    int64_t vol = 0, want = 0;
    for (auto& t : tr) vol += flexmi::box_volume(t.box);
    for (int64_t p = 0; p < dst.num_parts(); ++p) want += flexmi::box_volume(dst.part_box(p)) * dst.holders[p].size();
    CHECK(vol == want, "every destination element delivered once per holder");
    std::vector<int64_t> ids;
    std::vector<flexmi::Box> boxes;
    for (auto& t : tr) {
      ids.push_back(t.dst);
      boxes.push_back(t.box);
    }
    int64_t n = 0;
    for (int s : flexmi::split_launches(ids, boxes, 7)) n += s;
    CHECK(n == (int64_t)tr.size(), "launch split covers every piece");
  }
  bool threw = false;
  try {
    flexmi::ShardLayout bad;
    bad.shape = {4};
    bad.degrees = {2};
    bad.holders = {{0}};   // one holder list for two parts
    flexmi::reshard_transfers(bad, bad);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw, "invalid layout rejected");
}

void test_loader() {
  const int64_t N = 1000, B = 64, F = 5;   // samples, batch, features (int64 each)
  std::vector<int64_t> data(N * F);
  for (int64_t i = 0; i < N; ++i)
    for (int64_t f = 0; f < F; ++f) data[i * F + f] = i * 10 + f;
  for (int shuffle = 0; shuffle < 2; ++shuffle) {
    const int depth = 3;
    flexmi::BatchRing ring(B, N, depth, 3, shuffle != 0, 42);
    // rank view: rows [16, 48) of every batch, columns 1..3
    const int64_t lo = 16, hi = 48, col_off = 8, col_bytes = 3 * 8;
    int src = ring.add_source(data.data(), N, F * 8, col_off, col_bytes, lo, hi);
    std::vector<std::vector<int64_t>> slots(depth, std::vector<int64_t>((hi - lo) * 3));
    for (int s = 0; s < depth; ++s) ring.set_slot(src, s, slots[s].data());
    for (int cycle = 0; cycle < 2; ++cycle) {
      ring.start();
      const int64_t nb = ring.batches_per_epoch() * 2 + 3;   // crosses two epoch boundaries
      for (int64_t n = 0; n < nb; ++n) {
        const int s = ring.acquire();
        const auto ids = ring.batch_ids(n);
        bool ok = (int64_t)ids.size() == B;
        for (int64_t r = lo; r < hi && ok; ++r)
          for (int c = 0; c < 3; ++c) ok = ok && slots[s][(r - lo) * 3 + c] == ids[r] * 10 + 1 + c;
        CHECK(ok, "staged batch rows match the sampler");
        ring.release(s);
      }
      ring.stop();
    }
  }
}

}  // namespace

int main() {
  std::mt19937 rng(1234);
  test_codec(rng);
  test_shard(rng);
  test_loader();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("native selftest ok\n");
  return 0;
}
