#include "shard.h"

#include <algorithm>
#include <stdexcept>
#include <tuple>

namespace flexmi {

Range split_extent(int64_t n, int64_t d, int64_t k) {
  const int64_t b = (n + d - 1) / d;
  return {std::min(n, k * b), std::min(n, (k + 1) * b)};
}

bool box_intersect(const Box& a, const Box& b, Box& out) {
  out.clear();
  if (a.size() != b.size()) return false;
  out.reserve(a.size());
  for (size_t i = 0; i < a.size(); ++i) {
    const int64_t lo = std::max(a[i].first, b[i].first);
    const int64_t hi = std::min(a[i].second, b[i].second);
    if (lo >= hi) {
      out.clear();
      return false;
    }
    out.emplace_back(lo, hi);
  }
  return true;
}

int64_t box_volume(const Box& b) {
  int64_t v = 1;
  for (auto& r : b) v *= r.second - r.first;
  return v;
}

int64_t ShardLayout::num_parts() const {
  int64_t n = 1;
  for (auto d : degrees) n *= d;
  return n;
}

std::vector<int64_t> ShardLayout::part_coords(int64_t p) const {
  std::vector<int64_t> c(degrees.size());
  for (int i = (int)degrees.size() - 1; i >= 0; --i) {
    c[i] = p % degrees[i];
    p /= degrees[i];
  }
  return c;
}

Box ShardLayout::part_box(int64_t p) const {
  if (!boxes.empty()) return boxes.at(p);
  const auto c = part_coords(p);
  Box b;
  b.reserve(shape.size());
  for (size_t i = 0; i < shape.size(); ++i) b.push_back(split_extent(shape[i], degrees[i], c[i]));
  return b;
}

void ShardLayout::validate() const {
  if (shape.size() != degrees.size()) throw std::invalid_argument("ShardLayout: shape/degrees rank mismatch");
  for (auto d : degrees)
    if (d < 1) throw std::invalid_argument("ShardLayout: degrees must be >= 1");
  const int64_t np = num_parts();
  if ((int64_t)holders.size() != np) throw std::invalid_argument("ShardLayout: one holder list per part expected");
  for (auto& h : holders)
    if (h.empty()) throw std::invalid_argument("ShardLayout: every part needs a holder");
  if (!boxes.empty()) {
    if ((int64_t)boxes.size() != np) throw std::invalid_argument("ShardLayout: one box per part expected");
    for (auto& b : boxes)
      if (b.size() != shape.size()) throw std::invalid_argument("ShardLayout: box rank mismatch");
  }
}

std::vector<Transfer> reshard_transfers(const ShardLayout& src, const ShardLayout& dst) {
  src.validate();
  dst.validate();
  if (src.shape != dst.shape) throw std::invalid_argument("reshard_transfers: shapes differ");
  const bool reduce = src.partial && !dst.partial;
  const int64_t ns = src.num_parts(), nd = dst.num_parts();
  std::vector<Box> sboxes(ns);
  for (int64_t sp = 0; sp < ns; ++sp) sboxes[sp] = src.part_box(sp);
  std::vector<Transfer> out;
  Box inter;
  for (int64_t dp = 0; dp < nd; ++dp) {
    const Box dbox = dst.part_box(dp);
    for (int64_t sp = 0; sp < ns; ++sp) {
      if (!box_intersect(dbox, sboxes[sp], inter)) continue;
      const auto& sh = src.holders[sp];
      for (int d : dst.holders[dp]) {
        if (reduce) {
          for (int s : sh) out.push_back({s, d, inter, sp, dp});
        } else {
          int s = -1;
          for (int h : sh)
            if (h == d) s = d;
          if (s < 0) s = sh[(dp + sp) % (int64_t)sh.size()];
          out.push_back({s, d, inter, sp, dp});
        }
      }
    }
  }
  std::sort(out.begin(), out.end(), [](const Transfer& a, const Transfer& b) {
    return std::tie(a.src, a.dst, a.dst_part, a.src_part, a.box) < std::tie(b.src, b.dst, b.dst_part, b.src_part, b.box);
  });
  return out;
}

std::vector<int> split_launches(const std::vector<int64_t>& dst, const std::vector<Box>& boxes, int max_per_launch) {
  if (dst.size() != boxes.size()) throw std::invalid_argument("split_launches: one box per piece expected");
  std::vector<int> sizes;
  size_t start = 0;
  Box tmp;
  for (size_t i = 0; i < dst.size(); ++i) {
    bool clash = false;
    if (!boxes[i].empty()) {
      for (size_t j = start; j < i && !clash; ++j)
        clash = dst[j] == dst[i] && !boxes[j].empty() && box_intersect(boxes[j], boxes[i], tmp);
    }
    if (clash || (int)(i - start) == max_per_launch) {
      sizes.push_back((int)(i - start));
      start = i;
    }
  }
  if (start < dst.size()) sizes.push_back((int)(dst.size() - start));
  return sizes;
}

}  // namespace flexmi
