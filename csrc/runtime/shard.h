// Sharding algebra of the plan compiler: equal-block partitions, shard boxes, box intersections
// and reshard transfer lists.  This is what Legion did implicitly in the reference -- restriction
// partitions of logical regions (src/runtime/model.cc:457-875) plus the dependence analysis that
// inserted DMA copies between producer and consumer partitions (modelled as intersection copies in
// src/runtime/simulator.cc:295-326).  Here every cross-device byte is an explicit Transfer that the
// executor moves with one RCCL all_to_all per plan step.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace flexmi {

using Range = std::pair<int64_t, int64_t>;   // [lo, hi)
using Box = std::vector<Range>;

// How one logical tensor is distributed: degree per dim (user order, outer -> inner), holder ranks
// per part (row-major part index; >1 holder = replication), optional explicit boxes (overlapping
// halo boxes of spatial splits) and the partial-sum flag of gradient layouts.
struct ShardLayout {
  std::vector<int64_t> shape;
  std::vector<int64_t> degrees;
  std::vector<std::vector<int>> holders;
  std::vector<Box> boxes;   // empty = equal-block boxes from shape/degrees
  bool partial = false;

  int64_t num_parts() const;
  std::vector<int64_t> part_coords(int64_t p) const;
  Box part_box(int64_t p) const;
  void validate() const;   // throws std::invalid_argument
};

struct Transfer {
  int src, dst;
  Box box;           // global coordinates
  int64_t src_part, dst_part;
};

Range split_extent(int64_t n, int64_t d, int64_t k);
bool box_intersect(const Box& a, const Box& b, Box& out);
int64_t box_volume(const Box& b);

// Transfers turning src into dst.  partial src -> full dst: every partial holder contributes
// (sum); otherwise one source holder per destination piece (the destination itself when it
// holds the data, else holders rotate by (dst_part + src_part) to spread the load).  Sorted by
// (src, dst, dst_part, src_part, box) -- the order both ends of an all_to_all pack/unpack in.
std::vector<Transfer> reshard_transfers(const ShardLayout& src, const ShardLayout& dst);

// Split an ordered list of copy pieces into launches in which no two pieces write intersecting
// boxes of the same destination buffer (pieces of one launch run concurrently; partial-sum pieces
// add).  piece i: destination buffer id dst[i], box boxes[i] (empty box = never clashes).
// Returns the launch sizes.
std::vector<int> split_launches(const std::vector<int64_t>& dst, const std::vector<Box>& boxes, int max_per_launch);

}  // namespace flexmi
