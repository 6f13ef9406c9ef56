// Descriptor of the embedding sparse-SGD update fused into the fp32 interaction backward
// (csrc/kernels/interaction.hip fm_dot_interaction_bwd_f32_upd); built once per plan on the host
// (csrc/bindings/hip_ops.cpp dot_upd_desc) and read by the kernel from device memory.
#pragma once

constexpr int DOT_UPD_MAXF = 32;

struct DotUpd {
  float* W[DOT_UPD_MAXF];          // table (nullptr: this feature writes dZ as usual)
  const void* idx[DOT_UPD_MAXF];   // [B] lookup indices (bag 1)
  int* slot[DOT_UPD_MAXF];         // count-pass slots (lookups - 1, -1 = free) or nullptr: atomics only
  const int* own[DOT_UPD_MAXF];    // [B] 1 = this lookup arrived first at its row (count pass)
  long lo[DOT_UPD_MAXF];           // first row held by this shard
  int rows[DOT_UPD_MAXF];
  float scale[DOT_UPD_MAXF];
  const float* lr;
  int i64;
};
