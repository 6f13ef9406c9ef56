// Native batch loader: a ring of host staging slots filled by worker threads.
//
// Reference: every shard of every input ran a GPU task that gathered its sample indices from
// the zero-copy full dataset into a buffer and copied it to the GPU (SingleDataLoader
// load_input_2d/4d, python/flexflow_dataloader.cu:97-150; DLRM dlrm.cu:19-122).  Here the
// gather runs on host threads ahead of the training loop: batch n lands in slot n % depth
// (pinned memory owned by the caller), the consumer takes slots strictly in batch order and
// issues one async H2D copy per input, and releases the slot once that copy has completed.
// Each rank gathers only ITS rows/columns of every input (the tensor's home shard box).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>

namespace flexmi {

struct LoaderSource {
  const char* base = nullptr;   // full dataset, row-major [rows, row_bytes]
  int64_t rows = 0;
  int64_t row_bytes = 0;
  int64_t col_off = 0;          // byte offset of this rank's column block inside a row
  int64_t col_bytes = 0;        // bytes copied per row
  int64_t row_lo = 0, row_hi = 0;  // this rank's rows of every batch
  int64_t dst_pitch = 0;        // staging row pitch >= col_bytes (wider: zero-padded tensor rows)
  std::vector<char*> slot_ptr;  // staging buffer per slot: [shard_rows, dst_pitch]
};

class BatchRing {
 public:
  // batch: global batch rows; num_samples: dataset rows used per epoch (whole batches only)
  BatchRing(int64_t batch, int64_t num_samples, int depth, int threads, bool shuffle, uint64_t seed);
  ~BatchRing();

  // [row_lo, row_hi): the rows of every batch this rank holds for the source (its shard box)
  int add_source(const void* base, int64_t rows, int64_t row_bytes, int64_t col_off, int64_t col_bytes,
                 int64_t row_lo, int64_t row_hi, int64_t dst_pitch = -1);
  void set_slot(int source, int slot, void* ptr);
  void start();                 // spawn workers (sources and slots must be complete)
  void stop();                  // join workers; the ring can be start()ed again (from batch 0)
  int acquire();                // blocks until the next batch (in order) is staged; returns its slot
  void release(int slot);       // oldest acquired slot may be refilled (several may be held)
  int64_t batches_per_epoch() const { return bpe_; }
  int64_t consumed() const { return next_consume_; }
  int depth() const { return depth_; }
  // sample ids of all rows of batch n -- used by tests to check the gather
  std::vector<int64_t> batch_ids(int64_t n) const;

 private:
  enum State { FREE = 0, FILLING = 1, READY = 2 };
  void worker();
  void fill(int slot, int64_t n);
  const std::vector<int64_t>& perm_for_epoch(int64_t epoch);

  int64_t batch_, num_samples_, bpe_;
  int depth_, nthreads_;
  bool shuffle_;
  uint64_t seed_;
  std::vector<LoaderSource> src_;
  std::vector<int> state_;
  std::vector<int64_t> slot_batch_;
  int64_t next_claim_ = 0, next_consume_ = 0, next_acquire_ = 0;  // filled / released / handed out
  bool stopping_ = false;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_;
  // epoch permutations (shuffle): computed lazily, two kept
  mutable std::mutex perm_mu_;
  int64_t perm_epoch_[2] = {-1, -1};
  std::vector<int64_t> perm_[2];
};

}  // namespace flexmi
