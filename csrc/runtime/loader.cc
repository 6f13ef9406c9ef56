// Native batch loader ring (see loader.h).
#include "loader.h"

#include <algorithm>
#include <cstring>
#include <numeric>
#include <random>
#include <stdexcept>

namespace flexmi {

BatchRing::BatchRing(int64_t batch, int64_t num_samples, int depth, int threads, bool shuffle, uint64_t seed)
    : batch_(batch), num_samples_(num_samples), depth_(depth), nthreads_(threads), shuffle_(shuffle), seed_(seed) {
  if (batch <= 0) throw std::invalid_argument("bad batch");
  if (depth < 2) throw std::invalid_argument("depth must be >= 2");
  bpe_ = num_samples / batch;
  if (bpe_ <= 0) throw std::invalid_argument("num_samples < batch");
  state_.assign(depth, FREE);
  slot_batch_.assign(depth, -1);
}

BatchRing::~BatchRing() { stop(); }

int BatchRing::add_source(const void* base, int64_t rows, int64_t row_bytes, int64_t col_off, int64_t col_bytes,
                          int64_t row_lo, int64_t row_hi, int64_t dst_pitch) {
  if (row_lo < 0 || row_hi > batch_ || row_lo > row_hi) throw std::invalid_argument("bad shard rows");
  if (!threads_.empty()) throw std::logic_error("add_source after start");
  if (rows < num_samples_) throw std::invalid_argument("source has fewer rows than num_samples");
  if (col_off < 0 || col_bytes < 0 || col_off + col_bytes > row_bytes) throw std::invalid_argument("bad column block");
  if (dst_pitch < 0) dst_pitch = col_bytes;
  if (dst_pitch < col_bytes) throw std::invalid_argument("staging pitch narrower than the column block");
  LoaderSource s;
  s.base = static_cast<const char*>(base);
  s.rows = rows;
  s.row_bytes = row_bytes;
  s.col_off = col_off;
  s.col_bytes = col_bytes;
  s.row_lo = row_lo;
  s.row_hi = row_hi;
  s.dst_pitch = dst_pitch;
  s.slot_ptr.assign(depth_, nullptr);
  src_.push_back(s);
  return (int)src_.size() - 1;
}

void BatchRing::set_slot(int source, int slot, void* ptr) {
  src_.at(source).slot_ptr.at(slot) = static_cast<char*>(ptr);
}

const std::vector<int64_t>& BatchRing::perm_for_epoch(int64_t epoch) {
  // caller holds perm_mu_
  int k = (int)(epoch & 1);
  if (perm_epoch_[k] != epoch) {
    auto& p = perm_[k];
    p.resize(num_samples_);
    std::iota(p.begin(), p.end(), 0);
    std::mt19937_64 rng(seed_ * 0x9E3779B97F4A7C15ull + (uint64_t)epoch);
    std::shuffle(p.begin(), p.end(), rng);
    perm_epoch_[k] = epoch;
  }
  return perm_[k];
}

std::vector<int64_t> BatchRing::batch_ids(int64_t n) const {
  int64_t epoch = n / bpe_, b = n % bpe_;
  std::vector<int64_t> ids(batch_);
  if (!shuffle_) {
    for (int64_t i = 0; i < batch_; ++i) ids[i] = b * batch_ + i;
  } else {
    std::lock_guard<std::mutex> g(perm_mu_);
    auto& p = const_cast<BatchRing*>(this)->perm_for_epoch(epoch);
    for (int64_t i = 0; i < batch_; ++i) ids[i] = p[b * batch_ + i];
  }
  return ids;
}

void BatchRing::fill(int slot, int64_t n) {
  const std::vector<int64_t> ids = batch_ids(n);
  for (auto& s : src_) {
    char* dst = s.slot_ptr[slot];
    const int64_t nr = s.row_hi - s.row_lo;
    if (nr == 0) continue;
    const int64_t* id = ids.data() + s.row_lo;
    if (!shuffle_ && s.col_off == 0 && s.col_bytes == s.row_bytes && s.dst_pitch == s.col_bytes) {  // one block
      std::memcpy(dst, s.base + id[0] * s.row_bytes, (size_t)(nr * s.row_bytes));
      continue;
    }
    for (int64_t r = 0; r < nr; ++r)
      std::memcpy(dst + r * s.dst_pitch, s.base + id[r] * s.row_bytes + s.col_off, (size_t)s.col_bytes);
  }
}

void BatchRing::worker() {
  for (;;) {
    int64_t n;
    int slot;
    {
      std::unique_lock<std::mutex> lk(mu_);
      n = next_claim_++;
      slot = (int)(n % depth_);
      // the slot is reusable once batch n - depth has been consumed and released
      cv_.wait(lk, [&] { return stopping_ || (state_[slot] == FREE && n - depth_ < next_consume_); });
      if (stopping_) return;
      state_[slot] = FILLING;
      slot_batch_[slot] = n;
    }
    fill(slot, n);
    {
      std::lock_guard<std::mutex> lk(mu_);
      state_[slot] = READY;
    }
    cv_.notify_all();
  }
}

void BatchRing::start() {
  if (!threads_.empty()) return;
  for (auto& s : src_)
    for (auto* p : s.slot_ptr)
      if (!p) throw std::logic_error("start(): a slot buffer is not set");
  {
    std::lock_guard<std::mutex> lk(mu_);
    stopping_ = false;
    next_claim_ = next_consume_ = next_acquire_ = 0;
    std::fill(state_.begin(), state_.end(), (int)FREE);
    std::fill(slot_batch_.begin(), slot_batch_.end(), -1);
  }
  for (int i = 0; i < std::max(1, nthreads_); ++i) threads_.emplace_back([this] { worker(); });
}

void BatchRing::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stopping_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
  threads_.clear();
}

int BatchRing::acquire() {
  std::unique_lock<std::mutex> lk(mu_);
  if (threads_.empty()) throw std::logic_error("acquire() before start()");
  const int64_t n = next_acquire_;
  const int slot = (int)(n % depth_);
  cv_.wait(lk, [&] { return state_[slot] == READY && slot_batch_[slot] == n; });
  ++next_acquire_;
  return slot;
}

void BatchRing::release(int slot) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (state_.at(slot) != READY || slot_batch_[slot] != next_consume_)
      throw std::logic_error("release(): slots must be released in acquisition order");
    state_[slot] = FREE;
    ++next_consume_;
  }
  cv_.notify_all();
}

}  // namespace flexmi
