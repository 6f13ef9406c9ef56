// flexmi host communicator (see host_comm.h).
#include "host_comm.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <stdexcept>
#include <thread>
#include <vector>

namespace flexmi {

namespace {
constexpr uint32_t kReady = 0x464d4843u;   // "FMHC"
constexpr auto kTimeout = std::chrono::seconds(60);

void fail(const std::string& what) { throw std::runtime_error("host comm: " + what); }

// Session token shared by every rank of one run and (almost surely) different between runs: FNV-1a
// of FM_RUN_ID, else the torch.distributed launcher's TORCHELASTIC_RUN_ID + MASTER_PORT; 0 when
// none is set (then only world / slot size / the unlink by rank 0 guard against a stale region).
uint64_t session_token() {
  std::string key;
  for (const char* v : {"FM_RUN_ID", "TORCHELASTIC_RUN_ID", "MASTER_PORT"}) {
    const char* e = std::getenv(v);
    if (e) {
      key += e;
      key += '|';
    }
  }
  if (key.empty()) return 0;
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : key) h = (h ^ c) * 1099511628211ull;
  return h;
}
}  // namespace

HostComm::HostComm(const std::string& dir, int rank, int world, size_t slot_bytes)
    : rank_(rank), world_(world), slot_bytes_((slot_bytes + 255) / 256 * 256) {
  if (world < 1 || rank < 0 || rank >= world) fail("bad rank / world");
  if (dir.empty()) fail("world > 1 needs a rendezvous directory");
  if (slot_bytes_ == 0) slot_bytes_ = 256;
  path_ = dir + "/host_comm.shm";
  map_bytes_ = header_bytes_ + (size_t)world * slot_bytes_;
  const uint64_t token = session_token();
  if (rank == 0) {
    // a region left by a crashed run goes first, then initialise under a temporary name and
    // rename: peers never map a half-built region; the session token in the header keeps a peer
    // that raced ahead of this unlink from accepting a stale region of the same world / slot size
    ::unlink(path_.c_str());
    const std::string tmp = path_ + ".tmp";
    fd_ = ::open(tmp.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
    if (fd_ < 0) fail("create " + tmp);
    if (::ftruncate(fd_, (off_t)map_bytes_) != 0) fail("size " + tmp);
    void* p = ::mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (p == MAP_FAILED) fail("map " + tmp);
    base_ = static_cast<char*>(p);
    hdr_ = new (base_) Header();
    hdr_->arrived.store(0);
    hdr_->generation.store(0);
    hdr_->world = (uint32_t)world;
    hdr_->slot_bytes = slot_bytes_;
    hdr_->token = token;
    hdr_->ready.store(kReady, std::memory_order_release);
    if (::rename(tmp.c_str(), path_.c_str()) != 0) fail("publish " + path_);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    while (true) {
      fd_ = ::open(path_.c_str(), O_RDWR);
      if (fd_ >= 0) {
        struct stat st;
        if (::fstat(fd_, &st) == 0 && (size_t)st.st_size >= header_bytes_) {
          void* p = ::mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
          if (p != MAP_FAILED) {
            auto* h = reinterpret_cast<Header*>(p);
            if (h->ready.load(std::memory_order_acquire) == kReady && h->world == (uint32_t)world &&
                h->slot_bytes == slot_bytes_ && h->token == token && (size_t)st.st_size == map_bytes_) {
              base_ = static_cast<char*>(p);
              hdr_ = h;
              break;
            }
            ::munmap(p, (size_t)st.st_size);
          }
        }
        ::close(fd_);
        fd_ = -1;
      }
      if (std::chrono::steady_clock::now() - t0 > kTimeout) fail("no communicator from rank 0 at " + path_);
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  }
  barrier();   // everyone mapped
}

HostComm::~HostComm() {
  if (!hdr_) return;
  try {
    barrier();   // nobody still reads a peer slot
  } catch (...) {
  }
  ::munmap(base_, map_bytes_);
  if (fd_ >= 0) ::close(fd_);
  if (rank_ == 0) ::unlink(path_.c_str());
}

void HostComm::barrier() {
  if (world_ == 1) return;
  const uint32_t gen = hdr_->generation.load(std::memory_order_acquire);
  if (hdr_->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)world_) {
    hdr_->arrived.store(0, std::memory_order_relaxed);
    hdr_->generation.fetch_add(1, std::memory_order_acq_rel);   // releases every slot write
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  while (hdr_->generation.load(std::memory_order_acquire) == gen) {
    if (++spins > 1000) {
      std::this_thread::yield();
      if ((spins & 1023) == 0 && std::chrono::steady_clock::now() - t0 > kTimeout) fail("barrier timed out");
    }
  }
}

void HostComm::all_reduce_sum(float* buf, int64_t n) {
  if (world_ == 1 || n <= 0) return;
  const int64_t chunk = (int64_t)(slot_bytes_ / sizeof(float));
  for (int64_t c0 = 0; c0 < n; c0 += chunk) {
    const int64_t len = std::min<int64_t>(chunk, n - c0);
    std::memcpy(slot(rank_), buf + c0, (size_t)len * sizeof(float));
    barrier();
    std::vector<const float*> s(world_);
    for (int r = 0; r < world_; ++r) s[r] = reinterpret_cast<const float*>(slot(r));
    for (int64_t i = 0; i < len; ++i) {
      float v = s[0][i];
      for (int r = 1; r < world_; ++r) v += s[r][i];   // rank order on every rank
      buf[c0 + i] = v;
    }
    barrier();
  }
}

void HostComm::all_to_all(const float* send, const int64_t* send_counts, float* recv, const int64_t* recv_counts) {
  // slot layout: [this rank's send counts: world int64, padded to 256 B][send chunks by peer]
  const size_t cbytes = ((size_t)world_ * sizeof(int64_t) + 255) / 256 * 256;
  int64_t total = 0;
  for (int r = 0; r < world_; ++r) total += send_counts[r];
  if (cbytes + (size_t)total * sizeof(float) > slot_bytes_) fail("all_to_all send buffer exceeds the staging slot");
  std::memcpy(slot(rank_), send_counts, (size_t)world_ * sizeof(int64_t));
  std::memcpy(slot(rank_) + cbytes, send, (size_t)total * sizeof(float));
  barrier();
  int64_t out = 0;
  for (int p = 0; p < world_; ++p) {
    const int64_t* pc = reinterpret_cast<const int64_t*>(slot(p));
    if (pc[rank_] != recv_counts[p]) fail("all_to_all: peer " + std::to_string(p) + " sends a different count");
    int64_t off = 0;
    for (int r = 0; r < rank_; ++r) off += pc[r];
    std::memcpy(recv + out, reinterpret_cast<const float*>(slot(p) + cbytes) + off, (size_t)pc[rank_] * sizeof(float));
    out += pc[rank_];
  }
  barrier();
}

}  // namespace flexmi
