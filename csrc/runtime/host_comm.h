// flexmi host communicator: the collectives of the native model's CPU engine across PROCESSES
// (one per rank) without MPI, gloo or Python -- a file-backed shared mapping in the rendezvous
// directory, one staging slot per rank and a sense-reversing barrier on lock-free atomics.
//
// The reference moved every inter-device byte through Legion/Realm DMA; the
// native model issues explicit collectives instead (RCCL on the HIP engine).  This is the CPU
// engine's equivalent, used to run multi-rank plans (table-wise embeddings + data-parallel MLPs)
// in a C program on a host without GPUs:
//   * all_reduce_sum: every rank publishes its buffer, every rank sums the R slots in RANK ORDER
//     (identical fp32 operations everywhere -> bit-identical replicas);
//   * all_to_all: per-peer chunks, contiguous by peer in the send / receive buffers.
// Rendezvous: rank 0 creates <dir>/host_comm.shm, sizes it and publishes a ready word; the others
// map it once the word is set.  Every wait is bounded (60 s) and throws on timeout.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>

namespace flexmi {

class HostComm {
 public:
  // slot_bytes: the largest buffer any collective stages per rank (all_to_all: the whole send
  // buffer; all_reduce is chunked to it)
  HostComm(const std::string& dir, int rank, int world, size_t slot_bytes);
  ~HostComm();
  HostComm(const HostComm&) = delete;
  HostComm& operator=(const HostComm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  void barrier();
  void all_reduce_sum(float* buf, int64_t n);
  // send[sum(send_counts)] in peer order -> recv[sum(recv_counts)] in peer order (float counts)
  void all_to_all(const float* send, const int64_t* send_counts, float* recv, const int64_t* recv_counts);

 private:
  struct Header {
    std::atomic<uint32_t> ready;
    std::atomic<uint32_t> arrived;
    std::atomic<uint32_t> generation;
    uint32_t world;
    uint64_t slot_bytes;
    uint64_t token;      // per-run session token (session_token()): a stale region never matches
  };
  char* slot(int r) const { return base_ + header_bytes_ + (size_t)r * slot_bytes_; }

  int rank_, world_;
  size_t slot_bytes_, header_bytes_ = 256, map_bytes_ = 0;
  std::string path_;
  int fd_ = -1;
  char* base_ = nullptr;
  Header* hdr_ = nullptr;
};

}  // namespace flexmi
