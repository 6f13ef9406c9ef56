// Split-K reduce OFF the critical path (bf16 gemm.hip and fp32 gemm_f32.hip).
//
// A split-K GEMM writes per-slice fp32 slabs and a memory-bound reduce launch sums them into C.
// In a training step the split-K GEMMs are the weight-gradient GEMMs (dW: K = batch), and what
// follows each one on the stream is the compute-bound input-gradient GEMM of the same layer,
// which does not read dW.  When the caller arms it (the executor, for dW GEMMs whose gradient
// is read only by the optimizer / the gradient all-reduce), the reduce is issued on a SIDE
// stream forked from the GEMM (event), so it co-resides with the next GEMM's blocks (it needs no
// LDS and few registers) instead of serialising behind it.  A round-1 alternative -- every tile's
// last-arriving block summing the other slices in-launch -- measured SLOWER than the reduce
// launch (profiles/README.md: the last arriver reads the slabs serially at the cross-XCD rate).
//
// Ordering rules (the host functions below):
//   * fork:  the reduce waits for its GEMM (event on the GEMM's stream);
//   * guard: any later GEMM that writes the shared slab workspace (split-K) or accumulates into
//     its output (beta) first joins a pending reduce -- the slabs are reused, and a beta GEMM may
//     target the reduced gradient;
//   * join:  the caller joins before anything reads the gradients (bucket all-reduce, update) and
//     before every graph-segment boundary, so a captured fork is always joined inside its capture.
// The side stream and events are created on the first armed call outside a capture (the
// executor's eager warm-up step); a capture before that keeps the reduce on the GEMM's stream.
// OPT-IN (FM_GEMM_ASYNC_REDUCE=1 arms the executor's dW GEMMs): measured slower on the DLRM step
// (profiles/bench_ab_async_reduce_r3h.txt) -- the captured reduce still ran ahead of the next GEMM
// and the cross-stream edges added gaps to the replay.
#include <hip/hip_runtime.h>

#include <cstdlib>

namespace {

struct AsyncReduce {
  hipStream_t side = nullptr;
  hipEvent_t ev_in = nullptr, ev_done = nullptr;
  bool pending = false;
};
constexpr int MAXDEV = 64;
AsyncReduce g_ar[MAXDEV];
thread_local int g_armed = 0;

bool enabled() {   // FM_GEMM_ASYNC_REDUCE=0 also refuses armed calls of other callers
  static const bool on = !(getenv("FM_GEMM_ASYNC_REDUCE") != nullptr && atoi(getenv("FM_GEMM_ASYNC_REDUCE")) == 0);
  return on;
}

AsyncReduce* device_state() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXDEV) return nullptr;
  return &g_ar[dev];
}

}  // namespace

// arm (1) / disarm (0) the async reduce for the split-K GEMM launched next on this thread
extern "C" void fm_gemm_async_arm(int on) { g_armed = on; }

// make stream s wait for a pending async reduce (no-op when none is pending)
extern "C" void fm_gemm_join(hipStream_t s) {
  AsyncReduce* a = device_state();
  if (a == nullptr || !a->pending) return;
  (void)hipStreamWaitEvent(s, a->ev_done, 0);
  a->pending = false;
}

// the stream the reduce of a split-K GEMM just enqueued on s runs on: s itself unless armed
extern "C" hipStream_t fm_gemm_async_fork(hipStream_t s) {
  const int armed = g_armed;
  g_armed = 0;
  if (!armed || !enabled()) return s;
  AsyncReduce* a = device_state();
  if (a == nullptr) return s;
  if (a->side == nullptr) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return s;
    if (hipStreamCreateWithFlags(&a->side, hipStreamNonBlocking) != hipSuccess) {
      a->side = nullptr;
      return s;
    }
    if (hipEventCreateWithFlags(&a->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&a->ev_done, hipEventDisableTiming) != hipSuccess)
      return s;
  }
  if (hipEventRecord(a->ev_in, s) != hipSuccess || hipStreamWaitEvent(a->side, a->ev_in, 0) != hipSuccess) return s;
  return a->side;
}

// after the reduce was enqueued on the side stream returned by fm_gemm_async_fork
extern "C" void fm_gemm_async_forked(hipStream_t side) {
  AsyncReduce* a = device_state();
  if (a == nullptr || side != a->side) return;
  (void)hipEventRecord(a->ev_done, side);
  a->pending = true;
}
