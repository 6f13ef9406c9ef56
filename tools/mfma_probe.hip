// fp32 MFMA pipe probe for gfx950 (MI355X): where does an LDS-staged v_mfma_f32_16x16x4_f32 GEMM
// main loop lose issue slots?  Each kernel runs the same per-wave MFMA stream (64x64 wave tile:
// 16 accumulators, 64 MFMAs per 16-deep k-chunk) and adds one ingredient of the real loop:
//   P0 operands in registers only                P1 + fragment reads from LDS (double-buffered)
//   P2 + one s_barrier per 32-deep stage         P3 + 8 LDS-DMA (global_load_lds_dwordx4) per wave
//                                                   per stage, waited two stages later
// run with WPS = 1 (4 waves per block) and 2 (8 waves per block) waves per SIMD, one block per CU.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/bin/mfma_probe
// Prints one JSON line per (kernel, waves per SIMD): TF/s over the whole chip.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const void* gptr;
typedef __attribute__((address_space(3))) void* lptr;

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <int N>
__device__ inline void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ inline void mfma_chunk(f32x4 (&acc)[4][4], const float (&a)[4][4], const float (&b)[4][4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][s], a[i][s], acc[i][j], 0, 0, 0);
}

// fragment reads of one 16-deep chunk from a wave-private [64 rows][32 k] A and B image (swizzled)
__device__ inline void frags(const char* img, int kk, int lane, float (&a)[4][4], float (&b)[4][4]) {
  const int q = lane & 15, g = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int row = 16 * t + q;
    const int c = (4 * kk + g) ^ ((row >> 1) & 7);
    const f32x4 x = *reinterpret_cast<const f32x4*>(img + row * 128 + 16 * c);
    const f32x4 y = *reinterpret_cast<const f32x4*>(img + 8192 + row * 128 + 16 * c);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      a[t][s] = x[s];
      b[t][s] = y[s];
    }
  }
}

template <int P, int NW>
__global__ void __launch_bounds__(NW * 64, 1) probe(const float* __restrict__ src, float* __restrict__ out, int stages,
                                                   long src_floats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int DPW = 32 / NW;                      // DMA KiB per wave per stage (32 KiB per block)
  char* img = smem;                                 // fragment image shared by the waves (A 8 KB + B 8 KB)
  char* dma = smem + 16384;                         // DMA landing area: 32 KiB per slot, 3 slots
  for (int i = threadIdx.x; i < 16384 / 4; i += NW * 64) reinterpret_cast<float*>(img)[i] = src[(blockIdx.x * 977 + i) % src_floats];
  __syncthreads();
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a[2][4][4], b[2][4][4];
  if constexpr (P == 0) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        a[0][t][s] = src[(lane + 64 * (4 * t + s)) % src_floats];
        b[0][t][s] = src[(lane * 3 + 64 * (4 * t + s) + 7) % src_floats];
      }
    for (int st = 0; st < stages; ++st) {
      mfma_chunk(acc, a[0], b[0]);
      mfma_chunk(acc, a[0], b[0]);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    const long per_blk = 3L * 8 * 1024 / 4;         // floats one wave streams per 3 stages
    frags(img, 0, lane, a[0], b[0]);
    for (int st = 0; st < stages; ++st) {
      f32x4 stg[DPW];
      if constexpr (P == 4) {
        // register staging: DPW x 16 B per lane of global_load_dwordx4, stored to LDS after the
        // stage's first chunk (hipBLASLt's fp32 form)
        const long base = ((long)(blockIdx.x * NW + wave) * per_blk + (long)(st % 64) * 2048) % (src_floats - 2048);
#pragma unroll
        for (int i = 0; i < DPW; ++i) stg[i] = *reinterpret_cast<const f32x4*>(src + base + i * 256 + 4 * lane);
      }
      if constexpr (P == 3) {
        // DPW x 1 KiB DMA into this wave's part of slot st % 3 (never read: bandwidth + issue cost)
        char* slot = dma + (st % 3) * 32768 + wave * DPW * 1024;
        const long base = ((long)(blockIdx.x * NW + wave) * per_blk + (long)(st % 64) * 2048) % (src_floats - 2048);
#pragma unroll
        for (int i = 0; i < DPW; ++i)
          __builtin_amdgcn_global_load_lds((gptr)(src + base + i * 256 + 4 * lane), (lptr)(slot + i * 1024), 16, 0, 0);
      }
      frags(img, 1, lane, a[1], b[1]);
      mfma_chunk(acc, a[0], b[0]);
      if constexpr (P == 3) wait_vm<2 * DPW>();
      if constexpr (P == 4) {
        char* slot = dma + (st % 3) * 32768 + wave * DPW * 1024;
#pragma unroll
        for (int i = 0; i < DPW; ++i) *reinterpret_cast<f32x4*>(slot + i * 1024 + 16 * lane) = stg[i];
      }
      if constexpr (P >= 2) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      frags(img, 0, lane, a[0], b[0]);
      mfma_chunk(acc, a[1], b[1]);
    }
    if constexpr (P == 3) wait_vm<0>();
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int P, int NW>
void run(const float* src, float* out, long nsrc, int blocks, int stages, const char* tag = "") {
  const int lds = 16384 + (P >= 3 ? 3 * 32768 : 0);   // P3 / P4: three 32 KiB landing slots
  CHECK(hipFuncSetAttribute((const void*)probe<P, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe<P, NW>), dim3(blocks), dim3(NW * 64), lds, 0, src, out, stages, nsrc);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((probe<P, NW>), dim3(blocks), dim3(NW * 64), lds, 0, src, out, stages, nsrc);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double flop = 2.0 * blocks * NW * (double)stages * 128 * 1024;   // 128 MFMAs of 1024 MAC per stage
  printf("{\"probe\": \"P%d%s\", \"waves_per_simd\": %d, \"blocks\": %d, \"ms\": %.4f, \"TF\": %.1f}\n", P, tag,
         NW / 4, blocks, best, flop / (best * 1e-3) / 1e12);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int stages = argc > 1 ? atoi(argv[1]) : 2000;
  const long nsrc = 64L << 20;   // 256 MB source (beyond L2; the DMA streams it)
  std::vector<float> h(nsrc);
  unsigned x = 12345;
  for (long i = 0; i < nsrc; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = (float)((x >> 8) & 0xffff) / 65536.f - 0.5f;
  }
  float *src, *out;
  CHECK(hipMalloc(&src, nsrc * 4));
  CHECK(hipMalloc(&out, 1024 * 1024 * 4));
  CHECK(hipMemcpy(src, h.data(), nsrc * 4, hipMemcpyHostToDevice));
  const int blocks = 256;
  const long small = 1L << 20;   // 4 MB source: L2-resident streams (the GEMM operand re-read case)
  run<2, 4>(src, out, nsrc, blocks, stages);
  run<3, 4>(src, out, nsrc, blocks, stages, "-hbm");
  run<3, 4>(src, out, small, blocks, stages, "-l2");
  run<4, 4>(src, out, nsrc, blocks, stages, "-hbm");
  run<4, 4>(src, out, small, blocks, stages, "-l2");
  run<2, 8>(src, out, nsrc, blocks, stages / 2);
  run<3, 8>(src, out, nsrc, blocks, stages / 2, "-hbm");
  run<3, 8>(src, out, small, blocks, stages / 2, "-l2");
  run<4, 8>(src, out, nsrc, blocks, stages / 2, "-hbm");
  run<4, 8>(src, out, small, blocks, stages / 2, "-l2");
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
