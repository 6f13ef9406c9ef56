// bf16 MFMA pipe probe for gfx950 (MI355X): sustained v_mfma_f32_16x16x32_bf16 rate with operands
// in registers (16 independent accumulators per wave), the ceiling the bf16 and split-fp32 GEMMs
// are priced against.  Also the same stream plus one ds_read_b128 per 4 MFMAs (the split GEMM's
// fragment ratio) to check the LDS read path does not cap the pipe, and with 4 / 2 / 1 independent
// accumulator chains (the MFMA-to-MFMA srcC dependency latency).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_bf16_probe.hip -o tools/bin/mfma_bf16_probe
// Prints one JSON line per (probe, waves per SIMD): TF/s over the whole chip.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <int LDSR, int CH = 16>
__global__ void probe(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) char lds[16384];
  const int lane = threadIdx.x & 63;
  f32x4 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = s16x8{(short)(lane + i), 1, 2, 3, 4, 5, 6, 7};
    b[i] = s16x8{(short)(lane * 3 + i), 7, 6, 5, 4, 3, 2, 1};
  }
  for (int i = threadIdx.x; i < 16384 / 4; i += blockDim.x) reinterpret_cast<int*>(lds)[i] = i;
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (LDSR) {
        a[i] = *reinterpret_cast<const s16x8*>(lds + ((lane * 16 + it * 64 + i * 1024) & 16383));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[(i * 4 + j) % CH] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&a[i]),
                                                                  *reinterpret_cast<const bf16x8*>(&b[j]), acc[(i * 4 + j) % CH], 0,
                                                                  0, 0);
    }
  }
  f32x4 s = acc[0];
#pragma unroll
  for (int i = 1; i < 16; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

template <int LDSR, int CH = 16>
void run(const char* name, int wps, float* out, int iters) {
  dim3 grid(256), block(64 * 4 * wps);
  hipLaunchKernelGGL((probe<LDSR, CH>), grid, block, 0, 0, out, iters);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((probe<LDSR, CH>), grid, block, 0, 0, out, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  const double flops = 256.0 * 4 * wps * (double)iters * 16 * 16 * 16 * 32 * 2;
  printf("{\"probe\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"TF\": %.1f}\n", name, wps, ms, flops / ms / 1e9);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  float* out;
  CHECK(hipMalloc(&out, 256 * 1024 * sizeof(float)));
  for (int wps = 1; wps <= 2; ++wps) {
    run<0>("regs", wps, out, iters);
    run<1>("regs+ds_read", wps, out, iters);
    run<0, 4>("regs,4chains", wps, out, iters);
    run<0, 2>("regs,2chains", wps, out, iters);
    run<0, 1>("regs,1chain", wps, out, iters);
  }
  CHECK(hipFree(out));
  return 0;
}
