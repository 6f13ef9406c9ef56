// Image input pipeline on the GPU: decoded uint8 RGB batches (NHWC, as a JPEG/PNG decoder and
// the host resize produce them) -> normalized NCHW fp32 / bf16 network input in ONE pass:
//   out[n][c][y][x] = (src[n][y][x][c] / 256 - mean[c]) / std[c]
// The layout change (HWC -> CHW) is fused into the normalization, so the host never transposes
// and the device reads each decoded byte once.  Reference: apply_normalize +
// UtilityTasks::normalize_images_task (src/runtime/model.cu:151-164, same constants and the same
// /256 scaling), whose input is the CHW copy the CPU nearest_neighbor resize writes (:56-74).
//
// One thread per group of 4 consecutive x positions of one (n, y) row: a 12-byte gather of the
// 4 RGB triples (3 aligned 4-byte loads when W % 4 == 0) and three 4-wide stores, one per channel
// plane (16 B fp32 / 8 B bf16).  Memory bound: 3 B read + 12 B (fp32) written per pixel.
#include "common.h"

namespace {

template <typename T>
__global__ void __launch_bounds__(256) fm_image_normalize_kernel(const unsigned char* __restrict__ src, T* __restrict__ dst,
                                                                long N, int H, int W, float m0, float m1, float m2,
                                                                float is0, float is1, float is2) {
  const int WQ = (W + 3) / 4;
  const long total = N * H * (long)WQ;
  const long plane = (long)H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int xq = (int)(i % WQ);
    const long ny = i / WQ;
    const int y = (int)(ny % H);
    const long n = ny / H;
    const int x0 = 4 * xq;
    const unsigned char* s = src + (ny * W + x0) * 3;
    float v[3][4];
    if (x0 + 3 < W && (W & 3) == 0) {
      const unsigned int* s4 = reinterpret_cast<const unsigned int*>(s);   // 12 bytes, 4-B aligned
      unsigned int w[3] = {s4[0], s4[1], s4[2]};
#pragma unroll
      for (int k = 0; k < 12; ++k) v[k % 3][k / 3] = (float)((w[k / 4] >> (8 * (k % 4))) & 0xffu);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c][e] = (x0 + e < W) ? (float)s[3 * e + c] : 0.f;
    }
    const float mean[3] = {m0, m1, m2}, istd[3] = {is0, is1, is2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      T* d = dst + (n * 3 + c) * plane + (long)y * W + x0;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (x0 + e < W) d[e] = fromf<T>((v[c][e] * (1.f / 256.f) - mean[c]) * istd[c]);
    }
  }
}

}  // namespace

// src: uint8 [N][H][W][3]; dst: [N][3][H][W] fp32 (bf16 = 0) or bf16 (bf16 = 1)
extern "C" void fm_image_normalize(const unsigned char* src, void* dst, long N, int H, int W, const float* mean,
                                   const float* stdv, int bf16, hipStream_t s) {
  const long total = N * H * (long)((W + 3) / 4);
  if (total <= 0) return;
  const unsigned grid = (unsigned)fm_grid(total);
  if (bf16)
    hipLaunchKernelGGL(fm_image_normalize_kernel<unsigned short>, dim3(grid), dim3(256), 0, s, src, (unsigned short*)dst, N,
                       H, W, mean[0], mean[1], mean[2], 1.f / stdv[0], 1.f / stdv[1], 1.f / stdv[2]);
  else
    hipLaunchKernelGGL(fm_image_normalize_kernel<float>, dim3(grid), dim3(256), 0, s, src, (float*)dst, N, H, W, mean[0],
                       mean[1], mean[2], 1.f / stdv[0], 1.f / stdv[1], 1.f / stdv[2]);
}
