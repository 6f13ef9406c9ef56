// Lab for the multi-plane DMA GEMM main loop (csrc/kernels/gemm_mp.h): times block / wave tile /
// stage-count variants on the DLRM shapes, bf16 (NP = 1) and split-fp32 planes (NP = 3), and checks
// sampled outputs against a float64 host reference of the same operands.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/kernels tools/gemm_mp_lab.hip -o tools/bin/gemm_mp_lab
// Prints one JSON line per variant.
#include "gemm_mp.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <int BM, int BN, int NP, bool AK, bool BKC, int WM, int WN, int ST, int LAB>
__global__ void __launch_bounds__(WM * WN * 64, 1) lab_kernel(mp::Opnds o, float* C, int M, int N, int K, int tiles_m,
                                                             int tiles_n, int ksplit, long long* stamps) {
  using L = mp::Loop<BM, BN, NP, AK, BKC, WM, WN, ST, LAB>;
  const long long t0 = stamps ? __builtin_amdgcn_s_memtime() : 0;
  long long* st = stamps ? stamps + ((long)(blockIdx.z * gridDim.x + blockIdx.x) * (WM * WN) + (threadIdx.x >> 6)) * 5 : nullptr;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int tm, tn;
  if (M >= N) { tn = bid % tiles_n; tm = bid / tiles_n; }
  else { tm = bid % tiles_m; tn = bid / tiles_m; }
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = K / L::BK;
  const int per = (ktiles + ksplit - 1) / ksplit;
  const int kt0 = blockIdx.z * per, kt1 = min(ktiles, kt0 + per);
  f32x4_t acc[L::MR][L::NR];
  L::run(o, m0, n0, kt0, kt1, smem, acc, st ? st + 1 : nullptr);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  float* Cz = C + (long)blockIdx.z * M * N;
#pragma unroll
  for (int i = 0; i < L::MR; ++i)
#pragma unroll
    for (int j = 0; j < L::NR; ++j) {
      const int m = m0 + wm * L::TM + 16 * i + (lane & 15);
      const int n = n0 + wn * L::TN + 16 * j + 4 * (lane >> 4);
      *reinterpret_cast<f32x4_t*>(Cz + (long)m * N + n) = acc[i][j];
    }
  if (st && lane == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st[0] = t0;
    st[4] = __builtin_amdgcn_s_memtime();
  }
}

__global__ void reduce_k(const float* ws, float* C, long MN, int ks) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < MN / 4; i += (long)gridDim.x * blockDim.x) {
    f32x4_t s = slab_sum4(ws + i * 4, MN, ks);
    *reinterpret_cast<f32x4_t*>(C + i * 4) = s;
  }
}

static unsigned short bf_trunc(float x) {
  unsigned u;
  memcpy(&u, &x, 4);
  return (unsigned short)(u >> 16);
}
static float bf_to_f(unsigned short h) {
  unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static unsigned short bf_rne(float x) {
  unsigned u;
  memcpy(&u, &x, 4);
  return (unsigned short)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

// host split x = h + m + l by truncation
static void split3(float x, unsigned short& h, unsigned short& m, unsigned short& l) {
  h = bf_trunc(x);
  float r = x - bf_to_f(h);
  m = bf_trunc(r);
  float r2 = r - bf_to_f(m);
  l = bf_trunc(r2);
}

struct Buf {
  std::vector<float> f;               // fp32 values (NP = 3) or bf16 values as float (NP = 1)
  unsigned short* d = nullptr;        // NP planes on device
  long plane = 0;
};

static Buf make(long elems, int NP, unsigned seed) {
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  Buf b;
  b.f.resize(elems);
  std::vector<unsigned short> h(elems * NP);
  for (long i = 0; i < elems; ++i) {
    float x = U(g);
    if (NP == 1) {
      h[i] = bf_rne(x);
      b.f[i] = bf_to_f(h[i]);
    } else {
      b.f[i] = x;
      split3(x, h[i], h[elems + i], h[2 * elems + i]);
    }
  }
  b.plane = elems;
  CK(hipMalloc(&b.d, elems * NP * 2));
  CK(hipMemcpy(b.d, h.data(), elems * NP * 2, hipMemcpyHostToDevice));
  return b;
}

struct Shape {
  const char* name;
  int M, N, K;
  bool ak, bk;
};

template <int BM, int BN, int NP, bool AK, bool BKC, int WM, int WN, int ST, int LAB = 0>
void run(const char* vname, const Shape& s, int ksplit, int reps) {
  using L = mp::Loop<BM, BN, NP, AK, BKC, WM, WN, ST, LAB>;
  const int M = s.M, N = s.N, K = s.K;
  if (M % BM || N % BN || K % (L::BK * ksplit)) {
    printf("{\"variant\": \"%s\", \"shape\": \"%s\", \"skip\": \"shape\"}\n", vname, s.name);
    return;
  }
  Buf A = make((long)M * K, NP, 1), B = make((long)N * K, NP, 2);
  float *C, *ws = nullptr;
  CK(hipMalloc(&C, (long)M * N * 4));
  if (ksplit > 1) CK(hipMalloc(&ws, (long)M * N * 4 * ksplit));
  mp::Opnds o;
  o.A = A.d; o.lda = AK ? K : M; o.sA = 0; o.sAp = A.plane;
  o.B = B.d; o.ldb = BKC ? K : N; o.sB = 0; o.sBp = B.plane;
  const int tiles_m = M / BM, tiles_n = N / BN;
  dim3 grid(tiles_m * tiles_n, 1, ksplit);
  auto kern = lab_kernel<BM, BN, NP, AK, BKC, WM, WN, ST, LAB>;
  long long* stamps = nullptr;
  const long nst = (long)grid.x * grid.z * L::NW * 5;
  CK(hipMalloc(&stamps, nst * 8));
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, L::LDS));
  auto launch = [&](long long* sp = nullptr) {
    hipLaunchKernelGGL(kern, grid, dim3(L::NTH), L::LDS, 0, o, ksplit > 1 ? ws : C, M, N, K, tiles_m, tiles_n, ksplit, sp);
    if (ksplit > 1) hipLaunchKernelGGL(reduce_k, dim3(1024), dim3(256), 0, 0, ws, C, (long)M * N, ksplit);
  };
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  // one stamped launch: cycles per phase (wave means) and the clock they imply
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, grid, dim3(L::NTH), L::LDS, 0, o, ksplit > 1 ? ws : C, M, N, K, tiles_m, tiles_n, ksplit, stamps);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms1;
  CK(hipEventElapsedTime(&ms1, e0, e1));
  std::vector<long long> hs(nst);
  CK(hipMemcpy(hs.data(), stamps, nst * 8, hipMemcpyDeviceToHost));
  double pro = 0, loop = 0, wait = 0, epi = 0;
  long long tmin = hs[0], tmax = hs[4];
  const long nw = nst / 5;
  for (long w = 0; w < nw; ++w) {
    const long long* q = &hs[w * 5];
    pro += q[1] - q[0];
    loop += q[2] - q[1];
    wait += q[3];
    epi += q[4] - q[2];
    tmin = q[0] < tmin ? q[0] : tmin;
    tmax = q[4] > tmax ? q[4] : tmax;
  }
  pro /= nw; loop /= nw; wait /= nw; epi /= nw;
  CK(hipFree(stamps));
  std::vector<float> hc((long)M * N);
  CK(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
  // sampled float64 check: err / sum |a b|
  std::mt19937 g(7);
  double worst = 0;
  for (int t = 0; t < 256; ++t) {
    const int m = g() % M, n = g() % N;
    double ref = 0, mag = 0;
    for (int k = 0; k < K; ++k) {
      const double a = AK ? A.f[(long)m * K + k] : A.f[(long)k * M + m];
      const double b = BKC ? B.f[(long)n * K + k] : B.f[(long)k * N + n];
      ref += a * b;
      mag += fabs(a * b);
    }
    worst = fmax(worst, fabs(hc[(long)m * N + n] - ref) / mag);
  }
  const double fl = 2.0 * M * N * K;
  printf("{\"variant\": \"%s\", \"shape\": \"%s\", \"NP\": %d, \"ksplit\": %d, \"lab\": %d, \"us\": %.2f, \"TF\": %.1f, "
         "\"mfma_PF\": %.3f, \"rel_err\": %.3g, \"grid\": %d, \"cyc_pro\": %.0f, \"cyc_loop\": %.0f, \"cyc_wait\": %.0f, "
         "\"cyc_epi\": %.0f, \"cyc_span\": %lld, \"stamped_us\": %.2f, \"ideal_loop_cyc\": %.0f}\n",
         vname, s.name, NP, ksplit, LAB, us, fl / us / 1e6, fl * (NP == 1 ? 1 : 6) / us / 1e9, worst,
         tiles_m * tiles_n * ksplit, pro, loop, wait, epi, tmax - tmin, ms1 * 1e3,
         (double)BM * BN * (K / ksplit) * 2 * (NP == 1 ? 1 : 6) / 4096.0);
  fflush(stdout);
  CK(hipFree(A.d));
  CK(hipFree(B.d));
  CK(hipFree(C));
  if (ws) CK(hipFree(ws));
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const Shape fwd{"fwd_8192x1024x1024", 8192, 1024, 1024, true, true};
  const Shape dx{"dx_8192x1024x1024", 8192, 1024, 1024, true, false};
  const Shape dw{"dw_1024x1024x8192", 1024, 1024, 8192, false, false};
  const Shape f512{"fwd_8192x512x1024", 8192, 512, 1024, true, true};
  run<256, 128, 1, true, true, 4, 2, 2>("bf16_256x128_w64x64_s2", fwd, 1, reps);
  run<256, 128, 1, true, true, 4, 2, 2, 1>("bf16_256x128_w64x64_s2", fwd, 1, reps);
  run<256, 128, 1, true, true, 4, 2, 2, 2>("bf16_256x128_w64x64_s2", fwd, 1, reps);
  run<128, 128, 1, true, true, 2, 2, 2>("bf16_128x128_w64x64_s2", fwd, 1, reps);
  run<128, 128, 1, true, true, 2, 2, 2, 1>("bf16_128x128_w64x64_s2", fwd, 1, reps);
  run<256, 128, 3, true, true, 4, 2, 2>("x3_256x128_w64x64_s2", fwd, 1, reps);
  run<256, 128, 3, true, true, 4, 2, 2, 1>("x3_256x128_w64x64_s2", fwd, 1, reps);
  run<256, 128, 3, true, true, 4, 2, 2, 2>("x3_256x128_w64x64_s2", fwd, 1, reps);
  run<256, 128, 3, true, true, 2, 2, 2>("x3_256x128_w128x64_s2", fwd, 1, reps);
  run<256, 128, 3, true, true, 2, 2, 2, 1>("x3_256x128_w128x64_s2", fwd, 1, reps);
  return 0;
}
