// NHWC-staged implicit-GEMM convolution for gfx950 (MI355X / CDNA4), bf16 operands, fp32
// accumulate.  The NCHW kernels (conv_igemm.hip) gather every operand chunk from NCHW with
// per-element index math, halo masks and funnel shifts; PMC on ResNet-50 layers shows them
// instruction-bound (r2 3x3 fwd: ~21 VALU instructions per MFMA, 1x1 fwd 64:1, wgrad heavy on
// SALU; profiles/pmc_conv_nchw_r3l.txt).  This path first re-lays each image operand ONCE into a
// zero-padded NHWC copy ("staging"), after which every 16-B operand chunk of the implicit GEMM is
// 8 consecutive channels at one pixel -- one aligned buffer_load_b128 with no bounds math beyond
// the tile edges:
//
//   staged S[n][i][j][c], i in [0,Hp), j in [0,Wp), c in [0,Cp) (Cp = roundup(C, 8), zeros in the
//   halo, in the channel pad and, for the data gradient, around G)
//   pixel pix = (n, p, q) -> window origin  org(pix) = ((n*Hp + p*sh + oh)*Wp + q*sw + ow) * Cp
//   reduction chunk j of (r, s, c8)  ->  tap(j) = (r*Wp + s) * Cp + 8*c8
//
//   fwd    Y[k][pix]      = sum_{(r,s,c)}  Wf[k][(r,s,c)]  * Xs[org(pix) + tap]         (NCHW Y)
//   dgrad dX[c][pix]      = sum_{(r,s,k)}  Wd[c][(r,s,k)]  * Gs[org(pix) + tap]         (Gs = G
//          placed at (R-1-pt, S-1-pl), dilated by the stride; Wd = W flipped in (r,s) and
//          transposed; NCHW dX.  A stride-s layer multiplies s*s times the useful MACs here.)
//   wgrad dW2[k][(r,s,c)] = sum_pix Gs[orgG(pix) + k] * Xs[orgX(pix) + tap(r,s,c)]     (fp32)
//
// fwd / dgrad: A = weights K-contiguous [M][K] (plain rows), B = gathered pixels K-contiguous
// (the thread's pixel rows are fixed for the whole K loop: origins computed once; a k-tile costs
// one tap() per thread).  wgrad: both operands MN-contiguous (k = pixel rows, channel chunks
// along M / N) -> LDS images [k][R] read with ds_read_b64_tr_b16 like gemm.hip's MN operands.
// MFMA core, LDS images and swizzles are gemm.hip's (gemm_common.h): v_mfma_f32_16x16x32_bf16,
// BM x BN x 64 tiles, register-staged double-buffered LDS, one barrier per k-tile, XCD-aware
// tile order, 8-wave blocks for 128x128 tiles.  Epilogues: fwd bias + activation into NCHW y;
// dgrad (+)= into NCHW dx; wgrad fp32 [K][R*S*Cp] (float atomics across split-K slices), folded
// into dW[K][C][R][S] by fm_cnhwc_wprep mode 2.
// Replaces the reference's cuDNN calls (src/ops/conv_2d.cu:285-296 forward, :405-432 backward).
#include "gemm_common.h"

#include <algorithm>
#include <type_traits>

extern "C" int fm_gemm_dma_enabled();   // gemm_f32.hip

namespace {

constexpr unsigned OOBN = 0x80000000u;   // buffer offset past num_records: the load returns 0

enum { CN_FWD = 0, CN_DGRAD = 1, CN_WGRAD = 2 };

// pixel geometry of one staged operand (pixel = (n, p, q) of the GEMM's pixel index space)
struct PixG {
  FastDiv dPQ, dQ;
  int PQ, Q;
  int Hp, Wp, Cp;
  int sh, sw, oh, ow;
};

// reduction / column taps over (r, s, c8) with c8 fastest
struct TapG {
  FastDiv dC8, dS;
  int C8, S, Wp, Cp;
  int t0, rstep, sstep;   // tap (r, s, c8) at t0 + r*rstep + s*sstep + 8*c8 (a stride-phase sub-kernel
                          // walks every sh-th row / sw-th column of the staged G)
};

struct ConvN {
  const unsigned short* A;  long a_bytes;   // fwd/dgrad: weight matrix [M][K]; wgrad: staged G
  const unsigned short* B;  long b_bytes;   // staged image operand
  void* out;                                // fwd: y (bf16 NCHW); dgrad: dx (bf16 NCHW); wgrad: fp32 [M][N]
  const float* bias;
  int M, N, K;          // GEMM sizes (K = reduction length, a multiple of 8)
  int Mp;               // wgrad: staged channel count of A (loads below Mp read real memory)
  int npix;             // pixels of the pixel index space
  PixG ga, gb;
  TapG tb;
  const int* ptab;      // wgrad: {orgA, orgB} per pixel (fm_pix_table)
  float* db;            // wgrad: bias gradient (+)= sum over pixels of the staged G (may be null)
  FastDiv dOPQ;         // fwd/dgrad output pixels per image
  int OPQ;
  // fwd/dgrad second output: the result also stored straight into a CONSUMER's staged NHWC operand
  // (out2[n][p*d2h + t2][q*d2w + l2][m], rows / columns outside [0,H2) x [0,W2) dropped) so the
  // consumer skips its staging pass; write_nchw = 0 skips the NCHW store when nothing reads it
  unsigned short* out2;
  FastDiv dOQ;          // output pixels per row (p, q split of the output pixel)
  int OQ, H2, W2, C2, t2, l2, d2h, d2w, write_nchw;
  // strided NCHW output (a stride-phase data gradient): pixel (h', w') of the GEMM lands at
  // (o_oh + o_sh*h', o_ow + o_sw*w') of an o_H x o_W plane
  int strided_out, o_sh, o_sw, o_oh, o_ow, o_H, o_W;
  int act, accum, ksplit, kt_per, tiles_m, tiles_n;
};

FM_DEVICE __amdgpu_buffer_rsrc_t rsrc_n(const void* p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

FM_DEVICE u32x4_t ld16(__amdgpu_buffer_rsrc_t rs, bool ok, int elem_off) {
  return __builtin_bit_cast(u32x4_t,
                            __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? (unsigned)elem_off * 2u : OOBN, 0, 0));
}

FM_DEVICE void pix_nqp(const PixG& g, int pix, int& n, int& p, int& q) {
  n = fdiv(pix, g.dPQ);
  const int rem = pix - n * g.PQ;
  p = fdiv(rem, g.dQ);
  q = rem - p * g.Q;
}

FM_DEVICE int pix_org(const PixG& g, int n, int p, int q) {
  return ((n * g.Hp + p * g.sh + g.oh) * g.Wp + q * g.sw + g.ow) * g.Cp;
}

FM_DEVICE int tap_off(const TapG& t, int j) {
  const int rs = fdiv(j, t.dC8), c8 = j - rs * t.C8;
  const int r = fdiv(rs, t.dS), s = rs - r * t.S;
  return t.t0 + r * t.rstep + s * t.sstep + 8 * c8;
}

// ---- operand loaders (global -> registers -> LDS image) ----------------------------------
// K-contiguous rows (fwd/dgrad A: weight rows; B: gathered pixel rows).  Chunk ci = tid + NTH*i:
// row ci >> 3, k-chunk ci & 7 (the same for every i of a thread).
template <int R, int NTH, bool GATHER>
struct LoadKC {
  static constexpr int PER_T = R * 8 / NTH;
  u32x4_t v[PER_T];
  int org[PER_T];
  bool rok[PER_T];

  FM_DEVICE void init(const ConvN& p, int row0, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int row = row0 + ((tid + NTH * i) >> 3);
      if constexpr (GATHER) {
        rok[i] = row < p.N;
        int n, pp, q;
        pix_nqp(p.gb, rok[i] ? row : 0, n, pp, q);
        org[i] = pix_org(p.gb, n, pp, q);
      } else {
        rok[i] = row < p.M;
        org[i] = (rok[i] ? row : 0) * p.K;
      }
    }
  }

  FM_DEVICE void load(const ConvN& p, __amdgpu_buffer_rsrc_t rs, int kt, int tid) {
    const int j = kt * 8 + (tid & 7);       // reduction chunk of this thread
    const bool kok = j * 8 < p.K;
    int t;
    if constexpr (GATHER) t = tap_off(p.tb, kok ? j : 0);
    else t = 8 * j;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) v[i] = ld16(rs, kok && rok[i], org[i] + t);
  }

  FM_DEVICE void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      *reinterpret_cast<u32x4_t*>(lds + lds_off<true, R>(ci >> 3, ci & 7)) = v[i];
    }
  }
};

// K-contiguous rows staged by LDS-DMA (buffer_load_dwordx4 ... lds: no VGPR round trip, no
// ds_write): one wave-instruction fills 1 KiB of the image (8 rows x 128 B), lane L's 16 B landing at
// base + 16 L, so lane L loads the (row, k-chunk) the image's swizzle puts at its slot; out-of-range
// rows / chunks / halo taps read at OOBN, which the buffer unit returns as zeros.
template <int R, int NTH, bool GATHER>
struct LoadKCDma {
  static constexpr int PER_W = R * BK * 2 / 1024 / (NTH / 64);
  static_assert(PER_W >= 1 && (R * BK * 2) % (1024 * (NTH / 64)) == 0, "whole 1-KiB pieces per wave");
  int org[PER_W], ch[PER_W];
  bool rok[PER_W];

  FM_DEVICE void init(const ConvN& p, int row0, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int o = (wave * PER_W + i) * 1024 + 16 * lane;
      const int r = o / (BK * 2);
      ch[i] = ((o % (BK * 2)) / 16) ^ ((r >> 1) & 7);
      const int row = row0 + r;
      if constexpr (GATHER) {
        rok[i] = row < p.N;
        int n, pp, q;
        pix_nqp(p.gb, rok[i] ? row : 0, n, pp, q);
        org[i] = pix_org(p.gb, n, pp, q);
      } else {
        rok[i] = row < p.M;
        org[i] = (rok[i] ? row : 0) * p.K;
      }
    }
  }

  FM_DEVICE void issue(const ConvN& p, __amdgpu_buffer_rsrc_t rs, int kt, char* lds, int wave) const {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int j = kt * 8 + ch[i];
      const bool ok = rok[i] && j * 8 < p.K;
      int t;
      if constexpr (GATHER) t = tap_off(p.tb, ok ? j : 0);
      else t = 8 * j;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + (wave * PER_W + i) * 1024),
                                               16, ok ? (unsigned)(org[i] + t) * 2u : OOBN, 0, 0, 0);
    }
  }
};

// MN-contiguous (wgrad): k-row = pixel, chunks of 8 channels / taps along the R rows of the tile.
// Chunk ci = tid + NTH*i: k-row ci / (R/8), chunk ci % (R/8) (fixed per thread).  The window
// origins of a k-tile's pixels come from the per-pass origin table (fm_pix_table: {orgA, orgB} per
// pixel), read one k-tile AHEAD: load(kt) issues the data loads of k-tile kt with the origins in
// registers, then the table loads of k-tile kt+1 -- no pixel index math in the K loop.
template <int R, int NTH, bool IS_A>
struct LoadMN {
  static constexpr int PER_T = R * 8 / NTH;
  static constexpr int CPR = R / 8;       // chunks per k-row
  u32x4_t v[PER_T];
  int org[PER_T];
  int coff;       // fixed column offset of this thread's chunk (channel or tap)
  bool cok;

  FM_DEVICE void init(const ConvN& p, int col0, int tid, int kt0) {
    const int c = col0 + 8 * (tid % CPR);
    if constexpr (IS_A) {
      cok = c < p.Mp;
      coff = c;
    } else {
      cok = c < p.N;
      coff = tap_off(p.tb, cok ? c / 8 : 0);
    }
    const PixG& g = IS_A ? p.ga : p.gb;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int pix = kt0 * 64 + (tid + NTH * i) / CPR;
      int n, pp, q;
      pix_nqp(g, pix < p.npix ? pix : 0, n, pp, q);
      org[i] = pix_org(g, n, pp, q);
    }
  }

  FM_DEVICE void load(const ConvN& p, __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rtab, int kt, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int pix = kt * 64 + (tid + NTH * i) / CPR;
      v[i] = ld16(rs, cok && pix < p.npix, org[i] + coff);
    }
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {       // origins of k-tile kt+1 (0 past the table)
      const int pix = (kt + 1) * 64 + (tid + NTH * i) / CPR;
      org[i] = __builtin_amdgcn_raw_buffer_load_b32(rtab, pix < p.npix ? (unsigned)(2 * pix + (IS_A ? 0 : 1)) * 4u : OOBN,
                                                    0, 0);
    }
  }

  FM_DEVICE void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      *reinterpret_cast<u32x4_t*>(lds + lds_off<false, R>(ci / CPR, ci % CPR)) = v[i];
    }
  }

  // every chunk of this thread covers the same 8 channels: summing the staged chunks gives the
  // per-channel partial sums of G (the bias gradient) without another pass over G
  FM_DEVICE void accumulate(float (&s)[8]) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[2 * j] += bf2f((unsigned short)(v[i][j] & 0xFFFF));
        s[2 * j + 1] += bf2f((unsigned short)(v[i][j] >> 16));
      }
  }
};

// MN-contiguous (wgrad) operand staged by LDS-DMA: a 1-KiB piece is 1024 / (R*2) pixel k-rows of the
// [pixel][R] image; lane L loads the 8 channels / taps the MN swizzle puts at its slot, from the
// pixel's window origin (per-pass table, read one k-tile ahead into registers).
template <int R, int NTH, bool IS_A>
struct LoadMNDma {
  static constexpr int PER_W = R * BK * 2 / 1024 / (NTH / 64);
  static_assert(PER_W >= 1 && (R * BK * 2) % (1024 * (NTH / 64)) == 0, "whole 1-KiB pieces per wave");
  int org[PER_W], kr[PER_W], coff[PER_W];
  bool cok[PER_W];

  FM_DEVICE void table(const ConvN& p, __amdgpu_buffer_rsrc_t rtab, int kt) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int pix = kt * 64 + kr[i];
      org[i] = __builtin_amdgcn_raw_buffer_load_b32(rtab, pix < p.npix ? (unsigned)(2 * pix + (IS_A ? 0 : 1)) * 4u : OOBN,
                                                    0, 0);
    }
  }

  FM_DEVICE void init(const ConvN& p, __amdgpu_buffer_rsrc_t rtab, int col0, int wave, int lane, int kt0) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int o = (wave * PER_W + i) * 1024 + 16 * lane;
      kr[i] = o / (R * 2);
      const int c = col0 + 8 * (((o % (R * 2)) / 16) ^ MNSwz<R>::f(kr[i]));
      if constexpr (IS_A) {
        cok[i] = c < p.Mp;
        coff[i] = c;
      } else {
        cok[i] = c < p.N;
        coff[i] = tap_off(p.tb, cok[i] ? c / 8 : 0);
      }
    }
    table(p, rtab, kt0);
  }

  // k-tile kt into lds (origins in registers), then the origins of k-tile kt+1
  FM_DEVICE void issue(const ConvN& p, __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rtab, int kt, char* lds, int wave) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const bool ok = cok[i] && kt * 64 + kr[i] < p.npix;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + (wave * PER_W + i) * 1024),
                                               16, ok ? (unsigned)(org[i] + coff[i]) * 2u : OOBN, 0, 0, 0);
    }
    table(p, rtab, kt + 1);
  }
};

// {orgA, orgB} window origins of every pixel of a wgrad pass (both operands share the pixel space)
__global__ void __launch_bounds__(256) fm_pix_table(int* __restrict__ tab, int npix, PixG ga, PixG gb) {
  for (int pix = blockIdx.x * 256 + threadIdx.x; pix < npix; pix += gridDim.x * 256) {
    int n, p, q;
    pix_nqp(ga, pix, n, p, q);
    tab[2 * pix] = pix_org(ga, n, p, q);
    tab[2 * pix + 1] = pix_org(gb, n, p, q);
  }
}

// ---- the kernel -------------------------------------------------------------------------------
template <int BM, int BN, int MODE, int NTH, bool DMA = false>
__global__ void __launch_bounds__(NTH, 2) fm_conv_nhwc(ConvN p) {
  constexpr bool KCM = MODE != CN_WGRAD;     // both operands K-contiguous (fwd / dgrad)
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int WN = (NTH == 512 && BN >= 128) ? 4 : 2;
  constexpr int WM = NTH / 64 / WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 16, NR = TN / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int bid = xcd_remap(blockIdx.x, p.tiles_m * p.tiles_n);
  const int tm = bid % p.tiles_m, tn = bid / p.tiles_m;   // row tiles fastest: the big pixel operand is shared
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.kt_per, kt1 = min(ktiles, kt0 + p.kt_per);

  const auto rsa = rsrc_n(p.A, p.a_bytes);
  const auto rsb = rsrc_n(p.B, p.b_bytes);
  using LA = typename std::conditional<KCM, LoadKC<BM, NTH, false>, LoadMN<BM, NTH, true>>::type;
  using LB = typename std::conditional<KCM, LoadKC<BN, NTH, true>, LoadMN<BN, NTH, false>>::type;
  LA la;
  LB lb;
  const auto rst = rsrc_n(p.ptab, KCM ? 0 : (long)p.npix * 8);
  if constexpr (KCM && !DMA) {
    la.init(p, m0, tid);
    lb.init(p, n0, tid);
  } else if constexpr (!DMA) {
    la.init(p, m0, tid, kt0);
    lb.init(p, n0, tid, kt0);
  }
#define FM_CN_LOAD(kt)                \
  do {                                \
    if constexpr (KCM) {              \
      la.load(p, rsa, kt, tid);       \
      lb.load(p, rsb, kt, tid);       \
    } else {                          \
      la.load(p, rsa, rst, kt, tid);  \
      lb.load(p, rsb, rst, kt, tid);  \
    }                                 \
  } while (0)

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  float dbs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  bool dbrow = false;
  if constexpr (!KCM) dbrow = p.db != nullptr && tn == 0;
  if constexpr (DMA) {
    // LDS-DMA staging: k-tile kt+1 issued into the free stage before k-tile kt's MFMAs, vmcnt(0)
    // before the barrier that publishes it (profiles/conv_dma_ab_r6.txt); wgrad reads its bias
    // gradient back from the staged G image
    using DA = typename std::conditional<KCM, LoadKCDma<BM, NTH, false>, LoadMNDma<BM, NTH, true>>::type;
    using DB = typename std::conditional<KCM, LoadKCDma<BN, NTH, true>, LoadMNDma<BN, NTH, false>>::type;
    DA da;
    DB db;
    auto issue = [&](int kt, char* st) {
      if constexpr (KCM) {
        da.issue(p, rsa, kt, st, wave);
        db.issue(p, rsb, kt, st + A_BYTES, wave);
      } else {
        da.issue(p, rsa, rst, kt, st, wave);
        db.issue(p, rsb, rst, kt, st + A_BYTES, wave);
      }
    };
    if constexpr (KCM) {
      da.init(p, m0, wave, lane);
      db.init(p, n0, wave, lane);
    } else {
      da.init(p, rst, m0, wave, lane, kt0);
      db.init(p, rst, n0, wave, lane, kt0);
    }
    if (kt0 < kt1) {
      issue(kt0, smem);
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    }
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      if (kt + 1 < kt1) issue(kt + 1, smem + (cur ^ 1) * (A_BYTES + B_BYTES));
      const char* sa = smem + cur * (A_BYTES + B_BYTES);
      const char* sb = sa + A_BYTES;
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        bf16x8_t af[MR], bfr[NR];
#pragma unroll
        for (int i = 0; i < MR; ++i) af[i] = frag<KCM, BM>(sa, wm * TM + 16 * i, kk, lane);
#pragma unroll
        for (int j = 0; j < NR; ++j) bfr[j] = frag<KCM, BN>(sb, wn * TN + 16 * j, kk, lane);
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8v_t*>(&bfr[j]),
                                                                *reinterpret_cast<bf16x8v_t*>(&af[i]), acc[i][j], 0, 0, 0);
      }
      if constexpr (!KCM) {   // bias gradient: the register form's chunks, read back from the staged G
        if (dbrow) {
          constexpr int CPR = BM / 8, PER_T = BM * 8 / NTH;
#pragma unroll
          for (int i = 0; i < PER_T; ++i) {
            const int ci = tid + NTH * i;
            const u32x4_t w = *reinterpret_cast<const u32x4_t*>(sa + lds_off<false, BM>(ci / CPR, ci % CPR));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              dbs[2 * j] += bf2f((unsigned short)(w[j] & 0xFFFF));
              dbs[2 * j + 1] += bf2f((unsigned short)(w[j] >> 16));
            }
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's pieces of k-tile kt+1 landed
      __syncthreads();
    }
  } else {
  if (kt0 < kt1) {
    FM_CN_LOAD(kt0);
    if constexpr (!KCM) {
      if (dbrow) la.accumulate(dbs);
    }
    la.store(smem, tid);
    lb.store(smem + A_BYTES, tid);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) FM_CN_LOAD(kt + 1);
    const char* sa = smem + cur * (A_BYTES + B_BYTES);
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8_t af[MR], bfr[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) af[i] = frag<KCM, BM>(sa, wm * TM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < NR; ++j) bfr[j] = frag<KCM, BN>(sb, wn * TN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8v_t*>(&bfr[j]),
                                                              *reinterpret_cast<bf16x8v_t*>(&af[i]), acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* nx = smem + (cur ^ 1) * (A_BYTES + B_BYTES);
      if constexpr (!KCM) {
        if (dbrow) la.accumulate(dbs);
      }
      la.store(nx, tid);
      lb.store(nx + A_BYTES, tid);
    }
    __syncthreads();
  }
  }
#undef FM_CN_LOAD
  if constexpr (!KCM) {
    if (dbrow) {   // reduce the NTH/(BM/8) threads sharing each 8-channel column, 1 atomic per channel
      constexpr int CPR = BM / 8;
      float* red = reinterpret_cast<float*>(smem);   // LDS is free after the K loop
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(tid / CPR) * BM + (tid % CPR) * 8 + j] = dbs[j];
      __syncthreads();
      if (tid < BM && m0 + tid < p.M) {
        float x = 0.f;
        for (int t = 0; t < NTH / CPR; ++t) x += red[t * BM + tid];
        atomicAdd(p.db + m0 + tid, x);
      }
    }
  }

  // epilogue: lane owns C[m][n .. n+3], m = mbase + 16 i + (lane & 15), n = nbase + 16 j + 4 (lane >> 4)
  const int mbase = m0 + wm * TM, nbase = n0 + wn * TN;
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int m = mbase + 16 * i + (lane & 15);
    if (m >= p.M) continue;
    const float bm = (MODE == CN_FWD && p.bias) ? p.bias[m] : 0.f;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int n = nbase + 16 * j + 4 * (lane >> 4);
      if (n >= p.N) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r];
      if constexpr (MODE == CN_WGRAD) {
        // split-K slab z = blockIdx.z of [ksplit][M][N] (N % 8 == 0: one 16-B store)
        float* dw = reinterpret_cast<float*>(p.out) + ((long)blockIdx.z * p.M + m) * p.N + n;
        *reinterpret_cast<f32x4_t*>(dw) = f32x4_t{v[0], v[1], v[2], v[3]};
      } else {
        if constexpr (MODE == CN_FWD) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = act_fwd(p.act, v[r] + bm);
        }
        const bool add = MODE == CN_DGRAD && p.accum;
        unsigned short* out = reinterpret_cast<unsigned short*>(p.out);
        const int img = fdiv(n, p.dOPQ), px = n - img * p.OPQ;
        const long o = ((long)img * p.M + m) * p.OPQ + px;
        if (p.out2 != nullptr) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nn = n + r;
            if (nn >= p.N) break;
            const int im = fdiv(nn, p.dOPQ), pr = nn - im * p.OPQ;
            const int pp = fdiv(pr, p.dOQ), qq = pr - pp * p.OQ;
            const int i2 = pp * p.d2h + p.t2, j2 = qq * p.d2w + p.l2;
            if ((unsigned)i2 < (unsigned)p.H2 && (unsigned)j2 < (unsigned)p.W2)
              p.out2[(((long)im * p.H2 + i2) * p.W2 + j2) * p.C2 + m] = f2bf(v[r]);
          }
          if (!p.write_nchw) continue;
        }
        if (p.strided_out) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nn = n + r;
            if (nn >= p.N) break;
            const int im = fdiv(nn, p.dOPQ), pr = nn - im * p.OPQ;
            const int hh = fdiv(pr, p.dOQ), ww = pr - hh * p.OQ;
            unsigned short* d = out + (((long)im * p.M + m) * p.o_H + p.o_oh + p.o_sh * hh) * p.o_W + p.o_ow + p.o_sw * ww;
            *d = f2bf(v[r] + (add ? bf2f(*d) : 0.f));
          }
          continue;
        }
        if (n + 3 < p.N && px + 3 < p.OPQ && (o & 3) == 0) {
          bf16x4_t w4;
          if (add) {
            const bf16x4_t old = *reinterpret_cast<const bf16x4_t*>(out + o);
#pragma unroll
            for (int r = 0; r < 4; ++r) w4[r] = (short)f2bf(v[r] + bf2f((unsigned short)old[r]));
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) w4[r] = (short)f2bf(v[r]);
          }
          *reinterpret_cast<bf16x4_t*>(out + o) = w4;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nn = n + r;
            if (nn >= p.N) break;
            const int im = fdiv(nn, p.dOPQ), pr = nn - im * p.OPQ;
            unsigned short* d = out + ((long)im * p.M + m) * p.OPQ + pr;
            *d = f2bf(v[r] + (add ? bf2f(*d) : 0.f));
          }
        }
      }
    }
  }
}

// ---- staging: NCHW -> zero-padded NHWC ------------------------------------------------------
// dst [N][Hp][Wp][Cp]: dst[n][i][j][c] = v[n][c][(i - top)/dh][(j - left)/dw] where the division is
// exact and inside, 0 elsewhere (top / left may be negative: leading source rows / columns are
// skipped; dilation dh, dw > 1 spreads a strided convolution's G for its stride-1 data gradient).
// v = src, or for the gradient staging (GRAD) v = act'(y) * dy rounded to bf16 (one pass instead of
// an activation-backward pass + a copy; the bias gradient is summed by the wgrad kernel).
// Block = 64 destination columns x 64 channels of one destination row; loads coalesce along the
// source row (w), the 16-B stores along the channels.
template <bool GRAD>
__global__ void __launch_bounds__(256) fm_nhwc_stage(const unsigned short* __restrict__ src, const unsigned short* __restrict__ ysrc,
                                                     unsigned short* __restrict__ dst, int act,
                                                     int C, int H, int W, int Cp, int Hp, int Wp, int top, int left, int dh,
                                                     int dw) {
  // [channel][column] with 132-B rows (33 dwords): the store phase's lanes read 8 rows x 8 columns at
  // stride 8 rows = 264 dwords = 8 banks apart -> conflict-free (a 144-B pitch put every other
  // lane group on the same bank: 6.7 conflicts per LDS instruction, profiles/pmc_conv_nhwc_r4g.txt)
  __shared__ __attribute__((aligned(16))) unsigned short tile[64][66];
  const int j0 = blockIdx.y * 64, c0 = blockIdx.z * 64;
  const int ni = blockIdx.x;
  const int n = ni / Hp, i = ni - n * Hp;
  const int hd = i - top, h = hd / dh;
  const bool rowin = hd >= 0 && h * dh == hd && h < H;
  if (rowin) {
    if (dw == 1) {
      // 8 consecutive source columns per thread-chunk: one (unaligned) 16-B buffer load where the
      // chunk lies inside the row, element loads only for the chunks on the row's edges
      const long rowel = (long)H * W;
      const auto rs = rsrc_n(src, (long)gridDim.x / Hp * C * rowel * 2);
      const auto ry = rsrc_n(GRAD ? ysrc : src, (long)gridDim.x / Hp * C * rowel * 2);
      for (int e = threadIdx.x; e < 64 * 8; e += 256) {
        const int cc = e >> 3, ch = e & 7;
        const int c = c0 + cc, w0 = j0 + 8 * ch - left;
        u32x4_t v = {0u, 0u, 0u, 0u};
        if (c < C) {
          const long o = (((long)n * C + c) * H + h) * W + w0;
          if (w0 >= 0 && w0 + 8 <= W) {
            v = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(o * 2), 0, 0));
            if constexpr (GRAD) {
              if (act != ACT_NONE) {
                const u32x4_t yv =
                    __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(ry, (unsigned)(o * 2), 0, 0));
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  const unsigned short lo = f2bf(act_bwd(act, bf2f((unsigned short)(yv[u] & 0xFFFF)),
                                                         bf2f((unsigned short)(v[u] & 0xFFFF))));
                  const unsigned short hi = f2bf(act_bwd(act, bf2f((unsigned short)(yv[u] >> 16)),
                                                         bf2f((unsigned short)(v[u] >> 16))));
                  v[u] = (unsigned)lo | ((unsigned)hi << 16);
                }
              }
            }
          } else {
            unsigned short e8[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const int w = w0 + t;
              unsigned short x = 0;
              if (w >= 0 && w < W) {
                x = src[o + t];
                if constexpr (GRAD) {
                  if (act != ACT_NONE) x = f2bf(act_bwd(act, bf2f(ysrc[o + t]), bf2f(x)));
                }
              }
              e8[t] = x;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = (unsigned)e8[2 * u] | ((unsigned)e8[2 * u + 1] << 16);
          }
        }
        unsigned* tw = reinterpret_cast<unsigned*>(&tile[cc][8 * ch]);   // 4-B aligned (132-B rows)
#pragma unroll
        for (int u = 0; u < 4; ++u) tw[u] = v[u];
      }
    } else {
      for (int e = threadIdx.x; e < 64 * 64; e += 256) {
        const int cc = e >> 6, jj = e & 63;
        const int c = c0 + cc, wd = j0 + jj - left, w = wd / dw;
        unsigned short v = 0;
        if (c < C && wd >= 0 && w * dw == wd && w < W) {
          const long o = (((long)n * C + c) * H + h) * W + w;
          v = src[o];
          if constexpr (GRAD) {
            if (act != ACT_NONE) v = f2bf(act_bwd(act, bf2f(ysrc[o]), bf2f(v)));
          }
        }
        tile[cc][jj] = v;
      }
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 512; e += 256) {
    const int jj = e >> 3, cg = e & 7;
    const int j = j0 + jj, c = c0 + 8 * cg;
    if (j >= Wp || c >= Cp) continue;
    u32x4_t o = {0u, 0u, 0u, 0u};
    if (rowin) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        o[u] = (unsigned)tile[8 * cg + 2 * u][jj] | ((unsigned)tile[8 * cg + 2 * u + 1][jj] << 16);
    }
    *reinterpret_cast<u32x4_t*>(dst + (((long)n * Hp + i) * Wp + j) * Cp + c) = o;
  }
}

// Narrow images (Wp < 32): the row kernel above would leave most of its 64 columns empty (Inception
// 17x17 / 8x8, ResNet 14x14 / 7x7).  This form tiles 64 consecutive destination PIXELS of one
// image (flattened i*Wp + j, crossing rows) x 64 channels: a per-block LDS table maps each pixel
// slot to its source offset (or -1 in the halo / dilation gaps), the loads walk the slots (runs
// of one source row are contiguous) and the 16-B stores of a block cover one contiguous
// [64 pixels][Cp] run of the destination.
template <bool GRAD>
__global__ void __launch_bounds__(256) fm_nhwc_stage_flat(const unsigned short* __restrict__ src,
                                                          const unsigned short* __restrict__ ysrc,
                                                          unsigned short* __restrict__ dst, int act, int C, int H, int W,
                                                          int Cp, int Hp, int Wp, int top, int left, int dh, int dw,
                                                          int blocks_per_img) {
  __shared__ __attribute__((aligned(16))) unsigned short tile[64][66];   // 132-B rows: conflict-free reads
  __shared__ int soff[64];
  const int n = blockIdx.x / blocks_per_img;
  const int pix0 = (blockIdx.x - n * blocks_per_img) * 64;
  const int c0 = blockIdx.y * 64;
  const int npix = Hp * Wp;
  if (threadIdx.x < 64) {
    const int pi = pix0 + threadIdx.x;
    int off = -1;
    if (pi < npix) {
      const int i = pi / Wp, j = pi - i * Wp;
      const int hd = i - top, wd = j - left;
      const int h = hd / dh, w = wd / dw;
      if (hd >= 0 && wd >= 0 && h * dh == hd && w * dw == wd && h < H && w < W) off = h * W + w;
    }
    soff[threadIdx.x] = off;
  }
  __syncthreads();
  const long plane = (long)H * W;
  // 8 element loads in flight per thread (clamped addresses, predicated use) before the LDS stores
#pragma unroll
  for (int b0 = 0; b0 < 64 * 64; b0 += 256 * 8) {
    unsigned short v[8], yv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = b0 + u * 256 + (int)threadIdx.x;
      const int cc = e >> 6, jj = e & 63;
      const int c = min(c0 + cc, C - 1), off = max(soff[jj], 0);
      const long o = ((long)n * C + c) * plane + off;
      v[u] = src[o];
      if constexpr (GRAD) yv[u] = act != ACT_NONE ? ysrc[o] : (unsigned short)0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = b0 + u * 256 + (int)threadIdx.x;
      const int cc = e >> 6, jj = e & 63;
      unsigned short x = (c0 + cc < C && soff[jj] >= 0) ? v[u] : (unsigned short)0;
      if constexpr (GRAD) {
        if (act != ACT_NONE && x != 0) x = f2bf(act_bwd(act, bf2f(yv[u]), bf2f(x)));
      }
      tile[cc][jj] = x;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 512; e += 256) {
    const int jj = e >> 3, cg = e & 7;
    const int pi = pix0 + jj, c = c0 + 8 * cg;
    if (pi >= npix || c >= Cp) continue;
    u32x4_t o;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      o[u] = (unsigned)tile[8 * cg + 2 * u][jj] | ((unsigned)tile[8 * cg + 2 * u + 1][jj] << 16);
    *reinterpret_cast<u32x4_t*>(dst + ((long)n * npix + pi) * Cp + c) = o;
  }
}

template <bool GRAD>
void stage_launch(const void* src, const void* y, void* dst, int act, int N, int C, int H, int W, int Cp, int Hp, int Wp, int top,
                  int left, int dh, int dw, hipStream_t s) {
  // image widths below 128 take the flattened-pixel kernel (32 / 64 / 128 measured,
  // profiles/ab_stage_wgrad_r3y.txt)
  if (Wp < 128) {
    const int bpi = (Hp * Wp + 63) / 64;
    hipLaunchKernelGGL(fm_nhwc_stage_flat<GRAD>, dim3(N * bpi, (Cp + 63) / 64), dim3(256), 0, s, (const unsigned short*)src,
                       (const unsigned short*)y, (unsigned short*)dst, act, C, H, W, Cp, Hp, Wp, top, left, dh, dw, bpi);
    return;
  }
  dim3 grid(N * Hp, (Wp + 63) / 64, (Cp + 63) / 64);
  hipLaunchKernelGGL(fm_nhwc_stage<GRAD>, grid, dim3(256), 0, s, (const unsigned short*)src, (const unsigned short*)y,
                     (unsigned short*)dst, act, C, H, W, Cp, Hp, Wp, top, left, dh, dw);
}

// weight re-layouts: mode 0 (fwd)  out[k][(r*S+s)*Cp + c] = w[k][c][r][s]            (0 for c >= C)
//                    mode 1 (dgrad) out[c][(r*S+s)*Kp + k] = w[k][c][R-1-r][S-1-s]    (0 for k >= K)
//                    mode 3 both (fwd into out, dgrad into out2): one launch per forward
FM_DEVICE void wprep_body(const unsigned short* __restrict__ w, unsigned short* __restrict__ out,
                          unsigned short* __restrict__ out2, int K, int C, int R, int S, int Cp, int Kp, int mode) {
  // 32-bit index math (the host checks the sizes): 64-bit divisions are emulated, ~4x the work
  const int RS = R * S;
  const int t0 = K * RS * Cp, t1 = C * RS * Kp;
  const int total = mode == 0 ? t0 : mode == 1 ? t1 : t0 + t1;
  for (int oo = blockIdx.x * 256 + threadIdx.x; oo < total; oo += gridDim.x * 256) {
    // mode 3: both layouts in one launch (fwd matrix into out, dgrad matrix into out2)
    const bool second = mode == 1 || (mode == 3 && oo >= t0);
    const int o = mode == 3 && second ? oo - t0 : oo;
    unsigned short* dst = mode == 3 && second ? out2 : out;
    if (!second) {
      const int t = o / Cp, c = o - t * Cp;
      const int k = t / RS, rs = t - k * RS;
      dst[o] = c < C ? w[(k * C + c) * RS + rs] : (unsigned short)0;
    } else {
      const int t = o / Kp, k = o - t * Kp;
      const int c = t / RS, rs = t - c * RS;
      const int r = rs / S, s = rs - r * S;
      dst[o] = k < K ? w[(k * C + c) * RS + (R - 1 - r) * S + (S - 1 - s)] : (unsigned short)0;
    }
  }
}

__global__ void fm_cnhwc_wprep(const unsigned short* __restrict__ w, unsigned short* __restrict__ out,
                               unsigned short* __restrict__ out2, int K, int C, int R, int S, int Cp, int Kp, int mode) {
  wprep_body(w, out, out2, K, C, R, S, Cp, Kp, mode);
}

// every NHWC layer's two weight matrices (mode 3) in one launch, blockIdx.y = layer: the step's
// re-layouts as one kernel instead of one ~7 us launch per convolution (ResNet-50: 53 per step)
constexpr int WPREP_MAX = 32;
struct WprepJob {
  const unsigned short* w;
  unsigned short *out, *out2;
  int K, C, R, S, Cp, Kp;
};
struct WprepSet {
  WprepJob j[WPREP_MAX];
};
__global__ void fm_cnhwc_wprep_multi(WprepSet s) {
  const WprepJob& d = s.j[blockIdx.y];
  wprep_body(d.w, d.out, d.out2, d.K, d.C, d.R, d.S, d.Cp, d.Kp, 3);
}

PixG make_pix(int PQ, int Q, int Hp, int Wp, int Cp, int sh, int sw, int oh, int ow) {
  PixG g;
  g.dPQ = make_fastdiv(PQ);
  g.dQ = make_fastdiv(Q);
  g.PQ = PQ; g.Q = Q; g.Hp = Hp; g.Wp = Wp; g.Cp = Cp;
  g.sh = sh; g.sw = sw; g.oh = oh; g.ow = ow;
  return g;
}

TapG make_tap(int Cp, int S, int Wp) {
  TapG t;
  t.C8 = Cp / 8;
  t.dC8 = make_fastdiv(t.C8);
  t.S = S;
  t.dS = make_fastdiv(S);
  t.Wp = Wp;
  t.Cp = Cp;
  t.t0 = 0;
  t.rstep = Wp * Cp;
  t.sstep = Cp;
  return t;
}

// stride-phase sub-kernel of the dgrad matrix: out[c][(ri*Ss + si)*Kp + k] =
// w[k][c][R-1-(r0 + sh*ri)][S-1-(s0 + sw*si)] (0 for k >= K)
__global__ void fm_cnhwc_wphase(const unsigned short* __restrict__ w, unsigned short* __restrict__ out, int K, int C, int R,
                                int S, int Kp, int r0, int s0, int sh, int sw, int Rs, int Ss) {
  const long total = (long)C * Rs * Ss * Kp;
  for (long o = blockIdx.x * 256L + threadIdx.x; o < total; o += (long)gridDim.x * 256) {
    const int k = (int)(o % Kp);
    const long t = o / Kp;
    const int rs = (int)(t % (Rs * Ss)), c = (int)(t / (Rs * Ss));
    const int ri = rs / Ss, si = rs - ri * Ss;
    const int r = R - 1 - (r0 + sh * ri), q = S - 1 - (s0 + sw * si);
    out[o] = k < K ? w[(((long)k * C + c) * R + r) * S + q] : (unsigned short)0;
  }
}

// wgrad fold: dw[k][c][r][s] += sum_z g2[z][k][(r*S+s)*Cp + c] over the split-K slabs.  Block = 32
// consecutive slab elements x 8 split groups (coalesced 128-B slab reads, the split sum reduced in
// LDS) -- hundreds of splits stay parallel instead of one serial loop per output.
__global__ void __launch_bounds__(256) fm_cnhwc_fold(const float* __restrict__ g2, float* __restrict__ dw, int K, int C, int RS,
                                                     int Cp, int nsplit) {
  __shared__ float red[8][33];
  const long slab = (long)K * RS * Cp;
  const int ol = threadIdx.x & 31, zg = threadIdx.x >> 5;
  const long o = blockIdx.x * 32L + ol;
  float acc = 0.f;
  if (o < slab) {
    // 4 independent slab loads in flight per thread
    float a4[4] = {0.f, 0.f, 0.f, 0.f};
    int z = zg;
    for (; z + 24 < nsplit; z += 32) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a4[u] += g2[(long)(z + 8 * u) * slab + o];
    }
    for (; z < nsplit; z += 8) a4[0] += g2[(long)z * slab + o];
    acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
  }
  red[zg][ol] = acc;
  __syncthreads();
  if (threadIdx.x < 32 && o < slab) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += red[g][ol];
    const int c = (int)(o % Cp);
    if (c < C) {
      const long q = o / Cp;
      const int rs = (int)(q % RS), k = (int)(q / RS);
      dw[((long)k * C + c) * RS + rs] += t;
    }
  }
}

// launch plan: tile shape (0: 128x128 / 8 waves, 1: 64x128, 2: 64x64 / 4 waves), tiles, k split.
// 128x128 when it still gives >= 256 tiles, else the smaller tiles that fill the 256 CUs.  wgrad
// (M = K out channels, N = R*S*Cp taps) takes 128-row tiles for M > 64 and 64x64 for N <= 64, and
// splits its long pixel reduction until ~2 blocks per CU (>= 8 k-tiles each); the splits write
// fp32 slabs [ksplit][M][N] that fm_cnhwc_fold sums while folding.
struct Plan {
  int shape, tiles_m, tiles_n, ksplit, kt_per;
};

// per-pass tile-shape override (-1: the heuristic below), set by the per-layer measured selection
// around one layer's launches (fm_conv_nhwc_set_shape); the split-K workspace size follows it
int g_cn_shape[3] = {-1, -1, -1};

Plan make_plan(int mode, int M, int N, int K) {
  auto tiles = [&](int bm, int bn) { return (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  Plan q;
  if (g_cn_shape[mode] >= 0) q.shape = g_cn_shape[mode];
  else if (mode == CN_WGRAD) q.shape = N <= 64 ? 2 : M > 64 ? 0 : 1;
  else if (M > 64 && tiles(128, 128) >= 256) q.shape = 0;
  else if (tiles(64, 128) >= 256) q.shape = 1;
  else q.shape = 2;
  const int bm = q.shape == 0 ? 128 : 64, bn = q.shape == 2 ? 64 : 128;
  q.tiles_m = (M + bm - 1) / bm;
  q.tiles_n = (N + bn - 1) / bn;
  const int ktiles = (K + BK - 1) / BK;
  int ks = 1;
  // split-K target of the weight gradient: 512 blocks
  // (256 / 1024 measured: AlexNet b256 86.8 k / 97.9 k vs 98.2-99.9 k img/s, ResNet-50 b64 6.31 k / 6.44 k vs
  // 6.60 k; profiles/conv_wgrad_split_ab_r7.txt)
  constexpr int wg_blocks = 512;
  if (mode == CN_WGRAD) ks = std::max(1, std::min(wg_blocks / std::max(q.tiles_m * q.tiles_n, 1), ktiles / 8));
  q.kt_per = (ktiles + ks - 1) / ks;
  q.ksplit = (ktiles + q.kt_per - 1) / q.kt_per;
  return q;
}

template <int BM, int BN, int MODE, int NTH>
void go(ConvN& p, const Plan& q, hipStream_t s) {
  p.tiles_m = q.tiles_m;
  p.tiles_n = q.tiles_n;
  p.ksplit = q.ksplit;
  p.kt_per = q.kt_per;
  const int lds = 2 * (BM + BN) * BK * 2;
  // operands staged by LDS-DMA (FM_GEMM_DMA=0: register staging, for A/B)
  const bool dma = fm_gemm_dma_enabled();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fm_conv_nhwc<BM, BN, MODE, NTH>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    (void)hipFuncSetAttribute((const void*)fm_conv_nhwc<BM, BN, MODE, NTH, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds);
    attr = true;
  }
  if (dma)
    hipLaunchKernelGGL((fm_conv_nhwc<BM, BN, MODE, NTH, true>), dim3(p.tiles_m * p.tiles_n, 1, p.ksplit), dim3(NTH), lds, s, p);
  else
    hipLaunchKernelGGL((fm_conv_nhwc<BM, BN, MODE, NTH>), dim3(p.tiles_m * p.tiles_n, 1, p.ksplit), dim3(NTH), lds, s, p);
}

// 128x128 tiles as 8-wave blocks (a 4-wave form with 64x64 per wave measured slower,
// profiles/ab_conv_nhwc_4wave_r3v.txt)
template <int MODE>
int dispatch(ConvN& p, hipStream_t s) {
  const Plan q = make_plan(MODE, p.M, p.N, p.K);
  if (q.shape == 0) go<128, 128, MODE, 512>(p, q, s);
  else if (q.shape == 1) go<64, 128, MODE, 256>(p, q, s);
  else go<64, 64, MODE, 256>(p, q, s);
  return q.ksplit;
}

}  // namespace

// tile shape of pass mode (0 fwd, 1 dgrad, 2 wgrad) for the launches that follow: 0 = 128x128 (8
// waves), 1 = 64x128, 2 = 64x64 (4 waves), -1 = the size heuristic
extern "C" void fm_conv_nhwc_set_shape(int mode, int shape) {
  if (mode >= 0 && mode < 3) g_cn_shape[mode] = shape >= 0 && shape < 3 ? shape : -1;
}

// stage src [N][C][H][W] (bf16) into dst [N][Hp][Wp][Cp] at (top, left), zeros elsewhere
extern "C" void fm_nhwc_stage_run(const void* src, void* dst, int N, int C, int H, int W, int Cp, int Hp, int Wp, int top,
                                  int left, int dh, int dw, hipStream_t s) {
  stage_launch<false>(src, nullptr, dst, ACT_NONE, N, C, H, W, Cp, Hp, Wp, top, left, dh, dw, s);
}

// gradient staging: dst = stage(act'(y) * dy) (y unused when act == none)
extern "C" void fm_nhwc_stage_grad_run(const void* dy, const void* y, void* dst, int act, int N, int C, int H, int W, int Cp,
                                       int Hp, int Wp, int top, int left, int dh, int dw, hipStream_t s) {
  stage_launch<true>(dy, y, dst, act, N, C, H, W, Cp, Hp, Wp, top, left, dh, dw, s);
}

extern "C" void fm_cnhwc_wprep_run(const void* w, void* out, void* out2, const float* g2, float* dw, int K, int C, int R, int S,
                                   int Cp, int Kp, int mode, int nsplit, hipStream_t s) {
  if (mode == 2) {
    const long slab = (long)K * R * S * Cp;
    hipLaunchKernelGGL(fm_cnhwc_fold, dim3((unsigned)((slab + 31) / 32)), dim3(256), 0, s, g2, dw, K, C, R * S, Cp, nsplit);
    return;
  }
  const long t0 = (long)K * R * S * Cp, t1 = (long)C * R * S * Kp;
  const long total = mode == 0 ? t0 : mode == 1 ? t1 : t0 + t1;
  if (total + 256L * 1024 >= (1L << 31)) return;   // (2^31 - 1 index range; no conv weight comes near)
  hipLaunchKernelGGL(fm_cnhwc_wprep, dim3(fm_grid(total, 256, 1024)), dim3(256), 0, s, (const unsigned short*)w,
                     (unsigned short*)out, (unsigned short*)out2, K, C, R, S, Cp, Kp, mode);
}

extern "C" void fm_cnhwc_wprep_multi_run(int n, const void* const* w, void* const* out, void* const* out2, const int* K,
                                         const int* C, const int* R, const int* S, const int* Cp, const int* Kp,
                                         hipStream_t s) {
  for (int b = 0; b < n; b += WPREP_MAX) {
    WprepSet set{};
    const int m = std::min(WPREP_MAX, n - b);
    long mx = 0;
    for (int i = 0; i < m; ++i) {
      const int k = b + i;
      set.j[i] = WprepJob{(const unsigned short*)w[k], (unsigned short*)out[k], (unsigned short*)out2[k], K[k], C[k],
                          R[k], S[k], Cp[k], Kp[k]};
      mx = std::max(mx, (long)K[k] * R[k] * S[k] * Cp[k] + (long)C[k] * R[k] * S[k] * Kp[k]);
    }
    hipLaunchKernelGGL(fm_cnhwc_wprep_multi, dim3(fm_grid(mx, 256, 1024), m), dim3(256), 0, s, set);
  }
}

// fp32 floats of the wgrad split-K slab workspace for these sizes (ksplit * K * R*S*Cp)
extern "C" long fm_conv_nhwc_wgrad_ws(int N, int K, int P, int Q, int R, int S, int Cp) {
  const Plan q = make_plan(CN_WGRAD, K, R * S * Cp, N * P * Q);
  return (long)q.ksplit * K * R * S * Cp;
}

// fwd: xs staged [N][Hp][Wp][Cp] (window origin of output (p, q) at row p*sh, col q*sw),
// wf [K][R*S*Cp] (mode 0), y [N][K][P][Q] bf16, bias fp32 [K] or null
// out2 (may be null): the consumer's staged input [N][H2][W2][C2], this output at (t2, l2), or with
// dilation (d2h, d2w); write_nchw = 0: y is not written
extern "C" void fm_conv_nhwc_fwd(const void* xs, long xs_bytes, const void* wf, const float* bias, void* y, int N, int K,
                                 int P, int Q, int R, int S, int Cp, int Hp, int Wp, int sh, int sw, int act, void* out2,
                                 int H2, int W2, int C2, int t2, int l2, int d2h, int d2w, int write_nchw, hipStream_t s) {
  ConvN p{};
  p.A = (const unsigned short*)wf; p.a_bytes = (long)K * R * S * Cp * 2;
  p.B = (const unsigned short*)xs; p.b_bytes = xs_bytes;
  p.out = y; p.bias = bias; p.act = act;
  p.M = K; p.N = N * P * Q; p.K = R * S * Cp;
  p.npix = p.N;
  p.gb = make_pix(P * Q, Q, Hp, Wp, Cp, sh, sw, 0, 0);
  p.tb = make_tap(Cp, S, Wp);
  p.OPQ = P * Q; p.dOPQ = make_fastdiv(P * Q);
  p.out2 = (unsigned short*)out2;
  p.OQ = Q; p.dOQ = make_fastdiv(Q);
  p.H2 = H2; p.W2 = W2; p.C2 = C2; p.t2 = t2; p.l2 = l2; p.d2h = d2h; p.d2w = d2w;
  p.write_nchw = out2 == nullptr ? 1 : write_nchw;
  dispatch<CN_FWD>(p, s);
}

// dgrad: gs staged G [N][Hg][Wg][Kp] with G at (R-1-pt, S-1-pl) dilated by the stride, wd [C][R*S*Kp] (mode 1),
// dx [N][C][H][W] bf16 (accum: +=)
static void dgrad_phases(const void* gs, long gs_bytes, const void* w, void* wsub, void* dx, int accum, int N, int C, int H,
                         int W, int K, int R, int S, int Kp, int Hg, int Wg, int gt, int gl, int sh, int sw, void* out2, int H2,
                         int W2, int C2, int t2, int l2, int d2h, int d2w, int write_nchw, hipStream_t s);

extern "C" void fm_conv_nhwc_dgrad(const void* gs, long gs_bytes, const void* wd, void* dx, int accum, int N, int C, int H,
                                   int W, int R, int S, int Kp, int Hg, int Wg, void* out2, int H2, int W2, int C2, int t2,
                                   int l2, int d2h, int d2w, int write_nchw, hipStream_t s) {
  ConvN p{};
  p.A = (const unsigned short*)wd; p.a_bytes = (long)C * R * S * Kp * 2;
  p.B = (const unsigned short*)gs; p.b_bytes = gs_bytes;
  p.out = dx; p.accum = accum;
  p.M = C; p.N = N * H * W; p.K = R * S * Kp;
  p.npix = p.N;
  p.gb = make_pix(H * W, W, Hg, Wg, Kp, 1, 1, 0, 0);
  p.tb = make_tap(Kp, S, Wg);
  p.OPQ = H * W; p.dOPQ = make_fastdiv(H * W);
  p.out2 = (unsigned short*)out2;
  p.OQ = W; p.dOQ = make_fastdiv(W);
  p.H2 = H2; p.W2 = W2; p.C2 = C2; p.t2 = t2; p.l2 = l2; p.d2h = d2h; p.d2w = d2w;
  p.write_nchw = out2 == nullptr ? 1 : write_nchw;
  dispatch<CN_DGRAD>(p, s);
}

// wgrad: g2 fp32 slabs [ksplit][K][R*S*Cp] (fm_conv_nhwc_wgrad_ws floats; returns ksplit) = sum over output pixels of
// Gs[orgG + k] * Xs[orgX + tap]; gs staged G [N][Hg][Wg][Kp], pixel (p, q) at (gt + p*gsh, gl + q*gsw)
// (gsh, gsw > 1: the stride-dilated G of the data gradient); xs as in fwd; ptab: int scratch of
// 2 * N*P*Q entries (the pass's pixel origin table: built when build_tab, else reused -- it depends
// on the geometry only, so an op builds it once)
extern "C" int fm_conv_nhwc_wgrad(const void* gs, long gs_bytes, const void* xs, long xs_bytes, float* g2, float* db, int N,
                                  int K, int Kp, int P, int Q, int Hg, int Wg, int gt, int gl, int gsh, int gsw, int R, int S,
                                  int Cp, int Hp, int Wp, int sh, int sw, int* ptab, int build_tab, hipStream_t s) {
  ConvN p{};
  p.A = (const unsigned short*)gs; p.a_bytes = gs_bytes;
  p.B = (const unsigned short*)xs; p.b_bytes = xs_bytes;
  p.out = g2;
  p.M = K; p.Mp = Kp; p.N = R * S * Cp; p.K = N * P * Q;
  p.npix = p.K;
  p.ga = make_pix(P * Q, Q, Hg, Wg, Kp, gsh, gsw, gt, gl);
  p.gb = make_pix(P * Q, Q, Hp, Wp, Cp, sh, sw, 0, 0);
  p.tb = make_tap(Cp, S, Wp);
  p.ptab = ptab;
  p.db = db;
  if (build_tab) hipLaunchKernelGGL(fm_pix_table, dim3(fm_grid(p.npix, 256, 2048)), dim3(256), 0, s, ptab, p.npix, p.ga, p.gb);
  return dispatch<CN_WGRAD>(p, s);
}

// Strided data gradient by stride phases: output pixels (a + sh*h', b + sw*w') of phase (a, b) only
// meet the taps r' = r0 + sh*i, s' = s0 + sw*j of the flipped kernel (r0 = (gt - a) mod sh) at
// nonzero rows of the stride-dilated staged G -- so each phase is a dense GEMM over its sub-kernel
// (Rs x Ss taps) with a strided NCHW store, and the phases together do exactly the layer's MACs
// (the dilated form computed every tap of every output pixel: sh*sw times the work).  wsub: bf16
// scratch of C * R*S * Kp (the phases' sub-kernels partition the R*S taps).
static void dgrad_phases(const void* gs, long gs_bytes, const void* w, void* wsub, void* dx, int accum, int N, int C, int H,
                         int W, int K, int R, int S, int Kp, int Hg, int Wg, int gt, int gl, int sh, int sw, void* out2, int H2,
                         int W2, int C2, int t2, int l2, int d2h, int d2w, int write_nchw, hipStream_t s) {
  bool empty_phase = false;
  for (int a = 0; a < sh && a < H; ++a)
    for (int b = 0; b < sw && b < W; ++b) {
      const int r0 = ((gt - a) % sh + sh) % sh, s0 = ((gl - b) % sw + sw) % sw;
      if (r0 >= R || s0 >= S) empty_phase = true;
    }
  // phases without taps receive no gradient: zero the outputs first (the others overwrite theirs)
  if (empty_phase && !accum) {
    if (write_nchw || out2 == nullptr) (void)hipMemsetAsync(dx, 0, (size_t)N * C * H * W * 2, s);
  }
  long woff = 0;
  for (int a = 0; a < sh && a < H; ++a)
    for (int b = 0; b < sw && b < W; ++b) {
      const int r0 = ((gt - a) % sh + sh) % sh, s0 = ((gl - b) % sw + sw) % sw;
      if (r0 >= R || s0 >= S) continue;
      const int Rs = (R - r0 + sh - 1) / sh, Ss = (S - s0 + sw - 1) / sw;
      const int Ha = (H - a + sh - 1) / sh, Wb = (W - b + sw - 1) / sw;
      unsigned short* wp = (unsigned short*)wsub + woff;
      const long nw = (long)C * Rs * Ss * Kp;
      woff += nw;
      hipLaunchKernelGGL(fm_cnhwc_wphase, dim3(fm_grid(nw, 256, 1024)), dim3(256), 0, s, (const unsigned short*)w, wp, K, C, R,
                         S, Kp, r0, s0, sh, sw, Rs, Ss);
      ConvN p{};
      p.A = wp; p.a_bytes = nw * 2;
      p.B = (const unsigned short*)gs; p.b_bytes = gs_bytes;
      p.out = dx; p.accum = accum;
      p.M = C; p.N = N * Ha * Wb; p.K = Rs * Ss * Kp;
      p.npix = p.N;
      p.gb = make_pix(Ha * Wb, Wb, Hg, Wg, Kp, sh, sw, a, b);
      p.tb = make_tap(Kp, Ss, Wg);
      p.tb.t0 = (r0 * Wg + s0) * Kp;
      p.tb.rstep = sh * Wg * Kp;
      p.tb.sstep = sw * Kp;
      p.OPQ = Ha * Wb; p.dOPQ = make_fastdiv(Ha * Wb);
      p.OQ = Wb; p.dOQ = make_fastdiv(Wb);
      p.strided_out = 1;
      p.o_sh = sh; p.o_sw = sw; p.o_oh = a; p.o_ow = b; p.o_H = H; p.o_W = W;
      p.out2 = (unsigned short*)out2;
      p.H2 = H2; p.W2 = W2; p.C2 = C2;
      p.t2 = t2 + a * d2h; p.l2 = l2 + b * d2w; p.d2h = d2h * sh; p.d2w = d2w * sw;
      p.write_nchw = out2 == nullptr ? 1 : write_nchw;
      dispatch<CN_DGRAD>(p, s);
    }
}

// strided data gradient (sh or sw > 1) over the stride-dilated staged G, by stride phases
extern "C" void fm_conv_nhwc_dgrad_strided(const void* gs, long gs_bytes, const void* w, void* wsub, void* dx, int accum, int N,
                                           int C, int H, int W, int K, int R, int S, int Kp, int Hg, int Wg, int gt, int gl,
                                           int sh, int sw, void* out2, int H2, int W2, int C2, int t2, int l2, int d2h,
                                           int d2w, int write_nchw, hipStream_t s) {
  dgrad_phases(gs, gs_bytes, w, wsub, dx, accum, N, C, H, W, K, R, S, Kp, Hg, Wg, gt, gl, sh, sw, out2, H2, W2, C2, t2, l2,
               d2h, d2w, write_nchw, s);
}
