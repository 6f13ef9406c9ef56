// DLRM dot feature interaction on MFMA (absent in the reference: caveat C3; the closest reference
// path is the DotCompressor test model built from concat/reshape/transpose/batch_matmul,
// src/ops/tests/test_harness.py:96-186, i.e. cuBLAS strided-batched GEMMs + copies).
//
// Forward, one wave per sample b:  Z = [x; e_1; ..; e_{F-1}] (F <= 32 rows of D bf16)
//   G = Z Z^T with v_mfma_f32_32x32x16_bf16: the A and B fragments of a Gram matrix are the SAME
//   register (lane l holds Z[l&31][k0 + 8(l>>5) .. +7]), D/16 MFMAs per sample;
//   out[b] = [x | strictly-lower(G) | 0-pad] assembled in LDS and written with 16-B stores.
// Backward: S = dG + dG^T gathered from dOut's packed triangle; dZ = S Z with the same MFMA
//   (A = S rows gathered per lane from the staged dOut row with precomputed positions, B = Z
//   columns via the transposing ds_read_b64_tr_b16);
//   dZ_0 += dOut[:, :D].  Inputs/grads are pointer tables, so it also reads/writes concat slices.
#include "common.h"

#include <cstdlib>

namespace {

constexpr int MAXF = 32;
struct PtrTab {
  const unsigned short* p[MAXF];
};
struct MPtrTab {
  unsigned short* p[MAXF];
};

typedef __attribute__((address_space(3))) bf16x4_t lds_v4_t;

FM_DEVICE int pair_pos(int i, int j, int self) { return self ? (i * (i + 1) / 2 + j) : (i * (i - 1) / 2 + j); }

__global__ void __launch_bounds__(256) fm_dot_fwd(PtrTab Z, long ldz, unsigned short* __restrict__ out, long ldo,
                                                 long B, int F, int D, int W, int self) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned short* row = reinterpret_cast<unsigned short*>(smem) + wave * W;
  const int waves_total = gridDim.x * (blockDim.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  for (long b = blockIdx.x * (blockDim.x >> 6) + wave; b < B; b += waves_total) {
    f32x16_t acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    const unsigned short* zr = (r < F) ? (Z.p[r] + b * ldz) : nullptr;
    for (int k0 = 0; k0 < D; k0 += 16) {
      bf16x8_t f;
      if (zr) f = *reinterpret_cast<const bf16x8_t*>(zr + k0 + 8 * h);
      else f = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<bf16x8v_t*>(&f), *reinterpret_cast<bf16x8v_t*>(&f),
                                                    acc, 0, 0, 0);
    }
    // stage x and the padding
    for (int c = lane; c < D; c += 64) row[c] = Z.p[0][b * ldz + c];
    const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
    for (int c = D + npairs + lane; c < W; c += 64) row[c] = 0;
    // scatter the lower triangle: lane holds G[i][j], j = lane&31, i = (q&3) + 8(q>>2) + 4h
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int i = (q & 3) + 8 * (q >> 2) + 4 * h;
      int j = r;
      if (i < F && (self ? j <= i : j < i)) row[D + pair_pos(i, j, self)] = f2bf(acc[q]);
    }
    FM_WAVE_LDS_SYNC();
    // coalesced write of the assembled row
    unsigned short* o = out + b * ldo;
    for (int c = lane * 8; c < W; c += 64 * 8) *reinterpret_cast<u32x4_t*>(o + c) = *reinterpret_cast<const u32x4_t*>(row + c);
    FM_WAVE_LDS_SYNC();
  }
}

__global__ void __launch_bounds__(256) fm_dot_bwd(PtrTab Z, long ldz, const unsigned short* __restrict__ dout, long ldo,
                                                 MPtrTab dZ, long lddz, unsigned acc_mask, long B, int F, int D,
                                                 int self) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int Dp = (D + 31) & ~31;  // LDS image padded to whole 32-column MFMA tiles
  const int zbytes = 32 * Dp * 2;
  char* base = smem + wave * (zbytes + 32 * 32 * 2);
  unsigned short* zs = reinterpret_cast<unsigned short*>(base);            // [32][D]
  unsigned short* ss = reinterpret_cast<unsigned short*>(base + zbytes);   // [32][32]
  const int waves_total = gridDim.x * (blockDim.x >> 6);
  const int chunks_per_row = Dp / 8;
  for (long b = blockIdx.x * (blockDim.x >> 6) + wave; b < B; b += waves_total) {
    // stage Z (rows >= F zero)
    for (int c = lane; c < 32 * chunks_per_row; c += 64) {
      int i = c / chunks_per_row, k = (c % chunks_per_row) * 8;
      u32x4_t v = {0u, 0u, 0u, 0u};
      if (i < F && k < D) v = *reinterpret_cast<const u32x4_t*>(Z.p[i] + b * ldz + k);
      *reinterpret_cast<u32x4_t*>(zs + i * Dp + k) = v;
    }
    // build S = dG + dG^T (bf16) from the packed triangle
    const unsigned short* dp = dout + b * ldo + D;
    for (int e = lane; e < 32 * 32; e += 64) {
      int i = e >> 5, j = e & 31;
      float v = 0.f;
      if (i < F && j < F) {
        if (i > j) v = bf2f(dp[pair_pos(i, j, self)]);
        else if (j > i) v = bf2f(dp[pair_pos(j, i, self)]);
        else if (self) v = 2.f * bf2f(dp[pair_pos(i, i, self)]);
      }
      ss[e] = f2bf(v);
    }
    FM_WAVE_LDS_SYNC();
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    for (int nt = 0; nt < Dp / 32; ++nt) {
      f32x16_t acc;
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[t] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(ss + (lane & 31) * 32 + 16 * ks + 8 * (lane >> 5));
        int krow = 16 * ks + 8 * (g >> 1) + q;
        int col = 32 * nt + 16 * (g & 1) + 4 * p;
        bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_t*)(zs + krow * Dp + col));
        bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_t*)(zs + (krow + 4) * Dp + col));
        bf16x8_t bb;
        bb.lo = lo;
        bb.hi = hi;
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<bf16x8v_t*>(&a), *reinterpret_cast<bf16x8v_t*>(&bb),
                                                      acc, 0, 0, 0);
      }
      const int n = 32 * nt + (lane & 31);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        int i = (t & 3) + 8 * (t >> 2) + 4 * (lane >> 5);
        if (i < F && n < D && dZ.p[i] != nullptr) {
          float v = acc[t];
          if (i == 0) v += bf2f(dout[b * ldo + n]);
          unsigned short* d = dZ.p[i] + b * lddz + n;
          if (acc_mask & (1u << i)) v += bf2f(*d);
          *d = f2bf(v);
        }
      }
    }
    FM_WAVE_LDS_SYNC();
  }
}


// ---------------------------------------------------------------------------------------------
// Specialised kernels for a compile-time D (32/64/128; DLRM uses 128) and 16-B aligned rows:
// every global access is a 16-B vector access issued before its first use (no dependent
// round trips per sample), the x part of the output comes straight from the MFMA operand
// registers, and the backward stages dOut and Z with vector loads and writes dZ through an
// LDS transpose with 16-B stores (the generic kernels above issue 2-B scalar loads/stores).
template <int DT>
__global__ void __launch_bounds__(256) fm_dot_fwd_t(PtrTab Z, long ldz, unsigned short* __restrict__ out, long ldo,
                                                   long B, int F, int W, int self) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KS = DT / 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned short* row = reinterpret_cast<unsigned short*>(smem) + wave * W;
  const int waves_total = gridDim.x * (blockDim.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  // persistent waves: the Z rows of the NEXT sample are loaded before this sample's MFMAs and
  // output writes, so every wave keeps one sample's loads in flight behind its compute
  const unsigned short* zbase = (r < F) ? Z.p[r] : Z.p[0];
  const bool zok = r < F;
  long b = blockIdx.x * (blockDim.x >> 6) + wave;
  bf16x8_t f[KS];
  {
    const unsigned short* zr = zbase + min(b, B - 1) * ldz + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) f[ks] = *reinterpret_cast<const bf16x8_t*>(zr + 16 * ks);
  }
  for (; b < B; b += waves_total) {
    bf16x8_t fn[KS];
    {
      const unsigned short* zr = zbase + min(b + waves_total, B - 1) * ldz + 8 * h;   // clamped: unconditional
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) fn[ks] = *reinterpret_cast<const bf16x8_t*>(zr + 16 * ks);
    }
    if (!zok) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) f[ks] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
    f32x16_t acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<bf16x8v_t*>(&f[ks]), *reinterpret_cast<bf16x8v_t*>(&f[ks]),
                                                    acc, 0, 0, 0);
    if (r == 0) {   // lanes 0 / 32 hold row 0 = the dense features x
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<bf16x8_t*>(row + 16 * ks + 8 * h) = f[ks];
    }
    for (int c = DT + npairs + lane; c < W; c += 64) row[c] = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int i = (q & 3) + 8 * (q >> 2) + 4 * h;
      if (i < F && (self ? r <= i : r < i)) row[DT + pair_pos(i, r, self)] = f2bf(acc[q]);
    }
    FM_WAVE_LDS_SYNC();
    unsigned short* o = out + b * ldo;
    for (int c = lane * 8; c < W; c += 64 * 8) *reinterpret_cast<u32x4_t*>(o + c) = *reinterpret_cast<const u32x4_t*>(row + c);
    FM_WAVE_LDS_SYNC();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) f[ks] = fn[ks];
  }
}

template <int DT>
__global__ void __launch_bounds__(256) fm_dot_bwd_t(PtrTab Z, long ldz, const unsigned short* __restrict__ dout, long ldo,
                                                   MPtrTab dZ, long lddz, unsigned acc_mask, long B, int F, int W, int self) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CPR = DT / 8;                 // 16-B chunks per Z row
  constexpr int ZCH = 32 * CPR / 64;          // Z chunks per lane (rows >= F are zero)
  constexpr int NT = DT / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wpad = (W + 7) & ~7;
  char* base = smem + wave * (32 * DT * 2 + wpad * 2);
  unsigned short* zs = reinterpret_cast<unsigned short*>(base);                        // [32][DT]
  unsigned short* ds = reinterpret_cast<unsigned short*>(base + 32 * DT * 2);          // dOut row [W]
  const int waves_total = gridDim.x * (blockDim.x >> 6);
  // MFMA A operand of dZ = S Z (S = dG + dG^T from dOut's packed triangle) straight from the staged
  // dOut row: lane (r = lane&31, h = lane>>5) holds S[r][16ks + 8h + e], whose dOut position is
  // the same for every sample -- computed once here instead of building S in LDS per sample
  short apos[2][8];           // -1: zero entry
  unsigned dmask = 0;         // diagonal entries (self interaction: 2 x dG_ii)
  {
    const int r = lane & 31;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = 16 * ks + 8 * (lane >> 5) + e;
        int pos = -1;
        if (r < F && j < F) {
          if (r > j) pos = pair_pos(r, j, self);
          else if (j > r) pos = pair_pos(j, r, self);
          else if (self) {
            pos = pair_pos(r, r, self);
            dmask |= 1u << (8 * ks + e);
          }
        }
        apos[ks][e] = (short)pos;
      }
  }
  // persistent waves with the next sample's Z rows and dOut row prefetched into registers
  // (clamped addresses: every load unconditional) while this sample is processed
  const bool dload = lane * 8 < W;
  auto load = [&](long bb, u32x4_t (&zv)[ZCH], u32x4_t& dv) {
    bb = min(bb, B - 1);
#pragma unroll
    for (int t = 0; t < ZCH; ++t) {
      const int c = lane + 64 * t, i = c / CPR, k = (c % CPR) * 8;
      zv[t] = *reinterpret_cast<const u32x4_t*>(Z.p[i < F ? i : 0] + bb * ldz + k);
    }
    dv = *reinterpret_cast<const u32x4_t*>(dout + bb * ldo + (dload ? lane * 8 : 0));
  };
  long b = blockIdx.x * (blockDim.x >> 6) + wave;
  u32x4_t zv[ZCH], dv;
  load(b, zv, dv);
  for (; b < B; b += waves_total) {
    u32x4_t zn[ZCH], dn;
    load(b + waves_total, zn, dn);
#pragma unroll
    for (int t = 0; t < ZCH; ++t) {
      const int i = (lane + 64 * t) / CPR;
      if (i >= F) zv[t] = u32x4_t{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int t = 0; t < ZCH; ++t) {
      const int c = lane + 64 * t, i = c / CPR, k = (c % CPR) * 8;
      *reinterpret_cast<u32x4_t*>(zs + i * DT + k) = zv[t];
    }
    if (dload) *reinterpret_cast<u32x4_t*>(ds + lane * 8) = dv;
    FM_WAVE_LDS_SYNC();
    const unsigned short* dp = ds + DT;
    bf16x8_t afr[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int pos = apos[ks][e];
        float v = bf2f(dp[pos < 0 ? 0 : pos]);      // unconditional (clamped) LDS read
        v = pos < 0 ? 0.f : v;
        if ((dmask >> (8 * ks + e)) & 1u) v *= 2.f;
        afr[ks][e] = (short)f2bf(v);
      }
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    f32x16_t acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[nt][t] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t a = afr[ks];
        int krow = 16 * ks + 8 * (g >> 1) + q;
        int col = 32 * nt + 16 * (g & 1) + 4 * p;
        bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_t*)(zs + krow * DT + col));
        bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_t*)(zs + (krow + 4) * DT + col));
        bf16x8_t bb;
        bb.lo = lo;
        bb.hi = hi;
        acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<bf16x8v_t*>(&a),
                                                          *reinterpret_cast<bf16x8v_t*>(&bb), acc[nt], 0, 0, 0);
      }
    }
    FM_WAVE_LDS_SYNC();    // every lane is done reading zs: reuse it for the dZ tile
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = 32 * nt + (lane & 31);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        int i = (t & 3) + 8 * (t >> 2) + 4 * (lane >> 5);
        zs[i * DT + n] = f2bf(acc[nt][t]);
      }
    }
    FM_WAVE_LDS_SYNC();
    for (int c = lane; c < F * CPR; c += 64) {
      const int i = c / CPR, k = (c % CPR) * 8;
      unsigned short* d = dZ.p[i];
      if (d == nullptr) continue;
      d += b * lddz + k;
      bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(zs + i * DT + k);
      const bool add_x = i == 0, add_old = (acc_mask >> i) & 1u;
      if (add_x || add_old) {
        bf16x8_t x = add_x ? *reinterpret_cast<const bf16x8_t*>(ds + k) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
        bf16x8_t o = add_old ? *reinterpret_cast<const bf16x8_t*>(d) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[e] = (short)f2bf(bf2f((unsigned short)v[e]) + bf2f((unsigned short)x[e]) + bf2f((unsigned short)o[e]));
      }
      *reinterpret_cast<bf16x8_t*>(d) = v;
    }
    FM_WAVE_LDS_SYNC();
#pragma unroll
    for (int t = 0; t < ZCH; ++t) zv[t] = zn[t];
    dv = dn;
  }
}

// ---------------------------------------------------------------------------------------------
// fp32 (reference-precision) interaction on the exact f32-input MFMA v_mfma_f32_32x32x2_f32.
// Forward: lane (r = lane&31, h = lane>>5) holds row r of Z restricted to the k-half h (the Gram
// matrix sums over k in any order, so half h takes k in [h*D/2, (h+1)*D/2) and MFMA step s uses
// k = h*D/2 + s); the same register is the A and B operand.  Backward: dZ = S Z with the A operand
// S[r][2ks + h] gathered from the staged dOut row through per-lane positions (computed once) and
// B = Z[2ks + h][32nt + r] from the fp32 Z rows staged in LDS.  DT = D (16/32/64/128) or 0 for a
// runtime D (scalar loads, any even D).
struct PtrTabF {
  const float* p[MAXF];
};
struct MPtrTabF {
  float* p[MAXF];
};
FM_DEVICE const float* zrow(const PtrTabF& Z, long ldz, int i, long b) { return Z.p[i] + b * ldz; }

template <int DT>
__global__ void __launch_bounds__(256) fm_dot_fwd_f32(PtrTabF Z, long ldz, float* __restrict__ out, long ldo, long B,
                                                     int F, int Drt, int W, int self) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int D = DT > 0 ? DT : Drt;
  const int half = D / 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* row = reinterpret_cast<float*>(smem) + wave * W;
  const int waves_total = gridDim.x * (blockDim.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  const bool zok = r < F;
  const float* zbase = (zok ? Z.p[r] : Z.p[0]) + h * half;
  constexpr int NV = DT > 0 ? DT / 8 : 1;    // float4 per lane (k-half of DT floats)
  // persistent waves, one register set: zn[v] holds this sample's chunk v and is reloaded with the
  // NEXT sample's chunk right after its four MFMAs are issued (no loop-carried register copies,
  // which would make the compiler wait for the whole prefetch at the loop back edge).  Lanes with
  // r >= F read row 0: their Gram rows/columns are never written out.
  f32x4_t zn[NV];
  const long b_first = blockIdx.x * (blockDim.x >> 6) + wave;
  if constexpr (DT > 0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) zn[v] = *reinterpret_cast<const f32x4_t*>(zbase + min(b_first, B - 1) * ldz + 4 * v);
  }
  for (long b = b_first; b < B; b += waves_total) {
    f32x16_t acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    if constexpr (DT > 0) {
      const long bn = min(b + waves_total, B - 1);
#pragma unroll
      for (int v = 0; v < NV; ++v) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(zn[v][e], zn[v][e], acc, 0, 0, 0);
        if (r == 0) *reinterpret_cast<f32x4_t*>(row + h * half + 4 * v) = zn[v];
        zn[v] = *reinterpret_cast<const f32x4_t*>(zbase + bn * ldz + 4 * v);
        __builtin_amdgcn_sched_barrier(0);   // keep the reload between this chunk's MFMAs and the next's
      }
    } else {
      for (int k = 0; k < half; ++k) {
        const float a = zok ? zbase[b * ldz + k] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, acc, 0, 0, 0);
        if (r == 0) row[h * half + k] = a;
      }
    }
    for (int c = D + npairs + lane; c < W; c += 64) row[c] = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = (q & 3) + 8 * (q >> 2) + 4 * h;
      if (i < F && (self ? r <= i : r < i)) row[D + pair_pos(i, r, self)] = acc[q];
    }
    FM_WAVE_LDS_SYNC();
    float* o = out + b * ldo;
    if (DT > 0 && (W & 3) == 0 && (ldo & 3) == 0 && W <= 1024) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {     // fixed trip count: straight-line code keeps the waitcnts exact
        const int c = lane * 4 + 256 * t;
        if (c < W) *reinterpret_cast<f32x4_t*>(o + c) = *reinterpret_cast<const f32x4_t*>(row + c);
      }
    } else if ((W & 3) == 0 && (ldo & 3) == 0) {
      for (int c = lane * 4; c < W; c += 256) *reinterpret_cast<f32x4_t*>(o + c) = *reinterpret_cast<const f32x4_t*>(row + c);
    } else {
      for (int c = lane; c < W; c += 64) o[c] = row[c];
    }
    FM_WAVE_LDS_SYNC();
  }
}

template <int DT>
__global__ void __launch_bounds__(256) fm_dot_bwd_f32(PtrTabF Z, long ldz, const float* __restrict__ dout, long ldo,
                                                     MPtrTabF dZ, long lddz, unsigned acc_mask, long B, int F, int Drt,
                                                     int W, int self, int act0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int D = DT > 0 ? DT : Drt;
  const int Dp = (D + 31) & ~31;                 // staged Z rows padded to whole 32-column tiles
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wpad = (W + 3) & ~3;
  float* zs = reinterpret_cast<float*>(smem) + (long)wave * (32 * Dp + wpad);   // [32][Dp]
  float* ds = zs + 32 * Dp;                                                     // dOut row [W]
  const int waves_total = gridDim.x * (blockDim.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  // A operand positions: lane holds S[r][j = 2ks + h] (ks = 0..15) = dOut pair (r, j) (+ diag x2)
  short apos[16];
  unsigned dmask = 0;
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int j = 2 * ks + h;
    int pos = -1;
    if (r < F && j < F) {
      if (r > j) pos = pair_pos(r, j, self);
      else if (j > r) pos = pair_pos(j, r, self);
      else if (self) {
        pos = pair_pos(r, r, self);
        dmask |= 1u << ks;
      }
    }
    apos[ks] = (short)pos;
  }
  // DT > 0: persistent waves with the next sample's Z rows and dOut row prefetched into registers
  // (clamped addresses, every load unconditional) while this sample is staged and multiplied
  constexpr int DPT = DT > 0 ? ((DT + 31) & ~31) : 32;
  constexpr int CPRP = DPT / 4;                    // float4 chunks per staged Z row
  constexpr int ZCH = DT > 0 ? 32 * CPRP / 64 : 1;
  constexpr int DCH = 4;                           // dOut float4 chunks per lane (W <= 1024)
  f32x4_t zv[ZCH], dv[DCH];
  auto load = [&](long bb) {
    bb = min(bb, B - 1);
#pragma unroll
    for (int t = 0; t < ZCH; ++t) {
      const int c = lane + 64 * t, i = c / CPRP, k = (c % CPRP) * 4;
      const bool ok = i < F && k < D;
      zv[t] = *reinterpret_cast<const f32x4_t*>(Z.p[ok ? i : 0] + bb * ldz + (ok ? k : 0));
      if (!ok) zv[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int t = 0; t < DCH; ++t) {
      const int c = 4 * (lane + 64 * t);
      dv[t] = *reinterpret_cast<const f32x4_t*>(dout + bb * ldo + (c < W ? c : 0));
    }
  };
  const bool vec = DT > 0;
  const long b_first = blockIdx.x * (blockDim.x >> 6) + wave;
  if (vec) load(b_first);
  for (long b = b_first; b < B; b += waves_total) {
    // stage Z (rows >= F and columns >= D zero) and the dOut row
    if (vec) {
#pragma unroll
      for (int t = 0; t < ZCH; ++t) {
        const int c = lane + 64 * t, i = c / CPRP, k = (c % CPRP) * 4;
        *reinterpret_cast<f32x4_t*>(zs + i * Dp + k) = zv[t];
      }
#pragma unroll
      for (int t = 0; t < DCH; ++t) {
        const int c = 4 * (lane + 64 * t);
        if (c < W) *reinterpret_cast<f32x4_t*>(ds + c) = dv[t];
      }
      load(b + waves_total);
    } else {
      for (int e = lane; e < 32 * Dp; e += 64) {
        const int i = e / Dp, k = e % Dp;
        zs[e] = (i < F && k < D) ? Z.p[i][b * ldz + k] : 0.f;
      }
      for (int c = lane; c < W; c += 64) ds[c] = dout[b * ldo + c];
    }
    FM_WAVE_LDS_SYNC();
    const float* dp = ds + D;
    float a[16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int pos = apos[ks];
      float v = dp[pos < 0 ? 0 : pos];
      v = pos < 0 ? 0.f : v;
      if ((dmask >> ks) & 1u) v *= 2.f;
      a[ks] = v;
    }
    for (int nt = 0; nt < Dp / 32; ++nt) {
      f32x16_t acc;
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[t] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 16; ++ks)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ks], zs[(2 * ks + h) * Dp + 32 * nt + r], acc, 0, 0, 0);
      const int n = 32 * nt + r;
      if (n < D) {
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const int i = (t & 3) + 8 * (t >> 2) + 4 * h;
          if (i >= F || dZ.p[i] == nullptr) continue;
          float v = acc[t];
          if (i == 0) {
            v += ds[n];
            if (act0 != ACT_NONE) v = act_bwd(act0, zs[n], v);   // z0 staged as row 0
          }
          float* d = dZ.p[i] + b * lddz + n;
          if ((acc_mask >> i) & 1u) v += *d;
          *d = v;
        }
      }
    }
    FM_WAVE_LDS_SYNC();
  }
}

// fp32 forward with COALESCED loads: the per-lane row layout above (lane (r, h) reads 16 B of row
// r per instruction, 54 rows x 16 B per wave-instruction) is request-bound at ~2.9 TB/s.  Here a
// wave-instruction loads whole rows (D/4 lanes per row, 64 / (D/4) rows per instruction, 16 B
// per lane), stages the sample's Z (F <= 32 rows) in a per-wave LDS tile padded to D + 4 floats a
// row (the row-per-lane ds_read_b128 of the MFMA operands is then bank-conflict free), and keeps
// the NEXT sample's rows in flight in registers while this sample's MFMAs and stores run.
template <int D, typename ZT = PtrTabF, bool X3 = false>
__global__ void __launch_bounds__(256, 2) fm_dot_fwd_f32s(ZT Z, long ldz, float* __restrict__ out, long ldo, long B,
                                                          int F, int W, int self) {
  constexpr int LPR = D / 4, RPI = 64 / LPR, NI = 32 / RPI, RS = D + 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wpad = (W + 3) & ~3;
  float* zs = reinterpret_cast<float*>(smem) + (long)wave * (32 * RS + wpad);
  float* row = zs + 32 * RS;
  const int waves_total = gridDim.x * (blockDim.x >> 6);
  const int lr = lane / LPR, lc = lane - lr * LPR;
  const int r = lane & 31, h = lane >> 5;
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  f32x4_t zr[NI];
  auto load = [&](long bb) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = i * RPI + lr;
      zr[i] = *reinterpret_cast<const f32x4_t*>(zrow(Z, ldz, j < F ? j : F - 1, bb) + 4 * lc);
    }
  };
  const long b_first = blockIdx.x * (blockDim.x >> 6) + wave;
  load(min(b_first, B - 1));
  for (long b = b_first; b < B; b += waves_total) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = i * RPI + lr;
      if (j < F) *reinterpret_cast<f32x4_t*>(zs + j * RS + 4 * lc) = zr[i];
    }
    FM_WAVE_LDS_SYNC();
    load(min(b + waves_total, B - 1));
    f32x16_t acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    if constexpr (X3) {
      // exact three-way bf16 split of every fp32 value (gemm_x3.hip): G = sum of the six products
      // with plane indices summing to <= 2 on v_mfma_f32_32x32x16_bf16 (32 cycles per 16 k against
      // 8 x 16 for 32x32x2f32); lane (r, h) holds Z[r][16 s + 8 h .. + 7] for both operands
#pragma unroll
      for (int st = 0; st < D / 16; ++st) {
        const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(zs + r * RS + 16 * st + 8 * h);
        const f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(zs + r * RS + 16 * st + 8 * h + 4);
        unsigned ph[4], pm[4], pl[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float a = u < 2 ? x0[2 * u] : x1[2 * u - 4], b = u < 2 ? x0[2 * u + 1] : x1[2 * u - 3];
          fm_split3_pair(a, b, ph[u], pm[u], pl[u]);
        }
        const bf16x8v_t H = __builtin_bit_cast(bf16x8v_t, u32x4_t{ph[0], ph[1], ph[2], ph[3]});
        const bf16x8v_t Mm = __builtin_bit_cast(bf16x8v_t, u32x4_t{pm[0], pm[1], pm[2], pm[3]});
        const bf16x8v_t L = __builtin_bit_cast(bf16x8v_t, u32x4_t{pl[0], pl[1], pl[2], pl[3]});
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(L, H, acc, 0, 0, 0);    // small terms first
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(H, L, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Mm, Mm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Mm, H, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(H, Mm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(H, H, acc, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int v = 0; v < D / 8; ++v) {
        const f32x4_t x = *reinterpret_cast<const f32x4_t*>(zs + r * RS + h * (D / 2) + 4 * v);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[e], x[e], acc, 0, 0, 0);
      }
    }
    // output row: [ z_0 (D) | pairs | zero pad ]
    for (int c = 4 * lane; c < D; c += 256) *reinterpret_cast<f32x4_t*>(row + c) = *reinterpret_cast<const f32x4_t*>(zs + c);
    for (int c = D + npairs + lane; c < W; c += 64) row[c] = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = (q & 3) + 8 * (q >> 2) + 4 * h;
      if (i < F && (self ? r <= i : r < i)) row[D + pair_pos(i, r, self)] = acc[q];
    }
    FM_WAVE_LDS_SYNC();
    float* o = out + b * ldo;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = lane * 4 + 256 * t;
      if (c < W) *reinterpret_cast<f32x4_t*>(o + c) = *reinterpret_cast<const f32x4_t*>(row + c);
    }
    FM_WAVE_LDS_SYNC();
  }
}

// fp32 backward with the B operand straight from global memory (D = 32E, E = 1/2/4): the column
// map of N-tile e is n = E*r + e, so lane (r, h) loads Z_j[E r .. E r + E-1] of each row
// j = 2ks + h with ONE E-float load and that register feeds the E MFMAs of step ks; the E
// accumulators then hold C[i][E r .. E r + E-1] for the lane's 16 rows i -> E-float stores of
// whole 32E-column rows.  No Z staging in LDS (only the dOut row, for the per-lane S gather),
// so a wave keeps the NEXT sample's Z rows and dOut chunks in flight in registers while this
// sample's (F+1)/2 x E MFMAs run.  Steps past F are skipped (uniform), not padded to 32.
template <int E> struct VecF { using type = float __attribute__((ext_vector_type(E))); };
template <> struct VecF<1> { using type = float; };

template <int E, int NKS, bool ACC, typename ZT = PtrTabF>
__global__ void __launch_bounds__(256, 2) fm_dot_bwd_f32r(ZT Z, long ldz, const float* __restrict__ dout, long ldo,
                                                         MPtrTabF dZ, long lddz, unsigned acc_mask, long B, int F,
                                                         int W, int self, int act0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int D = 32 * E;
  constexpr int DCH = 4;                           // dOut float4 chunks per lane (W <= 1024)
  using vecE = typename VecF<E>::type;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wpad = (W + 3) & ~3;
  float* ds = reinterpret_cast<float*>(smem) + (long)wave * wpad;
  const int waves_total = gridDim.x * (blockDim.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  // A operand positions: S[r][j = 2ks + h]; j >= F -> 0 (the B row loaded for it is row F-1)
  short apos[NKS];
  unsigned dmask = 0;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int j = 2 * ks + h;
    int pos = -1;
    if (r < F && j < F) {
      if (r > j) pos = pair_pos(r, j, self);
      else if (j > r) pos = pair_pos(j, r, self);
      else if (self) {
        pos = pair_pos(r, r, self);
        dmask |= 1u << ks;
      }
    }
    apos[ks] = (short)pos;
  }
  // zn[ks] holds row 2ks+h of the CURRENT sample; right after its E MFMAs are issued it is
  // reloaded with the NEXT sample's row (one register set; the loads overlap the remaining
  // steps and the stores).  All loops have compile-time trip counts (NKS steps, rows >= F
  // clamped) so the compiler's vmcnt waits stay exact instead of draining the prefetch.
  vecE zn[NKS];
  f32x4_t dn[DCH];
  auto load_row = [&](long bb, int ks) {
    const float* p0 = zrow(Z, ldz, min(2 * ks, F - 1), bb);
    const float* p1 = zrow(Z, ldz, min(2 * ks + 1, F - 1), bb);
    zn[ks] = *reinterpret_cast<const vecE*>((h ? p1 : p0) + E * r);
  };
  auto load_dout = [&](long bb) {
#pragma unroll
    for (int t = 0; t < DCH; ++t) {
      const int c = 4 * (lane + 64 * t);
      dn[t] = *reinterpret_cast<const f32x4_t*>(dout + bb * ldo + (c < W ? c : 0));
    }
  };
  const long b_first = blockIdx.x * (blockDim.x >> 6) + wave;
  {
    const long b0 = min(b_first, B - 1);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) load_row(b0, ks);
    load_dout(b0);
  }
  for (long b = b_first; b < B; b += waves_total) {
    const long bn = min(b + waves_total, B - 1);
#pragma unroll
    for (int t = 0; t < DCH; ++t) {
      const int c = 4 * (lane + 64 * t);
      if (c < W) *reinterpret_cast<f32x4_t*>(ds + c) = dn[t];
    }
    FM_WAVE_LDS_SYNC();
    load_dout(bn);
    const float* dp = ds + D;
    float a[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int pos = apos[ks];
      float v = dp[pos < 0 ? 0 : pos];
      v = pos < 0 ? 0.f : v;
      if ((dmask >> ks) & 1u) v *= 2.f;
      a[ks] = v;
    }
    const vecE x0 = *reinterpret_cast<const vecE*>(ds + E * r);   // dZ_0 += dOut[:, :D]
    const vecE z0 = zn[0];         // lanes h = 0: row 0 of this sample (for act0; zn is reloaded below)
    f32x16_t acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[e][t] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        float bz;
        if constexpr (E == 1) bz = zn[ks];
        else bz = zn[ks][e];
        acc[e] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ks], bz, acc[e], 0, 0, 0);
      }
      load_row(bn, ks);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int i0 = (t & 3) + 8 * (t >> 2);
      if (i0 >= F) continue;                                   // uniform
      const int i = i0 + 4 * h;
      float* q0 = dZ.p[i0];
      float* q1 = dZ.p[i0 + 4];
      float* q = h ? q1 : q0;
      vecE v;
      if constexpr (E == 1) v = acc[0][t];
      else {
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = acc[e][t];
      }
      if (i == 0) {
        v += x0;
        // act0: the activation backward of feature 0's producer (the bottom MLP's last layer,
        // whose output z0 is), so that layer skips its own act-bwd pass
        if (act0 != ACT_NONE) {
          if constexpr (E == 1) v = act_bwd(act0, z0, v);
          else {
#pragma unroll
            for (int e = 0; e < E; ++e) v[e] = act_bwd(act0, z0[e], v[e]);
          }
        }
      }
      if (i < F && q != nullptr) {
        float* d = q + b * lddz + E * r;
        if constexpr (ACC) {
          if ((acc_mask >> i) & 1u) v += *reinterpret_cast<const vecE*>(d);
        }
        *reinterpret_cast<vecE*>(d) = v;
      }
    }
    FM_WAVE_LDS_SYNC();
  }
}

FM_HOST_DEVICE bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// persistent-grid size of the interaction kernels (4 waves per block; each wave loops over
// samples with the next one prefetched)
long dot_block_cap() { return 512L; }

}  // namespace

extern "C" void fm_dot_interaction_fwd_f32(const float* const* z, int F, long ldz, float* out, long ldo, long B, int D,
                                           int W, int self, hipStream_t s) {
  PtrTabF t;
  for (int i = 0; i < MAXF; ++i) t.p[i] = i < F ? z[i] : nullptr;
  const int waves = 4;
  const long blocks = std::min<long>((B + waves - 1) / waves, dot_block_cap());
  bool fast = (D == 16 || D == 32 || D == 64 || D == 128) && ldz % 4 == 0;
  for (int i = 0; i < F; ++i) fast = fast && al16(z[i]);
  // the staged kernel with the Gram on the bf16 matrix cores through the exact three-way split:
  // 8192 x 27 x 128 forward 35.6 -> 29.4 us against the fp32 MFMA, MLPerf fp32 step -6 us
  // (profiles/dot_fwd_x3_ab_r5y.txt; the fp32-MFMA and unstaged A/B forms deleted in r6)
  if (fast && D >= 32 && F <= 32 && (W & 3) == 0 && (ldo & 3) == 0 && W <= 1024 && al16(out)) {
    const size_t lds_s = (size_t)waves * (32 * (D + 4) + ((W + 3) & ~3)) * 4;
    auto ks = D == 128 ? fm_dot_fwd_f32s<128, PtrTabF, true> : D == 64 ? fm_dot_fwd_f32s<64, PtrTabF, true>
                                                                       : fm_dot_fwd_f32s<32, PtrTabF, true>;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)fm_dot_fwd_f32s<128, PtrTabF, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                96 << 10);
      (void)hipFuncSetAttribute((const void*)fm_dot_fwd_f32s<64, PtrTabF, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                96 << 10);
      (void)hipFuncSetAttribute((const void*)fm_dot_fwd_f32s<32, PtrTabF, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                96 << 10);
      attr = true;
    }
    hipLaunchKernelGGL(ks, dim3((int)blocks), dim3(64 * waves), lds_s, s, t, ldz, out, ldo, B, F, W, self);
    return;
  }
  const size_t lds = (size_t)waves * W * 4;
  auto k = !fast ? fm_dot_fwd_f32<0> : D == 128 ? fm_dot_fwd_f32<128> : D == 64 ? fm_dot_fwd_f32<64>
                                     : D == 32 ? fm_dot_fwd_f32<32> : fm_dot_fwd_f32<16>;
  hipLaunchKernelGGL(k, dim3((int)blocks), dim3(64 * waves), lds, s, t, ldz, out, ldo, B, F, D, W, self);
}

// act0: activation backward (of z[0]'s producer) applied to dz[0]; ACT_NONE = plain gradient
extern "C" void fm_dot_interaction_bwd_f32(const float* const* z, int F, long ldz, const float* dout, long ldo,
                                           float* const* dz, long lddz, unsigned acc_mask, long B, int D, int self,
                                           int act0, hipStream_t s) {
  PtrTabF t;
  MPtrTabF g;
  for (int i = 0; i < MAXF; ++i) {
    t.p[i] = i < F ? z[i] : nullptr;
    g.p[i] = i < F ? dz[i] : nullptr;
  }
  const int waves = 4;
  const long blocks = std::min<long>((B + waves - 1) / waves, dot_block_cap());
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  const int W = D + npairs;                        // dOut columns read
  const int Dp = (D + 31) & ~31;
  bool fast = (D == 16 || D == 32 || D == 64 || D == 128) && ldz % 4 == 0 && ldo % 4 == 0 && al16(dout) && W <= 1024;
  for (int i = 0; i < F; ++i) fast = fast && al16(z[i]);
  if ((D == 32 || D == 64 || D == 128) && ldo % 4 == 0 && al16(dout) && W <= 1024) {
    const int E = D / 32;
    auto alE = [&](const void* q) { return ((uintptr_t)q & (4 * E - 1)) == 0; };
    bool ok = ldz % E == 0 && lddz % E == 0;
    for (int i = 0; i < F; ++i) ok = ok && alE(z[i]) && (dz[i] == nullptr || alE(dz[i]));
    if (ok) {
      const int wpad = (W + 3) & ~3;
      const bool acc = acc_mask != 0;
      const bool k14 = E == 4 && (F + 1) / 2 == 14 && !acc;   // DLRM: 26 tables + dense (F = 27)
      auto k = k14 ? fm_dot_bwd_f32r<4, 14, false>
             : E == 4 ? (acc ? fm_dot_bwd_f32r<4, 16, true> : fm_dot_bwd_f32r<4, 16, false>)
             : E == 2 ? (acc ? fm_dot_bwd_f32r<2, 16, true> : fm_dot_bwd_f32r<2, 16, false>)
                      : (acc ? fm_dot_bwd_f32r<1, 16, true> : fm_dot_bwd_f32r<1, 16, false>);
      hipLaunchKernelGGL(k, dim3((int)blocks), dim3(64 * waves), (size_t)waves * wpad * 4, s, t, ldz, dout, ldo, g, lddz,
                         acc_mask, B, F, W, self, act0);
      return;
    }
  }
  const int Wr = fast ? ((W + 3) & ~3) : W;        // the vector path stages whole 16-B chunks
  const size_t lds = (size_t)waves * (32 * Dp + ((Wr + 3) & ~3)) * 4;
  auto k = !fast ? fm_dot_bwd_f32<0> : D == 128 ? fm_dot_bwd_f32<128> : D == 64 ? fm_dot_bwd_f32<64>
                                     : D == 32 ? fm_dot_bwd_f32<32> : fm_dot_bwd_f32<16>;
  hipLaunchKernelGGL(k, dim3((int)blocks), dim3(64 * waves), lds, s, t, ldz, dout, ldo, g, lddz, acc_mask, B, F, D, Wr,
                     self, act0);
}

extern "C" void fm_dot_interaction_fwd(const void* const* z, int F, long ldz, void* out, long ldo, long B, int D, int W,
                                       int self, hipStream_t s) {
  PtrTab t;
  for (int i = 0; i < MAXF; ++i) t.p[i] = i < F ? (const unsigned short*)z[i] : nullptr;
  int waves = 4;
  long blocks = std::min<long>((B + waves - 1) / waves, dot_block_cap());
  bool fast = (D == 32 || D == 64 || D == 128) && F <= 32 && ldz % 8 == 0 && ldo % 8 == 0 && W % 8 == 0 && al16(out);
  for (int i = 0; i < F; ++i) fast = fast && al16(z[i]);
  if (fast) {
    auto k = D == 128 ? fm_dot_fwd_t<128> : D == 64 ? fm_dot_fwd_t<64> : fm_dot_fwd_t<32>;
    hipLaunchKernelGGL(k, dim3((int)blocks), dim3(64 * waves), waves * W * 2, s, t, ldz, (unsigned short*)out, ldo, B,
                       F, W, self);
    return;
  }
  hipLaunchKernelGGL(fm_dot_fwd, dim3((int)blocks), dim3(64 * waves), waves * W * 2, s, t, ldz, (unsigned short*)out,
                     ldo, B, F, D, W, self);
}

extern "C" void fm_dot_interaction_bwd(const void* const* z, int F, long ldz, const void* dout, long ldo, void* const* dz,
                                       long lddz, unsigned acc_mask, long B, int D, int self, hipStream_t s) {
  PtrTab t;
  MPtrTab g;
  for (int i = 0; i < MAXF; ++i) {
    t.p[i] = i < F ? (const unsigned short*)z[i] : nullptr;
    g.p[i] = i < F ? (unsigned short*)dz[i] : nullptr;
  }
  int waves = 4;
  long blocks = std::min<long>((B + waves - 1) / waves, dot_block_cap());
  const int npairs = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
  const int W = ((D + npairs) + 7) & ~7;    // dOut columns read (x part + packed triangle)
  bool fast = (D == 32 || D == 64 || D == 128) && F <= 32 && ldz % 8 == 0 && ldo % 8 == 0 && lddz % 8 == 0 && al16(dout);
  for (int i = 0; i < F; ++i) fast = fast && al16(z[i]) && (dz[i] == nullptr || al16(dz[i]));
  if (fast) {
    auto k = D == 128 ? fm_dot_bwd_t<128> : D == 64 ? fm_dot_bwd_t<64> : fm_dot_bwd_t<32>;
    size_t lds = waves * (32 * D * 2 + W * 2);
    hipLaunchKernelGGL(k, dim3((int)blocks), dim3(64 * waves), lds, s, t, ldz, (const unsigned short*)dout, ldo, g, lddz,
                       acc_mask, B, F, W, self);
    return;
  }
  const int Dp = (D + 31) & ~31;
  size_t lds = waves * (32 * Dp * 2 + 32 * 32 * 2);
  hipLaunchKernelGGL(fm_dot_bwd, dim3((int)blocks), dim3(64 * waves), lds, s, t, ldz, (const unsigned short*)dout, ldo,
                     g, lddz, acc_mask, B, F, D, self);
}
