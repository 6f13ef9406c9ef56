// Implicit-GEMM convolution on MFMA for gfx950 (MI355X / CDNA4): forward, data gradient and
// weight gradient straight from NCHW activations and [K][C][R][S] weights -- no im2col
// columns, no NCHW<->NHWC transposes, no col2im.
//
// Replaces the reference's cuDNN calls (src/ops/conv_2d.cu:285-296 forward + bias + ReLU,
// :405-432 backward filter / data / bias, algorithm search :216-243 / :872-930).
//
//   fwd    Y[k, (n,p,q)]   = sum_(c,r,s)  W[k, (c,r,s)]   * X[n, c, p*sh+r-pt, q*sw+s-pl]
//   dgrad dX[c, (n,h,w)]   = sum_(k,r,s) Wt[c, (k,r,s)]   * G[n, k, (h+pt-r)/sh, (w+pl-s)/sw]
//   wgrad dW[k, (c,r,s)]  += sum_(n,p,q)  G[n, k, (p,q)]  * X[n, c, p*sh+r-pt, q*sw+s-pl]
//
// G = act'(y) * dY is written (with db) by fm_conv_act_bwd; the weight operand is re-laid by
// fm_conv_wprep into a row-padded matrix (fwd: W [K][CRS8], dgrad: Wt [C][KRS8]) so every A
// tile streams 16-B chunks.  The image operand is GATHERED per tile into LDS.  Two gathers:
//
// * PIXEL-VECTOR (bf16, unit stride -- every AlexNet / ResNet 3x3 / Inception layer but the
//   strided ones): output rows are padded to Qp = roundup(Q, 8) columns, so 8 consecutive GEMM
//   columns are 8 consecutive pixels of ONE image row; for a stride-1 conv they read 8
//   consecutive source pixels -> ONE 16-B buffer load per 8 elements (unaligned allowed), a
//   funnel shift for the left halo and a mask for the right halo / row tail.  fwd and dgrad use
//   an MN-contiguous LDS image [k][pixel] (fragments through ds_read_b64_tr_b16, the same image
//   as gemm.hip's MN operands); wgrad's reduction runs over (n, p, q<Qp) so both of its operands
//   stay K-contiguous and load 8 pixels per instruction too.
// * ELEMENT (fp32 -- MFMA-bound at 157 TF anyway -- and strided convs): thread t owns ONE row of a
//   K-contiguous image and chunks t/R, t/R + 256/R, ...; the chunk index is wave-uniform, so the
//   reduction-index decomposition of each element is scalar work and a lane pays a few VALU + one
//   buffer_load per element.
// Out-of-range elements load through a buffer offset past num_records (returns 0): no branches.
// MFMA: bf16 -> v_mfma_f32_16x16x32_bf16; fp32 -> v_mfma_f32_16x16x4_f32 with the k-permutation
// of gemm_f32.hip (lane group g takes k = 16kk + 4g + s of each row chunk).  Tile BM x 128 x
// (128 B of k), 256 threads = 2x2 waves, register-staged double-buffered LDS (next tile's gathers
// issued before this tile's MFMAs), XCD-aware tile order.  Epilogues: fwd bias + activation into
// NCHW y; dgrad (+)= into NCHW dx; wgrad split over (n,p,q) with fp32 atomics into dW.
#include "gemm_common.h"

#include <algorithm>

namespace {

constexpr int CT = 256;
constexpr unsigned OOB = 0x80000000u;   // buffer offset past num_records: the load returns 0

enum { CONV_FWD = 0, CONV_DGRAD = 1, CONV_WGRAD = 2 };

struct ConvP {
  const void* a;  long a_bytes;        // fwd: Wpad [K][lda]; dgrad: Wt [C][lda]; wgrad: G [N][K][P][Q]
  const void* b;  long b_bytes;        // fwd: X;             dgrad: G;           wgrad: X
  void* out;                           // fwd: Y (T); dgrad: dX (T); wgrad: dW (fp32)
  const float* bias;
  int N, C, H, W, K, R, S, P, Q, sh, sw, pt, pl;
  int M, Ncols, Kred, lda;             // GEMM sizes of this pass (Kred = true reduction length)
  int Qp;                              // pixel-vector path: padded columns per image row
  int act, accum, ksplit, kt_per;
  int tiles_m, tiles_n;
  int a_nel, b_nel;                    // operand sizes in elements (pixel-vector loads stay inside)
  FastDiv dRS, dS;                     // reduction index (ch, r, s) decomposition
  FastDiv dPer, dQp;                   // wgrad pixel-vector reduction index (n, p, q0)
  FastDiv dSh, dSw;                    // strided dgrad: divisibility by the stride
  int adv_c, adv_r, adv_s;             // one bf16 k-tile (64) in (ch, r, s) digits
};

template <typename T> struct TB;
template <> struct TB<unsigned short> { static constexpr int E = 8; };
template <> struct TB<float> { static constexpr int E = 4; };

template <typename T>
FM_DEVICE unsigned ldb1(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  if constexpr (sizeof(T) == 2) return (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0);
  else return (unsigned)__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
}

FM_DEVICE u32x4_t ldb16(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  return __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}

FM_DEVICE __amdgpu_buffer_rsrc_t make_rsrc(const void* p, long bytes) {
  // uniform inputs (kernel arguments) -> the descriptor lives in SGPRs, no waterfall loops
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// Pixel-vector chunks: 8 bf16 of one source row read by ONE 16-B buffer load at the (unaligned)
// position of element 0; elements outside the valid window [lowz, cnt) -- left halo (read from
// the previous row), right halo / row tail (read from the next row) -- are cleared with a mask
// from a 72-entry LDS table (entry lowz * 9 + cnt).  Only a chunk within 8 elements of the
// tensor's first / last element needs its load moved inside the tensor (a load straddling
// num_records comes back as zeros) and a funnel shift; that rare divergent branch lives in
// px_finish.  Split in two so the load latency overlaps the MFMAs: px_issue starts the load and
// packs the fix-up into ``meta``.
constexpr int MASK_ENTRIES = 72;
constexpr int MASK_BYTES = MASK_ENTRIES * 16;

FM_DEVICE void init_mask_table(char* tab, int tid) {
  if (tid < MASK_ENTRIES) {
    const int lowz = tid / 9, cnt = tid % 9;
    u32x4_t m;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool a = lowz <= 2 * j && 2 * j < cnt, b = lowz <= 2 * j + 1 && 2 * j + 1 < cnt;
      m[j] = (a ? 0x0000FFFFu : 0u) | (b ? 0xFFFF0000u : 0u);
    }
    *reinterpret_cast<u32x4_t*>(tab + tid * 16) = m;
  }
}

// want: tensor position of element 0; w0: its source column (< 0: left halo); inside: elements
// t < inside lie inside the row / window
FM_DEVICE u32x4_t px_issue(__amdgpu_buffer_rsrc_t rs, bool ok, int want, int w0, int inside, int nel, unsigned& meta) {
  const int cnt = min(8, inside), lowz = max(0, -w0);
  ok = ok && cnt > lowz;
  const int L = min(max(want, 0), nel - 8);             // the load stays inside the tensor
  const int delta = want - L;                           // 0 except within 8 elements of its ends
  meta = ok ? (unsigned)(lowz * 9 + cnt) | ((unsigned)(delta + 8) << 8) : (8u << 8);
  return ldb16(rs, ok ? (unsigned)L * 2u : OOB);
}

FM_DEVICE u32x4_t px_finish(u32x4_t v, unsigned meta, const char* tab) {
  const int delta = (int)((meta >> 8) & 15) - 8;
  if (delta != 0) {                                     // rare: shift the moved load into place
    unsigned long lo = (unsigned long)v[0] | ((unsigned long)v[1] << 32);
    unsigned long hi = (unsigned long)v[2] | ((unsigned long)v[3] << 32);
    if (delta < 0) {
      const int b = -16 * delta;
      if (b >= 64) {
        hi = lo << (b - 64);
        lo = 0;
      } else {
        hi = (hi << b) | (lo >> (64 - b));
        lo <<= b;
      }
    } else {
      const int b = 16 * delta;
      if (b >= 64) {
        lo = hi >> (b - 64);
        hi = 0;
      } else {
        lo = (lo >> b) | (hi << (64 - b));
        hi >>= b;
      }
    }
    v = u32x4_t{(unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32)};
  }
  return v & *reinterpret_cast<const u32x4_t*>(tab + (meta & 127) * 16);
}

// One operand tile (R rows x 128 B of reduction index) gathered into registers, then LDS.
// ROLE: 0 = padded weight matrix [rows][lda] (16-B chunks), 1 = fwd image columns (element),
// 2 = dgrad G columns (element), 3 = wgrad G rows (element), 4 = wgrad image rows (element),
// 5 = fwd / dgrad pixel-vector columns (MN-contiguous image), 6 = wgrad G rows (pixel-vector),
// 7 = wgrad image rows (pixel-vector).
#define ERAW(t) e[ELT ? i : 0][t]
template <typename T, int R, int ROLE, int MODE>
struct Gather {
  static constexpr int E = TB<T>::E;                 // elements per 16-B chunk
  static constexpr int BKE = 128 / (int)sizeof(T);   // reduction elements per k-tile
  static constexpr int PER_T = R * 8 / CT;
  static constexpr bool PIX = ROLE >= 5;            // pixel-vector chunks (fixed up in finish)
  static constexpr bool ELT = ROLE >= 1 && ROLE <= 4;   // element gathers (packed in finish)
  u32x4_t v[PER_T];
  unsigned meta[PER_T];                               // PIX: px_finish fix-up
  unsigned e[ELT ? PER_T : 1][TB<T>::E];              // ELT: raw element loads
  bool vec_done = false;                              // ELT role 3 took the 16-B chunk path
  int row;        // this thread's tile row (global index)
  bool rowok;
  int base;       // role-specific element offset of the row
  int hb, wb;     // role-specific spatial coordinates of the row
  int rr, ss;     // rows (c, r, s): the row's (r, s)
  // role 5: per chunk, the reduction index (ch, r, s) of its k-row as ch * Hs * Ws, r, r * Ws, s,
  // advanced by 64 (one k-tile) with carries -- no divisions or multiplies in the main loop
  int cho[ROLE == 5 ? PER_T : 1], r5[ROLE == 5 ? PER_T : 1], rw5[ROLE == 5 ? PER_T : 1], s5[ROLE == 5 ? PER_T : 1];

  FM_DEVICE void init(const ConvP& p, int row0, int nrows, int tid, int kt0) {
    const int HW = p.H * p.W, PQ = p.P * p.Q;
    if constexpr (ROLE == 5) {
      // this thread's pixel chunk: 8 columns (tid % 16) of the 128-column tile, fixed for the block
      const bool fwd = MODE == CONV_FWD;
      const int Cs = fwd ? p.C : p.K, Hs = fwd ? p.H : p.P, Ws = fwd ? p.W : p.Q;
      row = row0 + 8 * (tid & 15);
      rowok = row < nrows;
      const int rw = rowok ? row : 0;
      const int Po = fwd ? p.P : p.H;
      const int per = Po * p.Qp;
      const int n = rw / per, rem = rw - n * per;
      const int orow = rem / p.Qp;                        // output row
      wb = rem - orow * p.Qp;                             // first output column of the chunk
      hb = fwd ? orow - p.pt : orow + p.pt;               // source row = hb +/- r
      wb = fwd ? wb - p.pl : wb + p.pl;                   // source column = wb +/- s
      base = n * Cs * Hs * Ws + hb * Ws + wb;             // + ch*Hs*Ws +/- r*Ws +/- s
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int k = kt0 * 64 + (tid >> 4) + 16 * i;
        const int ch = k / (p.R * p.S), rsi = k - ch * p.R * p.S;
        r5[i] = rsi / p.S;
        s5[i] = rsi - r5[i] * p.S;
        cho[i] = ch * Hs * Ws;
        rw5[i] = r5[i] * Ws;
      }
      return;
    }
    row = row0 + tid % R;
    rowok = row < nrows;
    const int rw = rowok ? row : 0;
    if constexpr (ROLE == 0) {
      base = rw * p.lda;
    } else if constexpr (ROLE == 1) {
      const int n = rw / PQ, pq = rw - n * PQ, pp = pq / p.Q, qq = pq - pp * p.Q;
      hb = pp * p.sh - p.pt;
      wb = qq * p.sw - p.pl;
      base = n * p.C * HW + hb * p.W + wb;
    } else if constexpr (ROLE == 2) {
      const int n = rw / HW, hw = rw - n * HW, h = hw / p.W, w = hw - h * p.W;
      hb = h + p.pt;
      wb = w + p.pl;
      base = n * p.K * PQ;
    } else if constexpr (ROLE == 3 || ROLE == 6) {
      base = rw * PQ;
    } else {
      const int RS = p.R * p.S, c = rw / RS, rs = rw - c * RS;
      rr = rs / p.S;
      ss = rs - rr * p.S;
      base = c * HW + rr * p.W + ss;
      hb = c;
    }
  }

  // finish the chunks issued by load(): pixel fix-up shifts / element packing (after the MFMAs
  // of the current tile, so the loads' latency is hidden behind them)
  FM_DEVICE void finish(const char* tab) {
    if constexpr (PIX) {
#pragma unroll
      for (int i = 0; i < PER_T; ++i) v[i] = px_finish(v[i], meta[i], tab);
    } else if constexpr (ELT) {
      if (vec_done) return;
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        if constexpr (sizeof(T) == 2) {
          v[i] = u32x4_t{e[i][0] | (e[i][1] << 16), e[i][2] | (e[i][3] << 16), e[i][4] | (e[i][5] << 16),
                         e[i][6] | (e[i][7] << 16)};
        } else {
          v[i] = u32x4_t{e[i][0], e[i][1], e[i][2], e[i][3]};
        }
      }
    }
  }

  // issue this thread's loads of k-tile kt (results land in v / e, completed by finish())
  FM_DEVICE void load(const ConvP& p, __amdgpu_buffer_rsrc_t rs, int kt, int tid) {
    if constexpr (ROLE == 5) {
      // k-row (tid >> 4) + 16 i of the 64-row k-tile; source position base + ch*Hs*Ws +/- r*Ws +/- s
      const bool fwd = MODE == CONV_FWD;
      const int Hs = fwd ? p.H : p.P, Ws = fwd ? p.W : p.Q;
      const int kb = kt * 64 + (tid >> 4);
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int hs = fwd ? hb + r5[i] : hb - r5[i];
        const int w0 = fwd ? wb + s5[i] : wb - s5[i];
        const bool ok = rowok && kb + 16 * i < p.Kred && (unsigned)hs < (unsigned)Hs;
        const int want = fwd ? base + cho[i] + rw5[i] + s5[i] : base + cho[i] - rw5[i] - s5[i];
        v[i] = px_issue(rs, ok, want, w0, Ws - w0, p.b_nel, meta[i]);
        // advance (ch, r, s) by one k-tile (64 = adv_c*RS + adv_r*S + adv_s)
        s5[i] += p.adv_s;
        const bool c1 = s5[i] >= p.S;
        s5[i] -= c1 ? p.S : 0;
        r5[i] += p.adv_r + (c1 ? 1 : 0);
        rw5[i] += p.adv_r * Ws + (c1 ? Ws : 0);
        const bool c2 = r5[i] >= p.R;
        r5[i] -= c2 ? p.R : 0;
        rw5[i] -= c2 ? p.R * Ws : 0;
        cho[i] += (p.adv_c + (c2 ? 1 : 0)) * Hs * Ws;
      }
      return;
    }
    const int c0 = __builtin_amdgcn_readfirstlane(tid / R);
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int kb = kt * BKE + (c0 + i * (CT / R)) * E;   // wave-uniform first reduction index
      if constexpr (ROLE == 0) {
        v[i] = ldb16(rs, (rowok && kb < p.Kred) ? (unsigned)(base + kb) * sizeof(T) : OOB);
        continue;
      } else if constexpr (ROLE == 6 || ROLE == 7) {
        // k = (n, p, q < Qp): 8 consecutive q of one output row
        const int n = fdiv(kb, p.dPer), rem = kb - n * (p.P * p.Qp), pp = fdiv(rem, p.dQp), q0 = rem - pp * p.Qp;
        const bool okk = rowok && kb < p.Kred;
        if constexpr (ROLE == 6) {       // G[n, row, pp, q0 ..]: lanes differ only in the row
          v[i] = px_issue(rs, okk, (n * p.K * p.P + pp) * p.Q + q0 + base, q0, p.Q - q0, p.a_nel, meta[i]);
        } else {                         // X[n, c, pp + r - pt, q0 + s - pl ..]
          const int hs = pp + rr - p.pt, w0 = q0 + ss - p.pl;
          v[i] = px_issue(rs, okk && (unsigned)hs < (unsigned)p.H, n * p.C * p.H * p.W + (pp - p.pt) * p.W + q0 - p.pl + base,
                          w0, min(p.W - w0, p.Q - q0), p.b_nel, meta[i]);   // t < Q - q0: padded q load as 0
        }
        continue;
      } else if constexpr (ROLE == 1) {
        // k = (c, r, s)
        const int RS = p.R * p.S;
        int c = kb / RS, rem = kb - c * RS, r = rem / p.S, s = rem - r * p.S;
        const int HW = p.H * p.W;
#pragma unroll
        for (int t = 0; t < E; ++t) {
          const bool ok = rowok && kb + t < p.Kred && (unsigned)(hb + r) < (unsigned)p.H &&
                          (unsigned)(wb + s) < (unsigned)p.W;
          ERAW(t) = ldb1<T>(rs, ok ? (unsigned)(base + c * HW + r * p.W + s) * sizeof(T) : OOB);
          if (++s == p.S) { s = 0; if (++r == p.R) { r = 0; ++c; } }
        }
      } else if constexpr (ROLE == 2) {
        // k = (k_out, r, s); G[n, k, (hb - r)/sh, (wb - s)/sw]
        const int RS = p.R * p.S, PQ = p.P * p.Q;
        int k = kb / RS, rem = kb - k * RS, r = rem / p.S, s = rem - r * p.S;
#pragma unroll
        for (int t = 0; t < E; ++t) {
          int hp = hb - r, wp = wb - s;
          bool ok = rowok && kb + t < p.Kred;
          if (p.sh == 1 && p.sw == 1) {
            ok = ok && (unsigned)hp < (unsigned)p.P && (unsigned)wp < (unsigned)p.Q;
          } else {
            const int qh = fdiv(max(hp, 0), p.dSh), qw = fdiv(max(wp, 0), p.dSw);
            ok = ok && hp >= 0 && wp >= 0 && qh * p.sh == hp && qw * p.sw == wp && qh < p.P && qw < p.Q;
            hp = qh;
            wp = qw;
          }
          ERAW(t) = ldb1<T>(rs, ok ? (unsigned)(base + k * PQ + hp * p.Q + wp) * sizeof(T) : OOB);
          if (++s == p.S) { s = 0; if (++r == p.R) { r = 0; ++k; } }
        }
      } else if constexpr (ROLE == 3) {
        // k = (n, pq); G[n, row, pq]
        const int PQ = p.P * p.Q;
        int n = kb / PQ, pq = kb - n * PQ;
        vec_done = PQ % E == 0;
        if (vec_done) {      // the chunk is one contiguous, aligned run inside image n
          v[i] = ldb16(rs, (rowok && kb < p.Kred) ? (unsigned)(n * p.K * PQ + base + pq) * sizeof(T) : OOB);
          continue;
        }
#pragma unroll
        for (int t = 0; t < E; ++t) {
          const bool ok = rowok && kb + t < p.Kred;
          ERAW(t) = ldb1<T>(rs, ok ? (unsigned)(n * p.K * PQ + base + pq) * sizeof(T) : OOB);
          if (++pq == PQ) { pq = 0; ++n; }
        }
      } else {
        // k = (n, p, q); X[n, c, p*sh - pt + r, q*sw - pl + s]
        const int PQ = p.P * p.Q, CHW = p.C * p.H * p.W;
        int n = kb / PQ, pq = kb - n * PQ, pp = pq / p.Q, qq = pq - pp * p.Q;
#pragma unroll
        for (int t = 0; t < E; ++t) {
          const int uh = pp * p.sh - p.pt, uw = qq * p.sw - p.pl;
          const bool ok = rowok && kb + t < p.Kred && (unsigned)(uh + rr) < (unsigned)p.H &&
                          (unsigned)(uw + ss) < (unsigned)p.W;
          ERAW(t) = ldb1<T>(rs, ok ? (unsigned)(n * CHW + uh * p.W + uw + base) * sizeof(T) : OOB);
          if (++qq == p.Q) { qq = 0; if (++pp == p.P) { pp = 0; ++n; } }
        }
      }
    }
  }

  FM_DEVICE void store(char* lds, int tid) const {
    if constexpr (ROLE == 5) {   // MN-contiguous image [64 k][R pixels]
#pragma unroll
      for (int i = 0; i < PER_T; ++i)
        *reinterpret_cast<u32x4_t*>(lds + lds_off<false, R>((tid >> 4) + 16 * i, tid & 15)) = v[i];
      return;
    }
    const int r = tid % R, c0 = tid / R;
#pragma unroll
    for (int i = 0; i < PER_T; ++i)
      *reinterpret_cast<u32x4_t*>(lds + lds_off<true, R>(r, c0 + i * (CT / R))) = v[i];
  }
};

template <typename T, int MR, int NR, int BN, bool BMN>
FM_DEVICE void mma_tile(const char* la, const char* lb, int abase, int bbase, int lane, f32x4_t (&acc)[MR][NR]) {
  const int rowl = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    u32x4_t af[MR], bf[NR];
#pragma unroll
    for (int i = 0; i < MR; ++i)
      af[i] = *reinterpret_cast<const u32x4_t*>(la + lds_off<true, 0>(abase + 16 * i + rowl, 4 * kk + g));
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      if constexpr (BMN) bf[j] = __builtin_bit_cast(u32x4_t, frag<false, BN>(lb, bbase + 16 * j, kk, lane));
      else bf[j] = *reinterpret_cast<const u32x4_t*>(lb + lds_off<true, 0>(bbase + 16 * j + rowl, 4 * kk + g));
    }
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        if constexpr (sizeof(T) == 2) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v_t, bf[j]),
                                                              __builtin_bit_cast(bf16x8v_t, af[i]), acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(bf[j][s]), __uint_as_float(af[i][s]),
                                                             acc[i][j], 0, 0, 0);
        }
      }
  }
}

template <typename T>
FM_DEVICE void st4(T* dst, const float (&v)[4], bool add) {
  if constexpr (sizeof(T) == 2) {
    bf16x4_t o;
    if (add) {
      const bf16x4_t old = *reinterpret_cast<const bf16x4_t*>(dst);
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r] + bf2f((unsigned short)old[r]));
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
    }
    *reinterpret_cast<bf16x4_t*>(dst) = o;
  } else {
    f32x4_t o = {v[0], v[1], v[2], v[3]};
    if (add) o += *reinterpret_cast<const f32x4_t*>(dst);
    *reinterpret_cast<f32x4_t*>(dst) = o;
  }
}

template <typename T, int BM, int MODE, bool PV>
__global__ void __launch_bounds__(CT, 2) fm_conv_igemm(ConvP p) {
  constexpr int BN = 128;
  constexpr int MR = BM / 32, NR = BN / 32;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int AROLE = MODE == CONV_WGRAD ? (PV ? 6 : 3) : 0;
  constexpr int BROLE = MODE == CONV_WGRAD ? (PV ? 7 : 4) : PV ? 5 : MODE == CONV_FWD ? 1 : 2;
  constexpr bool BMN = BROLE == 5;
  extern __shared__ __attribute__((aligned(16))) char smem[];   // 2 x (A, B) tiles + the mask table
  char* tab = smem + 2 * (A_BYTES + B_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int bid = xcd_remap(blockIdx.x, p.tiles_m * p.tiles_n);
  const int tm = bid % p.tiles_m, tn = bid / p.tiles_m;   // row tiles fastest: the big column operand is shared
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.z;
  constexpr int BKE = 128 / (int)sizeof(T);
  const int ktiles = (p.Kred + BKE - 1) / BKE;
  const int kt0 = split * p.kt_per, kt1 = min(ktiles, kt0 + p.kt_per);

  const auto rsa = make_rsrc(p.a, p.a_bytes);
  const auto rsb = make_rsrc(p.b, p.b_bytes);
  Gather<T, BM, AROLE, MODE> ga;
  Gather<T, BN, BROLE, MODE> gb;
  ga.init(p, m0, p.M, tid, kt0);
  gb.init(p, n0, p.Ncols, tid, kt0);
  init_mask_table(tab, tid);
  __syncthreads();

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    ga.load(p, rsa, kt0, tid);
    gb.load(p, rsb, kt0, tid);
    ga.finish(tab);
    gb.finish(tab);
    ga.store(smem, tid);
    gb.store(smem + A_BYTES, tid);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {
      ga.load(p, rsa, kt + 1, tid);
      gb.load(p, rsb, kt + 1, tid);
    }
    const char* la = smem + cur * (A_BYTES + B_BYTES);
    mma_tile<T, MR, NR, BN, BMN>(la, la + A_BYTES, wm * (BM / 2), wn * (BN / 2), lane, acc);
    if (more) {
      ga.finish(tab);
      gb.finish(tab);
      char* nx = smem + (cur ^ 1) * (A_BYTES + B_BYTES);
      ga.store(nx, tid);
      gb.store(nx + A_BYTES, tid);
    }
    __syncthreads();
  }

  // epilogue: lane owns row m = mbase + 16 i + (lane & 15), columns n .. n+3, n = nbase + 16 j + 4 (lane >> 4)
  const int mbase = m0 + wm * (BM / 2), nbase = n0 + wn * (BN / 2);
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int m = mbase + 16 * i + (lane & 15);
    if (m >= p.M) continue;
    const float bm = (MODE == CONV_FWD && p.bias) ? p.bias[m] : 0.f;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int n = nbase + 16 * j + 4 * (lane >> 4);
      if (n >= p.Ncols) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r];
      if constexpr (MODE == CONV_WGRAD) {
        float* dw = reinterpret_cast<float*>(p.out) + (long)m * p.Ncols + n;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (n + r >= p.Ncols) break;
          if (p.ksplit > 1) atomicAdd(dw + r, v[r]);
          else dw[r] += v[r];
        }
      } else {
        // NCHW destination, row m = channel
        const bool add = MODE == CONV_DGRAD && p.accum;
        if constexpr (MODE == CONV_FWD) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = act_fwd(p.act, v[r] + bm);
        }
        T* out = reinterpret_cast<T*>(p.out);
        const int CH = MODE == CONV_FWD ? p.K : p.C;
        const int Ho = MODE == CONV_FWD ? p.P : p.H, Wo = MODE == CONV_FWD ? p.Q : p.W;
        if constexpr (PV) {
          // padded columns: n .. n+3 lie in one output row (Qp % 8 == 0), valid while q < Wo
          const int per = Ho * p.Qp;
          const int img = n / per, rem = n - img * per, hrow = rem / p.Qp, q = rem - hrow * p.Qp;
          T* d = out + (((long)img * CH + m) * Ho + hrow) * Wo + q;
          const int cnt = min(4, Wo - q);
          if (cnt == 4 && ((((long)img * CH + m) * Ho + hrow) * Wo + q) % 4 == 0) {
            st4<T>(d, v, add);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (r < cnt) st<T>(d + r, v[r] + (add ? ld<T>(d + r) : 0.f));
          }
        } else {
          const int PIX = Ho * Wo;
          const int img = n / PIX, px = n - img * PIX;
          const long o = ((long)img * CH + m) * PIX + px;
          if (n + 3 < p.Ncols && px + 3 < PIX && (o & 3) == 0) {
            st4<T>(out + o, v, add);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int nn = n + r;
              if (nn >= p.Ncols) break;
              const int im = nn / PIX, pr = nn - im * PIX;
              T* d = out + ((long)im * CH + m) * PIX + pr;
              st<T>(d, v[r] + (add ? ld<T>(d) : 0.f));
            }
          }
        }
      }
    }
  }
}

// G = act'(y) * dY (written only when act != none) and db[k] += sum over (n, p, q) of G.  Block
// (k, image range); the block's threads stream the (image, 16-B chunk) pairs of its planes
// (planes start anywhere: unaligned 16-B buffer accesses; scalar tail per plane).
template <typename T>
__global__ void __launch_bounds__(256) fm_conv_act_bwd(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ g,
                                                      float* __restrict__ db, int N, int K, int PQ, int act, int nper,
                                                      FastDiv dch) {
  constexpr int E = 16 / (int)sizeof(T);
  __shared__ float red[4];
  const long bytes = (long)N * K * PQ * (long)sizeof(T);
  const auto rdy = make_rsrc(dy, bytes), ry = make_rsrc(y, bytes), rg = make_rsrc(g, bytes);
  const int k = blockIdx.x;
  const int n0 = blockIdx.y * nper, n1 = min(N, n0 + nper);
  const int chunks = (PQ + E - 1) / E;
  const int work = (n1 - n0) * chunks;
  const bool wr = act != ACT_NONE;
  float s = 0.f;
  for (int w = threadIdx.x; w < work; w += 256) {
    const int nn = fdiv(w, dch), c = w - nn * chunks;
    const int off = ((n0 + nn) * K + k) * PQ + c * E, cnt = min(E, PQ - c * E);
    if (cnt == E) {
      const u32x4_t vd = ldb16(rdy, (unsigned)off * sizeof(T));
      if (!wr) {
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int j = 0; j < 4; ++j) s += bf2f((unsigned short)(vd[j] & 0xFFFF)) + bf2f((unsigned short)(vd[j] >> 16));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) s += __uint_as_float(vd[j]);
        }
        continue;
      }
      const u32x4_t vy = ldb16(ry, (unsigned)off * sizeof(T));
      u32x4_t o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (sizeof(T) == 2) {
          const float d0 = act_bwd(act, bf2f((unsigned short)(vy[j] & 0xFFFF)), bf2f((unsigned short)(vd[j] & 0xFFFF)));
          const float d1 = act_bwd(act, bf2f((unsigned short)(vy[j] >> 16)), bf2f((unsigned short)(vd[j] >> 16)));
          const unsigned short b0 = f2bf(d0), b1 = f2bf(d1);
          s += bf2f(b0) + bf2f(b1);
          o[j] = (unsigned)b0 | ((unsigned)b1 << 16);
        } else {
          const float d = act_bwd(act, __uint_as_float(vy[j]), __uint_as_float(vd[j]));
          s += d;
          o[j] = __float_as_uint(d);
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(o, rg, (unsigned)off * sizeof(T), 0, 0);
    } else {
      for (int t = 0; t < cnt; ++t) {
        float d = ld<T>(dy + off + t);
        if (wr) {
          d = act_bwd(act, ld<T>(y + off + t), d);
          st<T>(g + off + t, d);
          d = ld<T>(g + off + t);
        }
        s += d;
      }
    }
  }
  if (!db) return;
  s = wave_reduce_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(db + k, red[0] + red[1] + red[2] + red[3]);
}

// weight operand prep: mode 0 (fwd) out[k][lda] = W[k][crs] (crs < C*RS, else 0);
// mode 1 (dgrad) out[c][lda] = W[k][c][rs] at column k*RS + rs (else 0)
template <typename T>
__global__ void fm_conv_wprep(const T* __restrict__ w, T* __restrict__ out, int K, int C, int RS, int lda, int mode) {
  const int rows = mode ? C : K;
  const long n = (long)rows * lda;
  const int cols = mode ? K * RS : C * RS;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int row = (int)(i / lda), col = (int)(i - (long)row * lda);
    T v = (T)0;
    if (col < cols) {
      if (mode == 0) {
        v = w[(long)row * cols + col];
      } else {
        const int k = col / RS, rs = col - k * RS;
        v = w[((long)k * C + row) * RS + rs];
      }
    }
    out[i] = v;
  }
}

// Space-to-depth for strided convolutions with few input channels (AlexNet's 11x11/4 stem on 3
// channels): a stride-s conv over X equals a stride-1 conv over X' (C*s*s channels, phase
// (a, b) of the padded input: X'[n, (c*s + a)*s + b, i, j] = Xpad[n, c, i*s + a, j*s + b]) with the
// kernel re-laid the same way (ceil(R/s) x ceil(S/s) taps, zero where r >= R) -- so the stem runs
// on the pixel-vector path.  inv = 1: scatter back (the data gradient; acc adds).
template <typename T>
__global__ void __launch_bounds__(256) fm_conv_s2d(const T* __restrict__ src, T* __restrict__ dst, int total, FastDiv dWs,
                                                   FastDiv dHs, FastDiv dss, FastDiv ds, int C, int H, int W, int s, int pt,
                                                   int pl, int Hs, int Ws, int inv, int acc) {
  const int o = blockIdx.x * 256 + threadIdx.x;     // element of xs [N, C*s*s, Hs, Ws]
  if (o >= total) return;
  int t = fdiv(o, dWs);
  const int j = o - t * Ws;
  int u = fdiv(t, dHs);
  const int i = t - u * Hs;                         // u = n * C*s*s + cp
  const int nc = fdiv(u, dss), ab = u - nc * s * s; // nc = n * C + c
  const int a = fdiv(ab, ds), b = ab - a * s;
  const int h = i * s + a - pt, w = j * s + b - pl;
  const bool in = h >= 0 && h < H && w >= 0 && w < W;
  const long xo = ((long)nc * H + h) * W + w;
  if (!inv) {
    dst[o] = in ? src[xo] : (T)0;
  } else if (in) {
    const float v = ld<T>(src + o) + (acc ? ld<T>(dst + xo) : 0.f);
    st<T>(dst + xo, v);
  }
}

// kernel re-layout for space-to-depth: fwd ws[k][(c*s+a)*s+b][i][j] = w[k][c][i*s+a][j*s+b] (0 past R / S);
// inv: dW[k][c][r][q] += dWs[k][(c*s + r%s)*s + q%s][r/s][q/s] (fp32 gradients)
template <typename T>
__global__ void fm_conv_w_s2d(const T* __restrict__ w, T* __restrict__ ws, const float* __restrict__ dws,
                              float* __restrict__ dw, int K, int C, int R, int S, int s, int Rs, int Ss, int inv) {
  const long total = inv ? (long)K * C * R * S : (long)K * C * s * s * Rs * Ss;
  for (long o = blockIdx.x * 256L + threadIdx.x; o < total; o += (long)gridDim.x * 256) {
    if (!inv) {
      const int j = (int)(o % Ss);
      long t = o / Ss;
      const int i = (int)(t % Rs);
      t /= Rs;
      const int cp = (int)(t % (C * s * s));
      const int k = (int)(t / (C * s * s));
      const int c = cp / (s * s), a = (cp / s) % s, b = cp % s;
      const int r = i * s + a, q = j * s + b;
      ws[o] = (r < R && q < S) ? w[(((long)k * C + c) * R + r) * S + q] : (T)0;
    } else {
      const int q = (int)(o % S);
      long t = o / S;
      const int r = (int)(t % R);
      t /= R;
      const int c = (int)(t % C);
      const int k = (int)(t / C);
      const int cp = (c * s + r % s) * s + q % s;
      dw[o] += dws[(((long)k * C * s * s + cp) * Rs + r / s) * Ss + q / s];
    }
  }
}

template <typename T, int MODE>
int launch(ConvP& p, hipStream_t s) {
  const int BKE = 128 / (int)sizeof(T);
  p.a_nel = (int)(p.a_bytes / (long)sizeof(T));
  p.b_nel = (int)(p.b_bytes / (long)sizeof(T));
  const bool pv = sizeof(T) == 2 && p.sh == 1 && p.sw == 1 && p.a_nel >= 8 && p.b_nel >= 8;
  const int Ho = MODE == CONV_DGRAD ? p.H : p.P, Wo = MODE == CONV_DGRAD ? p.W : p.Q;
  p.Qp = (Wo + 7) / 8 * 8;
  if (pv && MODE != CONV_WGRAD) p.Ncols = p.N * Ho * p.Qp;
  if (pv && MODE == CONV_WGRAD) p.Kred = p.N * p.P * p.Qp;
  p.dRS = make_fastdiv(p.R * p.S);
  p.dS = make_fastdiv(p.S);
  p.dPer = make_fastdiv(p.P * p.Qp);
  p.dQp = make_fastdiv(p.Qp);
  p.dSh = make_fastdiv(p.sh);
  p.adv_c = 64 / (p.R * p.S);
  p.adv_r = (64 / p.S) % p.R;
  p.adv_s = 64 % p.S;
  p.dSw = make_fastdiv(p.sw);
  const bool small_m = p.M <= 64;
  const int BM = small_m ? 64 : 128;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.Ncols + 127) / 128;
  const int ktiles = (p.Kred + BKE - 1) / BKE;
  p.ksplit = 1;
  if (MODE == CONV_WGRAD) {   // long (n,p,q) reduction: split it until ~2 blocks per CU
    const int tiles = p.tiles_m * p.tiles_n;
    p.ksplit = std::max(1, std::min(512 / std::max(tiles, 1), ktiles / 4));
  }
  p.kt_per = (ktiles + p.ksplit - 1) / p.ksplit;
  p.ksplit = (ktiles + p.kt_per - 1) / p.kt_per;
  dim3 grid(p.tiles_m * p.tiles_n, 1, p.ksplit);
#define FM_CONV_GO(BMv, PVv)                                                                         \
  do {                                                                                               \
    const int lds = 2 * (BMv * 128 + 128 * 128) + MASK_BYTES;                                        \
    static bool attr = false;                                                                        \
    if (!attr) {                                                                                     \
      (void)hipFuncSetAttribute((const void*)fm_conv_igemm<T, BMv, MODE, PVv>,                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds);                    \
      attr = true;                                                                                   \
    }                                                                                                \
    hipLaunchKernelGGL((fm_conv_igemm<T, BMv, MODE, PVv>), grid, dim3(CT), lds, s, p);               \
  } while (0)
  if constexpr (sizeof(T) == 2) {   // the pixel-vector gathers are bf16 only
    if (pv) {
      if (small_m) FM_CONV_GO(64, true);
      else FM_CONV_GO(128, true);
      return 0;
    }
  }
  if (small_m) FM_CONV_GO(64, false);
  else FM_CONV_GO(128, false);
#undef FM_CONV_GO
  return 0;
}

ConvP geom(int N, int C, int H, int W, int K, int R, int S, int P, int Q, int sh, int sw, int pt, int pl) {
  ConvP p{};
  p.N = N; p.C = C; p.H = H; p.W = W; p.K = K; p.R = R; p.S = S; p.P = P; p.Q = Q;
  p.sh = sh; p.sw = sw; p.pt = pt; p.pl = pl;
  return p;
}

template <typename T>
void wprep(const void* w, void* out, int K, int C, int RS, int lda, int mode, hipStream_t s) {
  const long n = (long)(mode ? C : K) * lda;
  hipLaunchKernelGGL(fm_conv_wprep<T>, dim3((unsigned)std::min<long>((n + 255) / 256, 1024)), dim3(256), 0, s,
                     (const T*)w, (T*)out, K, C, RS, lda, mode);
}

}  // namespace

// Row stride of the padded weight scratch: fwd [K][conv_lda(C*R*S)], dgrad [C][conv_lda(K*R*S)].
extern "C" int fm_conv_lda(int cols) { return (cols + 7) / 8 * 8; }

// shapes: x [N,C,H,W], w [K,C,R,S], y [N,K,P,Q]; pads (pt, pl) = top / left of this shard, the
// bottom / right halo is implied by P, Q.  Every tensor must stay under 2 GiB (32-bit buffer
// offsets; the host binding checks).  wpad: scratch of K * fm_conv_lda(C*R*S) elements.
extern "C" int fm_conv_fwd(const void* x, const void* w, void* wpad, const float* bias, void* y, int bf16, int N, int C,
                           int H, int W, int K, int R, int S, int P, int Q, int sh, int sw, int pt, int pl, int act,
                           hipStream_t s) {
  ConvP p = geom(N, C, H, W, K, R, S, P, Q, sh, sw, pt, pl);
  const long es = bf16 ? 2 : 4;
  p.Kred = C * R * S;
  p.lda = fm_conv_lda(p.Kred);
  if (bf16) wprep<unsigned short>(w, wpad, K, C, R * S, p.lda, 0, s);
  else wprep<float>(w, wpad, K, C, R * S, p.lda, 0, s);
  p.a = wpad; p.a_bytes = (long)K * p.lda * es;
  p.b = x; p.b_bytes = (long)N * C * H * W * es;
  p.out = y; p.bias = bias; p.act = act;
  p.M = K; p.Ncols = N * P * Q;
  return bf16 ? launch<unsigned short, CONV_FWD>(p, s) : launch<float, CONV_FWD>(p, s);
}

// wt: scratch of C * fm_conv_lda(K*R*S) elements; g: act'(y)*dY or dY itself [N,K,P,Q]
extern "C" int fm_conv_dgrad(const void* g, const void* w, void* wt, void* dx, int accum, int bf16, int N, int C, int H,
                             int W, int K, int R, int S, int P, int Q, int sh, int sw, int pt, int pl, hipStream_t s) {
  ConvP p = geom(N, C, H, W, K, R, S, P, Q, sh, sw, pt, pl);
  const long es = bf16 ? 2 : 4;
  p.Kred = K * R * S;
  p.lda = fm_conv_lda(p.Kred);
  if (bf16) wprep<unsigned short>(w, wt, K, C, R * S, p.lda, 1, s);
  else wprep<float>(w, wt, K, C, R * S, p.lda, 1, s);
  p.a = wt; p.a_bytes = (long)C * p.lda * es;
  p.b = g; p.b_bytes = (long)N * K * P * Q * es;
  p.out = dx; p.accum = accum;
  p.M = C; p.Ncols = N * H * W;
  return bf16 ? launch<unsigned short, CONV_DGRAD>(p, s) : launch<float, CONV_DGRAD>(p, s);
}

// dw fp32 [K][C*R*S] ACCUMULATES
extern "C" int fm_conv_wgrad(const void* g, const void* x, float* dw, int bf16, int N, int C, int H, int W, int K, int R,
                             int S, int P, int Q, int sh, int sw, int pt, int pl, hipStream_t s) {
  ConvP p = geom(N, C, H, W, K, R, S, P, Q, sh, sw, pt, pl);
  const long es = bf16 ? 2 : 4;
  p.a = g; p.a_bytes = (long)N * K * P * Q * es;
  p.b = x; p.b_bytes = (long)N * C * H * W * es;
  p.out = dw;
  p.M = K; p.Ncols = C * R * S; p.Kred = N * P * Q;
  return bf16 ? launch<unsigned short, CONV_WGRAD>(p, s) : launch<float, CONV_WGRAD>(p, s);
}

// g = act'(y) * dy (skipped when act == none), db (fp32 [K], may be null) ACCUMULATES sum of g
extern "C" void fm_conv_act_bwd(const void* dy, const void* y, void* g, float* db, int bf16, int N, int K, int PQ, int act,
                                hipStream_t s) {
  if (act == ACT_NONE && db == nullptr) return;
  if (act == ACT_NONE) g = const_cast<void*>(dy);   // nothing written
  const int want = std::max(1, std::min(N, 2048 / std::max(K, 1)));   // ~2048 blocks over (k, image range)
  const int nper = (N + want - 1) / want;
  const int ny = (N + nper - 1) / nper;
  const FastDiv dch = make_fastdiv((PQ + (bf16 ? 8 : 4) - 1) / (bf16 ? 8 : 4));
  if (bf16)
    hipLaunchKernelGGL(fm_conv_act_bwd<unsigned short>, dim3(K, ny), dim3(256), 0, s, (const unsigned short*)dy,
                       (const unsigned short*)y, (unsigned short*)g, db, N, K, PQ, act, nper, dch);
  else
    hipLaunchKernelGGL(fm_conv_act_bwd<float>, dim3(K, ny), dim3(256), 0, s, (const float*)dy, (const float*)y, (float*)g,
                       db, N, K, PQ, act, nper, dch);
}

// space-to-depth helpers (see fm_conv_s2d): inv = 0: xs = S2D(x); inv = 1: x (+)= S2D^-1(xs)
extern "C" void fm_conv_s2d_run(const void* x, void* xs, int bf16, int N, int C, int H, int W, int s, int pt, int pl, int Hs,
                                int Ws, int inv, int acc, hipStream_t st) {
  const int total = N * C * s * s * Hs * Ws;        // host binding: < 2^31 elements
  const dim3 grid((total + 255) / 256);
  const FastDiv dWs = make_fastdiv(Ws), dHs = make_fastdiv(Hs), dss = make_fastdiv(s * s), ds = make_fastdiv(s);
  if (bf16)
    hipLaunchKernelGGL(fm_conv_s2d<unsigned short>, grid, dim3(256), 0, st, (const unsigned short*)(inv ? xs : x),
                       (unsigned short*)(inv ? const_cast<void*>(x) : xs), total, dWs, dHs, dss, ds, C, H, W, s, pt, pl, Hs,
                       Ws, inv, acc);
  else
    hipLaunchKernelGGL(fm_conv_s2d<float>, grid, dim3(256), 0, st, (const float*)(inv ? xs : x),
                       (float*)(inv ? const_cast<void*>(x) : xs), total, dWs, dHs, dss, ds, C, H, W, s, pt, pl, Hs, Ws, inv,
                       acc);
}

// inv = 0: ws = S2D(w); inv = 1: dw += S2D^-1(dws)
extern "C" void fm_conv_w_s2d_run(const void* w, void* ws, const float* dws, float* dw, int bf16, int K, int C, int R, int S,
                                  int s, int Rs, int Ss, int inv, hipStream_t st) {
  const long total = inv ? (long)K * C * R * S : (long)K * C * s * s * Rs * Ss;
  const int grid = (int)std::min<long>((total + 255) / 256, 1024);
  if (bf16)
    hipLaunchKernelGGL(fm_conv_w_s2d<unsigned short>, dim3(grid), dim3(256), 0, st, (const unsigned short*)w,
                       (unsigned short*)ws, dws, dw, K, C, R, S, s, Rs, Ss, inv);
  else
    hipLaunchKernelGGL(fm_conv_w_s2d<float>, dim3(grid), dim3(256), 0, st, (const float*)w, (float*)ws, dws, dw, K, C, R, S,
                       s, Rs, Ss, inv);
}
