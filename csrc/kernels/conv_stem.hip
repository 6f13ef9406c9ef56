// Stem convolutions on MFMA: the strided few-channel first layer of AlexNet (11x11 / 4 on 3
// channels) and ResNet (7x7 / 2), 64 filters, bf16.  The reference runs these through cuDNN like
// every other convolution (src/ops/conv_2d.cu:405-565 forward, :566-640 filter gradient); on the
// generic implicit-GEMM paths they cost 20 % of an AlexNet step (a space-to-depth pass over the
// whole image, then a stride-1 kernel whose K = 48 x 9 tiles badly, profiles/prof_r8_alexnet_*).
//
// Both kernels stage a tile of the input straight from NCHW global memory into an LDS image in
// SPACE-TO-DEPTH NHWC order: s2d pixel (y', x') holds the s*s phases of every input channel,
// channel c' = (c*s + a)*s + b = x[c][y'*s + a - pt][x'*s + b - pl] (zero outside the image), so the
// stride-s R x S convolution is a stride-1 ceil(R/s) x ceil(S/s) convolution over CP = C*s*s
// channels and every 8 consecutive GEMM k (one tap, 8 channels) are 16 contiguous bytes of one
// pixel.  GEMM k = tap * CP + c'.
//   forward  D[pixel][filter]: A = the pixel's 16-B channel run (ds_read_b128), B = the filter
//            fragments, held in registers for the block's lifetime (built once from the weights);
//            bias + activation in the epilogue, 4 consecutive output columns per 8-B store.
//   wgrad    D[filter][k] summed over pixels: A = g = act'(y) * dy, 8 consecutive output columns
//            per 16-B global load; B = the im2col columns, 8 consecutive pixels of one channel --
//            stride CP in the NHWC image, so read with ds_read_b64_tr_b16 (4 pixel rows x 16
//            channels per 16-lane group, delivered channel-major).  Every block keeps a [64][K]
//            fp32 partial over its tiles; fm_stem_wgrad_reduce sums the partials and scatters the
//            valid (tap, channel) entries into dW[64][C][R][S] (and db).
// Tiles: 2 output rows x 64 output columns per block iteration, 4 waves, persistent blocks (two per
// CU, register-bound; the LDS image is 30 KiB), so one block's global staging overlaps the other's
// MFMAs.
#include "common.h"

#include <algorithm>

namespace {

typedef __attribute__((address_space(3))) bf16x4_t st_lds_v4_t;

constexpr int STK = 64;    // filters
constexpr int STQ = 60;    // output columns per tile (the MFMA groups cover 64; see StemLoader)
constexpr int STP = 2;     // output rows per tile (one per wave pair)
constexpr int STT = 256;   // threads per block

struct StemP {
  const unsigned short* x;    // [N, C, H, W]
  const unsigned short* w;    // forward: weight fragments [KS][4][64 lanes][8] (fm_stem_wprep)
  const float* bias;          // [64] fp32 or null
  unsigned short* y;          // forward output / wgrad: the forward output (activation derivative)
  const unsigned short* dy;   // wgrad: [N, 64, P, Q]
  float* part;                // wgrad: [gridDim.x][64][KP + 4] fp32 partials (column KP: db)
  int N, C, H, W, R, S, P, Q, pt, pl, act;
  int tiles_q, tiles_p, ntiles;
};

template <int CP, int RS, int SS>
struct StemGeo {
  static constexpr int CPS = CP + 8;                   // pixel stride in the LDS image (conflict padding)
  static constexpr int NTAP = RS * SS;
  static constexpr int KS = (NTAP * CP + 31) / 32;     // k steps of 32
  static constexpr int KP = KS * 32;
  static constexpr int XH = STP + RS - 1;
  static constexpr int XW = STQ + SS - 1;              // staged s2d columns
  static constexpr int XWA = 64 + SS - 1;              // allocated (and read: 4 groups of 16) columns
  static constexpr int LDS_ELEMS = XH * XWA * CPS;
};

FM_DEVICE void tile_of(const StemP& p, int tile, int& n, int& p0, int& q0) {
  const int tq = tile % p.tiles_q;
  const int t = tile / p.tiles_q;
  const int tp = t % p.tiles_p;
  n = t / p.tiles_p;
  p0 = tp * STP;
  q0 = tq * STQ;
}

// Global NCHW -> LDS space-to-depth NHWC image of one tile.  A row task (c, a, y') is the source row
// segment of XW*S_ <= 249 elements at s2d row y', phase a; a half-wave (32 lanes) loads it with 16-B
// loads aligned down from its first element (so two row tasks per wave instruction), and each lane
// scatters its 8 elements to (pixel col/S_, channel (c*S_ + a)*S_ + col%S_) with 2-B LDS stores.  (The
// first version loaded 2 B per lane at an 8-B lane stride: ~33 texture-addresser cycles per load
// instruction, 60 % TA-busy -- the kernel's bound.)  Positions outside the image are written as zeros
// every tile.  Split into a register prefetch (load) and the LDS write (store), so the forward can
// keep the next tile's loads in flight under this tile's MFMAs; row tasks bounded for C <= 3.
constexpr int ST_RAWN = 256;                            // elements of one raw row buffer (32 lanes x 8)
constexpr int ST_RAW_BYTES = 4 * 2 * ST_RAWN * 2;       // per block: 4 waves x 2 row tasks

template <int CP, int RS, int SS, int S_, int NR = (3 * S_ * (STP + RS - 1) + 7) / 8, int NTH = STT>
struct StemLoader {
  using G = StemGeo<CP, RS, SS>;
  static constexpr int XWS = G::XW * S_;
  static_assert(XWS + 7 <= 256, "a row task spans at most 32 lanes x 8 elements");
  static constexpr int RPR = NTH / 32;                   // row tasks per round (one per half-wave)
  static constexpr int NRT = (3 * S_ * G::XH + RPR - 1) / RPR;   // rounds per tile
  u32x4_t v[NR];                                        // rounds ub .. ub + NR - 1

  FM_DEVICE static void row_of(const StemP& p, int r, int n, int p0, int q0, int& yr, int& ch, bool& rok, int& g0) {
    yr = r % G::XH;
    const int t = r / G::XH;
    const int a = t % S_, c = t / S_;
    ch = (c * S_ + a) * S_;
    const int yy = (p0 + yr) * S_ + a - p.pt;
    rok = yy >= 0 && yy < p.H;
    g0 = ((n * p.C + c) * p.H + yy) * p.W + q0 * S_ - p.pl;   // global index of the task's first element
  }

  FM_DEVICE void load(const StemP& p, int n, int p0, int q0, int ub = 0) {
    const int nrow = p.C * S_ * G::XH;
    const int lane = threadIdx.x & 63, j = lane & 31;
    const int total = p.N * p.C * p.H * p.W;
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int r = ((int)threadIdx.x >> 5) + RPR * (ub + u);
      int yr, ch, g0;
      bool rok;
      row_of(p, min(r, nrow - 1), n, p0, q0, yr, ch, rok, g0);
      const int base = g0 - (g0 & 7) + 8 * j;
      if (r >= nrow || !rok) {
        v[u] = u32x4_t{0u, 0u, 0u, 0u};                  // a row outside the image: no loads
      } else if (base >= 0 && base + 8 <= total) {
        v[u] = *reinterpret_cast<const u32x4_t*>(p.x + base);
      } else {
        // a chunk overhanging the tensor (its first / last row): element loads
        unsigned e16[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int gi = base + e;
          const bool ok = r < nrow && rok && gi >= 0 && gi < total;
          e16[e] = ok ? p.x[ok ? gi : 0] : 0u;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) v[u][i] = e16[2 * i] | (e16[2 * i + 1] << 16);
      }
    }
  }

  // raw: this wave's 2 x ST_RAWN-element row buffers.  The 16-B chunks go to the raw row first
  // (ds_write_b128, lanes contiguous: conflict-free); each lane then gathers whole s2d pixels (S_
  // phases) from it and writes them with one 8- / 4-B store.  (Scattering the 8 elements of a chunk
  // with 2-B stores directly -- lanes 8 elements apart, so two pixels = 56 dwords apart -- conflicted
  // 8-16 ways and was the forward's LDS bound.)
  FM_DEVICE void store(const StemP& p, unsigned short* xs, unsigned short* raw, int n, int p0, int q0, int ub = 0) const {
    const int nrow = p.C * S_ * G::XH;
    const int lane = threadIdx.x & 63, j = lane & 31;
    unsigned short* rw = raw + (lane >> 5) * ST_RAWN;
    const int xx0 = q0 * S_ - p.pl;
    constexpr int KK = (G::XW + 31) / 32;
    // the image columns of this lane's pixels (the same for every row task of the tile): bit e of
    // cm[kk] = source column xx0 + k*S_ + e inside the image
    unsigned cm[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      cm[kk] = 0;
#pragma unroll
      for (int e = 0; e < S_; ++e) {
        const int xx = xx0 + (j + 32 * kk) * S_ + e;
        cm[kk] |= (xx >= 0 && xx < p.W) ? (1u << e) : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int r = ((int)threadIdx.x >> 5) + RPR * (ub + u);
      int yr, ch, g0;
      bool rok;
      row_of(p, min(r, nrow - 1), n, p0, q0, yr, ch, rok, g0);
      *reinterpret_cast<u32x4_t*>(rw + 8 * j) = v[u];
      FM_WAVE_LDS_SYNC();
      const int rot = g0 & 7;                            // raw index of row position 0
      unsigned short* drow = xs + yr * G::XWA * G::CPS + ch;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int k = j + 32 * kk;                       // s2d pixel of this row task
        if (r < nrow && k < G::XW) {
          const unsigned m = rok ? cm[kk] : 0u;
          unsigned e16[S_];
          if ((rot & 1) == 0) {                          // 4-B aligned pairs
#pragma unroll
            for (int e = 0; e < S_; e += 2) {
              const unsigned d = *reinterpret_cast<const unsigned*>(rw + k * S_ + e + rot);
              e16[e] = (m >> e) & 1 ? (d & 0xffffu) : 0u;
              e16[e + 1] = (m >> (e + 1)) & 1 ? (d >> 16) : 0u;
            }
          } else {
#pragma unroll
            for (int e = 0; e < S_; ++e) e16[e] = (m >> e) & 1 ? (unsigned)rw[k * S_ + e + rot] : 0u;
          }
          if constexpr (S_ == 4)
            *reinterpret_cast<uint2*>(drow + k * G::CPS) = uint2{e16[0] | (e16[1] << 16), e16[2] | (e16[3] << 16)};
          else
            *reinterpret_cast<unsigned*>(drow + k * G::CPS) = e16[0] | (e16[1] << 16);
        }
      }
      FM_WAVE_LDS_SYNC();                                // the gathers read the raw row before it is reused
    }
  }
};

// GEMM k -> raw weight element of filter f (or -1 for a padding k)
template <int CP, int RS, int SS, int S_>
FM_DEVICE int stem_widx(int f, int k, int C, int R, int S) {
  constexpr int NTAP = RS * SS;
  const int t = k / CP, cp = k - t * CP;
  if (t >= NTAP) return -1;
  const int ra = t / SS, sa = t - ra * SS;
  const int c = cp / (S_ * S_), a = (cp / S_) % S_, b = cp % S_;
  const int r = ra * S_ + a, sc = sa * S_ + b;
  if (c >= C || r >= R || sc >= S) return -1;
  return ((f * C + c) * R + r) * S + sc;
}

// weights [64][C][R][S] -> forward B fragments: wf[ks][nt][lane][e] = W(filter nt*16 + lane%16,
// k = ks*32 + (lane/16)*8 + e), zero for padding k
template <int CP, int RS, int SS, int S_>
__global__ void __launch_bounds__(256) fm_stem_wprep(const unsigned short* __restrict__ w, unsigned short* __restrict__ wf,
                                                     int C, int R, int S) {
  using G = StemGeo<CP, RS, SS>;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= G::KS * 2048) return;
  const int j8 = e & 7, ln = (e >> 3) & 63, nt = (e >> 9) & 3, ks = e >> 11;
  const int wi = stem_widx<CP, RS, SS, S_>(nt * 16 + (ln & 15), ks * 32 + (ln >> 4) * 8 + j8, C, R, S);
  wf[e] = wi >= 0 ? w[wi] : (unsigned short)0;
}

// ACT: ACT_NONE / ACT_RELU compiled in; any other activation code is evaluated at run time (-1)
template <int ACT>
FM_DEVICE float stem_act(int act, float x) {
  if constexpr (ACT == ACT_NONE) return x;
  else if constexpr (ACT == ACT_RELU) return fmaxf(x, 0.f);
  else return act_fwd(act, x);
}
template <int ACT>
FM_DEVICE float stem_act_bwd(int act, float y, float dy) {
  if constexpr (ACT == ACT_NONE) return dy;
  else if constexpr (ACT == ACT_RELU) return y > 0.f ? dy : 0.f;
  else return act_bwd(act, y, dy);
}

// image offset of GEMM k run k0 (8 channels of one tap; the tap clamped: padding k meet zero weights)
template <int CP, int RS, int SS>
constexpr int stem_koff(int k0) {
  using G = StemGeo<CP, RS, SS>;
  const int t = k0 / CP < G::NTAP - 1 ? k0 / CP : G::NTAP - 1;
  return ((t / SS) * G::XWA + t % SS) * G::CPS + k0 % CP;
}
FM_DEVICE int sel4(int i, int a, int b, int c, int d) { return i < 2 ? (i == 0 ? a : b) : (i == 2 ? c : d); }

template <int CP, int RS, int SS, int S_, int ACT>
__global__ void __launch_bounds__(STT, 2) fm_stem_fwd(StemP p) {
  using G = StemGeo<CP, RS, SS>;
  extern __shared__ __attribute__((aligned(16))) unsigned short xs[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rw = wave >> 1, h = wave & 1;              // output row rw of the tile; filters 32h .. 32h+31
  const int l16 = lane & 15, kg = lane >> 4;
  // B fragments for the block's lifetime (fm_stem_wprep's [ks][nt][lane][8] layout): 16-B loads
  bf16x8_t bw[G::KS][2];
#pragma unroll
  for (int ks = 0; ks < G::KS; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bw[ks][j] = *reinterpret_cast<const bf16x8_t*>(p.w + (((ks * 4 + 2 * h + j) * 64) + lane) * 8);
  // zero both images: the padding channels (c' >= C*s*s) are never staged
  for (int e = tid * 8; e < 2 * G::LDS_ELEMS; e += STT * 8)
    *reinterpret_cast<u32x4_t*>(xs + e) = u32x4_t{0u, 0u, 0u, 0u};
  float bias2[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bias2[j] = p.bias ? p.bias[(2 * h + j) * 16 + l16] : 0.f;
  const int lbase = (rw * G::XWA + l16) * G::CPS;
  unsigned short* raw = xs + 2 * G::LDS_ELEMS + wave * 2 * ST_RAWN;
  StemLoader<CP, RS, SS, S_> ld;
  int buf = 0;
  if ((int)blockIdx.x < p.ntiles) {
    int n, p0, q0;
    tile_of(p, blockIdx.x, n, p0, q0);
    __syncthreads();                                    // the zero fill is done
    ld.load(p, n, p0, q0);
    ld.store(p, xs, raw, n, p0, q0);
  }
  __syncthreads();
  for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    int n, p0, q0;
    tile_of(p, tile, n, p0, q0);
    const int next = tile + gridDim.x;
    if (next < p.ntiles) {                              // the next tile's loads fly under this tile's MFMAs
      int n1, p1, q1;
      tile_of(p, next, n1, p1, q1);
      ld.load(p, n1, p1, q1);
    }
    const unsigned short* xb = xs + buf * G::LDS_ELEMS;
    f32x4_t acc[4][2];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[g][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < G::KS; ++ks) {
      // this lane's k run: tap t (clamped: padding k meet zero weights), channels cp .. cp+7
      // the lane's k run k0 = 32 ks + 8 kg: its image offset is one of four compile-time constants
      // (selected by kg) instead of a run-time division per k step
      const int koff = lbase + sel4(kg, stem_koff<CP, RS, SS>(ks * 32), stem_koff<CP, RS, SS>(ks * 32 + 8),
                                    stem_koff<CP, RS, SS>(ks * 32 + 16), stem_koff<CP, RS, SS>(ks * 32 + 24));
      if ((ks & 1) == 0) __builtin_amdgcn_sched_barrier(0);    // bound the A reads in flight
      u32x4_t af[4];
#pragma unroll
      for (int g = 0; g < 4; ++g)   // group g: columns 16g .. 16g+15 of row rw
        af[g] = *reinterpret_cast<const u32x4_t*>(xb + koff + g * 16 * G::CPS);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v_t, af[g]),
                                                              __builtin_bit_cast(bf16x8v_t, bw[ks][j]), acc[g][j], 0, 0, 0);
    }
    // epilogue: lane holds pixels 4kg .. 4kg+3 of its group's 16 columns, filter (2h + j)*16 + l16
    const bool vec = (p.Q & 3) == 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int pp = p0 + rw;
      const int q = q0 + g * 16 + 4 * kg;
      if (pp >= p.P || q >= p.Q || q - q0 >= STQ) continue;   // STQ % 4 == 0: whole quads
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int f = (2 * h + j) * 16 + l16;
        unsigned short* dst = p.y + (((long)n * STK + f) * p.P + pp) * p.Q + q;
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = stem_act<ACT>(p.act, acc[g][j][i] + bias2[j]);
        if (vec) {
          bf16x4_t pk;
#pragma unroll
          for (int i = 0; i < 4; ++i) pk[i] = (short)f2bf(o[i]);
          *reinterpret_cast<bf16x4_t*>(dst) = pk;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (q + i < p.Q) dst[i] = f2bf(o[i]);
        }
      }
    }
    if (next < p.ntiles) {
      int n1, p1, q1;
      tile_of(p, next, n1, p1, q1);
      ld.store(p, xs + (buf ^ 1) * G::LDS_ELEMS, raw, n1, p1, q1);
    }
    __syncthreads();
    buf ^= 1;
  }
}

// weight gradient: every block sums its tiles into a [64][KP] register partial.  Wave w owns the k
// column blocks 7w .. 7w+6 for all 64 filters, so every im2col fragment is read from the LDS once per
// block; g = act'(y) * dy of the tile is staged in the LDS beside the image ([64][GROW], rows padded
// for conflict-free 16-B fragment reads).
constexpr int ST_GROW = STP * 64 + 8;
static_assert(STP == 2, "the g-tile chunk map assumes two output rows per tile");

template <int CP, int RS, int SS, int S_, int ACT>
__global__ void __launch_bounds__(STT, 2) fm_stem_wgrad(StemP p) {
  using G = StemGeo<CP, RS, SS>;
  constexpr int NT = G::KP / 16;                        // k column blocks of 16
  constexpr int NTW = (NT + 3) / 4;                     // per wave
  extern __shared__ __attribute__((aligned(16))) unsigned short xs[];
  unsigned short* gs = xs + G::LDS_ELEMS;               // [64][ST_GROW]
  unsigned short* raw = gs + STK * ST_GROW + ((int)threadIdx.x >> 6) * 2 * ST_RAWN;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kg = lane >> 4;
  const int tq4 = l16 >> 2, tp4 = l16 & 3;             // transposed read: block row tq4, columns 4tp4 ..
  for (int e = tid * 8; e < G::LDS_ELEMS; e += STT * 8)
    *reinterpret_cast<u32x4_t*>(xs + e) = u32x4_t{0u, 0u, 0u, 0u};
  f32x4_t acc[4][NTW];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[m][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dbs[4] = {0.f, 0.f, 0.f, 0.f};                 // filter tid/16 + 16i (the g chunks of this thread)
  const bool vec = (p.Q & 7) == 0;
  for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    int n, p0, q0;
    tile_of(p, tile, n, p0, q0);
    __syncthreads();                                    // the previous tile's reads are done
    // g tile: chunk c = (filter c/16, row (c/8)&1, 8 columns 8(c&7)); 4 chunks per thread
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + STT * i;
      const int f = c >> 4, r = (c >> 3) & 1, c8 = (c & 7) * 8;
      const int pp = p0 + r, q = q0 + c8;
      const int qend = min(p.Q, q0 + STQ);             // this tile's columns
      const long o = (((long)n * STK + f) * p.P + min(pp, p.P - 1)) * p.Q;
      float gv[8];
      if (pp >= p.P || q >= qend) {                     // outside the tile: zeros, no loads
#pragma unroll
        for (int e = 0; e < 8; ++e) gv[e] = 0.f;
      } else if (vec && q + 8 <= qend) {
        const bf16x8_t d = *reinterpret_cast<const bf16x8_t*>(p.dy + o + q);
        bf16x8_t yv = d;
        if constexpr (ACT != ACT_NONE) yv = *reinterpret_cast<const bf16x8_t*>(p.y + o + q);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dd = bf2f((unsigned short)d[e]);
          gv[e] = stem_act_bwd<ACT>(p.act, bf2f((unsigned short)yv[e]), dd);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool ok = pp < p.P && q + e < qend;
          const long oi = o + (ok ? q + e : 0);
          const float dd = bf2f(p.dy[oi]);
          const float g = ACT == ACT_NONE ? dd : stem_act_bwd<ACT>(p.act, bf2f(p.y[oi]), dd);
          gv[e] = ok ? g : 0.f;
        }
      }
      bf16x8_t gb;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        gb[e] = (short)f2bf(gv[e]);
        dbs[i] += gv[e];
      }
      *reinterpret_cast<bf16x8_t*>(gs + f * ST_GROW + r * 64 + c8) = gb;
    }
    __builtin_amdgcn_sched_barrier(0);                 // the g tile's registers die before the image loads
    {
      using L = StemLoader<CP, RS, SS, S_, 2>;        // two rounds of loads in flight (registers)
      L ld;
#pragma unroll
      for (int ub = 0; ub < L::NRT; ub += 2) {
        ld.load(p, n, p0, q0, ub);
        ld.store(p, xs, raw, n, p0, q0, ub);
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < STP; ++r)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        // pixels of this step: row r, columns hh*32 + kg*8 + 0..7
        u32x4_t ga[4];
#pragma unroll
        for (int m = 0; m < 4; ++m)
          ga[m] = *reinterpret_cast<const u32x4_t*>(gs + (m * 16 + l16) * ST_GROW + r * 64 + hh * 32 + kg * 8);
        // block rows of the transposed reads: pixel kg*8 + tq4 (lo) and kg*8 + 4 + tq4 (hi)
        const int pix = (r * G::XWA + hh * 32 + kg * 8 + tq4) * G::CPS;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          // k columns nt*16 .. +15: 16 consecutive channels of one tap (clamped past the last tap)
          const int nt = min(wave * NTW + j, NT - 1);
          const int t = min(nt * 16 / CP, G::NTAP - 1), cp = nt * 16 - (nt * 16 / CP) * CP;
          const int boff = ((t / SS) * G::XWA + t % SS) * G::CPS + cp + 4 * tp4;
          const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((st_lds_v4_t*)(xs + pix + boff));
          const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((st_lds_v4_t*)(xs + pix + 4 * G::CPS + boff));
          bf16x8_t bx;
          bx.lo = lo;
          bx.hi = hi;
#pragma unroll
          for (int m = 0; m < 4; ++m)
            acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v_t, ga[m]),
                                                                __builtin_bit_cast(bf16x8v_t, bx), acc[m][j], 0, 0, 0);
        }
      }
  }
  // partial out: lane holds D[filter m*16 + 4kg + i][k (wave*NTW + j)*16 + l16]
  float* part = p.part + (long)blockIdx.x * STK * (G::KP + 4);
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wave * NTW + j;
    if (nt >= NT) break;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[(m * 16 + 4 * kg + i) * (G::KP + 4) + nt * 16 + l16] = acc[m][j][i];
  }
  // db: the 16 threads tid/16 == const hold one filter's chunks
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = dbs[i];
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    if ((tid & 15) == 0) part[((tid >> 4) + 16 * i) * (G::KP + 4) + G::KP] = v;
  }
}

// Pipelined weight gradient (the form the launcher uses): 8 waves per block, one block per CU; wave
// w owns filters 32*(w&1) .. +31 and the k column blocks 7*(w>>1) .. +6 (NT/4 of them), so the
// accumulators take 56 registers and the NEXT tile's image and g loads (28 registers) stay in
// flight under this tile's MFMAs; images and g tiles double-buffered in LDS, one barrier per tile.
// (The 4-wave form above staged synchronously: 67 % of its wave cycles waiting on memory.)
constexpr int SW_NTH = 512;

template <int CP, int RS, int SS, int S_>
struct StemGLoader {                                   // the g tile of one block tile: 2 chunks per thread
  u32x4_t d[2], y[2];
  FM_DEVICE void load(const StemP& p, int n, int p0, int q0, bool need_y) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = (int)threadIdx.x + SW_NTH * i;
      const int f = c >> 4, r = (c >> 3) & 1, c8 = (c & 7) * 8;
      const int pp = p0 + r, q = q0 + c8;
      const int qend = min(p.Q, q0 + STQ);
      const long o = (((long)n * STK + f) * p.P + min(pp, p.P - 1)) * p.Q;
      d[i] = u32x4_t{0u, 0u, 0u, 0u};
      y[i] = u32x4_t{0u, 0u, 0u, 0u};
      if (pp >= p.P || q >= qend) continue;            // outside the tile: zeros
      if ((p.Q & 7) == 0 && q + 8 <= qend) {
        d[i] = *reinterpret_cast<const u32x4_t*>(p.dy + o + q);
        if (need_y) y[i] = *reinterpret_cast<const u32x4_t*>(p.y + o + q);
      } else {
        unsigned dv[8], yv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool ok = q + e < qend;
          const long oi = o + (ok ? q + e : 0);
          dv[e] = ok ? (unsigned)p.dy[oi] : 0u;
          yv[e] = ok && need_y ? (unsigned)p.y[oi] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[i][k] = dv[2 * k] | (dv[2 * k + 1] << 16);
          y[i][k] = yv[2 * k] | (yv[2 * k + 1] << 16);
        }
      }
    }
  }
  template <int ACT>
  FM_DEVICE void store(const StemP& p, unsigned short* gs, float (&dbs)[2]) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = (int)threadIdx.x + SW_NTH * i;
      const int f = c >> 4, r = (c >> 3) & 1, c8 = (c & 7) * 8;
      u32x4_t o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float g2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float dd = bf2f((unsigned short)(d[i][k] >> (16 * h)));
          const float yy = bf2f((unsigned short)(y[i][k] >> (16 * h)));
          g2[h] = stem_act_bwd<ACT>(p.act, yy, dd);
          dbs[i] += g2[h];
        }
        o[k] = (unsigned)f2bf(g2[0]) | ((unsigned)f2bf(g2[1]) << 16);
      }
      *reinterpret_cast<u32x4_t*>(gs + f * ST_GROW + r * 64 + c8) = o;
    }
  }
};

template <int CP, int RS, int SS, int S_, int ACT>
__global__ void __launch_bounds__(SW_NTH, 1) fm_stem_wgrad2(StemP p) {
  using G = StemGeo<CP, RS, SS>;
  constexpr int NT = G::KP / 16;                        // k column blocks of 16
  constexpr int NTW = (NT + 3) / 4;                     // per wave (four k quarters)
  constexpr int BUF = G::LDS_ELEMS + STK * ST_GROW;     // one image + one g tile (elements)
  using L = StemLoader<CP, RS, SS, S_, (3 * S_ * (STP + RS - 1) + SW_NTH / 32 - 1) / (SW_NTH / 32), SW_NTH>;
  extern __shared__ __attribute__((aligned(16))) unsigned short xs[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kg = lane >> 4;
  const int tq4 = l16 >> 2, tp4 = l16 & 3;
  const int mh = wave & 1, kq = wave >> 1;
  unsigned short* raw = xs + 2 * BUF + wave * 2 * ST_RAWN;
  for (int e = tid * 8; e < 2 * BUF; e += SW_NTH * 8)
    *reinterpret_cast<u32x4_t*>(xs + e) = u32x4_t{0u, 0u, 0u, 0u};
  f32x4_t acc[2][NTW];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[m][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dbs[2] = {0.f, 0.f};                           // filters tid/16 and tid/16 + 32
  L ld;
  StemGLoader<CP, RS, SS, S_> gl;
  int buf = 0;
  if ((int)blockIdx.x < p.ntiles) {
    int n, p0, q0;
    tile_of(p, blockIdx.x, n, p0, q0);
    __syncthreads();                                    // the zero fill is done
    ld.load(p, n, p0, q0);
    gl.load(p, n, p0, q0, ACT != ACT_NONE);
    ld.store(p, xs, raw, n, p0, q0);
    gl.template store<ACT>(p, xs + G::LDS_ELEMS, dbs);
  }
  __syncthreads();
  for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    const int next = tile + gridDim.x;
    int n1 = 0, p1 = 0, q1 = 0;
    if (next < p.ntiles) {                              // the next tile's loads fly under this tile's MFMAs
      tile_of(p, next, n1, p1, q1);
      ld.load(p, n1, p1, q1);
      gl.load(p, n1, p1, q1, ACT != ACT_NONE);
    }
    const unsigned short* xb = xs + buf * BUF;
    const unsigned short* gsb = xb + G::LDS_ELEMS;
#pragma unroll
    for (int r = 0; r < STP; ++r)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        u32x4_t ga[2];
#pragma unroll
        for (int m = 0; m < 2; ++m)
          ga[m] = *reinterpret_cast<const u32x4_t*>(gsb + ((2 * mh + m) * 16 + l16) * ST_GROW + r * 64 + hh * 32 + kg * 8);
        const int pix = (r * G::XWA + hh * 32 + kg * 8 + tq4) * G::CPS;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int nt = min(kq * NTW + j, NT - 1);
          const int t = min(nt * 16 / CP, G::NTAP - 1), cp = nt * 16 - (nt * 16 / CP) * CP;
          const int boff = ((t / SS) * G::XWA + t % SS) * G::CPS + cp + 4 * tp4;
          const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((st_lds_v4_t*)(xb + pix + boff));
          const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((st_lds_v4_t*)(xb + pix + 4 * G::CPS + boff));
          bf16x8_t bx;
          bx.lo = lo;
          bx.hi = hi;
#pragma unroll
          for (int m = 0; m < 2; ++m)
            acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v_t, ga[m]),
                                                                __builtin_bit_cast(bf16x8v_t, bx), acc[m][j], 0, 0, 0);
        }
      }
    if (next < p.ntiles) {
      unsigned short* nb = xs + (buf ^ 1) * BUF;
      ld.store(p, nb, raw, n1, p1, q1);
      gl.template store<ACT>(p, nb + G::LDS_ELEMS, dbs);
    }
    __syncthreads();
    buf ^= 1;
  }
  float* part = p.part + (long)blockIdx.x * STK * (G::KP + 4);
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = kq * NTW + j;
    if (nt >= NT) break;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[((2 * mh + m) * 16 + 4 * kg + i) * (G::KP + 4) + nt * 16 + l16] = acc[m][j][i];
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float v = dbs[i];
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    if ((tid & 15) == 0) part[((tid >> 4) + 32 * i) * (G::KP + 4) + G::KP] = v;
  }
}

// dW[f][c][r][s] += sum over blocks of part[.][f][k(c, r, s)]; db[f] += sum of part[.][f][KP].  A block
// takes 32 consecutive partial columns x 8 block slices (8 loads in flight per thread), then folds the
// 8 slice sums in a fixed order (deterministic).
template <int CP, int RS, int SS, int S_>
__global__ void __launch_bounds__(256) fm_stem_wgrad_reduce(const float* __restrict__ part, int nblk, float* __restrict__ dw,
                                                            float* __restrict__ db, int C, int R, int S) {
  using G = StemGeo<CP, RS, SS>;
  constexpr int LD = G::KP + 4;
  __shared__ float red[8][33];
  const int col = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int i = blockIdx.x * 32 + col;                 // flat [64][LD] index
  const bool live = i < STK * LD;
  const int per = (nblk + 7) / 8;
  const int b0 = sl * per, b1 = min(nblk, b0 + per);
  float s = 0.f;
  if (live) {
    int b = b0;
    for (; b + 8 <= b1; b += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(b + u) * STK * LD + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < b1; ++b) s += part[(long)b * STK * LD + i];
  }
  red[sl][col] = s;
  __syncthreads();
  if (sl != 0 || !live) return;
#pragma unroll
  for (int u = 1; u < 8; ++u) s += red[u][col];
  const int f = i / LD, k = i - f * LD;
  if (k < G::KP) {
    const int dst = stem_widx<CP, RS, SS, S_>(f, k, C, R, S);
    if (dst >= 0) dw[dst] += s;
  } else if (k == G::KP && db != nullptr) {
    db[f] += s;
  }
}

// wgrad form: the pipelined 8-wave kernel for the 48-channel (stride-4) stems -- AlexNet 245 -> 135
// us; the 4-wave kernel for the 16-channel (stride-2) ones, where the pipelined form measured
// slower (ResNet-50 b64 142 vs 208 us, profiles/stem_forms_r7.txt)
template <int CP, int RS, int SS, int S_, int ACT>
void stem_launch(StemP& p, int mode, float* dw, float* db, int grid, bool pipelined, hipStream_t st) {
  using G = StemGeo<CP, RS, SS>;
  const int lds = G::LDS_ELEMS * 2;
  if (mode == 0) {
    const int lds2 = 2 * lds + ST_RAW_BYTES;            // double-buffered image + raw rows
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)fm_stem_fwd<CP, RS, SS, S_, ACT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                lds2);
      attr = true;
    }
    hipLaunchKernelGGL((fm_stem_fwd<CP, RS, SS, S_, ACT>), dim3(grid), dim3(STT), lds2, st, p);
    return;
  }
  if (pipelined) {
    // two (image + g tile) buffers + 8 waves' raw rows
    const int lds_w = 2 * (lds + STK * ST_GROW * 2) + 8 * 2 * ST_RAWN * 2;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)fm_stem_wgrad2<CP, RS, SS, S_, ACT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                lds_w);
      attr = true;
    }
    hipLaunchKernelGGL((fm_stem_wgrad2<CP, RS, SS, S_, ACT>), dim3(grid), dim3(SW_NTH), lds_w, st, p);
  } else {
    const int lds_w = lds + STK * ST_GROW * 2 + ST_RAW_BYTES;   // the image + the g tile + raw rows
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)fm_stem_wgrad<CP, RS, SS, S_, ACT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                lds_w);
      attr = true;
    }
    hipLaunchKernelGGL((fm_stem_wgrad<CP, RS, SS, S_, ACT>), dim3(grid), dim3(STT), lds_w, st, p);
  }
  const int tot = STK * (G::KP + 4);
  hipLaunchKernelGGL((fm_stem_wgrad_reduce<CP, RS, SS, S_>), dim3((tot + 31) / 32), dim3(256), 0, st, p.part, grid, dw, db,
                     p.C, p.R, p.S);
}

template <int CP, int RS, int SS, int S_>
int stem_run(StemP& p, int mode, float* dw, float* db, int nsm, hipStream_t st) {
  using G = StemGeo<CP, RS, SS>;
  p.tiles_q = (p.Q + STQ - 1) / STQ;
  p.tiles_p = (p.P + STP - 1) / STP;
  p.ntiles = p.N * p.tiles_p * p.tiles_q;
  const bool pipelined = CP == 48;                      // see stem_launch
  // 4-wave kernels: two blocks per CU; the pipelined wgrad: one 8-wave block per CU
  const int grid = std::max(1, std::min(p.ntiles, (mode == 1 && pipelined ? 1 : 2) * nsm));
  if (mode == 0) {
    // the caller's raw weights -> fragments in the scratch (p.part as 16-bit storage)
    unsigned short* wf = reinterpret_cast<unsigned short*>(p.part);
    hipLaunchKernelGGL((fm_stem_wprep<CP, RS, SS, S_>), dim3((G::KS * 2048 + 255) / 256), dim3(256), 0, st, p.w, wf, p.C,
                       p.R, p.S);
    p.w = wf;
  }
  if (p.act == ACT_RELU) stem_launch<CP, RS, SS, S_, ACT_RELU>(p, mode, dw, db, grid, pipelined, st);
  else if (p.act == ACT_NONE) stem_launch<CP, RS, SS, S_, ACT_NONE>(p, mode, dw, db, grid, pipelined, st);
  else stem_launch<CP, RS, SS, S_, -1>(p, mode, dw, db, grid, pipelined, st);
  return 0;
}

// supported geometries: 1-3 channels (StemLoader's row-task bound), 64 filters, (11x11 / 4) or (7x7 / 2) class stems
int stem_kind(int C, int K, int R, int S, int s) {
  if (K != STK || C < 1) return 0;
  if (s == 4 && C * 16 <= 48 && R <= 12 && S <= 12) return 1;   // CP 48, 3 x 3 taps
  if (s == 2 && C <= 3 && R <= 8 && S <= 8) return 2;           // CP 16, 4 x 4 taps
  return 0;
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (n <= 0) n = 256;
  }
  return n;
}

}  // namespace

// 1 when the stem kernels take this convolution (bf16, 64 filters, the stride / kernel classes above)
extern "C" int fm_stem_supported(int C, int K, int R, int S, int sh, int sw) {
  return sh == sw && stem_kind(C, K, R, S, sh) != 0;
}

// 16-bit elements of the forward's weight-fragment scratch
extern "C" long fm_stem_wf_elems(int C, int K, int R, int S, int s) {
  const int kind = stem_kind(C, K, R, S, s);
  return kind == 1 ? StemGeo<48, 3, 3>::KS * 2048L : kind == 2 ? StemGeo<16, 4, 4>::KS * 2048L : 0;
}

// fp32 partial-buffer elements the weight gradient needs (one [64][KP + 4] slab per block)
extern "C" long fm_stem_wgrad_ws(int C, int K, int R, int S, int s) {
  const int kind = stem_kind(C, K, R, S, s);
  const int kp = kind == 1 ? StemGeo<48, 3, 3>::KP : StemGeo<16, 4, 4>::KP;
  return kind ? (long)2 * num_cus() * STK * (kp + 4) : 0;
}

// wf: scratch of fm_stem_wf_elems 16-bit elements (the weight fragments)
extern "C" int fm_stem_fwd_run(const void* x, const void* w, void* wf, const float* bias, void* y, int N, int C, int H, int W,
                               int R, int S, int P, int Q, int s, int pt, int pl, int act, hipStream_t st) {
  StemP p{};
  p.x = (const unsigned short*)x; p.w = (const unsigned short*)w; p.bias = bias; p.y = (unsigned short*)y;
  p.part = reinterpret_cast<float*>(wf);
  p.N = N; p.C = C; p.H = H; p.W = W; p.R = R; p.S = S; p.P = P; p.Q = Q; p.pt = pt; p.pl = pl; p.act = act;
  const int kind = stem_kind(C, STK, R, S, s);
  if (kind == 1) return stem_run<48, 3, 3, 4>(p, 0, nullptr, nullptr, num_cus(), st);
  if (kind == 2) return stem_run<16, 4, 4, 2>(p, 0, nullptr, nullptr, num_cus(), st);
  return -1;
}

// dw (fp32 [64*C*R*S]) and db (fp32 [64] or null) ACCUMULATE; y = the forward output (ReLU mask)
extern "C" int fm_stem_wgrad_run(const void* x, const void* y, const void* dy, float* dw, float* db, float* ws, int N, int C,
                                 int H, int W, int R, int S, int P, int Q, int s, int pt, int pl, int act, hipStream_t st) {
  StemP p{};
  p.x = (const unsigned short*)x; p.y = (unsigned short*)const_cast<void*>(y); p.dy = (const unsigned short*)dy;
  p.part = ws;
  p.N = N; p.C = C; p.H = H; p.W = W; p.R = R; p.S = S; p.P = P; p.Q = Q; p.pt = pt; p.pl = pl; p.act = act;
  const int kind = stem_kind(C, STK, R, S, s);
  if (kind == 1) return stem_run<48, 3, 3, 4>(p, 1, dw, db, num_cus(), st);
  if (kind == 2) return stem_run<16, 4, 4, 2>(p, 1, dw, db, num_cus(), st);
  return -1;
}
