// 3x3, stride 1, zero-padding 1, bias-free convolution, NCHW fp32, on
// v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation).
//
// Replaces the first (kxk) Conv2d of the guided-upsampling blocks' three
// branches — feature_conv, guide_conv and comb_conv
// (src/GuideDepth/model/modules.py:43-74, built with kernel_size=3 at
// GuideDepth.py:21-33) — at the full-resolution, small-channel shapes where
// MIOpen's Winograd / implicit-GEMM kernels run at 10-45 TFLOP/s:
// 16->16 @ 480x640, 32->32 @ 240x320 (weight gradient) and the 3-channel
// guide convolutions 3->{16,32,64}.  The conv bias is folded into the
// following BatchNorm (nn.py conv_bn), so the kernels are bias-free.
//
// Forward (and data gradient = the same kernel on the flipped, transposed
// weights): implicit GEMM with M = output pixels, N = output channels,
// K = (tap, input channel).  A block stages an input tile of
// C_in x (TH+2) x 66 (zero halo) and the weights in LDS; each wave owns
// RPW output rows x 64 columns x all output channels.  K is ordered tap-major
// so the 4 k-lanes of one MFMA step read 4 channels at the same tap: every
// operand read is one ds_read_b32 at a compile-time offset from a per-lane
// base, conflict-free (plane stride = 16 mod 64 words).
//
// Weight gradient: M = output channels, N = (tap, input channel), K =
// pixels.  Each block walks a strided list of 8x64 pixel tiles (x with halo
// and gy staged in LDS), accumulating its gW partial in registers; waves
// split the tile's rows (and, for wide problems, the N blocks).  Block
// partials land in a slab that a two-stage, fixed-order reduction sums, so
// the result is bitwise reproducible (no atomics).
#include <cstdlib>

#include "common.h"

namespace {

using f4 = __attribute__((__vector_size__(4 * sizeof(float)))) float;

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int kTW = 64;       // output columns per tile (4 MFMA row tiles)
constexpr int kXW = kTW + 2;  // staged input columns (one-pixel halo each side)

constexpr int cpad4(int c) { return (c + 3) / 4 * 4; }
// LDS plane stride (words) for `rows` staged rows of kXW, = `mod` (mod 64).
constexpr int plane_words(int rows, int mod) { return (rows * kXW + 63) / 64 * 64 + mod; }
// Weight-row stride (words): the four k-lane groups of a B read land on
// disjoint 16-bank quarters (16 -> 16, 32 -> 48, 64 -> 80, all = 16k mod 64
// with k odd or the groups spread 0/16/32/48).
constexpr int wrow_words(int co) { return co == 16 ? 16 : (co == 32 ? 48 : 80); }

// --------------------------------------------------------------- staging
// A CIP x XR x kXW input tile (rows r0-1.., cols c0-1..), zero outside the
// image and for channels >= CI, held in registers between its global loads
// and its LDS writes so that the loads of tile i+1 are in flight while tile i
// is multiplied.  Each wave copies whole tile rows (wave-uniform channel /
// row, lane = column 0..63); the two right-halo columns of all of the wave's
// rows go one element per lane in NH extra loads.  Out-of-range elements load
// element 0 and are zeroed by a select (no divergent branches around loads).
template <int CI, int CIP, int XR>
struct HaloTile {
  static constexpr int ROWS = CIP * XR;
  static constexpr int RPWV = (ROWS + 3) / 4;      // tile rows per wave
  static constexpr int NH = (2 * RPWV + 63) / 64;  // right-halo loads per lane
  static_assert(RPWV <= 64 && NH <= 32, "mask widths");
  float a[RPWV];
  float b[NH];
  // In-range flags, applied at store time: loads are unconditional (clamped
  // addresses) and nothing reads their values until the next tile's store,
  // so no select or divergent branch makes the wave wait for them early.
  uint64_t am;
  unsigned bm;

  __device__ __forceinline__ void load(const float* __restrict__ xi, int h, int w, int r0,
                                       int c0, int lane, int wvu) {
    const int gc = c0 - 1 + lane;
    const bool cok = gc >= 0 && gc < w;
    am = 0;
#pragma unroll
    for (int k = 0; k < RPWV; ++k) {
      const int ri = wvu + 4 * k;
      const int c = ri / XR, r = ri % XR, gr = r0 - 1 + r;
      const bool ok = (ROWS % 4 == 0 || ri < ROWS) && (CI == CIP || c < CI) && gr >= 0 &&
                      gr < h && cok;
      a[k] = xi[ok ? (unsigned)((c * h + gr) * w + gc) : 0u];  // 32-bit offsets: image < 2^31
      am |= ok ? (uint64_t)1 << k : (uint64_t)0;
    }
    bm = 0;
#pragma unroll
    for (int q = 0; q < NH; ++q) {
      const int e = 64 * q + lane;  // (row k = e / 2, column 64 + e % 2)
      const int ri = wvu + 4 * (e >> 1);
      const int c = ri / XR, r = ri % XR, gr = r0 - 1 + r, g2 = c0 + 63 + (e & 1);
      const bool ok = e < 2 * RPWV && ri < ROWS && c < CI && gr >= 0 && gr < h && g2 < w;
      b[q] = xi[ok ? (unsigned)((c * h + gr) * w + g2) : 0u];
      bm |= ok ? 1u << q : 0u;
    }
  }

  template <int PS>
  __device__ __forceinline__ void store(float* sx, int lane, int wvu) const {
#pragma unroll
    for (int k = 0; k < RPWV; ++k) {
      const int ri = wvu + 4 * k;
      if (ROWS % 4 == 0 || ri < ROWS)
        sx[(ri / XR) * PS + (ri % XR) * kXW + lane] = (am >> k) & 1 ? a[k] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < NH; ++q) {
      const int e = 64 * q + lane;
      const int ri = wvu + 4 * (e >> 1);
      if (e < 2 * RPWV && ri < ROWS)
        sx[(ri / XR) * PS + (ri % XR) * kXW + 64 + (e & 1)] = (bm >> q) & 1u ? b[q] : 0.f;
    }
  }
};

// A CO x TH x 64 gradient tile (rows r0.., cols c0..) as float4: 16 lanes
// per row, 4 rows per wave instruction; zero outside the image.  FULL (w a
// multiple of 64, so every tile is full width): one unconditional float4 load
// per row at a clamped address -- no per-element branches, so all the tile's
// loads are in flight together (the generic path's conditional scalar loads
// made the compiler drain the queue row by row).
template <int CO, int TH, bool FULL>
struct GradTile {
  static constexpr int ROWS = CO * TH;
  static constexpr int PER = (ROWS + 15) / 16;
  static_assert(PER <= 32, "mask width");
  float4 v[PER];
  unsigned vm;  // rows in range (FULL), applied at store time like HaloTile's

  __device__ __forceinline__ void load(const float* __restrict__ gi, int h, int w, int r0,
                                       int c0, int lane, int wvu) {
    const int gc = c0 + 4 * (lane & 15);
    vm = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int ri = 16 * i + 4 * wvu + (lane >> 4);
      const int c = ri / TH, gr = r0 + ri % TH;
      const bool rok = (ROWS % 16 == 0 || ri < ROWS) && gr < h;
      if constexpr (FULL) {
        v[i] = *reinterpret_cast<const float4*>(gi + (rok ? (unsigned)((c * h + gr) * w + gc) : 0u));
        vm |= rok ? 1u << i : 0u;
      } else {
        const float* src = gi + (rok ? ((int64_t)c * h + gr) * w + gc : 0);
        const bool vec = (w & 3) == 0 && gc + 3 < w;
        if (vec) {
          const float4 t = *reinterpret_cast<const float4*>(src);
          v[i] = rok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          float4 t;
          t.x = rok && gc < w ? src[0] : 0.f;
          t.y = rok && gc + 1 < w ? src[1] : 0.f;
          t.z = rok && gc + 2 < w ? src[2] : 0.f;
          t.w = rok && gc + 3 < w ? src[3] : 0.f;
          v[i] = t;
        }
      }
    }
  }

  template <int PSG>
  __device__ __forceinline__ void store(float* sg, int lane, int wvu) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int ri = 16 * i + 4 * wvu + (lane >> 4);
      if (ROWS % 16 == 0 || ri < ROWS) {
        float4 t = v[i];
        if (FULL && !((vm >> i) & 1u)) t = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(sg + (ri / TH) * PSG + (ri % TH) * kTW + 4 * (lane & 15)) = t;
      }
    }
  }
};

struct TileGeo {
  int img, r0, c0;
};

// Tiles walked by a persistent block: t0, t0 + step, ... < end.  XCD-aware
// (blocks b and b + 8 share an XCD and its L2 under round-robin placement):
// the 8 block groups take 8 contiguous ranges of the tile list, so the tiles
// vertically next to a tile (+- tiles_w, whose halo rows it re-reads) are
// processed at about the same time in the SAME L2.  Speed only: any
// placement gives the same tiles to the same blocks.
struct TileWalk {
  int t0, step, end;
};

__device__ __forceinline__ TileWalk tile_walk(int ntiles) {
  const int b = blockIdx.x, g = gridDim.x;
  if (g % 8 != 0 || ntiles < g) return {b, g, ntiles};
  const int span = (ntiles + 7) / 8, grp = b & 7;
  const int end = (grp + 1) * span < ntiles ? (grp + 1) * span : ntiles;
  return {grp * span + (b >> 3), g >> 3, end};
}

__device__ __forceinline__ TileGeo tile_geo(int tile, int th, int tiles_w, int tiles_per_img) {
  const int t = tile % tiles_per_img;
  return {tile / tiles_per_img, (t / tiles_w) * th, (t % tiles_w) * kTW};
}

// --------------------------------------------------------------- forward
// Persistent: block b multiplies tiles b, b + grid, ...; the next tile's
// input is loaded into registers before the current tile's MFMAs.
// STATS (forward only): also the output's per-channel shifted sums over
// this block's tiles -> stats[(co * gridDim.x + block) * 4] = (shift, count,
// sum (y - shift), sum (y - shift)^2), the following BatchNorm's statistics
// without re-reading y.
template <int CI, int CO, int RPW, bool FLIP, bool STATS = false>
__global__ void __launch_bounds__(256, 2)
    conv3x3_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                       float* __restrict__ y, int h, int w, int tiles_w, int tiles_per_img,
                       int ntiles, float* __restrict__ stats = nullptr) {
  static_assert(!(STATS && FLIP), "statistics are a forward epilogue");
  constexpr int CIP = cpad4(CI);
  constexpr int TH = 4 * RPW;
  constexpr int XR = TH + 2;
  constexpr int PS = plane_words(XR, 16);
  constexpr int WS = wrow_words(CO);
  constexpr int NB = CO / 16;
  __shared__ float sx[CIP * PS];
  __shared__ float sw[9 * CIP * WS];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int64_t img_in = (int64_t)CI * h * w, img_out = (int64_t)CO * h * w;

  // weights -> sw[(tap * CIP + ci) * WS + co]; FLIP: W'[co][ci][tap] =
  // W[ci][co][8 - tap] (the data gradient is this convolution of gy).
  {
    constexpr int WN = 9 * CIP * CO;
    constexpr int WPER = (WN + 255) / 256;
    float v[WPER];
#pragma unroll
    for (int i = 0; i < WPER; ++i) {
      const int e = tid + 256 * i;
      const int co = e % CO, rest = e / CO, ci = rest % CIP, tap = rest / CIP;
      const bool ok = e < WN && ci < CI;
      const int src = FLIP ? (ci * CO + co) * 9 + (8 - tap) : (co * CI + ci) * 9 + tap;
      const float t = wt[ok ? src : 0];
      v[i] = ok ? t : 0.f;
    }
#pragma unroll
    for (int i = 0; i < WPER; ++i) {
      const int e = tid + 256 * i;
      const int co = e % CO, rest = e / CO, ci = rest % CIP, tap = rest / CIP;
      if (e < WN) sw[(tap * CIP + ci) * WS + co] = v[i];
    }
  }

  const int li = lane & 15, lk = lane >> 4;
  const float* ax = sx + lk * PS + li + wv * RPW * kXW;
  const float* bw = sw + lk * WS + li;
  const bool vec = (w & 3) == 0;

  mde::Sh run[STATS ? NB : 1];  // output channel 16 nb + li, this lane's pixels
#pragma unroll
  for (int nb = 0; nb < (STATS ? NB : 1); ++nb) run[nb] = {0.f, 0.f, 0.f, 0.f};
  bool first = true;  // wave-uniform: the wave's first tile sets the shifts
  HaloTile<CI, CIP, XR> T;
  const TileWalk tw = tile_walk(ntiles);
  int tile = tw.t0;
  if (tile < tw.end) {
    const TileGeo g = tile_geo(tile, TH, tiles_w, tiles_per_img);
    T.load(x + g.img * img_in, h, w, g.r0, g.c0, lane, wvu);
  }
  for (; tile < tw.end; tile += tw.step) {
    const TileGeo g = tile_geo(tile, TH, tiles_w, tiles_per_img);
    __syncthreads();  // previous tile's operands consumed (and weights staged)
    T.template store<PS>(sx, lane, wvu);
    __syncthreads();
    const int nxt = tile + tw.step;
    if (nxt < tw.end) {
      const TileGeo gn = tile_geo(nxt, TH, tiles_w, tiles_per_img);
      T.load(x + gn.img * img_in, h, w, gn.r0, gn.c0, lane, wvu);
    }

    f4 acc[RPW][4][NB];
#pragma unroll
    for (int q = 0; q < RPW; ++q)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[q][m][nb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap % 3;
#pragma unroll
      for (int cs = 0; cs < CIP / 4; ++cs) {
        float b[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) b[nb] = bw[(tap * CIP + 4 * cs) * WS + nb * 16];
#pragma unroll
        for (int q = 0; q < RPW; ++q)
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const float a = ax[4 * cs * PS + (q + dy) * kXW + m * 16 + dx];
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) acc[q][m][nb] = mfma4(a, b[nb], acc[q][m][nb]);
          }
      }
    }

    if constexpr (STATS) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        if (first) {  // one shift per channel and wave: lane (li, lk = 0)'s first output
          const bool ok0 = g.r0 + wv * RPW < h && g.c0 < w;
          run[nb].ref = __shfl(ok0 ? acc[0][0][nb][0] : 0.f, li, 64);
        }
#pragma unroll
        for (int q = 0; q < RPW; ++q)
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int row = g.r0 + wv * RPW + q, col = g.c0 + m * 16 + 4 * lk + i;
              mde::sh_add(run[nb], acc[q][m][nb][i], row < h && col < w);
            }
      }
      first = false;
    }
    // D layout: lane holds pixels 4*lk + i (i = 0..3) of output channel li.
    float* yi = y + g.img * img_out;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int row = g.r0 + wv * RPW + q;
      if (row >= h) continue;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int col = g.c0 + m * 16 + 4 * lk;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          float* dst = yi + ((int64_t)(nb * 16 + li) * h + row) * w + col;
          const f4 v = acc[q][m][nb];
          if (vec && col + 3 < w) {
            *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (col + i < w) dst[i] = v[i];
          }
        }
      }
    }
  }
  if constexpr (STATS) {
    // lanes li, li + 16, +32, +48 share the channel's shift: plain-sum
    // butterfly over lk, then the 4 waves in order through LDS (sx is free:
    // every wave is past its last tile's reads once all pass the barrier)
    __syncthreads();
    float* part = sx;  // [4][CO][4]
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const mde::Sh a = mde::sh_xor_sum(mde::sh_xor_sum(run[nb], 16), 32);
      if (lk == 0) {
        float* p4 = part + (wv * CO + 16 * nb + li) * 4;
        p4[0] = a.ref;
        p4[1] = a.n;
        p4[2] = a.s1;
        p4[3] = a.s2;
      }
    }
    __syncthreads();
    if (tid < CO) {
      mde::Sh a{part[tid * 4], part[tid * 4 + 1], part[tid * 4 + 2], part[tid * 4 + 3]};
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const float* p4 = part + (k * CO + tid) * 4;
        a = mde::sh_merge(a, {p4[0], p4[1], p4[2], p4[3]});
      }
      float* o4 = stats + ((int64_t)tid * gridDim.x + blockIdx.x) * 4;
      o4[0] = a.ref;
      o4[1] = a.n;
      o4[2] = a.s1;
      o4[3] = a.s2;
    }
  }
}

// ------------------------------------------------------- weight gradient
template <int CI, int CO, int TH, int PW>
struct WgradCfg {
  static constexpr int CIP = cpad4(CI);
  static constexpr int XR = TH + 2;
  static constexpr int PSX = plane_words(XR, 4);  // = 4 (mod 64)
  static constexpr int PSG = TH * kTW + 4;        // = 4 (mod 64)
  static constexpr int NREAL = 9 * CIP;           // n = tap * CIP + ci
  static constexpr int NP = (NREAL + 15) / 16 * 16;
  static constexpr int NBLK = NP / 16;
  static constexpr int MB = CO / 16;
  static constexpr int TWAYS = 4 / PW;            // waves splitting the N blocks
  static constexpr int NBW = (NBLK + TWAYS - 1) / TWAYS;
  static constexpr int RPWG = TH / PW;            // tile rows per wave
  static constexpr int ZERO = CIP * PSX;          // zero pad for n >= NREAL
  static constexpr int STAGE = ZERO + XR * kXW + CO * PSG;
  // PW == 1: each wave owns whole N blocks over all rows -> stores its
  // accumulators straight to the block partial (no LDS reduction)
  static constexpr int RED = PW == 1 ? 0 : PW * MB * NBLK * 256;
  static constexpr int SMEM = STAGE > RED ? STAGE : RED;
  static constexpr int M = CO * NP;               // partial elements per block
};

template <int CI, int CO, int TH, int PW, bool FULL>
__global__ void __launch_bounds__(256, 2)
    conv3x3_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                         float* __restrict__ part, int h, int w, int tiles_w,
                         int tiles_per_img, int ntiles) {
  using C = WgradCfg<CI, CO, TH, PW>;
  __shared__ float smem[C::SMEM];
  float* sx = smem;
  float* sg = smem + C::ZERO + C::XR * kXW;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int pg = wv % PW, tg = wv / PW;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int64_t img_in = (int64_t)CI * h * w, img_out = (int64_t)CO * h * w;

  // per-lane B offsets of this wave's N blocks (tap shift folded in)
  int boff[C::NBW];
#pragma unroll
  for (int j = 0; j < C::NBW; ++j) {
    const int n = 16 * (tg + C::TWAYS * j) + li;
    if (n < C::NREAL) {
      const int tap = n / C::CIP, ci = n % C::CIP;
      boff[j] = ci * C::PSX + (tap / 3) * kXW + tap % 3 + lk;
    } else {
      boff[j] = C::ZERO + lk;
    }
  }
  const int aoff = li * C::PSG + lk;

  f4 acc[C::MB][C::NBW];
#pragma unroll
  for (int mb = 0; mb < C::MB; ++mb)
#pragma unroll
    for (int j = 0; j < C::NBW; ++j) acc[mb][j] = f4{0.f, 0.f, 0.f, 0.f};

  for (int e = tid; e < C::XR * kXW; e += 256) smem[C::ZERO + e] = 0.f;
  HaloTile<CI, C::CIP, C::XR> T;
  GradTile<CO, TH, FULL> G;
  const TileWalk tw = tile_walk(ntiles);
  int tile = tw.t0;
  if (tile < tw.end) {
    const TileGeo g = tile_geo(tile, TH, tiles_w, tiles_per_img);
    G.load(gy + g.img * img_out, h, w, g.r0, g.c0, lane, wvu);
    T.load(x + g.img * img_in, h, w, g.r0, g.c0, lane, wvu);
  }
  for (; tile < tw.end; tile += tw.step) {
    __syncthreads();  // previous tile's operands consumed
    T.template store<C::PSX>(sx, lane, wvu);
    G.template store<C::PSG>(sg, lane, wvu);
    __syncthreads();
    const int nxt = tile + tw.step;
    if (nxt < tw.end) {
      const TileGeo gn = tile_geo(nxt, TH, tiles_w, tiles_per_img);
      G.load(gy + gn.img * img_out, h, w, gn.r0, gn.c0, lane, wvu);
      T.load(x + gn.img * img_in, h, w, gn.r0, gn.c0, lane, wvu);
    }

    for (int rr = 0; rr < C::RPWG; ++rr) {
      const int row = pg * C::RPWG + rr;
      const float* ga = sg + aoff + row * kTW;
      const float* xb = sx + row * kXW;
#pragma unroll 4
      for (int s = 0; s < kTW / 4; ++s) {
        float a[C::MB];
#pragma unroll
        for (int mb = 0; mb < C::MB; ++mb) a[mb] = ga[mb * 16 * C::PSG + 4 * s];
#pragma unroll
        for (int j = 0; j < C::NBW; ++j) {
          const float b = xb[boff[j] + 4 * s];
#pragma unroll
          for (int mb = 0; mb < C::MB; ++mb) acc[mb][j] = mfma4(a[mb], b, acc[mb][j]);
        }
      }
    }
  }

  float* out = part + (int64_t)blockIdx.x * C::M;
  if constexpr (PW == 1) {
    // lane holds co = 16 mb + 4 lk + i, n = 16 nb + li of its N blocks
#pragma unroll
    for (int mb = 0; mb < C::MB; ++mb)
#pragma unroll
      for (int j = 0; j < C::NBW; ++j) {
        const int nb = tg + C::TWAYS * j;
        if (nb < C::NBLK) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            out[(16 * mb + 4 * lk + i) * C::NP + 16 * nb + li] = acc[mb][j][i];
        }
      }
    return;
  }
  // sum the PW pixel-group partials through LDS, then one block partial:
  // red[pg][mb][nb][co16][n16]; lane holds co16 = 4*lk + i, n16 = li.
  __syncthreads();
#pragma unroll
  for (int mb = 0; mb < C::MB; ++mb)
#pragma unroll
    for (int j = 0; j < C::NBW; ++j) {
      const int nb = tg + C::TWAYS * j;
      if (nb < C::NBLK) {
        float* d = smem + ((pg * C::MB + mb) * C::NBLK + nb) * 256 + li;
#pragma unroll
        for (int i = 0; i < 4; ++i) d[(4 * lk + i) * 16] = acc[mb][j][i];
      }
    }
  __syncthreads();
  for (int e = tid; e < C::M; e += 256) {
    const int co = e / C::NP, n = e % C::NP;
    const int mb = co / 16, nb = n / 16;
    const int o = ((mb * C::NBLK + nb) * 256) + (co % 16) * 16 + n % 16;
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < PW; ++p) s += smem[p * C::MB * C::NBLK * 256 + o];
    out[e] = s;
  }
}

// Stage 1: part [G][M] -> part2 [S][M] (S interleaved groups of blocks).
__global__ void __launch_bounds__(256)
    wgrad_reduce1_kernel(const float* __restrict__ part, float* __restrict__ part2,
                         int g, int m) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= m) return;
  const int s = blockIdx.y, ns = gridDim.y;
  float a0 = 0.f, a1 = 0.f;
  int b = s;
  for (; b + ns < g; b += 2 * ns) {
    a0 += part[(int64_t)b * m + e];
    a1 += part[(int64_t)(b + ns) * m + e];
  }
  if (b < g) a0 += part[(int64_t)b * m + e];
  part2[(int64_t)s * m + e] = a0 + a1;
}

// Stage 2: sum the S groups and scatter n = tap * cip + ci to gw[co][ci][tap].
__global__ void __launch_bounds__(256)
    wgrad_reduce2_kernel(const float* __restrict__ part2, float* __restrict__ gw, int ns,
                         int co_n, int ci_n, int cip, int np) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= co_n * np) return;
  const int co = e / np, n = e % np;
  const int tap = n / cip, ci = n % cip;
  if (tap >= 9 || ci >= ci_n) return;
  float s = 0.f;
  for (int k = 0; k < ns; ++k) s += part2[(int64_t)k * co_n * np + e];
  gw[(co * ci_n + ci) * 9 + tap] = s;
}

constexpr int kReduceSplit = 32;

// ---------------------------------------------------------------- dispatch
enum Pass { kFwd = 0, kDgrad = 1, kWgrad = 2 };

// Resident blocks of a kernel on the whole device (persistent grids).
template <auto Kernel>
int resident_blocks() {
  static const int cached = [] {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, Kernel, 256, 0);
    return (cus > 0 ? cus : 256) * (per > 0 ? per : 1);
  }();
  return cached;
}

template <int CI, int CO, int RPW, bool FLIP, bool STATS = false>
int fwd_grid(int64_t n, int64_t h, int64_t w, int* tiles_w, int* tiles_per_img, int* ntiles) {
  constexpr int TH = 4 * RPW;
  *tiles_w = (int)mde::cdiv(w, kTW);
  *tiles_per_img = (int)(mde::cdiv(h, TH) * *tiles_w);
  const int64_t nt = n * *tiles_per_img;
  if (nt > 0x7fffffff) return 0;
  *ntiles = (int)nt;
  const int res = resident_blocks<conv3x3_fwd_kernel<CI, CO, RPW, FLIP, STATS>>();
  return nt < res ? (int)nt : res;
}

template <int CI, int CO, int RPW, bool FLIP, bool STATS = false>
int launch_fwd(const float* in, const float* wt, float* out, int64_t n, int64_t h, int64_t w,
               double bytes, int kid, hipStream_t s, float* stats = nullptr) {
  const double flops = 2.0 * 9 * CI * CO * (double)(n * h * w);
  int tiles_w, tiles_per_img, ntiles;
  const int grid = fwd_grid<CI, CO, RPW, FLIP, STATS>(n, h, w, &tiles_w, &tiles_per_img, &ntiles);
  if (grid <= 0) return MDE_ERR_INVALID_ARG;
  MDE_LAUNCH_MFMA(kid, bytes, flops, s, (conv3x3_fwd_kernel<CI, CO, RPW, FLIP, STATS>),
                  dim3(grid), dim3(256), 0, in, wt, out, (int)h, (int)w, tiles_w, tiles_per_img,
                  ntiles, stats);
  return MDE_OK;
}

struct WgradPlan {
  int th, tiles_w, tiles_per_img, ntiles, grid, m, np, cip;
};

constexpr int kWgradGrid = 1024;

template <int CI, int CO, int TH, int PW>
WgradPlan wgrad_plan(int64_t n, int64_t h, int64_t w) {
  using C = WgradCfg<CI, CO, TH, PW>;
  WgradPlan p;
  p.th = TH;
  p.tiles_w = (int)mde::cdiv(w, kTW);
  p.tiles_per_img = (int)(mde::cdiv(h, TH) * p.tiles_w);
  const int64_t nt = n * p.tiles_per_img;
  p.ntiles = nt > 0x7fffffff ? 0x7fffffff : (int)nt;
  p.grid = p.ntiles < kWgradGrid ? p.ntiles : kWgradGrid;
  p.m = C::M;
  p.np = C::NP;
  p.cip = C::CIP;
  return p;
}

template <int CI, int CO, int TH, int PW>
int launch_wgrad(const float* x, const float* gy, float* gw, int64_t n, int64_t h, int64_t w,
                 float* ws, double bytes, hipStream_t s) {
  const WgradPlan p = wgrad_plan<CI, CO, TH, PW>(n, h, w);
  const double flops = 2.0 * 9 * CI * CO * (double)(n * h * w);
  float* part = ws;
  float* part2 = ws + (int64_t)p.grid * p.m;
  // the 3-channel guide convs' weight gradients have ~12 flop per byte, under the
  // fp32 MFMA ridge (157 TF / 8 TB/s ~ 20): timed as HBM-bound under their own id
  if (CI == 3) {
    if (w % kTW == 0)
      MDE_LAUNCH(mde::K_C3_WGRAD_GUIDE, bytes, s, (conv3x3_wgrad_kernel<CI, CO, TH, PW, true>),
                 dim3(p.grid), dim3(256), 0, x, gy, part, (int)h, (int)w, p.tiles_w,
                 p.tiles_per_img, p.ntiles);
    else
      MDE_LAUNCH(mde::K_C3_WGRAD_GUIDE, bytes, s, (conv3x3_wgrad_kernel<CI, CO, TH, PW, false>),
                 dim3(p.grid), dim3(256), 0, x, gy, part, (int)h, (int)w, p.tiles_w,
                 p.tiles_per_img, p.ntiles);
  } else if (w % kTW == 0) {
    MDE_LAUNCH_MFMA(mde::K_C3_WGRAD, bytes, flops, s, (conv3x3_wgrad_kernel<CI, CO, TH, PW, true>),
                    dim3(p.grid), dim3(256), 0, x, gy, part, (int)h, (int)w, p.tiles_w,
                    p.tiles_per_img, p.ntiles);
  } else {
    MDE_LAUNCH_MFMA(mde::K_C3_WGRAD, bytes, flops, s, (conv3x3_wgrad_kernel<CI, CO, TH, PW, false>),
                    dim3(p.grid), dim3(256), 0, x, gy, part, (int)h, (int)w, p.tiles_w,
                    p.tiles_per_img, p.ntiles);
  }
  const int split = p.grid < kReduceSplit ? p.grid : kReduceSplit;
  MDE_LAUNCH(mde::K_C3_WREDUCE, 4.0 * p.grid * p.m, s, wgrad_reduce1_kernel,
             dim3((unsigned)mde::cdiv(p.m, 256), split), dim3(256), 0, part, part2, p.grid, p.m);
  MDE_LAUNCH(mde::K_C3_WREDUCE, 4.0 * split * p.m, s, wgrad_reduce2_kernel,
             dim3((unsigned)mde::cdiv(p.m, 256)), dim3(256), 0, part2, gw, split, CO, CI, p.cip,
             p.np);
  return MDE_OK;
}

// Supported (cin, cout) per pass.  Forward: the guide convs (3 -> 16/32/64),
// 16 -> 16 and 32 -> 32; data gradient: 16 -> 16 and 32 -> 32 (the guide
// convs read the image, which needs no gradient); weight gradient: all.
bool supported(int64_t cin, int64_t cout, int pass) {
  const bool guide = cin == 3 && (cout == 16 || cout == 32 || cout == 64);
  const bool square = (cin == 16 && cout == 16) || (cin == 32 && cout == 32);
  switch (pass) {
    case kFwd:
      return guide || square;
    case kDgrad:
      return square;
    case kWgrad:
      return guide || square;
    default:
      return false;
  }
}

// Tuning experiments only (tools/kbench.py): MDE_C3_VARIANT selects alternative
// tile shapes for the 16->16 / 32->32 kernels; 0 (unset) is the shipped choice.
int variant() {
  static const int v = [] {
    const char* e = std::getenv("MDE_C3_VARIANT");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

// The tile loaders index one image with 32-bit offsets: 64 channels x h x w
// (the widest supported image) must stay under 2^31 elements.
bool dims_ok(int64_t n, int64_t h, int64_t w) {
  return n > 0 && h > 0 && w > 0 && h < (1 << 24) && w < (1 << 24) &&
         64 * h * w < ((int64_t)1 << 31);
}

}  // namespace

extern "C" {

int mde_conv3x3_supported(int64_t cin, int64_t cout, int pass) {
  return supported(cin, cout, pass) ? 1 : 0;
}

int mde_conv3x3_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t cin,
                    int64_t cout, int64_t h, int64_t w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !weight || !y || !dims_ok(n, h, w)) return MDE_ERR_INVALID_ARG;
  if (!supported(cin, cout, kFwd)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const float* in = (const float*)x;
  float* out = (float*)y;
  const double bytes = 4.0 * n * h * w * (double)(cin + cout);
  const int k = mde::K_C3_FWD;
  if (cin == 3 && cout == 16) return launch_fwd<3, 16, 2, false>(in, weight, out, n, h, w, bytes, k, s);
  if (cin == 3 && cout == 32) return launch_fwd<3, 32, 1, false>(in, weight, out, n, h, w, bytes, k, s);
  if (cin == 3 && cout == 64) return launch_fwd<3, 64, 1, false>(in, weight, out, n, h, w, bytes, k, s);
  if (cin == 16 && variant() == 1) return launch_fwd<16, 16, 2, false>(in, weight, out, n, h, w, bytes, k, s);
  if (cin == 16) return launch_fwd<16, 16, 1, false>(in, weight, out, n, h, w, bytes, k, s);
  return launch_fwd<32, 32, 1, false>(in, weight, out, n, h, w, bytes, k, s);
}

// Forward with the BatchNorm statistics epilogue: stats [cout][blocks][4]
// (shift, count, s1, s2), blocks = mde_conv3x3_stats_blocks(...).
int mde_conv3x3_stats_blocks(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w) {
  if (!supported(cin, cout, kFwd) || !dims_ok(n, h, w)) return 0;
  int a, b, c;
  if (cin == 3 && cout == 16) return fwd_grid<3, 16, 2, false, true>(n, h, w, &a, &b, &c);
  if (cin == 3 && cout == 32) return fwd_grid<3, 32, 1, false, true>(n, h, w, &a, &b, &c);
  if (cin == 3 && cout == 64) return fwd_grid<3, 64, 1, false, true>(n, h, w, &a, &b, &c);
  if (cin == 16) return fwd_grid<16, 16, 1, false, true>(n, h, w, &a, &b, &c);
  return fwd_grid<32, 32, 1, false, true>(n, h, w, &a, &b, &c);
}

int mde_conv3x3_fwd_stats(const void* x, const float* weight, void* y, float* stats, int64_t n,
                          int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype,
                          void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !weight || !y || !stats || !dims_ok(n, h, w)) return MDE_ERR_INVALID_ARG;
  if (!supported(cin, cout, kFwd)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const float* in = (const float*)x;
  float* out = (float*)y;
  const double bytes = 4.0 * n * h * w * (double)(cin + cout);
  const int k = mde::K_C3_FWD;
  if (cin == 3 && cout == 16)
    return launch_fwd<3, 16, 2, false, true>(in, weight, out, n, h, w, bytes, k, s, stats);
  if (cin == 3 && cout == 32)
    return launch_fwd<3, 32, 1, false, true>(in, weight, out, n, h, w, bytes, k, s, stats);
  if (cin == 3 && cout == 64)
    return launch_fwd<3, 64, 1, false, true>(in, weight, out, n, h, w, bytes, k, s, stats);
  if (cin == 16)
    return launch_fwd<16, 16, 1, false, true>(in, weight, out, n, h, w, bytes, k, s, stats);
  return launch_fwd<32, 32, 1, false, true>(in, weight, out, n, h, w, bytes, k, s, stats);
}

int mde_conv3x3_bwd_data(const void* gy, const float* weight, void* gx, int64_t n, int64_t cin,
                         int64_t cout, int64_t h, int64_t w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !weight || !gx || !dims_ok(n, h, w)) return MDE_ERR_INVALID_ARG;
  if (!supported(cin, cout, kDgrad)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const float* in = (const float*)gy;
  float* out = (float*)gx;
  const double bytes = 4.0 * n * h * w * (double)(cin + cout);
  const int k = mde::K_C3_DGRAD;
  if (cin == 16 && variant() == 1) return launch_fwd<16, 16, 2, true>(in, weight, out, n, h, w, bytes, k, s);
  if (cin == 16) return launch_fwd<16, 16, 1, true>(in, weight, out, n, h, w, bytes, k, s);
  return launch_fwd<32, 32, 1, true>(in, weight, out, n, h, w, bytes, k, s);
}

size_t mde_conv3x3_wgrad_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w) {
  if (!supported(cin, cout, kWgrad) || !dims_ok(n, h, w)) return 0;
  WgradPlan p;
  if (cin == 3 && cout == 16) p = wgrad_plan<3, 16, 8, 4>(n, h, w);
  else if (cin == 3 && cout == 32) p = wgrad_plan<3, 32, 8, 4>(n, h, w);
  else if (cin == 3) p = wgrad_plan<3, 64, 4, 4>(n, h, w);
  else if (cin == 16 && variant() == 1) p = wgrad_plan<16, 16, 8, 4>(n, h, w);
  else if (cin == 16 && variant() == 2) p = wgrad_plan<16, 16, 4, 2>(n, h, w);
  else if (cin == 16) p = wgrad_plan<16, 16, 4, 4>(n, h, w);
  else if (variant() == 1) p = wgrad_plan<32, 32, 4, 2>(n, h, w);
  else if (variant() == 2) p = wgrad_plan<32, 32, 4, 1>(n, h, w);
  else p = wgrad_plan<32, 32, 2, 2>(n, h, w);
  const int split = p.grid < kReduceSplit ? p.grid : kReduceSplit;
  return sizeof(float) * ((size_t)p.grid + (size_t)split) * (size_t)p.m;
}

int mde_conv3x3_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t cin,
                      int64_t cout, int64_t h, int64_t w, void* workspace, int dtype,
                      void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !x || !gweight || !workspace || !dims_ok(n, h, w)) return MDE_ERR_INVALID_ARG;
  if (!supported(cin, cout, kWgrad)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const float* xi = (const float*)x;
  const float* g = (const float*)gy;
  float* ws = (float*)workspace;
  const double bytes = 4.0 * n * h * w * (double)(cin + cout);
  if (cin == 3 && cout == 16) return launch_wgrad<3, 16, 8, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 3 && cout == 32) return launch_wgrad<3, 32, 8, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 3) return launch_wgrad<3, 64, 4, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 16 && variant() == 1) return launch_wgrad<16, 16, 8, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 16 && variant() == 2) return launch_wgrad<16, 16, 4, 2>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 16) return launch_wgrad<16, 16, 4, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (variant() == 1) return launch_wgrad<32, 32, 4, 2>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (variant() == 2) return launch_wgrad<32, 32, 4, 1>(xi, g, gweight, n, h, w, ws, bytes, s);
  return launch_wgrad<32, 32, 2, 2>(xi, g, gweight, n, h, w, ws, bytes, s);
}

}  // extern "C"
