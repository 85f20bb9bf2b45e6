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

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Resident blocks of a kernel on the whole device (persistent grids; the
// occupancy query is for 256-thread blocks).
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

constexpr int kTW = 64;       // output columns per tile (4 MFMA row tiles)
constexpr int kXW = kTW + 2;  // staged input columns (one-pixel halo each side)

constexpr int cpad4(int c) { return (c + 3) / 4 * 4; }
// LDS plane stride (words) for `rows` staged rows of kXW, = `mod` (mod 64).
constexpr int plane_words(int rows, int mod) { return (rows * kXW + 63) / 64 * 64 + mod; }
// Weight-row stride (words): the four k-lane groups of a B read land on
// disjoint 16-bank quarters (16 -> 16, 32 -> 48, 64 -> 80, all = 16k mod 64
// with k odd or the groups spread 0/16/32/48).
constexpr int wrow_words(int co) { return co == 16 ? 16 : (co == 32 ? 48 : 80); }

// v rounded to bf16 precision (RNE; the hardware conversion, as autocast's cast)
__device__ __forceinline__ float rbf(float v) {
  return __uint_as_float((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v) << 16);
}

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

  // RB: values rounded to bf16 precision (RNE) as they are staged -- the
  // autocast guide conv computes on the bf16 image
  template <int PS, bool RB = false>
  __device__ __forceinline__ void store(float* sx, int lane, int wvu) const {
#pragma unroll
    for (int k = 0; k < RPWV; ++k) {
      const int ri = wvu + 4 * k;
      if (ROWS % 4 == 0 || ri < ROWS) {
        const float v = (am >> k) & 1 ? a[k] : 0.f;
        sx[(ri / XR) * PS + (ri % XR) * kXW + lane] = RB ? rbf(v) : v;
      }
    }
#pragma unroll
    for (int q = 0; q < NH; ++q) {
      const int e = 64 * q + lane;
      const int ri = wvu + 4 * (e >> 1);
      if (e < 2 * RPWV && ri < ROWS) {
        const float v = (bm >> q) & 1u ? b[q] : 0.f;
        sx[(ri / XR) * PS + (ri % XR) * kXW + 64 + (e & 1)] = RB ? rbf(v) : v;
      }
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
// TO = bf16 (the autocast guide convs, modules.py:52-54 under bf16 autocast):
// image and weights rounded to bf16 precision on staging (autocast's input
// casts), exact f32 products and f32 accumulation as the bf16 MFMA, output
// rounded to bf16 (RNE) -- the statistics epilogue sees the rounded values.
template <int CI, int CO, int RPW, bool FLIP, bool STATS = false, typename TO = float>
__global__ void __launch_bounds__(256, 2)
    conv3x3_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                       TO* __restrict__ y, int h, int w, int tiles_w, int tiles_per_img,
                       int ntiles, float* __restrict__ stats = nullptr) {
  static_assert(!(STATS && FLIP), "statistics are a forward epilogue");
  constexpr bool RB = sizeof(TO) == 2;
  constexpr int CIP = cpad4(CI);
  constexpr int TH = 4 * RPW;
  constexpr int XR = TH + 2;
  constexpr int PS = plane_words(XR, 16);
  constexpr int WS = wrow_words(CO);
  constexpr int NB = CO / 16;
  __shared__ float sx[CIP * PS];
  __shared__ float sw[9 * CIP * WS];
  // staged output (the 3-input-channel guide convs, see the epilogue): lines
  // of 64 pixels + a 16-byte pad, where the tile fits 40 KB
  constexpr int kSOL = 64 + 16 / (int)sizeof(TO);
  constexpr bool SO = CI == 3 && !FLIP && TH * CO * kSOL * (int)sizeof(TO) <= 40 * 1024;
  __shared__ __attribute__((aligned(16))) TO so[SO ? TH * CO * kSOL : 4];

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
      v[i] = ok ? (RB ? rbf(t) : t) : 0.f;
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
    T.template store<PS, RB>(sx, lane, wvu);
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

    if constexpr (RB) {  // the bf16 output's values (statistics of what is stored)
#pragma unroll
      for (int q = 0; q < RPW; ++q)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int i = 0; i < 4; i += 2) {  // hardware RNE conversion, two at a time
              using bf2v = __bf16 __attribute__((ext_vector_type(2)));
              const uint32_t p = __builtin_bit_cast(
                  uint32_t, bf2v{(__bf16)acc[q][m][nb][i], (__bf16)acc[q][m][nb][i + 1]});
              acc[q][m][nb][i] = __uint_as_float(p << 16);
              acc[q][m][nb][i + 1] = __uint_as_float(p & 0xffff0000u);
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
        for (int q = 0; q < RPW; ++q) {
          const int row = g.r0 + wv * RPW + q;
          if (row < h && g.c0 + 64 <= w) {
            // a whole 64-pixel row segment (wave-uniform): no per-pixel bounds
            // tests (they were most of the epilogue's VALU); same sums
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const float d = acc[q][m][nb][i] - run[nb].ref;
                run[nb].s1 += d;
                run[nb].s2 = fmaf(d, d, run[nb].s2);
              }
            run[nb].n += 16.f;
          } else {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int col = g.c0 + m * 16 + 4 * lk + i;
                mde::sh_add(run[nb], acc[q][m][nb][i], row < h && col < w);
              }
          }
        }
      }
      first = false;
    }
    // D layout: lane holds pixels 4*lk + i (i = 0..3) of output channel li.
    TO* yi = y + g.img * img_out;
    if constexpr (SO) {
      // The guide convs (3 input channels) are output-bound: their direct
      // stores wrote 32 / 64-byte pieces of 16 channel planes per instruction
      // (1.3-3.3 TB/s).  Through LDS instead: the block's [TH rows][CO][64]
      // tile, then 16-byte pieces of whole 64-pixel row segments (the
      // conv3x3_bf_fwd2 epilogue).  `so` is rewritten only after the next
      // tile's two loop-top barriers, so one barrier here suffices.
      if (vec) {
#pragma unroll
        for (int q = 0; q < RPW; ++q)
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
              const f4 v = acc[q][m][nb];
              TO* sp = so + ((wv * RPW + q) * CO + nb * 16 + li) * kSOL + m * 16 + 4 * lk;
              if constexpr (RB) {  // already bf16 values: the high halves, two a word
                *reinterpret_cast<uint2*>(sp) = make_uint2(
                    __builtin_amdgcn_perm(__float_as_uint(v[1]), __float_as_uint(v[0]), 0x07060302u),
                    __builtin_amdgcn_perm(__float_as_uint(v[3]), __float_as_uint(v[2]), 0x07060302u));
              } else {
                mde::st4(sp, make_float4(v[0], v[1], v[2], v[3]));
              }
            }
        __syncthreads();
        constexpr int PX = 16 / (int)sizeof(TO);  // pixels per 16-byte piece
        constexpr int PPL = 64 / PX;              // pieces per 64-pixel line
        constexpr int NP = TH * CO * PPL;
        static_assert(NP % 256 == 0, "whole pieces per thread");
#pragma unroll
        for (int k = 0; k < NP / 256; ++k) {
          const int e = tid + 256 * k, line = e / PPL, pc = e % PPL;
          const int r = line / CO, co = line % CO;
          const int grow = g.r0 + r, col = g.c0 + PX * pc;
          const uint4 u = *reinterpret_cast<const uint4*>(so + line * kSOL + PX * pc);
          TO* dst = yi + ((int64_t)co * h + grow) * w + col;
          if (grow < h && col + PX <= w)
            *reinterpret_cast<uint4*>(dst) = u;
          else if (grow < h && col < w)  // bf16, w % 4 == 0: the first 4 pixels
            *reinterpret_cast<uint2*>(dst) = make_uint2(u.x, u.y);
        }
        continue;
      }
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int row = g.r0 + wv * RPW + q;
      if (row >= h) continue;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int col = g.c0 + m * 16 + 4 * lk;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          TO* dst = yi + ((int64_t)(nb * 16 + li) * h + row) * w + col;
          const f4 v = acc[q][m][nb];
          if (vec && col + 3 < w) {
            mde::st4(dst, make_float4(v[0], v[1], v[2], v[3]));
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (col + i < w) mde::st1(dst + i, v[i]);
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

// Weight-gradient reduction, one launch, fixed summation order: block
// (x, grp) owns 64 elements; its 16 waves sum the interleaved partial subsets
// b = w, w + 16, ... (four accumulators per lane, so 16 loads per lane are in
// flight), then wave 0 adds the 16 subset sums in order and scatters them to
// gw.  (Two launches of 256-thread blocks spent ~11 us each, latency-bound;
// a one-launch last-block hand-off between blocks needs agent-scope fences,
// which write back L2 on every block: 53 us.)
struct ReduceMap {
  int wide;             // > 0: the wide-channel layout [co wide][tap 9][ci 32] per group
                        // (wide = the group's output channels, 64 or 32)
  int np, cip;          // regular layout [co][n = tap * cip + ci] (np columns)
  int ci_n, co_n;
};

__device__ __forceinline__ int64_t gw_index(const ReduceMap& r, int grp, int e) {
  if (r.wide) {
    const int ngo = r.co_n / r.wide, col = e / 288, n = e % 288;
    const int co = (grp % ngo) * r.wide + col, ci = (grp / ngo) * 32 + n % 32;
    if (ci >= r.ci_n) return -1;  // a padded input-channel group's zero rows
    return ((int64_t)co * r.ci_n + ci) * 9 + n / 32;
  }
  const int co = e / r.np, n = e % r.np, tap = n / r.cip, ci = n % r.cip;
  if (tap >= 9 || ci >= r.ci_n) return -1;
  return ((int64_t)co * r.ci_n + ci) * 9 + tap;
}

constexpr int kRedWaves = 16;

__global__ void __launch_bounds__(64 * kRedWaves)
    wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ gw, int g, int m,
                        ReduceMap map) {
  __shared__ float red[kRedWaves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane, grp = blockIdx.y;
  const float* pg = part + (int64_t)grp * g * m + e;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (e < m) {
    int b = wv;
#pragma unroll 4
    for (; b + 3 * kRedWaves < g; b += 4 * kRedWaves) {
      a0 += pg[(int64_t)b * m];
      a1 += pg[(int64_t)(b + kRedWaves) * m];
      a2 += pg[(int64_t)(b + 2 * kRedWaves) * m];
      a3 += pg[(int64_t)(b + 3 * kRedWaves) * m];
    }
    for (; b < g; b += kRedWaves) a0 += pg[(int64_t)b * m];
  }
  red[wv][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wv != 0 || e >= m) return;
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < kRedWaves; ++k) sum += red[k][lane];
  const int64_t o = gw_index(map, grp, e);
  if (o >= 0) gw[o] = sum;
}

// float4 variant (m % 4 == 0): block (x, grp, z) sums rows [z R, z R + R) of
// 256 columns, 8 waves on interleaved row subsets (four float4 accumulators a
// lane: 64 bytes in flight per lane), wave 0 adds the 8 subset sums in order.
// FINAL: scatter to gw; else the slice sum overwrites the slice's first row
// (only this block reads those rows of these columns), and a second launch
// sums the S slice rows (stride R m).  Slices keep >= ~512 blocks in flight
// when the partial rows are many and the columns few (the 16 -> 16 kernel's
// 1024 rows of 2304 columns: 9 column blocks alone), where one block per
// column range serialised hundreds of loads per lane.
constexpr int kRed4Waves = 8;

template <bool FINAL>
__global__ void __launch_bounds__(64 * kRed4Waves)
    wgrad_reduce4_kernel(float* __restrict__ part, float* __restrict__ gw, int rows, int m,
                         int64_t rstride, int64_t gstride, int slice, ReduceMap map) {
  __shared__ float4 red[kRed4Waves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int e4 = blockIdx.x * 64 + lane, grp = blockIdx.y;
  const int m4 = m >> 2;
  const int b0 = blockIdx.z * slice, b1 = b0 + slice < rows ? b0 + slice : rows;
  const int64_t rs4 = rstride >> 2;
  float4* pg = reinterpret_cast<float4*>(part + (int64_t)grp * gstride) + e4;
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0, a3 = a0;
  if (e4 < m4) {
    int b = b0 + wv;
    for (; b + 3 * kRed4Waves < b1; b += 4 * kRed4Waves) {
      const float4 v0 = pg[(int64_t)b * rs4], v1 = pg[(int64_t)(b + kRed4Waves) * rs4];
      const float4 v2 = pg[(int64_t)(b + 2 * kRed4Waves) * rs4];
      const float4 v3 = pg[(int64_t)(b + 3 * kRed4Waves) * rs4];
      a0 = a0 + v0;
      a1 = a1 + v1;
      a2 = a2 + v2;
      a3 = a3 + v3;
    }
    for (; b < b1; b += kRed4Waves) a0 = a0 + pg[(int64_t)b * rs4];
  }
  red[wv][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wv != 0 || e4 >= m4) return;
  float4 sum = red[0][lane];
#pragma unroll
  for (int k = 1; k < kRed4Waves; ++k) sum = sum + red[k][lane];
  if constexpr (FINAL) {
    const float v[4] = {sum.x, sum.y, sum.z, sum.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t o = gw_index(map, grp, 4 * e4 + j);
      if (o >= 0) gw[o] = v[j];
    }
  } else {
    pg[(int64_t)b0 * rs4] = sum;
  }
}

// Weight-gradient workspace: the partials, [groups][g][m].
inline size_t wgrad_ws_bytes(int groups, int g, int m) {
  return sizeof(float) * (size_t)groups * (size_t)g * (size_t)m;
}

// Slices for the float4 reduction: enough (x, grp, z) blocks to fill the chip,
// >= 16 rows a slice (MDE_WRED_SLICES=1: one launch always, A/B).
inline int reduce_slices(int groups, int g, int m) {
  static const int force = [] {
    const char* e = std::getenv("MDE_WRED_SLICES");
    return e ? std::atoi(e) : 0;
  }();
  if (force > 0) return force < g ? force : g;
  const int blocks = (int)mde::cdiv(m, 256) * groups;
  // >= 64 column blocks (the wide kernels' 64 x 288-element groups): one
  // launch -- a second launch costs more than it saves there (per-shape A/B,
  // profiles/r04_wgrad_reduce_ab.txt); fewer: slices to fill the chip
  if (blocks >= 64) return 1;
  int sl = (int)mde::cdiv(512, blocks);
  const int cap = g / 16 > 1 ? g / 16 : 1;
  return sl < 1 ? 1 : (sl > cap ? cap : sl);
}

inline int launch_reduce(const float* part, float* gw, int groups, int g, int m,
                         const ReduceMap& map, hipStream_t s) {
  if (m % 4) {
    MDE_LAUNCH(mde::K_C3_WREDUCE, 4.0 * groups * (double)g * m + 4.0 * groups * m, s,
               wgrad_reduce_kernel, dim3((unsigned)mde::cdiv(m, 64), groups),
               dim3(64 * kRedWaves), 0, part, gw, g, m, map);
    return MDE_OK;
  }
  float* pw = const_cast<float*>(part);  // slice sums are written over consumed partial rows
  const int sl = reduce_slices(groups, g, m);
  const unsigned cx = (unsigned)mde::cdiv(m, 256);
  const int64_t gs = (int64_t)g * m;
  if (sl <= 1) {
    MDE_LAUNCH(mde::K_C3_WREDUCE, 4.0 * groups * (double)g * m + 4.0 * groups * m, s,
               wgrad_reduce4_kernel<true>, dim3(cx, groups, 1), dim3(64 * kRed4Waves), 0, pw, gw,
               g, m, (int64_t)m, gs, g, map);
    return MDE_OK;
  }
  const int rows = (int)mde::cdiv(g, sl);  // rows a slice
  const int ns = (int)mde::cdiv(g, rows);  // slices actually used
  MDE_LAUNCH(mde::K_C3_WREDUCE, 4.0 * groups * (double)(g + ns) * m, s,
             wgrad_reduce4_kernel<false>, dim3(cx, groups, ns), dim3(64 * kRed4Waves), 0, pw, gw,
             g, m, (int64_t)m, gs, rows, map);
  MDE_LAUNCH(mde::K_C3_WREDUCE, 4.0 * groups * (double)ns * m + 4.0 * groups * m, s,
             wgrad_reduce4_kernel<true>, dim3(cx, groups, 1), dim3(64 * kRed4Waves), 0, pw, gw,
             ns, m, (int64_t)rows * m, gs, ns, map);
  return MDE_OK;
}

// ------------------------------------------- wide-channel weight gradient
// DDRNet's 64 / 128 / 256-channel 3x3 / stride-1 convs (the BasicBlocks of
// src/GuideDepth/model/DDRNet_23_slim.py:41-72, at cfg2 60x80, 30x40, 15x20),
// whose weight gradient MIOpen runs as NHWC implicit GEMM behind
// NCHW <-> NHWC transposes.  Here in NCHW, no transposes:
//   gW[co][ci][tap] = sum over pixels p of gy[co][p] * x[ci][p + tap offset].
// Block groups (blockIdx.y) own 64 output x 32 input channels; a group's
// blocks (blockIdx.x) split the pixel tiles (split-K) -- a tile is `th` rows
// x `wc` columns (K = th * wc <= 192 pixels).  x rows r0-1 .. r0+th are staged
// with a zero border at pitch wc + 2, so tap (dy, dx) of pixel p is the
// constant offset dy * (wc + 2) + dx from p's base address (a per-tile
// pixel -> base table in LDS); gy rows r0 .. r0+th-1 are staged at pitch K.
// MFMA (v_mfma_f32_16x16x4_f32): M = output channels (wave w: the 16-channel
// tile w), N = (tap, input channel) = 18 tiles of 16, K = 4 pixels per step:
// per step a lane reads its pixel base, one gy value and 18 x values
// (conflict-free: both plane pitches = 2 mod 32) for 18 MFMAs.  The next
// tile's operands are loaded into registers while the current one is
// multiplied.  Block partials -> fixed-order two-stage reduction.
constexpr int kWCI = 32, kWCO = 64;
constexpr int kWNT = 9 * kWCI / 16;      // 18 N tiles: nt = 2 * tap + channel half
constexpr int kWPX = 386;                // x plane pitch: >= (th + 2)(wc + 2), = 2 mod 32
constexpr int kWPG = 194;                // gy plane pitch: >= K rounded to 4, = 2 mod 32
constexpr int kWK = 192;                 // pixels per tile, at most
constexpr int kWXL = (kWPX + 63) / 64;   // x loads per channel and lane (7)
constexpr int kWGL = kWK / 64;           // gy loads per channel and lane (3)
constexpr int kWM = kWCO * 9 * kWCI;     // partial elements per group: [co 64][tap 9][ci 32]

struct WideGeo {
  int th, wc, tiles_w, tiles_per_img, ntiles;
};

// th x wc tiles: whole rows when w <= 126, else 64-column strips
inline bool wide_geo(int64_t n, int64_t h, int64_t w, WideGeo* g) {
  const int wc = w <= 126 ? (int)w : 64;
  int th = kWK / wc;
  const int thx = kWPX / (wc + 2) - 2;
  if (thx < th) th = thx;
  if (th > (int)h) th = (int)h;
  if (th < 1) return false;
  g->th = th;
  g->wc = wc;
  g->tiles_w = (int)mde::cdiv(w, wc);
  const int64_t tpi = mde::cdiv(h, th) * g->tiles_w;
  const int64_t nt = n * tpi;
  if (tpi > 0x7fffffff || nt > 0x7fffffff) return false;
  g->tiles_per_img = (int)tpi;
  g->ntiles = (int)nt;
  return true;
}

__global__ void __launch_bounds__(256, 1)
    conv3x3_wgrad_wide_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                              float* __restrict__ part, int ci_n, int co_n, int h, int w,
                              WideGeo g) {
  __shared__ float sx[kWCI * kWPX];
  __shared__ float sg[kWCO * kWPG];
  __shared__ int tab[kWK];
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, lk = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ngo = co_n / kWCO;
  const int cog = blockIdx.y % ngo, cig = blockIdx.y / ngo;
  const int wc = g.wc, th = g.th, W2 = wc + 2, K = th * wc, KP = (K + 3) & ~3;
  const int XE = (th + 2) * W2;
  const int hw = h * w;
  for (int p = tid; p < KP; p += 256) tab[p] = p < K ? (p / wc) * W2 + p % wc : 0;
  for (int e = tid; e < kWCO * (KP - K); e += 256) {
    const int c = e / (KP - K);
    sg[c * kWPG + K + e % (KP - K)] = 0.f;  // K padding: gy = 0 (never rewritten)
  }
  // tile-invariant staging geometry of this lane: x element e = lane + 64 i of
  // a channel's staged plane is tile row rr, staged column cc (image column
  // c0 + cc - 1); gy element p = lane + 64 i is tile row p / wc, column p % wc
  int xrr[kWXL], xcc[kWXL];
#pragma unroll
  for (int i = 0; i < kWXL; ++i) {
    const int e = lane + 64 * i;
    const int rr = e / W2, cc = e - rr * W2;
    xrr[i] = e < XE ? rr : -4096;  // out of the plane: never in range
    xcc[i] = cc;
  }
  int gcol[kWGL], grow[kWGL];
#pragma unroll
  for (int i = 0; i < kWGL; ++i) {
    const int p = lane + 64 * i;
    grow[i] = p < K ? p / wc : -4096;
    gcol[i] = p % wc;
  }
  int boff[kWNT];
#pragma unroll
  for (int nt = 0; nt < kWNT; ++nt) {
    const int tap = nt >> 1;
    boff[nt] = (16 * (nt & 1) + li) * kWPX + (tap / 3) * W2 + tap % 3;
  }
  const int aoff = (16 * wv + li) * kWPG + lk;

  f4 acc[kWNT];
#pragma unroll
  for (int nt = 0; nt < kWNT; ++nt) acc[nt] = f4{0.f, 0.f, 0.f, 0.f};

  // this wave stages x channels 8 wv .. 8 wv + 7 and gy channels 16 wv .. 16 wv + 15
  const float* xg = x + ((int64_t)cig * kWCI + 8 * wv) * hw;
  const float* gg = gy + ((int64_t)cog * kWCO + 16 * wv) * hw;
  // in-range flags are applied at store time, so nothing waits on a load
  // before the next tile's LDS stores
  float vx[8][kWXL], vg[16][kWGL];
  unsigned xm = 0, gm = 0;
  auto load = [&](int tile) {
    const int img = tile / g.tiles_per_img, t = tile - img * g.tiles_per_img;
    const int r0 = (t / g.tiles_w) * th, c0 = (t % g.tiles_w) * wc;
    const float* xi = xg + (int64_t)img * ci_n * hw;
    const float* gi = gg + (int64_t)img * co_n * hw;
    // clamped coordinates: every load is a real element at a per-lane
    // address (a select of a uniform fallback address makes the compiler
    // split each load into a vector and a scalar branch)
    xm = 0;
#pragma unroll
    for (int i = 0; i < kWXL; ++i) {
      const int gr = r0 - 1 + xrr[i], gc = c0 - 1 + xcc[i];
      const bool ok = gr >= 0 && gr < h && gc >= 0 && gc < w;  // a strip's halo columns are real
      xm |= ok ? 1u << i : 0u;
      const int o = clampi(gr, 0, h - 1) * w + clampi(gc, 0, w - 1);
#pragma unroll
      for (int c = 0; c < 8; ++c) vx[c][i] = xi[(unsigned)(c * hw + o)];
    }
    gm = 0;
#pragma unroll
    for (int i = 0; i < kWGL; ++i) {
      const bool ok = grow[i] >= 0 && r0 + grow[i] < h && c0 + gcol[i] < w;
      gm |= ok ? 1u << i : 0u;
      const int o = clampi(r0 + grow[i], 0, h - 1) * w + clampi(c0 + gcol[i], 0, w - 1);
#pragma unroll
      for (int c = 0; c < 16; ++c) vg[c][i] = gi[(unsigned)(c * hw + o)];
    }
  };
  // XCD-aware walk (tile_walk): the tiles above / below a tile (whose rows
  // its halo re-reads) and the other channel groups of the same strip
  // (blockIdx.y, same blockIdx.x % 8 -> same XCD) go through one L2
  const TileWalk tw = tile_walk(g.ntiles);
  int tile = tw.t0;
  if (tile < tw.end) load(tile);
  for (; tile < tw.end; tile += tw.step) {
    __syncthreads();  // the previous tile's operands are consumed
#pragma unroll
    for (int i = 0; i < kWXL; ++i) {
      const int e = lane + 64 * i;
      if (e < XE) {
#pragma unroll
        for (int c = 0; c < 8; ++c) sx[(8 * wv + c) * kWPX + e] = (xm >> i) & 1u ? vx[c][i] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < kWGL; ++i) {
      const int p = lane + 64 * i;
      if (p < K) {
#pragma unroll
        for (int c = 0; c < 16; ++c) sg[(16 * wv + c) * kWPG + p] = (gm >> i) & 1u ? vg[c][i] : 0.f;
      }
    }
    __syncthreads();
    if (tile + tw.step < tw.end) load(tile + tw.step);
#pragma unroll 2
    for (int s = 0; s < KP / 4; ++s) {
      const int t = tab[4 * s + lk];
      const float a = sg[aoff + 4 * s];
#pragma unroll
      for (int nt = 0; nt < kWNT; ++nt) acc[nt] = mfma4(a, sx[boff[nt] + t], acc[nt]);
    }
  }
  // lane: co = 16 wv + 4 lk + i, n = 16 nt + li = 32 tap + ci
  float* out = part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * kWM;
#pragma unroll
  for (int nt = 0; nt < kWNT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(16 * wv + 4 * lk + i) * (9 * kWCI) + 16 * nt + li] = acc[nt][i];
}

// Fixed-strip variant (output width a multiple of SW, SW % 4 == 0; tiles of
// TH output rows x SW output columns): a K step's four pixels never straddle a
// row, so with the K loop fully unrolled every operand address is a per-lane
// base plus a compile-time offset (no pixel table, no address arithmetic),
// and the LDS is sized to the tile (<= 80 KB) so that two blocks share a CU.
// A strip's halo columns are the neighbouring strips' pixels (zero only at
// the image edge).  Same partial layout as the generic kernel.
// S = 2 (DDRNet's stride-2 3x3 convs, DDRNet_23_slim.py:41-72 with stride 2,
// down3 / down4 :254-265): the 2 TH + 1 input rows under a tile are staged
// split by column parity like the stem kernel's, O[j] = x[2(c0+j) - 1]
// (j = 0..SW) then E[j] = x[2(c0+j)] (j = 0..SW-1), so the column taps of
// output pixel p read O[p], E[p], O[p + 1] -- unit stride, as at S = 1.
template <int S, int SW, int TH, int COG = kWCO>
struct WideT {
  static constexpr int W2 = S == 1 ? SW + 2 : 2 * SW + 2;   // staged row pitch
  static constexpr int XROWS = S == 1 ? TH + 2 : 2 * TH + 1;
  static constexpr int K = TH * SW, XE = XROWS * W2;
  static constexpr int PX = (XE - 2 + 31) / 32 * 32 + 2;  // >= XE, = 2 mod 32
  static constexpr int PG = (K - 2 + 31) / 32 * 32 + 2;   // >= K, = 2 mod 32
  static constexpr int XL = (XE + 63) / 64, GL = (K + 63) / 64;
  static constexpr int SX = kWCI * PX, SMEM = SX + COG * PG;
  static constexpr int M = COG * 9 * kWCI;  // partial elements per group
  static_assert(SW % 4 == 0 && SMEM * 4 <= 80 * 1024, "two blocks per CU");
  // staged column of column tap dx for output column 0 of the row
  __device__ static constexpr int dxoff(int dx) {
    return S == 1 ? dx : (dx == 0 ? 0 : (dx == 1 ? SW + 1 : 1));
  }
  // input column (relative to S * c0) of staged column cc, or a value that is
  // never in range (the S = 2 row's pad column)
  __device__ static constexpr int incol(int cc) {
    return S == 1 ? cc - 1 : (cc <= SW ? 2 * cc - 1 : (cc <= 2 * SW ? 2 * (cc - SW - 1) : -(1 << 28)));
  }
};

// WPB waves per block: 4 (wave w = output-channel tile w x all 18 N tiles)
// or 8 (wave w = output-channel tile w & 3 x the 9 N tiles of input-channel
// half w >> 2: half the accumulators and staging registers per wave, so four
// waves per SIMD fit; measured 134.7 vs 140.4 us at 64->64 32x60x80).
// h, w: input sizes; ho, wo: gy sizes (= h, w at S = 1).
// COG = 32 (the 32 -> 32 convs, WPB = 4): wave w = output-channel tile
// w & 1 x the 9 N tiles of input-channel half w >> 1.
// PADC: ci_n not a multiple of 32 (the NewCRF projections' 24 / 40 / 112
// input channels, newcrf_layers.py:384-392): the last group's channels past
// ci_n are staged as zeros (never loaded) and their rows dropped by the
// reduction (gw_index).
template <int S, int SW, int TH, int WPB, int COG = kWCO, bool PADC = false>
__global__ void __launch_bounds__(64 * WPB, COG == kWCO ? 2 : 3)
    conv3x3_wgrad_wide_fixed_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                                    float* __restrict__ part, int ci_n, int co_n, int h, int w,
                                    int ho, int wo, int tiles_w, int tiles_per_img, int ntiles) {
  using P = WideT<S, SW, TH, COG>;
  static_assert(WPB == 4 || WPB == 8, "waves per block");
  static_assert(COG == kWCO || (COG == 32 && WPB == 4), "32-channel groups: 4 waves");
  constexpr int MTS = COG / 16;                    // output-channel tiles
  constexpr int NTW = MTS * kWNT / WPB;             // N tiles per wave
  constexpr int XC = kWCI / WPB, GC = COG / WPB;   // channels staged per wave
  __shared__ float sm[P::SMEM];
  float* sx = sm;
  float* sg = sm + P::SX;
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, lk = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  // this wave's output-channel tile and (when NTW == 9) input-channel half
  const int cot = NTW == kWNT ? wv : wv % MTS, hsel = NTW == kWNT ? 0 : wv / MTS;
  const int ngo = co_n / COG;
  const int cog = blockIdx.y % ngo, cig = blockIdx.y / ngo;
  const int hw = h * w, hwo = ho * wo;
  // staged element e = lane + 64 i of a channel's plane: input row S r0 - 1 +
  // xrr, input column S c0 + xcc; gy element p: tile row gpr, column gpc
  int xcc[P::XL], xrr[P::XL], gpr[P::GL], gpc[P::GL];
#pragma unroll
  for (int i = 0; i < P::XL; ++i) {
    const int e = lane + 64 * i;
    const int rr = e / P::W2;
    xrr[i] = e < P::XE ? rr : -4096;
    xcc[i] = P::incol(e - rr * P::W2);
  }
#pragma unroll
  for (int i = 0; i < P::GL; ++i) {
    const int p = lane + 64 * i < P::K ? lane + 64 * i : P::K - 1;
    gpr[i] = p / SW;
    gpc[i] = p % SW;
  }
  f4 acc[NTW];
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt) acc[nt] = f4{0.f, 0.f, 0.f, 0.f};
  const float* xg = x + ((int64_t)cig * kWCI + XC * wv) * hw;
  const float* gg = gy + ((int64_t)cog * COG + GC * wv) * hwo;
  const int cval = ci_n - (cig * kWCI + XC * wv);  // this wave's real staged channels (PADC)
  float vx[XC][P::XL], vg[GC][P::GL];
  unsigned xm = 0, gm = 0;
  auto load = [&](int tile) {
    const int img = tile / tiles_per_img, t = tile - img * tiles_per_img;
    const int r0 = (t / tiles_w) * TH, c0 = (t % tiles_w) * SW;
    const float* xi = xg + (int64_t)img * ci_n * hw;
    const float* gi = gg + (int64_t)img * co_n * hwo;
    // clamped coordinates (see the generic kernel): no uniform fallback address
    xm = 0;
#pragma unroll
    for (int i = 0; i < P::XL; ++i) {
      const int gr = S * r0 - 1 + xrr[i], gc = S * c0 + xcc[i];
      const bool ok = gr >= 0 && gr < h && gc >= 0 && gc < w;
      xm |= ok ? 1u << i : 0u;
      const int o = clampi(gr, 0, h - 1) * w + clampi(gc, 0, w - 1);
#pragma unroll
      for (int c = 0; c < XC; ++c)
        vx[c][i] = !PADC || c < cval ? xi[(unsigned)(c * hw + o)] : 0.f;
    }
    gm = 0;
#pragma unroll
    for (int i = 0; i < P::GL; ++i) {
      const int p = lane + 64 * i;
      const bool ok = p < P::K && r0 + p / SW < ho;
      gm |= ok ? 1u << i : 0u;
      const int o = clampi(r0 + gpr[i], 0, ho - 1) * wo + c0 + gpc[i];
#pragma unroll
      for (int c = 0; c < GC; ++c) vg[c][i] = gi[(unsigned)(c * hwo + o)];
    }
  };
  // XCD-aware walk (tile_walk): with gridDim.x % 8 == 0 every channel group
  // (blockIdx.y) of a strip and the strips above / below it (the halo rows)
  // are staged through the same XCD's L2
  const TileWalk tw = tile_walk(ntiles);
  int tile = tw.t0;
  if (tile < tw.end) load(tile);
  for (; tile < tw.end; tile += tw.step) {
    __syncthreads();  // the previous tile's operands are consumed
#pragma unroll
    for (int i = 0; i < P::XL; ++i) {
      const int e = lane + 64 * i;
      if (e < P::XE) {
#pragma unroll
        for (int c = 0; c < XC; ++c) sx[(XC * wv + c) * P::PX + e] = (xm >> i) & 1u ? vx[c][i] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < P::GL; ++i) {
      const int p = lane + 64 * i;
      if (p < P::K) {
#pragma unroll
        for (int c = 0; c < GC; ++c) sg[(GC * wv + c) * P::PG + p] = (gm >> i) & 1u ? vg[c][i] : 0.f;
      }
    }
    __syncthreads();
    if (tile + tw.step < tw.end) load(tile + tw.step);
    const float* xb = sx + (16 * hsel + li) * P::PX + lk;
    const float* gb = sg + (16 * cot + li) * P::PG + lk;
#pragma unroll 5
    for (int st = 0; st < P::K / 4; ++st) {
      // the step's first pixel: output row 4 st / SW -> staged row S x that
      const int so = S * (4 * st / SW) * P::W2 + (4 * st) % SW;
      const float a = gb[4 * st];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int tap = NTW == kWNT ? nt >> 1 : nt, half = NTW == kWNT ? nt & 1 : 0;
        acc[nt] = mfma4(a, xb[half * 16 * P::PX + (tap / 3) * P::W2 + P::dxoff(tap % 3) + so],
                        acc[nt]);
      }
    }
  }
  // lane: co = 16 cot + 4 lk + i, n = 32 tap + 16 half + li
  float* out = part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * P::M;
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt) {
    const int col = NTW == kWNT ? 16 * nt + li : 16 * (2 * nt + hsel) + li;
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(16 * cot + 4 * lk + i) * (9 * kWCI) + col] = acc[nt][i];
  }
}

// Fixed-strip geometry: (strip width, tile rows) with K = 80 pixels (K = 160
// spills at four waves per SIMD), or 0.
inline int wide_fixed_sw(int64_t w) {
  return w % 80 == 0 ? 80 : (w == 40 ? 40 : (w == 20 ? 20 : 0));
}

// Blocks of the fixed-strip wide weight gradients over all groups.  Each
// block leaves one 64 x 288 partial, so the slab (its HBM write and the
// reduction's read) scales with this: one 8-wave block per CU (256) for the
// 1/8- and smaller-resolution planes -- half the slab and PMC traffic 1.35x ->
// ~1.0x on the fetch side at equal time -- two per CU (512) for planes with
// >= 4096 strip tiles (64 -> 64 at 120 x 160: 385 vs 417 us), where the slab
// is small next to the inputs (profiles/r04_wide_blocks_ab.txt).
// >= 64 channel groups (NewCRF's 256 -> 512, 160 / 512 -> 1024 projections at
// 30 x 40 / 15 x 20: one to four blocks a group at 256): 768 blocks, three a
// CU in flight -- wide wgrad 2.485 -> 2.415 ms a cfg4 step for +0.01 ms of
// reduction (`gpurun_out/r06al`); DDRNet's <= 32 groups keep the rule above
// (768 for every shape: cfg4 wgrad 2.31 ms but cfg2's reduction +0.14 ms,
// cfg2 -0.4 %, `gpurun_out/r06ak`).
// MDE_WIDE_BLOCKS overrides (A/B).
inline int wide_blocks(int64_t ntiles, int groups) {
  static const int forced = [] {
    const char* e = std::getenv("MDE_WIDE_BLOCKS");
    const int v = e ? std::atoi(e) : 0;
    return v >= 8 ? v : 0;
  }();
  if (forced) return forced;
  if (groups >= 64) return 768;
  return ntiles >= 4096 ? 512 : 256;
}

struct WidePlan {
  WideGeo g;
  int groups, gx;
  int fixed_sw;  // > 0: the fixed-strip kernel (tiles of 80 / fixed_sw rows x fixed_sw columns)
};

inline bool wide_plan(int64_t n, int64_t ci, int64_t co, int64_t h, int64_t w, WidePlan* p) {
  if (co % kWCO || co < kWCO || ci < 16 || (ci % kWCI && ci % 8)) return false;
  if (!wide_geo(n, h, w, &p->g)) return false;
  p->fixed_sw = wide_fixed_sw(w);
  if (ci % kWCI && !p->fixed_sw) return false;  // padded channels: the fixed-strip kernel only
  if (p->fixed_sw) {  // tiles of 80 / fixed_sw rows x fixed_sw columns
    const int th = 80 / p->fixed_sw, tw = (int)(w / p->fixed_sw);
    const int64_t tpi = mde::cdiv(h, th) * tw, nt = n * tpi;
    if (nt > 0x7fffffff) return false;
    p->g.th = th;
    p->g.wc = p->fixed_sw;
    p->g.tiles_w = tw;
    p->g.tiles_per_img = (int)tpi;
    p->g.ntiles = (int)nt;
  }
  p->groups = (int)(mde::cdiv(ci, kWCI) * (co / kWCO));
  // one 100 KB-LDS block per CU (generic), two <= 80 KB blocks (fixed width)
  int gx = (p->fixed_sw ? wide_blocks(p->g.ntiles, p->groups) : 256) / p->groups;
  if (gx < 1) gx = 1;
  if (gx > p->g.ntiles) gx = p->g.ntiles;
  p->gx = gx;
  return true;
}

inline size_t wide_workspace(const WidePlan& p) {
  return wgrad_ws_bytes(p.groups, p.gx, kWM);
}

int launch_wgrad_wide(const float* x, const float* gy, float* gw, int64_t n, int64_t ci,
                      int64_t co, int64_t h, int64_t w, float* ws, hipStream_t s) {
  WidePlan p;
  if (!wide_plan(n, ci, co, h, w, &p)) return MDE_ERR_UNSUPPORTED;
  const double flops = 2.0 * 9 * ci * co * (double)(n * h * w);
  const double bytes = 4.0 * n * h * w * (double)(ci + co);
  const dim3 grid(p.gx, p.groups);
  const int tpi = p.g.tiles_per_img, nt = p.g.ntiles, tw = p.g.tiles_w;
  // MDE_WIDE_WPB=4 selects the 4-wave layout (A/B measurement only)
  static const int wpb = [] {
    const char* e = std::getenv("MDE_WIDE_WPB");
    return e ? std::atoi(e) : 8;
  }();
  const bool padc = ci % kWCI != 0;
#define MDE_WIDE_FIXED(WW, TT)                                                                  \
  do {                                                                                          \
    if (padc)                                                                                   \
      MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_WIDE, bytes, flops, s,                                    \
                      (conv3x3_wgrad_wide_fixed_kernel<1, WW, TT, 8, kWCO, true>), grid,        \
                      dim3(512), 0, x, gy, ws, (int)ci, (int)co, (int)h, (int)w, (int)h,        \
                      (int)w, tw, tpi, nt);                                                     \
    else if (wpb == 4)                                                                          \
      MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_WIDE, bytes, flops, s,                                         \
                      (conv3x3_wgrad_wide_fixed_kernel<1, WW, TT, 4>), grid, dim3(256), 0, x,   \
                      gy, ws, (int)ci, (int)co, (int)h, (int)w, (int)h, (int)w, tw, tpi, nt);   \
    else                                                                                        \
      MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_WIDE, bytes, flops, s,                                         \
                      (conv3x3_wgrad_wide_fixed_kernel<1, WW, TT, 8>), grid, dim3(512), 0, x,   \
                      gy, ws, (int)ci, (int)co, (int)h, (int)w, (int)h, (int)w, tw, tpi, nt);   \
  } while (0)
  if (p.fixed_sw == 80)
    MDE_WIDE_FIXED(80, 1);
  else if (p.fixed_sw == 40)
    MDE_WIDE_FIXED(40, 2);
  else if (p.fixed_sw == 20)
    MDE_WIDE_FIXED(20, 4);
  else
    MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_WIDE, bytes, flops, s, conv3x3_wgrad_wide_kernel, grid,
                    dim3(256), 0, x, gy, ws, (int)ci, (int)co, (int)h, (int)w, p.g);
#undef MDE_WIDE_FIXED
  return launch_reduce(ws, gw, p.groups, p.gx, kWM, ReduceMap{kWCO, 0, 0, (int)ci, (int)co}, s);
}

// 32 -> 32 at widths that are multiples of 80 (DDRNet's layer1 BasicBlocks at
// 120x160, the decoder's 32-channel convs at 240x320) on the fixed-strip kernel
// with 32-channel output groups (4 waves, three blocks per CU).
// MDE_C32_WIDE=0: the regular 32 -> 32 weight-gradient kernel (A/B).
inline bool c32_wide(int64_t w) {
  static const bool on = [] {
    const char* e = std::getenv("MDE_C32_WIDE");
    return !(e && e[0] == '0');
  }();
  return on && w % 80 == 0;
}

inline WidePlan c32_plan(int64_t n, int64_t h, int64_t w) {
  WidePlan p;
  const int tw = (int)(w / 80);
  const int64_t nt = n * h * tw;
  p.fixed_sw = 80;
  p.g.th = 1;
  p.g.wc = 80;
  p.g.tiles_w = tw;
  p.g.tiles_per_img = (int)(h * tw);
  p.g.ntiles = nt > 0x7fffffff ? 0x7fffffff : (int)nt;
  p.groups = 1;
  const int res = resident_blocks<conv3x3_wgrad_wide_fixed_kernel<1, 80, 1, 4, 32>>();
  p.gx = p.g.ntiles < res ? p.g.ntiles : res;
  return p;
}

int launch_wgrad_c32(const float* x, const float* gy, float* gw, int64_t n, int64_t h, int64_t w,
                     float* ws, hipStream_t s) {
  const WidePlan p = c32_plan(n, h, w);
  if (p.gx <= 0) return MDE_ERR_INVALID_ARG;
  constexpr int M = WideT<1, 80, 1, 32>::M;
  const double flops = 2.0 * 9 * 32 * 32 * (double)(n * h * w);
  const double bytes = 4.0 * n * h * w * 64.0;
  MDE_LAUNCH_MFMA(mde::K_C3_WGRAD, bytes, flops, s, (conv3x3_wgrad_wide_fixed_kernel<1, 80, 1, 4, 32>),
                  dim3(p.gx, 1), dim3(256), 0, x, gy, ws, 32, 32, (int)h, (int)w, (int)h, (int)w,
                  p.g.tiles_w, p.g.tiles_per_img, p.g.ntiles);
  return launch_reduce(ws, gw, 1, p.gx, M, ReduceMap{32, 0, 0, 32, 32}, s);
}

// The stem's 32 -> 32 stride-2 weight gradient on the same kernel (S = 2,
// 40-column strips, 32-channel output groups) when the output width is a
// multiple of 40; MDE_C32_WIDE=0 keeps the stem kernel (A/B).
int launch_wgrad_c32_s2(const float* x, const float* gy, float* gw, int64_t n, int64_t h,
                        int64_t w, float* ws, hipStream_t s) {
  const int ho = (int)((h - 1) / 2 + 1), wo = (int)((w - 1) / 2 + 1);
  const int tw = wo / 40, tpi = (int)mde::cdiv(ho, 2) * tw;
  const int64_t nt64 = n * (int64_t)tpi;
  if (nt64 > 0x7fffffff) return MDE_ERR_INVALID_ARG;
  const int nt = (int)nt64;
  const int res = resident_blocks<conv3x3_wgrad_wide_fixed_kernel<2, 40, 2, 4, 32>>();
  const int gx = nt < res ? nt : res;
  constexpr int M = WideT<2, 40, 2, 32>::M;
  const double flops = 2.0 * 9 * 32 * 32 * (double)n * ho * wo;
  const double bytes = 4.0 * n * (32.0 * h * w + 32.0 * ho * wo);
  MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_S2, bytes, flops, s,
                  (conv3x3_wgrad_wide_fixed_kernel<2, 40, 2, 4, 32>), dim3(gx, 1), dim3(256), 0, x,
                  gy, ws, 32, 32, (int)h, (int)w, ho, wo, tw, tpi, nt);
  return launch_reduce(ws, gw, 1, gx, M, ReduceMap{32, 0, 0, 32, 32}, s);
}

inline size_t c32_s2_workspace(int64_t n, int64_t h, int64_t w) {
  const int ho = (int)((h - 1) / 2 + 1), wo = (int)((w - 1) / 2 + 1);
  const int64_t nt = n * mde::cdiv(ho, 2) * (wo / 40);
  const int res = resident_blocks<conv3x3_wgrad_wide_fixed_kernel<2, 40, 2, 4, 32>>();
  const int gx = (int)(nt < res ? nt : res);
  return wgrad_ws_bytes(1, gx, WideT<2, 40, 2, 32>::M);
}

inline bool c32_s2(int64_t cin, int64_t cout, int64_t w) {
  const int64_t wo = (w - 1) / 2 + 1;
  return cin == 32 && cout == 32 && wo % 40 == 0 && c32_wide(80);
}

// Stride-2 wide weight gradient (fixed strips only: output width a multiple
// of 40, or 20; input width even).  h, w: input sizes.
inline int wide_s2_sw(int64_t wo) { return wo % 40 == 0 ? 40 : (wo == 20 ? 20 : 0); }

inline bool wide_s2_plan(int64_t n, int64_t ci, int64_t co, int64_t h, int64_t w, WidePlan* p) {
  if (ci % kWCI || co % kWCO || ci < kWCI || co < kWCO || w % 2) return false;
  const int64_t ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const int sw = wide_s2_sw(wo);
  if (!sw) return false;
  const int th = 80 / sw, tw = (int)(wo / sw);
  const int64_t tpi = mde::cdiv(ho, th) * tw, nt = n * tpi;
  if (nt > 0x7fffffff) return false;
  p->fixed_sw = sw;
  p->g.th = th;
  p->g.wc = sw;
  p->g.tiles_w = tw;
  p->g.tiles_per_img = (int)tpi;
  p->g.ntiles = (int)nt;
  p->groups = (int)((ci / kWCI) * (co / kWCO));
  int gx = wide_blocks(nt, p->groups) / p->groups;
  if (gx < 1) gx = 1;
  if (gx > p->g.ntiles) gx = p->g.ntiles;
  p->gx = gx;
  return true;
}

int launch_wgrad_wide_s2(const float* x, const float* gy, float* gw, int64_t n, int64_t ci,
                         int64_t co, int64_t h, int64_t w, float* ws, hipStream_t s) {
  WidePlan p;
  if (!wide_s2_plan(n, ci, co, h, w, &p)) return MDE_ERR_UNSUPPORTED;
  const int ho = (int)((h - 1) / 2 + 1), wo = (int)((w - 1) / 2 + 1);
  const double flops = 2.0 * 9 * ci * co * (double)n * ho * wo;
  const double bytes = 4.0 * n * ((double)ci * h * w + (double)co * ho * wo);
  const dim3 grid(p.gx, p.groups);
  const int tpi = p.g.tiles_per_img, nt = p.g.ntiles, tw = p.g.tiles_w;
  if (p.fixed_sw == 40)
    MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_S2, bytes, flops, s,
                    (conv3x3_wgrad_wide_fixed_kernel<2, 40, 2, 8>), grid, dim3(512), 0, x, gy, ws,
                    (int)ci, (int)co, (int)h, (int)w, ho, wo, tw, tpi, nt);
  else
    MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_S2, bytes, flops, s,
                    (conv3x3_wgrad_wide_fixed_kernel<2, 20, 4, 8>), grid, dim3(512), 0, x, gy, ws,
                    (int)ci, (int)co, (int)h, (int)w, ho, wo, tw, tpi, nt);
  return launch_reduce(ws, gw, p.groups, p.gx, kWM, ReduceMap{kWCO, 0, 0, (int)ci, (int)co}, s);
}

// ====================================================================== bf16
// bf16 activations / gradients on v_mfma_f32_16x16x32_bf16 (bf16 products,
// fp32 accumulation), for the autocast step (BASELINE cfg3): the same three
// passes as above at 16 -> 16 and 32 -> 32, without MIOpen's NCHW <-> NHWC
// transposes.  Weights stay fp32 in memory (autocast's master weights) and
// are rounded to bf16 (RNE, as autocast's cast) when a block loads them; the
// weight gradient is fp32.
//
// Staging (both kernels): the input tile (rows r0-1 .. r0+TH, the 64 tile
// columns) is stored as THREE column-shifted copies, copy d holding global
// columns c0 - 1 + d + t, t = 0..63, so every operand read of tap column d
// starts at an 8-/16-byte-aligned LDS address (an unaligned ds_read returns
// stale data or replays).  A lane loads one aligned 4-column chunk (8 B) of a
// tile row from HBM, takes its neighbours' chunks by DPP lane shifts and
// writes its 4 columns of each copy (3 ds_write_b64).  Plane (channel) pitch
// = 16 (mod 128) elements: conflict-free ds_read_b128 (weight gradient);
// the forward adds 64 elements between the two 8-channel halves, which makes
// its transposed reads (ds_read_b64_tr_b16) conflict-free.
//
// Forward / data gradient: M = 16 output pixels, N = 16 output channels,
// K = (tap, input channel) in steps of 32: one tap x 32 channels (CI = 32) or
// two taps x 16 channels (CI = 16; the tenth tap has zero weights).  The A
// operand (8 channels of one pixel per lane) comes from the channel-planar
// copies by two ds_read_b64_tr_b16 (4 channels x 16 pixels each); the B
// operand (weights) lives in registers.  Weight gradient: M = output
// channels, N = (tap, input channel), K = 32 pixels of a tile row; A = gy
// rows and B = x rows, 16 bytes per lane by ds_read_b128.
using mde::bf16;
using bf8v = __bf16 __attribute__((ext_vector_type(8)));
using f4v = float __attribute__((ext_vector_type(4)));
using s4v = short __attribute__((ext_vector_type(4)));
using u2v = uint32_t __attribute__((ext_vector_type(2)));
using u4v = uint32_t __attribute__((ext_vector_type(4)));
using lds_s4 = __attribute__((address_space(3))) s4v;

__device__ __forceinline__ f4v mfma_bf(u4v a, u4v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a),
                                                 __builtin_bit_cast(bf8v, b), c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t dpp_prev(uint32_t v) {  // lane - 1
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t dpp_next(uint32_t v) {  // lane + 1
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);
}

// Element layout of the shifted-copy tile: copy d, channel c, tile row r, col t.
template <int C, int XR, int GO>
struct CopyTile {
  static constexpr int PL = (XR * 64 + 127) / 128 * 128 + 16;   // plane pitch (elements)
  static constexpr int HALF = 8 * PL + GO;                       // 8-channel half pitch
  static constexpr int COPY = ((C + 7) / 8 * HALF + 127) / 128 * 128;
  static constexpr int ELEMS = 3 * COPY;
  __device__ static __forceinline__ int at(int d, int c, int r, int t) {
    return d * COPY + (c >> 3) * HALF + (c & 7) * PL + r * 64 + t;
  }
};

// Register stage of one tile: rows (channel, tile row) of 18 aligned 4-column
// chunks (global columns c0 - 4 + 4i, i = 0..17); three rows per wave
// instruction (lanes 0..53), the rows split over the block's 4 waves.
template <int C, int XR>
struct ChunkStage {
  static constexpr int ROWS = C * XR;
  static constexpr int PER = (ROWS + 11) / 12;  // 12 rows per block instruction
  u2v v[PER];
  __device__ __forceinline__ void load(const bf16* __restrict__ img, int h, int w, int r0,
                                       int c0, int lane, int wvu) {
    const int sub = lane / 18, i = lane - 18 * sub;  // row within the trio, chunk
    const int gc = c0 - 4 + 4 * i;
    const bool cok = lane < 54 && gc >= 0 && gc + 3 < w;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int row = 12 * k + 3 * wvu + sub;  // (channel, tile row) index
      const int c = row / XR, r = row - c * XR, gr = r0 - 1 + r;
      const bool ok = cok && row < ROWS && gr >= 0 && gr < h;
      const u2v t = *reinterpret_cast<const u2v*>(
          img + (ok ? (unsigned)((c * h + gr) * w + gc) : 0u));
      v[k] = ok ? t : u2v{0u, 0u};
    }
  }
  // copy d, tile columns 4j .. 4j+3 (j = i - 1) = global c0 - 1 + d + 4j .. :
  // d = 1 is chunk i itself; d = 0 the last element of chunk i - 1 and the
  // first three of chunk i; d = 2 the last three of chunk i and the first of
  // chunk i + 1 (neighbours by DPP lane shifts; all lanes execute them).
  template <int GO>
  __device__ __forceinline__ void store(bf16* sx, int lane, int wvu) const {
    using L = CopyTile<C, (ROWS / C), GO>;
    const int sub = lane / 18, i = lane - 18 * sub, j = i - 1;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t p1 = dpp_prev(v[k].y), n0 = dpp_next(v[k].x);
      const int row = 12 * k + 3 * wvu + sub;
      if (lane < 54 && j >= 0 && j < 16 && row < ROWS) {
        const int c = row / XR, r = row - c * XR;
        const u2v d1 = v[k];
        const u2v d0 = u2v{__builtin_amdgcn_alignbit(v[k].x, p1, 16),
                           __builtin_amdgcn_alignbit(v[k].y, v[k].x, 16)};
        const u2v d2 = u2v{__builtin_amdgcn_alignbit(v[k].y, v[k].x, 16),
                           __builtin_amdgcn_alignbit(n0, v[k].y, 16)};
        *reinterpret_cast<u2v*>(sx + L::at(0, c, r, 4 * j)) = d0;
        *reinterpret_cast<u2v*>(sx + L::at(1, c, r, 4 * j)) = d1;
        *reinterpret_cast<u2v*>(sx + L::at(2, c, r, 4 * j)) = d2;
      }
    }
  }
};

// fp32 weight -> bf16 (RNE) pair packed in a dword
__device__ __forceinline__ uint32_t pack_bf(float a, float b) {
  return (uint32_t)mde::f2bf(a) | ((uint32_t)mde::f2bf(b) << 16);
}

template <int CI, int CO, int RPW, bool FLIP, bool STATS>
__global__ void __launch_bounds__(256, 2)
    conv3x3_bf_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ wt,
                          bf16* __restrict__ y, int h, int w, int tiles_w, int tiles_per_img,
                          int ntiles, float* __restrict__ stats) {
  static_assert(CI == 16 || CI == 32, "bf16 forward: 16 or 32 input channels");
  static_assert(CO % 16 == 0, "output channels in 16-blocks");
  constexpr int TH = 4 * RPW, XR = TH + 2;
  constexpr int NB = CO / 16;
  constexpr int NS = CI == 16 ? 5 : 9;  // K steps of 32
  using L = CopyTile<CI, XR, 64>;
  __shared__ __attribute__((aligned(16))) bf16 sx[L::ELEMS];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int li = lane & 15, g = lane >> 4;
  const int64_t img_in = (int64_t)CI * h * w, img_out = (int64_t)CO * h * w;

  // B operands: lane (co = 16 nb + li, g) holds the 8 K values of step s:
  // K = 32 s + 8 g + j <-> (tap, channel) as the A reads below
  u4v wb[NS][NB];
#pragma unroll
  for (int st = 0; st < NS; ++st)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int co = 16 * nb + li;
      const int tap = CI == 32 ? st : 2 * st + (g >> 1);
      const int c8 = CI == 32 ? 8 * g : 8 * (g & 1);
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ci = c8 + j;
        const int src = FLIP ? (ci * CO + co) * 9 + (8 - tap) : (co * CI + ci) * 9 + tap;
        const float t = wt[tap < 9 ? src : 0];
        f[j] = tap < 9 ? t : 0.f;
      }
      wb[st][nb] = u4v{pack_bf(f[0], f[1]), pack_bf(f[2], f[3]), pack_bf(f[4], f[5]),
                       pack_bf(f[6], f[7])};
    }
  // A read addresses: lane 4q+p of group g supplies (channel c8g + q (+4),
  // tile row (row + dy), pixels 16m + 4p) of copy dx; per step s a constant
  // offset from the lane base.
  const int q = li >> 2, p = li & 3;
  int aoff[NS];
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int tap = CI == 32 ? st : (2 * st + (g >> 1) < 9 ? 2 * st + (g >> 1) : 8);
    const int c8 = CI == 32 ? 8 * g : 8 * (g & 1);
    aoff[st] = L::at(tap % 3, c8 + q, tap / 3, 4 * p);
  }

  mde::Sh run[STATS ? NB : 1];
#pragma unroll
  for (int nb = 0; nb < (STATS ? NB : 1); ++nb) run[nb] = {0.f, 0.f, 0.f, 0.f};
  bool first = true;
  ChunkStage<CI, XR> S;
  const TileWalk tw = tile_walk(ntiles);
  int tile = tw.t0;
  if (tile < tw.end) {
    const TileGeo gg = tile_geo(tile, TH, tiles_w, tiles_per_img);
    S.load(x + gg.img * img_in, h, w, gg.r0, gg.c0, lane, wvu);
  }
  for (; tile < tw.end; tile += tw.step) {
    const TileGeo gg = tile_geo(tile, TH, tiles_w, tiles_per_img);
    __syncthreads();
    S.template store<64>(sx, lane, wvu);
    __syncthreads();
    const int nxt = tile + tw.step;
    if (nxt < tw.end) {
      const TileGeo gn = tile_geo(nxt, TH, tiles_w, tiles_per_img);
      S.load(x + gn.img * img_in, h, w, gn.r0, gn.c0, lane, wvu);
    }
    f4v acc[RPW][4][NB];
#pragma unroll
    for (int qq = 0; qq < RPW; ++qq)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[qq][m][nb] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int qq = 0; qq < RPW; ++qq) {
      const int row = wv * RPW + qq;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int st = 0; st < NS; ++st) {
          const bf16* base = sx + aoff[st] + row * 64 + 16 * m;
          const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)base);
          const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + 4 * L::PL));
          const u2v l2 = __builtin_bit_cast(u2v, lo), h2 = __builtin_bit_cast(u2v, hi);
          const u4v a = u4v{l2.x, l2.y, h2.x, h2.y};
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) acc[qq][m][nb] = mfma_bf(a, wb[st][nb], acc[qq][m][nb]);
        }
      }
    }
    // D: lane holds pixels 16m + 4g + r (r = 0..3) of output channel 16nb + li
    bf16* yi = y + gg.img * img_out;
#pragma unroll
    for (int qq = 0; qq < RPW; ++qq) {
      const int row = gg.r0 + wv * RPW + qq;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int col = gg.c0 + 16 * m + 4 * g;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const f4v v = acc[qq][m][nb];
          const uint16_t b0 = mde::f2bf(v[0]), b1 = mde::f2bf(v[1]), b2 = mde::f2bf(v[2]),
                         b3 = mde::f2bf(v[3]);
          if constexpr (STATS) {
            if (first && qq == 0 && m == 0) {  // one shift per channel and wave
              const bool ok0 = gg.r0 + wv * RPW < h && gg.c0 < w;
              run[nb].ref = __shfl(ok0 ? mde::bf2f(b0) : 0.f, li, 64);
            }
            const bool rok = row < h;
            mde::sh_add(run[nb], mde::bf2f(b0), rok && col < w);
            mde::sh_add(run[nb], mde::bf2f(b1), rok && col + 1 < w);
            mde::sh_add(run[nb], mde::bf2f(b2), rok && col + 2 < w);
            mde::sh_add(run[nb], mde::bf2f(b3), rok && col + 3 < w);
          }
          if (row < h) {
            bf16* dst = yi + ((int64_t)(16 * nb + li) * h + row) * w + col;
            if (col + 3 < w) {
              *reinterpret_cast<u2v*>(dst) =
                  u2v{(uint32_t)b0 | ((uint32_t)b1 << 16), (uint32_t)b2 | ((uint32_t)b3 << 16)};
            } else {
              if (col < w) dst[0] = b0;
              if (col + 1 < w) dst[1] = b1;
              if (col + 2 < w) dst[2] = b2;
            }
          }
        }
      }
    }
    first = false;
  }
  if constexpr (STATS) {  // as the fp32 kernel: lk-butterfly, then the 4 waves in order
    __syncthreads();
    float* part = reinterpret_cast<float*>(sx);  // [4][CO][4]
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const mde::Sh a = mde::sh_xor_sum(mde::sh_xor_sum(run[nb], 16), 32);
      if (g == 0) {
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

// Row stage of the second bf16 forward (conv3x3_bf_fwd2_kernel): the tile's
// XR input rows x CI channels as (row, channel) lines, 16-byte buffer loads
// -- 8 lanes per 64-column line, 8 lines per wave instruction (line 32 k + 8
// wave + sub): every offset is a lane constant plus a uniform per-line one,
// past the buffer (zeros) for out-of-image rows and columns.  The halo
// columns c0 - 1 and c0 + 64 come from 2-byte loads by the 2 edge lanes of a
// line only (exec masked); the shifted copies take the neighbour columns by
// DPP row shifts.  (An 8-byte, 16-lanes-a-line stage with every lane loading
// a halo element kept the texture addresser ~75 % busy -- TA_TA_BUSY_sum /
// GRBM_GUI_ACTIVE -- at 207 us for the 16 -> 16 forward; this one: 194 us.)
template <int CI, int XR>
struct RowStage8 {
  static constexpr int K = XR * CI / 32;  // instructions per wave
  static_assert(XR * CI % 32 == 0, "whole instructions");
  u4v v[K];
  uint32_t hl[K];
  __device__ static __forceinline__ int line_r(int k, int wvu) {
    return CI == 32 ? k : 2 * k + (wvu >> 1);
  }
  __device__ static __forceinline__ int line_c(int wvu, int sub) {
    return CI == 32 ? 8 * wvu + sub : 8 * (wvu & 1) + sub;
  }
  __device__ __forceinline__ void load(const bf16* __restrict__ img, int h, int w, int r0, int c0,
                                       int lane, int wvu) {
    const int sub = lane >> 3, i = lane & 7;
    const int c = line_c(wvu, sub);
    const int hw = h * w;
    const int gc = c0 + 8 * i;
    // w % 4 == 0: an 8-column chunk is all in, all out, or (last 4 columns
    // out) read as 16 bytes whose second half lies past the row -- zeroed below
    const uint32_t vo = gc < w ? (uint32_t)(2 * (c * hw + gc)) : 0x7ffffff0u;
    const bool half = gc + 4 >= w;
    const int hc = i == 0 ? c0 - 1 : c0 + 64;
    const uint32_t vh = (unsigned)hc < (unsigned)w ? (uint32_t)(2 * (c * hw + hc)) : 0x7ffffff0u;
    const uint64_t a = (uint64_t)img;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, 2 * CI * hw, 0x00020000);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int gr = r0 - 1 + line_r(k, wvu);
      const int so = (unsigned)gr < (unsigned)h ? 2 * (gr * w) : 0x7ffffff0;
      u4v t = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(R, vo, so, 0));
      if (half) t = u4v{t[0], t[1], 0u, 0u};
      v[k] = t;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) hl[k] = 0u;
    if (i == 0 || i == 7) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int gr = r0 - 1 + line_r(k, wvu);
        const int so = (unsigned)gr < (unsigned)h ? 2 * (gr * w) : 0x7ffffff0;
        hl[k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(R, vh, so, 0);
      }
    }
  }
  template <int GO>
  __device__ __forceinline__ void store(bf16* sx, int lane, int wvu) const {
    using L = CopyTile<CI, XR, GO>;
    const int sub = lane >> 3, i = lane & 7;
    const int c = line_c(wvu, sub);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      // previous column (lane i - 1's last, or the left halo), next column
      // (lane i + 1's first, or the right halo); a 16-lane DPP row holds 2 lines
      const uint32_t pw = (uint32_t)__builtin_amdgcn_mov_dpp((int)v[k][3], 0x111, 0xf, 0xf, false);
      const uint32_t nx = (uint32_t)__builtin_amdgcn_mov_dpp((int)v[k][0], 0x101, 0xf, 0xf, false);
      const uint32_t p1 = i == 0 ? hl[k] << 16 : pw;
      const uint32_t n0 = i == 7 ? hl[k] : nx;
      const u4v d1 = v[k];
      const u4v d0 = u4v{__builtin_amdgcn_alignbit(v[k][0], p1, 16),
                         __builtin_amdgcn_alignbit(v[k][1], v[k][0], 16),
                         __builtin_amdgcn_alignbit(v[k][2], v[k][1], 16),
                         __builtin_amdgcn_alignbit(v[k][3], v[k][2], 16)};
      const u4v d2 = u4v{__builtin_amdgcn_alignbit(v[k][1], v[k][0], 16),
                         __builtin_amdgcn_alignbit(v[k][2], v[k][1], 16),
                         __builtin_amdgcn_alignbit(v[k][3], v[k][2], 16),
                         __builtin_amdgcn_alignbit(n0, v[k][3], 16)};
      const int r = line_r(k, wvu);
      *reinterpret_cast<u4v*>(sx + L::at(0, c, r, 8 * i)) = d0;
      *reinterpret_cast<u4v*>(sx + L::at(1, c, r, 8 * i)) = d1;
      *reinterpret_cast<u4v*>(sx + L::at(2, c, r, 8 * i)) = d2;
    }
  }
};

__device__ __forceinline__ uint32_t pk_bf(float a, float b) {
  using bf2v = __bf16 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, bf2v{(__bf16)a, (__bf16)b});
}

// The bf16 forward / data gradient of conv3x3_bf_fwd_kernel with (i) the row
// stage above instead of ChunkStage (linear addressing, no 18-chunk rows:
// the index arithmetic was ~60 % of the loop's VALU and SALU instructions,
// SQ_INSTS_VALU 15x SQ_INSTS_MFMA) and (ii) interior tiles stored through
// the hardware bf16 conversion without per-pixel bounds tests.  Same operand
// layouts, K order and summation order: bit-identical results.
// DEPTH: register stages (2 at 16 channels; the 32-channel kernel has no
// registers for a second).
template <int CI, int CO, int RPW, bool FLIP, bool STATS, int DEPTH = (CI == 16 ? 2 : 1)>
__global__ void __launch_bounds__(256, 2)
    conv3x3_bf_fwd2_kernel(const bf16* __restrict__ x, const float* __restrict__ wt,
                           bf16* __restrict__ y, int h, int w, int tiles_w, int tiles_per_img,
                           int ntiles, float* __restrict__ stats) {
  static_assert(CI == 16 || CI == 32, "bf16 forward: 16 or 32 input channels");
  static_assert(CO % 16 == 0, "output channels in 16-blocks");
  constexpr int TH = 4 * RPW, XR = TH + 2;
  constexpr int NB = CO / 16;
  constexpr int NS = CI == 16 ? 5 : 9;  // K steps of 32
  using L = CopyTile<CI, XR, 64>;
  __shared__ __attribute__((aligned(16))) bf16 sx[L::ELEMS];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int li = lane & 15, g = lane >> 4;
  const int64_t img_in = (int64_t)CI * h * w, img_out = (int64_t)CO * h * w;

  u4v wb[NS][NB];
#pragma unroll
  for (int st = 0; st < NS; ++st)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int co = 16 * nb + li;
      const int tap = CI == 32 ? st : 2 * st + (g >> 1);
      const int c8 = CI == 32 ? 8 * g : 8 * (g & 1);
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ci = c8 + j;
        const int src = FLIP ? (ci * CO + co) * 9 + (8 - tap) : (co * CI + ci) * 9 + tap;
        const float t = wt[tap < 9 ? src : 0];
        f[j] = tap < 9 ? t : 0.f;
      }
      wb[st][nb] = u4v{pack_bf(f[0], f[1]), pack_bf(f[2], f[3]), pack_bf(f[4], f[5]),
                       pack_bf(f[6], f[7])};
    }
  const int q = li >> 2, p = li & 3;
  int aoff[NS];
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int tap = CI == 32 ? st : (2 * st + (g >> 1) < 9 ? 2 * st + (g >> 1) : 8);
    const int c8 = CI == 32 ? 8 * g : 8 * (g & 1);
    aoff[st] = L::at(tap % 3, c8 + q, tap / 3, 4 * p);
  }

  mde::Sh run[STATS ? NB : 1];
#pragma unroll
  for (int nb = 0; nb < (STATS ? NB : 1); ++nb) run[nb] = {0.f, 0.f, 0.f, 0.f};
  bool first = true;
  // two register stages, the loop unrolled by two so each has fixed
  // registers and the waits count exactly the other stage's loads
  RowStage8<CI, XR> S0, S1;
  const TileWalk tw = tile_walk(ntiles);
  // unconditional (past the end: the last tile again, unused) so every step
  // issues the same loads and the waits stay exact
  auto fetch = [&](RowStage8<CI, XR>& S, int t) {
    const TileGeo gn = tile_geo(t < tw.end ? t : tw.end - 1, TH, tiles_w, tiles_per_img);
    S.load(x + gn.img * img_in, h, w, gn.r0, gn.c0, lane, wvu);
  };
  auto step = [&](RowStage8<CI, XR>& S, int tile) {
    const TileGeo gg = tile_geo(tile, TH, tiles_w, tiles_per_img);
    __syncthreads();
    S.template store<64>(sx, lane, wvu);
    __syncthreads();
    if constexpr (DEPTH == 1) fetch(S, tile + tw.step);  // in flight during this tile's math
    f4v acc[RPW][4][NB];
#pragma unroll
    for (int qq = 0; qq < RPW; ++qq)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[qq][m][nb] = f4v{0.f, 0.f, 0.f, 0.f};
    // K step outer, the 4 RPW accumulators inner: consecutive MFMAs are
    // independent (the m-inner chains of the first kernel issue-stalled on
    // their own results: SQ_WAIT_INST_ANY 58 % of wave cycles)
#pragma unroll
    for (int st = 0; st < NS; ++st) {
#pragma unroll
      for (int qq = 0; qq < RPW; ++qq) {
        const int row = wv * RPW + qq;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const bf16* base = sx + aoff[st] + row * 64 + 16 * m;
          const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)base);
          const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + 4 * L::PL));
          const u2v l2 = __builtin_bit_cast(u2v, lo), h2 = __builtin_bit_cast(u2v, hi);
          const u4v a = u4v{l2.x, l2.y, h2.x, h2.y};
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) acc[qq][m][nb] = mfma_bf(a, wb[st][nb], acc[qq][m][nb]);
        }
      }
    }
    // D: lane holds pixels 16m + 4g + r (r = 0..3) of output channel 16nb + li
    bf16* yi = y + gg.img * img_out;
    // Output through LDS: the block's [TH rows][CO][64] tile (line pitch 68:
    // conflict-free 8-byte writes) then full 128-byte line segments per 16
    // lanes (direct stores from the D layout wrote 32-byte pieces of 16
    // channel rows per instruction).
    constexpr int LP = 72;  // 16-byte aligned lines, 2-way at most on the 8-byte writes
    static_assert(TH * CO * LP <= L::ELEMS && TH * CO * 8 % 256 == 0, "output tile in LDS");
    __syncthreads();  // every wave's A reads of sx are done
#pragma unroll
    for (int qq = 0; qq < RPW; ++qq) {
      const int row = gg.r0 + wv * RPW + qq;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int col = gg.c0 + 16 * m + 4 * g;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const f4v v = acc[qq][m][nb];
          const u2v u{pk_bf(v[0], v[1]), pk_bf(v[2], v[3])};
          *reinterpret_cast<u2v*>(sx + ((wv * RPW + qq) * CO + 16 * nb + li) * LP + 16 * m + 4 * g) = u;
          if constexpr (STATS) {
            const float b[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
            if (first && qq == 0 && m == 0) {
              const bool ok0 = gg.r0 + wv * RPW < h && gg.c0 < w;
              run[nb].ref = __shfl(ok0 ? b[0] : 0.f, li, 64);
            }
            const bool ok = row < h && col < w;  // w % 4 == 0: all 4 columns or none
#pragma unroll
            for (int r = 0; r < 4; ++r) mde::sh_add(run[nb], b[r], ok);
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < TH * CO * 8 / 256; ++k) {  // 16-byte pieces, 8 lanes a line
      const int e = tid + 256 * k, line = e >> 3, ch = e & 7;
      const int r = line / CO, co = line % CO;
      const int grow = gg.r0 + r, col = gg.c0 + 8 * ch;
      const u4v u = *reinterpret_cast<const u4v*>(sx + line * LP + 8 * ch);
      bf16* dst = yi + ((int64_t)co * h + grow) * w + col;
      if (grow < h && col + 8 <= w)
        *reinterpret_cast<u4v*>(dst) = u;
      else if (grow < h && col < w)  // w % 4 == 0: the first half
        *reinterpret_cast<u2v*>(dst) = u2v{u[0], u[1]};
    }
    first = false;
    // DEPTH 2: the next-but-one tile's loads, after this tile's stores (a wait
    // for the stores' source registers then leaves these loads in flight)
    if constexpr (DEPTH == 2) fetch(S, tile + 2 * tw.step);
  };
  int tile = tw.t0;
  if constexpr (DEPTH == 1) {
    if (tile < tw.end) fetch(S0, tile);
    for (; tile < tw.end; tile += tw.step) step(S0, tile);
  } else {
    if (tile < tw.end) {
      fetch(S0, tile);
      fetch(S1, tile + tw.step);
    }
    while (tile < tw.end) {
      step(S0, tile);
      tile += tw.step;
      if (tile >= tw.end) break;
      step(S1, tile);
      tile += tw.step;
    }
  }
  if constexpr (STATS) {
    __syncthreads();
    float* part = reinterpret_cast<float*>(sx);  // [4][CO][4]
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const mde::Sh a = mde::sh_xor_sum(mde::sh_xor_sum(run[nb], 16), 32);
      if (g == 0) {
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

// gy tile of the bf16 weight gradient: CO planes of TH rows x 64 columns
// (plane pitch 16 mod 128), 16-byte loads: line L = 32 k + 8 wave + sub of
// the (channel, tile row) order, 8 lanes per 64-column line (channel L / TH,
// row L % TH: the row is a lane constant, the channel steps by 32 / TH per k,
// a uniform offset).
template <int CO, int TH>
struct GyStage8 {
  static constexpr int PL = (TH * 64 + 127) / 128 * 128 + 16;
  static constexpr int K = CO * TH / 32;
  static_assert(CO * TH % 32 == 0 && 32 % TH == 0, "whole instructions");
  u4v v[K];
  __device__ __forceinline__ void load(const bf16* __restrict__ img, int h, int w, int r0,
                                       int c0, int lane, int wvu) {
    const int sub = lane >> 3, i = lane & 7, l0 = 8 * wvu + sub;
    const int c = l0 / TH, gr = r0 + l0 % TH, gc = c0 + 8 * i;
    const int hw = h * w;
    const uint32_t vo = gr < h && gc < w ? (uint32_t)(2 * (c * hw + gr * w + gc)) : 0x7ffffff0u;
    const bool half = gc + 4 >= w;  // w % 4 == 0
    const uint64_t a = (uint64_t)img;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, 2 * CO * hw, 0x00020000);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      u4v t = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(R, vo, 2 * (32 / TH) * k * hw, 0));
      if (half) t = u4v{t[0], t[1], 0u, 0u};
      v[k] = t;
    }
  }
  __device__ __forceinline__ void store(bf16* sg, int lane, int wvu) const {
    const int sub = lane >> 3, i = lane & 7, l0 = 8 * wvu + sub;
    const int c = l0 / TH, r = l0 % TH;
#pragma unroll
    for (int k = 0; k < K; ++k)
      *reinterpret_cast<u4v*>(sg + (c + (32 / TH) * k) * PL + r * 64 + 8 * i) = v[k];
  }
};

// PW waves split a tile's K steps, 4 / PW wave groups split the N blocks.
template <int CI, int CO, int TH, int PW>
struct BfWgradCfg {
  static constexpr int XR = TH + 2;
  using LX = CopyTile<CI, XR, 0>;
  using GS = GyStage8<CO, TH>;
  static constexpr int MB = CO / 16;
  static constexpr int NP = 9 * CI;  // n = tap * CI + ci
  static constexpr int NBLK = NP / 16;
  static constexpr int TWAYS = 4 / PW;
  static constexpr int NBW = (NBLK + TWAYS - 1) / TWAYS;
  static constexpr int KS = 2 * TH;  // 32-pixel K steps per tile
  static constexpr int SG = (LX::ELEMS + 127) / 128 * 128;
  static constexpr int SMEM_BF = SG + CO * GS::PL;     // bf16 elements
  static constexpr int RED = PW * MB * NBLK * 256;     // fp32 block reduction
  static constexpr int SMEM_F = (SMEM_BF / 2 > RED ? SMEM_BF / 2 : RED);
  static constexpr int M = CO * NP;
};

template <int CI, int CO, int TH, int PW>
__global__ void __launch_bounds__(256, 2)
    conv3x3_bf_wgrad_kernel(const bf16* __restrict__ x, const bf16* __restrict__ gy,
                            float* __restrict__ part, int h, int w, int tiles_w,
                            int tiles_per_img, int ntiles) {
  using C = BfWgradCfg<CI, CO, TH, PW>;
  static_assert(CI % 16 == 0 && CO % 16 == 0, "16-channel blocks");
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM_F];
  bf16* sx = reinterpret_cast<bf16*>(smem);
  bf16* sg = sx + C::SG;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int li = lane & 15, g = lane >> 4;
  const int64_t img_in = (int64_t)CI * h * w, img_out = (int64_t)CO * h * w;

  const int pg = wvu % PW, tg = wvu / PW;  // K group, N group of this wave
  int boff[C::NBW];  // B (x) read base of each of the wave's N blocks
#pragma unroll
  for (int j = 0; j < C::NBW; ++j) {
    const int nb = tg + C::TWAYS * j;
    const int n = 16 * (nb < C::NBLK ? nb : 0) + li, tap = n / CI, ci = n % CI;
    boff[j] = C::LX::at(tap % 3, ci, tap / 3, 8 * g);
  }
  const int aoff = li * C::GS::PL + 8 * g;

  f4v acc[C::MB][C::NBW];
#pragma unroll
  for (int mb = 0; mb < C::MB; ++mb)
#pragma unroll
    for (int j = 0; j < C::NBW; ++j) acc[mb][j] = f4v{0.f, 0.f, 0.f, 0.f};

  RowStage8<CI, C::XR> S;
  typename C::GS G;
  const TileWalk tw = tile_walk(ntiles);
  int tile = tw.t0;
  if (tile < tw.end) {
    const TileGeo gg = tile_geo(tile, TH, tiles_w, tiles_per_img);
    G.load(gy + gg.img * img_out, h, w, gg.r0, gg.c0, lane, wvu);
    S.load(x + gg.img * img_in, h, w, gg.r0, gg.c0, lane, wvu);
  }
  for (; tile < tw.end; tile += tw.step) {
    __syncthreads();
    S.template store<0>(sx, lane, wvu);
    G.store(sg, lane, wvu);
    __syncthreads();
    const int nxt = tile + tw.step;
    if (nxt < tw.end) {
      const TileGeo gn = tile_geo(nxt, TH, tiles_w, tiles_per_img);
      G.load(gy + gn.img * img_out, h, w, gn.r0, gn.c0, lane, wvu);
      S.load(x + gn.img * img_in, h, w, gn.r0, gn.c0, lane, wvu);
    }
    // K steps kk = pg, pg + PW, ...: tile row kk / 2, columns 32 (kk & 1) + 8 g ..
#pragma unroll
    for (int kk = pg; kk < C::KS; kk += PW) {
      const int r = kk >> 1, c32 = 32 * (kk & 1);
      u4v a[C::MB];
#pragma unroll
      for (int mb = 0; mb < C::MB; ++mb)
        a[mb] = *reinterpret_cast<const u4v*>(sg + aoff + mb * 16 * C::GS::PL + r * 64 + c32);
#pragma unroll
      for (int j = 0; j < C::NBW; ++j) {
        if (tg + C::TWAYS * j < C::NBLK) {  // wave-uniform
          const u4v b = *reinterpret_cast<const u4v*>(sx + boff[j] + r * 64 + c32);
#pragma unroll
          for (int mb = 0; mb < C::MB; ++mb) acc[mb][j] = mfma_bf(a[mb], b, acc[mb][j]);
        }
      }
    }
  }
  // the PW K-group partials summed through LDS in group order, one block
  // partial: lane holds co = 16 mb + 4 g + i, n = 16 nb + li
  __syncthreads();
#pragma unroll
  for (int mb = 0; mb < C::MB; ++mb)
#pragma unroll
    for (int j = 0; j < C::NBW; ++j) {
      const int nb = tg + C::TWAYS * j;
      if (nb < C::NBLK) {
        float* d = smem + ((pg * C::MB + mb) * C::NBLK + nb) * 256 + li;
#pragma unroll
        for (int i = 0; i < 4; ++i) d[(4 * g + i) * 16] = acc[mb][j][i];
      }
    }
  __syncthreads();
  float* out = part + (int64_t)blockIdx.x * C::M;
  for (int e = tid; e < C::M; e += 256) {
    const int co = e / C::NP, n = e % C::NP;
    const int mb = co / 16, nb = n / 16;
    const int o = ((mb * C::NBLK + nb) * 256) + (co % 16) * 16 + n % 16;
    float sacc = 0.f;
#pragma unroll
    for (int k = 0; k < PW; ++k) sacc += smem[k * C::MB * C::NBLK * 256 + o];
    out[e] = sacc;
  }
}

// ------------------------------------------------ stride-2 weight gradient
// The DDRNet stem's two stride-2 convolutions (conv1 of
// src/GuideDepth/model/DDRNet_23_slim.py:229-236: 3 -> 32 and 32 -> 32, k3 s2
// p1), whose weight gradient MIOpen runs as NHWC implicit GEMM behind NCHW <->
// NHWC transposes (~0.69 ms per cfg2 step for the two).  NCHW here:
//   gW[co][ci][dy][dx] = sum_{n,r,c} gy[n][co][r][c] x[n][ci][2r + dy - 1][2c + dx - 1].
// A tile is one output row r x 64 output columns c0 .. c0+63 (K = 64 pixels).
// x rows 2r-1 .. 2r+1 are staged split by column parity, O[j] = x[2(c0+j) - 1]
// (j = 0..64) then E[j] = x[2(c0+j)] (j = 0..63), so the three column taps of
// output pixel p read O[p], E[p], O[p + 1]: unit stride in p, every operand
// one ds_read_b32 at a compile-time offset from a per-lane base.  A lane
// loads one aligned float2 per staged row (E[l], O[l + 1]); O[0] is a halo
// element.  MFMA (v_mfma_f32_16x16x4_f32): M = output channels, N = (tap, ci)
// tap-major, K = pixels; the waves split (M tiles, N tiles, K steps) as
// S2Cfg says, K-split partials are summed through LDS, and the block partials
// are reduced by wgrad_reduce_kernel (fixed order).
template <int CI, int CO>
struct S2Cfg {
  static constexpr int CIP = cpad4(CI);
  static constexpr int NREAL = 9 * CIP;             // n = tap * CIP + ci
  static constexpr int NP = (NREAL + 15) / 16 * 16;
  static constexpr int NT = NP / 16, MT = CO / 16;
  static constexpr int OE = 65;                     // E[0] within a staged row
  static constexpr int RW = 130;                    // staged row pitch (O 65 + E 64, + 1)
  static constexpr int PSX = (3 * RW - 2 + 31) / 32 * 32 + 2;  // >= 3 RW, = 2 (mod 32)
  static constexpr int PSG = kTW + 4;               // gy row pitch (float4-aligned)
  static constexpr int MW = CI >= 16 ? MT : 1;      // waves over M tiles
  static constexpr int NW = CI >= 16 ? 4 / MT : 1;  // ... over N tiles
  static constexpr int KW = 4 / (MW * NW);          // ... over K steps
  static constexpr int MTW = MT / MW, NTW = NT / NW;
  static constexpr int XR = CI * 3;                 // staged rows
  static constexpr int XRW = (XR + 3) / 4;          // staged rows per wave
  static constexpr int ZERO = CIP * PSX;            // 64 zeros: B of padded n
  static constexpr int SX = ZERO + 64;
  static constexpr int STAGE = SX + CO * PSG;
  static constexpr int RED = KW > 1 ? KW * MT * NT * 256 : 0;
  static constexpr int SMEM = STAGE > RED ? STAGE : RED;
  static constexpr int M = CO * NP;                 // partial elements per block
  static_assert(MW * NW * KW == 4 && MT % MW == 0 && NT % NW == 0 && 16 % KW == 0, "split");
  static_assert(XRW <= 32, "row mask");
};

template <int CI, int CO, bool FULL>
__global__ void __launch_bounds__(256, 2)
    conv3x3s2_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                           float* __restrict__ part, int h, int w, int ho, int wo, int tiles_w,
                           int tiles_per_img, int ntiles) {
  using C = S2Cfg<CI, CO>;
  __shared__ float smem[C::SMEM];
  float* sx = smem;
  float* sg = smem + C::SX;
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, lk = lane >> 4;
  const int wvu = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mw = wvu % C::MW, nw = (wvu / C::MW) % C::NW, kw = wvu / (C::MW * C::NW);
  const int64_t img_in = (int64_t)CI * h * w, img_out = (int64_t)CO * ho * wo;
  const int hw = h * w;
  // padded input channels (CI < CIP) and the padded-n zeros: never rewritten
  for (int e = CI * C::PSX + tid; e < C::SX; e += 256) sx[e] = 0.f;

  int boff[C::NTW];
#pragma unroll
  for (int j = 0; j < C::NTW; ++j) {
    const int n = 16 * (nw * C::NTW + j) + li;
    if (n < C::NREAL) {
      const int tap = n / C::CIP, ci = n % C::CIP, dy = tap / 3, dx = tap % 3;
      boff[j] = ci * C::PSX + dy * C::RW + (dx == 0 ? 0 : (dx == 1 ? C::OE : 1)) + lk;
    } else {
      boff[j] = C::ZERO + lk;
    }
  }
  int aoff[C::MTW];
#pragma unroll
  for (int i = 0; i < C::MTW; ++i) aoff[i] = (16 * (mw * C::MTW + i) + li) * C::PSG + lk;
  f4 acc[C::MTW][C::NTW];
#pragma unroll
  for (int i = 0; i < C::MTW; ++i)
#pragma unroll
    for (int j = 0; j < C::NTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // staging registers: this wave's rows k (staged row wvu + 4k = (ci, rr)),
  // one float2 (E[lane], O[lane + 1]) each, and the O[0] halo of row k in lane k
  float2 xv[C::XRW];
  float xh = 0.f;
  unsigned xm = 0;  // bit k: row k and this lane's columns in range
  bool hok = false;
  GradTile<CO, 1, FULL> G;  // FULL: wo % 64 == 0
  auto load = [&](int tile) {
    const int img = tile / tiles_per_img, t = tile - img * tiles_per_img;
    const int r = t / tiles_w, c0 = (t - r * tiles_w) * kTW;
    const float* xi = x + img * img_in;
    const int col = 2 * c0 + 2 * lane;  // even; w even, so col < w <=> col + 1 < w
    const bool cok = col < w;
    const int colc = col < w ? col : w - 2;
    xm = 0;
#pragma unroll
    for (int k = 0; k < C::XRW; ++k) {
      const int rk = wvu + 4 * k;
      const int ci = rk / 3 < CI ? rk / 3 : CI - 1, rr = rk % 3, ir = 2 * r - 1 + rr;
      const bool ok = (C::XR % 4 == 0 || rk < C::XR) && ir >= 0 && ir < h && cok;
      const int irc = ir < 0 ? 0 : (ir >= h ? h - 1 : ir);
      xv[k] = *reinterpret_cast<const float2*>(xi + (unsigned)(ci * hw + irc * w + colc));
      xm |= ok ? 1u << k : 0u;
    }
    {  // halo O[0] = x[2 c0 - 1] of row k = lane
      const int rk = wvu + 4 * lane;
      const int ci = rk / 3 < CI ? rk / 3 : CI - 1, rr = rk % 3, ir = 2 * r - 1 + rr;
      hok = lane < C::XRW && rk < C::XR && ir >= 0 && ir < h && c0 > 0;
      const int irc = ir < 0 ? 0 : (ir >= h ? h - 1 : ir);
      xh = xi[(unsigned)(ci * hw + irc * w + (c0 > 0 ? 2 * c0 - 1 : 0))];
    }
    G.load(gy + img * img_out, ho, wo, r, c0, lane, wvu);
  };
  const TileWalk tw = tile_walk(ntiles);
  int tile = tw.t0;
  if (tile < tw.end) load(tile);
  for (; tile < tw.end; tile += tw.step) {
    __syncthreads();  // the previous tile's operands are consumed
#pragma unroll
    for (int k = 0; k < C::XRW; ++k) {
      const int rk = wvu + 4 * k;
      if (C::XR % 4 == 0 || rk < C::XR) {
        float* row = sx + (rk / 3) * C::PSX + (rk % 3) * C::RW;
        const bool ok = (xm >> k) & 1u;
        row[C::OE + lane] = ok ? xv[k].x : 0.f;
        row[1 + lane] = ok ? xv[k].y : 0.f;
      }
    }
    if (lane < C::XRW) {
      const int rk = wvu + 4 * lane;
      if (rk < C::XR) sx[(rk / 3) * C::PSX + (rk % 3) * C::RW] = hok ? xh : 0.f;
    }
    G.template store<C::PSG>(sg, lane, wvu);
    __syncthreads();
    const int nxt = tile + tw.step;
    if (nxt < tw.end) load(nxt);
#pragma unroll
    for (int st = 0; st < 16 / C::KW; ++st) {
      const int s4 = 4 * (kw + C::KW * st);
      float a[C::MTW];
#pragma unroll
      for (int i = 0; i < C::MTW; ++i) a[i] = sg[aoff[i] + s4];
#pragma unroll
      for (int j = 0; j < C::NTW; ++j) {
        const float b = sx[boff[j] + s4];
#pragma unroll
        for (int i = 0; i < C::MTW; ++i) acc[i][j] = mfma4(a[i], b, acc[i][j]);
      }
    }
  }
  // lane holds co = 16 mt + 4 lk + i, n = 16 nt + li
  float* out = part + (int64_t)blockIdx.x * C::M;
  if constexpr (C::KW == 1) {
#pragma unroll
    for (int i = 0; i < C::MTW; ++i)
#pragma unroll
      for (int j = 0; j < C::NTW; ++j) {
        const int mt = mw * C::MTW + i, nt = nw * C::NTW + j;
#pragma unroll
        for (int q = 0; q < 4; ++q) out[(16 * mt + 4 * lk + q) * C::NP + 16 * nt + li] = acc[i][j][q];
      }
    return;
  }
  __syncthreads();  // staging reads done: smem becomes red[kw][mt][nt][16][16]
#pragma unroll
  for (int i = 0; i < C::MTW; ++i)
#pragma unroll
    for (int j = 0; j < C::NTW; ++j) {
      const int mt = mw * C::MTW + i, nt = nw * C::NTW + j;
      float* d = smem + ((kw * C::MT + mt) * C::NT + nt) * 256 + li;
#pragma unroll
      for (int q = 0; q < 4; ++q) d[(4 * lk + q) * 16] = acc[i][j][q];
    }
  __syncthreads();
  for (int e = tid; e < C::M; e += 256) {
    const int co = e / C::NP, n = e % C::NP;
    const int o = ((co / 16) * C::NT + n / 16) * 256 + (co % 16) * 16 + n % 16;
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < C::KW; ++k) sum += smem[k * C::MT * C::NT * 256 + o];
    out[e] = sum;
  }
}

// ---------------------------------------------------------------- dispatch
enum Pass { kFwd = 0, kDgrad = 1, kWgrad = 2 };

template <int CI, int CO, int RPW, bool FLIP, bool STATS = false, typename TO = float>
int fwd_grid(int64_t n, int64_t h, int64_t w, int* tiles_w, int* tiles_per_img, int* ntiles) {
  constexpr int TH = 4 * RPW;
  *tiles_w = (int)mde::cdiv(w, kTW);
  *tiles_per_img = (int)(mde::cdiv(h, TH) * *tiles_w);
  const int64_t nt = n * *tiles_per_img;
  if (nt > 0x7fffffff) return 0;
  *ntiles = (int)nt;
  const int res = resident_blocks<conv3x3_fwd_kernel<CI, CO, RPW, FLIP, STATS, TO>>();
  return nt < res ? (int)nt : res;
}

template <int CI, int CO, int RPW, bool FLIP, bool STATS = false, typename TO = float>
int launch_fwd(const float* in, const float* wt, TO* out, int64_t n, int64_t h, int64_t w,
               double bytes, int kid, hipStream_t s, float* stats = nullptr) {
  const double flops = 2.0 * 9 * CI * CO * (double)(n * h * w);
  int tiles_w, tiles_per_img, ntiles;
  const int grid =
      fwd_grid<CI, CO, RPW, FLIP, STATS, TO>(n, h, w, &tiles_w, &tiles_per_img, &ntiles);
  if (grid <= 0) return MDE_ERR_INVALID_ARG;
  MDE_LAUNCH_MFMA(kid, bytes, flops, s, (conv3x3_fwd_kernel<CI, CO, RPW, FLIP, STATS, TO>),
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
  // the 3-channel guide convs' weight gradients have ~12 flop per byte, under the
  // fp32 MFMA ridge (157 TF / 8 TB/s ~ 20): timed as HBM-bound under their own id
  if (CI == 3) {
    if (w % kTW == 0)
      MDE_LAUNCH(mde::K_C3_WGRAD_GUIDE, bytes, s, (conv3x3_wgrad_kernel<CI, CO, TH, PW, true>),
                 dim3(p.grid), dim3(256), 0, x, gy, ws, (int)h, (int)w, p.tiles_w,
                 p.tiles_per_img, p.ntiles);
    else
      MDE_LAUNCH(mde::K_C3_WGRAD_GUIDE, bytes, s, (conv3x3_wgrad_kernel<CI, CO, TH, PW, false>),
                 dim3(p.grid), dim3(256), 0, x, gy, ws, (int)h, (int)w, p.tiles_w,
                 p.tiles_per_img, p.ntiles);
  } else if (w % kTW == 0) {
    MDE_LAUNCH_MFMA(mde::K_C3_WGRAD, bytes, flops, s, (conv3x3_wgrad_kernel<CI, CO, TH, PW, true>),
                    dim3(p.grid), dim3(256), 0, x, gy, ws, (int)h, (int)w, p.tiles_w,
                    p.tiles_per_img, p.ntiles);
  } else {
    MDE_LAUNCH_MFMA(mde::K_C3_WGRAD, bytes, flops, s, (conv3x3_wgrad_kernel<CI, CO, TH, PW, false>),
                    dim3(p.grid), dim3(256), 0, x, gy, ws, (int)h, (int)w, p.tiles_w,
                    p.tiles_per_img, p.ntiles);
  }
  return launch_reduce(ws, gw, 1, p.grid, p.m, ReduceMap{0, p.np, p.cip, CI, CO}, s);
}

// ---- stride-2 weight gradient dispatch (3 -> 32, 32 -> 32; w even)
struct S2Plan {
  int ho, wo, tiles_w, tiles_per_img, ntiles, grid, m, np, cip;
};

template <int CI, int CO>
S2Plan s2_plan(int64_t n, int64_t h, int64_t w) {
  using C = S2Cfg<CI, CO>;
  S2Plan p;
  p.ho = (int)((h - 1) / 2 + 1);
  p.wo = (int)((w - 1) / 2 + 1);
  p.tiles_w = (int)mde::cdiv(p.wo, kTW);
  p.tiles_per_img = p.ho * p.tiles_w;
  const int64_t nt = n * p.tiles_per_img;
  p.ntiles = nt > 0x7fffffff ? 0x7fffffff : (int)nt;
  const int res = resident_blocks<conv3x3s2_wgrad_kernel<CI, CO, false>>();
  p.grid = p.ntiles < res ? p.ntiles : res;
  p.m = C::M;
  p.np = C::NP;
  p.cip = C::CIP;
  return p;
}

bool s2_supported(int64_t cin, int64_t cout) {
  return (cin == 3 || cin == 32) && cout == 32;
}

template <int CI, int CO>
int launch_wgrad_s2(const float* x, const float* gy, float* gw, int64_t n, int64_t h, int64_t w,
                    float* ws, hipStream_t s) {
  const S2Plan p = s2_plan<CI, CO>(n, h, w);
  if (p.grid <= 0) return MDE_ERR_INVALID_ARG;
  const double flops = 2.0 * 9 * CI * CO * (double)n * p.ho * p.wo;
  const double bytes = 4.0 * (double)n * ((double)CI * h * w + (double)CO * p.ho * p.wo);
  if (p.wo % kTW == 0)
    MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_S2, bytes, flops, s, (conv3x3s2_wgrad_kernel<CI, CO, true>),
                    dim3(p.grid), dim3(256), 0, x, gy, ws, (int)h, (int)w, p.ho, p.wo, p.tiles_w,
                    p.tiles_per_img, p.ntiles);
  else
    MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_S2, bytes, flops, s, (conv3x3s2_wgrad_kernel<CI, CO, false>),
                    dim3(p.grid), dim3(256), 0, x, gy, ws, (int)h, (int)w, p.ho, p.wo, p.tiles_w,
                    p.tiles_per_img, p.ntiles);
  return launch_reduce(ws, gw, 1, p.grid, p.m, ReduceMap{0, p.np, p.cip, CI, CO}, s);
}

// ---- bf16 dispatch
// conv3x3_bf_fwd2_kernel (row stage, interior fast stores) where the width
// allows (w % 4 == 0); MDE_C3BF_V2=0: the first kernel (A/B).
inline bool bf_v2(int64_t h, int64_t w) {
  static const bool on = [] {
    const char* e = std::getenv("MDE_C3BF_V2");
    return !(e && e[0] == '0');
  }();
  return on && w % 4 == 0 && 2 * 32 * h * w < (int64_t)1 << 30;  // 32-bit buffer offsets
}

template <int CI, int CO, int RPW, bool FLIP, bool STATS>
int bf_fwd_grid(int64_t n, int64_t h, int64_t w, int* tiles_w, int* tiles_per_img, int* ntiles) {
  constexpr int TH = 4 * RPW;
  *tiles_w = (int)mde::cdiv(w, kTW);
  *tiles_per_img = (int)(mde::cdiv(h, TH) * *tiles_w);
  const int64_t nt = n * *tiles_per_img;
  if (nt > 0x7fffffff) return 0;
  *ntiles = (int)nt;
  const int res = bf_v2(h, w) ? resident_blocks<conv3x3_bf_fwd2_kernel<CI, CO, RPW, FLIP, STATS>>()
                           : resident_blocks<conv3x3_bf_fwd_kernel<CI, CO, RPW, FLIP, STATS>>();
  return nt < res ? (int)nt : res;
}

// bf16 forward / data-gradient tile height: 8-row tiles (two rows per wave:
// twice the MFMAs per staging round and barrier, 1.25x instead of 1.5x halo
// rows) at 16 channels -- fwd 266 -> 246, dgrad 249 -> 225 us at 480 x 640 --
// 4-row tiles at 32 (8-row: 164 -> 194 us, one block per CU by registers),
// profiles/r04_bf_rpw_ab.txt.  MDE_BF_RPW=1 / 2 forces one (A/B).
inline int bf_rpw_forced() {
  static const int r = [] {
    const char* e = std::getenv("MDE_BF_RPW");
    return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
  }();
  return r;
}
inline int bf_rpw(int64_t ch) {
  const int f = bf_rpw_forced();
  return f ? f : (ch == 16 ? 2 : 1);
}

template <int CI, int CO, int RPW, bool FLIP, bool STATS = false>
int launch_bf_fwd(const bf16* in, const float* wt, bf16* out, int64_t n, int64_t h, int64_t w,
                  double bytes, int kid, hipStream_t s, float* stats = nullptr) {
  const double flops = 2.0 * 9 * CI * CO * (double)(n * h * w);
  int tiles_w, tiles_per_img, ntiles;
  const int grid =
      bf_fwd_grid<CI, CO, RPW, FLIP, STATS>(n, h, w, &tiles_w, &tiles_per_img, &ntiles);
  if (grid <= 0) return MDE_ERR_INVALID_ARG;
  if (bf_v2(h, w))
    MDE_LAUNCH_MFMA(kid, bytes, flops, s, (conv3x3_bf_fwd2_kernel<CI, CO, RPW, FLIP, STATS>),
                    dim3(grid), dim3(256), 0, in, wt, out, (int)h, (int)w, tiles_w, tiles_per_img,
                    ntiles, stats);
  else
    MDE_LAUNCH_MFMA(kid, bytes, flops, s, (conv3x3_bf_fwd_kernel<CI, CO, RPW, FLIP, STATS>),
                    dim3(grid), dim3(256), 0, in, wt, out, (int)h, (int)w, tiles_w, tiles_per_img,
                    ntiles, stats);
  return MDE_OK;
}

template <int CI, int CO, int TH, int PW>
WgradPlan bf_wgrad_plan(int64_t n, int64_t h, int64_t w) {
  using C = BfWgradCfg<CI, CO, TH, PW>;
  WgradPlan p;
  p.th = TH;
  p.tiles_w = (int)mde::cdiv(w, kTW);
  p.tiles_per_img = (int)(mde::cdiv(h, TH) * p.tiles_w);
  const int64_t nt = n * p.tiles_per_img;
  p.ntiles = nt > 0x7fffffff ? 0x7fffffff : (int)nt;
  const int res = resident_blocks<conv3x3_bf_wgrad_kernel<CI, CO, TH, PW>>();
  p.grid = p.ntiles < res ? p.ntiles : res;
  p.m = C::M;
  p.np = C::NP;
  p.cip = CI;
  return p;
}

template <int CI, int CO, int TH, int PW>
int launch_bf_wgrad(const bf16* x, const bf16* gy, float* gw, int64_t n, int64_t h, int64_t w,
                    float* ws, double bytes, hipStream_t s) {
  const WgradPlan p = bf_wgrad_plan<CI, CO, TH, PW>(n, h, w);
  if (p.grid <= 0) return MDE_ERR_INVALID_ARG;
  const double flops = 2.0 * 9 * CI * CO * (double)(n * h * w);
  MDE_LAUNCH_MFMA(mde::K_C3_WGRAD_BF16, bytes, flops, s, (conv3x3_bf_wgrad_kernel<CI, CO, TH, PW>),
                  dim3(p.grid), dim3(256), 0, x, gy, ws, (int)h, (int)w, p.tiles_w,
                  p.tiles_per_img, p.ntiles);
  return launch_reduce(ws, gw, 1, p.grid, p.m, ReduceMap{0, p.np, p.cip, CI, CO}, s);
}

// bf16 shapes: 16 -> 16 and 32 -> 32, every pass; 4-column chunks need w % 4 == 0
bool bf_supported(int64_t cin, int64_t cout) {
  return (cin == 16 && cout == 16) || (cin == 32 && cout == 32);
}

// Supported (cin, cout) per pass.  Forward: the guide convs (3 -> 16/32/64),
// 16 -> 16 and 32 -> 32; data gradient: 16 -> 16 and 32 -> 32 (the guide
// convs read the image, which needs no gradient); weight gradient: those and
// the wide-channel shapes.
// Wide channels (cin % 32 == 0, cout % 64 == 0; DDRNet's 64 / 128 / 256):
// weight gradient only.
bool wide(int64_t cin, int64_t cout) {
  return cin > 0 && cout > 0 && cin % kWCI == 0 && cout % kWCO == 0;
}

// input channels padded to the next 32 (the fixed-strip widths only: the
// workspace query returns 0 for other planes)
bool wide_pad(int64_t cin, int64_t cout) {
  return cin > 16 && cin % 8 == 0 && cin % kWCI != 0 && cout > 0 && cout % kWCO == 0;
}

bool supported(int64_t cin, int64_t cout, int pass) {
  const bool guide = cin == 3 && (cout == 16 || cout == 32 || cout == 64);
  const bool square = (cin == 16 && cout == 16) || (cin == 32 && cout == 32);
  switch (pass) {
    case kFwd:
      return guide || square;
    case kDgrad:
      return square;
    case kWgrad:
      return guide || square || wide(cin, cout) || wide_pad(cin, cout);
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

// stride-2 kernels: float2 loads of column pairs need an even width
bool s2_dims_ok(int64_t n, int64_t h, int64_t w) {
  return dims_ok(n, h, w) && w % 2 == 0;
}

}  // namespace

extern "C" {

int mde_conv3x3_guide_bf16_stats_blocks(int64_t n, int64_t cout, int64_t h, int64_t w) {
  int a, b, c;
  if (!dims_ok(n, h, w)) return 0;
  if (cout == 16) return fwd_grid<3, 16, 2, false, true, bf16>(n, h, w, &a, &b, &c);
  if (cout == 32) return fwd_grid<3, 32, 1, false, true, bf16>(n, h, w, &a, &b, &c);
  if (cout == 64) return fwd_grid<3, 64, 1, false, true, bf16>(n, h, w, &a, &b, &c);
  return 0;
}

int mde_conv3x3_guide_bf16_fwd(const float* x, const float* weight, void* y, float* stats,
                               int64_t n, int64_t cout, int64_t h, int64_t w, void* stream) {
  if (!x || !weight || !y || !dims_ok(n, h, w)) return MDE_ERR_INVALID_ARG;
  if (cout != 16 && cout != 32 && cout != 64) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  bf16* out = (bf16*)y;
  const double bytes = (double)n * h * w * (4.0 * 3 + 2.0 * cout);
  const int k = mde::K_C3_FWD;
  if (stats) {
    if (cout == 16)
      return launch_fwd<3, 16, 2, false, true, bf16>(x, weight, out, n, h, w, bytes, k, s, stats);
    if (cout == 32)
      return launch_fwd<3, 32, 1, false, true, bf16>(x, weight, out, n, h, w, bytes, k, s, stats);
    return launch_fwd<3, 64, 1, false, true, bf16>(x, weight, out, n, h, w, bytes, k, s, stats);
  }
  if (cout == 16) return launch_fwd<3, 16, 2, false, false, bf16>(x, weight, out, n, h, w, bytes, k, s);
  if (cout == 32) return launch_fwd<3, 32, 1, false, false, bf16>(x, weight, out, n, h, w, bytes, k, s);
  return launch_fwd<3, 64, 1, false, false, bf16>(x, weight, out, n, h, w, bytes, k, s);
}

int mde_conv3x3_supported(int64_t cin, int64_t cout, int pass, int dtype) {
  if (dtype == MDE_BF16) return bf_supported(cin, cout) && pass >= 0 && pass <= 2 ? 1 : 0;
  if (dtype != MDE_F32) return 0;
  return supported(cin, cout, pass) ? 1 : 0;
}

int mde_conv3x3_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t cin,
                    int64_t cout, int64_t h, int64_t w, int dtype, void* stream) {
  if (dtype == MDE_BF16) {
    if (!x || !weight || !y || !dims_ok(n, h, w) || w % 4) return MDE_ERR_INVALID_ARG;
    if (!bf_supported(cin, cout)) return MDE_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const double bytes = 2.0 * n * h * w * (double)(cin + cout);
#define MDE_BF(CC, R) \
  launch_bf_fwd<CC, CC, R, false>((const bf16*)x, weight, (bf16*)y, n, h, w, bytes, mde::K_C3_FWD_BF16, s)
    if (cin == 16) return bf_rpw(16) == 2 ? MDE_BF(16, 2) : MDE_BF(16, 1);
    return bf_rpw(32) == 2 ? MDE_BF(32, 2) : MDE_BF(32, 1);
#undef MDE_BF
  }
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
int mde_conv3x3_stats_blocks(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                             int dtype) {
  int a, b, c;
  if (dtype == MDE_BF16) {
    if (!bf_supported(cin, cout) || !dims_ok(n, h, w)) return 0;
    if (cin == 16)
      return bf_rpw(16) == 2 ? bf_fwd_grid<16, 16, 2, false, true>(n, h, w, &a, &b, &c)
                             : bf_fwd_grid<16, 16, 1, false, true>(n, h, w, &a, &b, &c);
    return bf_rpw(32) == 2 ? bf_fwd_grid<32, 32, 2, false, true>(n, h, w, &a, &b, &c)
                           : bf_fwd_grid<32, 32, 1, false, true>(n, h, w, &a, &b, &c);
  }
  if (!supported(cin, cout, kFwd) || !dims_ok(n, h, w)) return 0;
  if (cin == 3 && cout == 16) return fwd_grid<3, 16, 2, false, true>(n, h, w, &a, &b, &c);
  if (cin == 3 && cout == 32) return fwd_grid<3, 32, 1, false, true>(n, h, w, &a, &b, &c);
  if (cin == 3 && cout == 64) return fwd_grid<3, 64, 1, false, true>(n, h, w, &a, &b, &c);
  if (cin == 16 && variant() == 1) return fwd_grid<16, 16, 2, false, true>(n, h, w, &a, &b, &c);
  if (cin == 16) return fwd_grid<16, 16, 1, false, true>(n, h, w, &a, &b, &c);
  return fwd_grid<32, 32, 1, false, true>(n, h, w, &a, &b, &c);
}

int mde_conv3x3_fwd_stats(const void* x, const float* weight, void* y, float* stats, int64_t n,
                          int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype,
                          void* stream) {
  if (dtype == MDE_BF16) {
    if (!x || !weight || !y || !stats || !dims_ok(n, h, w) || w % 4) return MDE_ERR_INVALID_ARG;
    if (!bf_supported(cin, cout)) return MDE_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const double bytes = 2.0 * n * h * w * (double)(cin + cout);
#define MDE_BF(CC, R)                                                                   \
  launch_bf_fwd<CC, CC, R, false, true>((const bf16*)x, weight, (bf16*)y, n, h, w, bytes, \
                                        mde::K_C3_FWD_BF16, s, stats)
    if (cin == 16) return bf_rpw(16) == 2 ? MDE_BF(16, 2) : MDE_BF(16, 1);
    return bf_rpw(32) == 2 ? MDE_BF(32, 2) : MDE_BF(32, 1);
#undef MDE_BF
  }
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
  if (cin == 16 && variant() == 1)
    return launch_fwd<16, 16, 2, false, true>(in, weight, out, n, h, w, bytes, k, s, stats);
  if (cin == 16)
    return launch_fwd<16, 16, 1, false, true>(in, weight, out, n, h, w, bytes, k, s, stats);
  return launch_fwd<32, 32, 1, false, true>(in, weight, out, n, h, w, bytes, k, s, stats);
}

int mde_conv3x3_bwd_data(const void* gy, const float* weight, void* gx, int64_t n, int64_t cin,
                         int64_t cout, int64_t h, int64_t w, int dtype, void* stream) {
  if (dtype == MDE_BF16) {
    if (!gy || !weight || !gx || !dims_ok(n, h, w) || w % 4) return MDE_ERR_INVALID_ARG;
    if (!bf_supported(cin, cout)) return MDE_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const double bytes = 2.0 * n * h * w * (double)(cin + cout);
#define MDE_BF(CC, R)                                                                        \
  launch_bf_fwd<CC, CC, R, true>((const bf16*)gy, weight, (bf16*)gx, n, h, w, bytes,          \
                                 mde::K_C3_DGRAD_BF16, s)
    if (cin == 16) return bf_rpw(16) == 2 ? MDE_BF(16, 2) : MDE_BF(16, 1);
    return bf_rpw(32) == 2 ? MDE_BF(32, 2) : MDE_BF(32, 1);
#undef MDE_BF
  }
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

size_t mde_conv3x3_wgrad_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                                   int dtype) {
  WgradPlan p;
  if (dtype == MDE_BF16) {
    if (!bf_supported(cin, cout) || !dims_ok(n, h, w)) return 0;
    p = cin == 16 ? bf_wgrad_plan<16, 16, 4, 4>(n, h, w) : bf_wgrad_plan<32, 32, 2, 2>(n, h, w);
    return wgrad_ws_bytes(1, p.grid, p.m);
  }
  if (!supported(cin, cout, kWgrad) || !dims_ok(n, h, w)) return 0;
  if (wide(cin, cout) || wide_pad(cin, cout)) {
    WidePlan wp;
    return wide_plan(n, cin, cout, h, w, &wp) ? wide_workspace(wp) : 0;
  }
  if (cin == 3 && cout == 16) p = wgrad_plan<3, 16, 8, 4>(n, h, w);
  else if (cin == 3 && cout == 32) p = wgrad_plan<3, 32, 8, 4>(n, h, w);
  else if (cin == 3) p = wgrad_plan<3, 64, 4, 4>(n, h, w);
  else if (cin == 16 && variant() == 1) p = wgrad_plan<16, 16, 8, 4>(n, h, w);
  else if (cin == 16 && variant() == 2) p = wgrad_plan<16, 16, 4, 2>(n, h, w);
  else if (cin == 16) p = wgrad_plan<16, 16, 4, 4>(n, h, w);
  else if (c32_wide(w)) {
    const WidePlan wp = c32_plan(n, h, w);
    return wgrad_ws_bytes(1, wp.gx, WideT<1, 80, 1, 32>::M);
  } else if (variant() == 1) p = wgrad_plan<32, 32, 4, 2>(n, h, w);
  else if (variant() == 2) p = wgrad_plan<32, 32, 4, 1>(n, h, w);
  else p = wgrad_plan<32, 32, 2, 2>(n, h, w);
  return wgrad_ws_bytes(1, p.grid, p.m);
}

int mde_conv3x3_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t cin,
                      int64_t cout, int64_t h, int64_t w, void* workspace, int dtype,
                      void* stream) {
  if (dtype == MDE_BF16) {
    if (!gy || !x || !gweight || !workspace || !dims_ok(n, h, w) || w % 4)
      return MDE_ERR_INVALID_ARG;
    if (!bf_supported(cin, cout)) return MDE_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const double bytes = 2.0 * n * h * w * (double)(cin + cout);
    if (cin == 16)
      return launch_bf_wgrad<16, 16, 4, 4>((const bf16*)x, (const bf16*)gy, gweight, n, h, w,
                                           (float*)workspace, bytes, s);
    return launch_bf_wgrad<32, 32, 2, 2>((const bf16*)x, (const bf16*)gy, gweight, n, h, w,
                                         (float*)workspace, bytes, s);
  }
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !x || !gweight || !workspace || !dims_ok(n, h, w)) return MDE_ERR_INVALID_ARG;
  if (!supported(cin, cout, kWgrad)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const float* xi = (const float*)x;
  const float* g = (const float*)gy;
  float* ws = (float*)workspace;
  const double bytes = 4.0 * n * h * w * (double)(cin + cout);
  if (wide(cin, cout) || wide_pad(cin, cout))
    return launch_wgrad_wide(xi, g, gweight, n, cin, cout, h, w, ws, s);
  if (cin == 3 && cout == 16) return launch_wgrad<3, 16, 8, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 3 && cout == 32) return launch_wgrad<3, 32, 8, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 3) return launch_wgrad<3, 64, 4, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 16 && variant() == 1) return launch_wgrad<16, 16, 8, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 16 && variant() == 2) return launch_wgrad<16, 16, 4, 2>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (cin == 16) return launch_wgrad<16, 16, 4, 4>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (c32_wide(w)) return launch_wgrad_c32(xi, g, gweight, n, h, w, ws, s);
  if (variant() == 1) return launch_wgrad<32, 32, 4, 2>(xi, g, gweight, n, h, w, ws, bytes, s);
  if (variant() == 2) return launch_wgrad<32, 32, 4, 1>(xi, g, gweight, n, h, w, ws, bytes, s);
  return launch_wgrad<32, 32, 2, 2>(xi, g, gweight, n, h, w, ws, bytes, s);
}


/* Stride-2 3x3 weight gradient (k3 s2 p1, bias-free, NCHW fp32): x [n, cin, h, w]
 * (w even), gy [n, cout, (h-1)/2+1, (w-1)/2+1]; (cin, cout) = (3, 32) or (32, 32). */
int mde_conv3x3s2_supported(int64_t cin, int64_t cout, int dtype) {
  return dtype == MDE_F32 && (s2_supported(cin, cout) || wide(cin, cout)) ? 1 : 0;
}

size_t mde_conv3x3s2_wgrad_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                                     int dtype) {
  if (dtype != MDE_F32 || !s2_dims_ok(n, h, w)) return 0;
  if (wide(cin, cout)) {
    WidePlan wp;
    return wide_s2_plan(n, cin, cout, h, w, &wp) ? wide_workspace(wp) : 0;
  }
  if (!s2_supported(cin, cout)) return 0;
  if (c32_s2(cin, cout, w)) return c32_s2_workspace(n, h, w);
  const S2Plan p = cin == 3 ? s2_plan<3, 32>(n, h, w) : s2_plan<32, 32>(n, h, w);
  return wgrad_ws_bytes(1, p.grid, p.m);
}

int mde_conv3x3s2_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t cin,
                        int64_t cout, int64_t h, int64_t w, void* workspace, int dtype,
                        void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !x || !gweight || !workspace || !s2_dims_ok(n, h, w)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (wide(cin, cout))
    return launch_wgrad_wide_s2((const float*)x, (const float*)gy, gweight, n, cin, cout, h, w,
                                (float*)workspace, s);
  if (!s2_supported(cin, cout)) return MDE_ERR_UNSUPPORTED;
  if (c32_s2(cin, cout, w))
    return launch_wgrad_c32_s2((const float*)x, (const float*)gy, gweight, n, h, w,
                               (float*)workspace, s);
  if (cin == 3)
    return launch_wgrad_s2<3, 32>((const float*)x, (const float*)gy, gweight, n, h, w,
                                  (float*)workspace, s);
  return launch_wgrad_s2<32, 32>((const float*)x, (const float*)gy, gweight, n, h, w,
                                 (float*)workspace, s);
}

}  // extern "C"
