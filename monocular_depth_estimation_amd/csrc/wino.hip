// Winograd F(2x2, 3x3) for the wide stride-1 3x3 convolutions of DDRNet-23-slim
// (the BasicBlocks, DAPPM's process convs and the seg head:
// src/GuideDepth/model/DDRNet_23_slim.py:41-72,121-171,201-210, cfg2 at
// 120x160 / 60x80 / 30x40 / 15x20), forward and data gradient, NCHW fp32.
//
//   Y = A^T [ (G g G^T) (.) (B^T d B) ] A      (Lavin & Gray, F(2x2, 3x3))
//
// per 2x2 output tile: d = the 4x4 input patch (zero padded), g = a 3x3
// filter.  The 16 element-wise products, summed over input channels, are 16
// independent GEMMs  M[xi][co][tile] = sum_ci U[xi][co][ci] V[xi][ci][tile]:
// 16 MACs per 4 outputs instead of 36 (2.25x fewer MFMA cycles than the direct
// band-GEMM kernel, which runs at the fp32 MFMA rate MIOpen's Winograd matches).
//
//  * U = G g G^T is computed once per weight update by wino_weight_kernel
//    (16 x Cout x Cin floats, L2-resident) -- the data gradient uses the
//    flipped, transposed filter (a stride-1 / pad-1 3x3 conv's input gradient
//    is the same conv with g'[ci][co] = rot180(g[co][ci])).
//  * A block owns 4 x 8 tiles (8 x 16 output pixels) x CO_B output channels.
//    Per chunk of 16 input channels its 256 threads each transform two
//    (channel, tile) patches (B^T d B: adds only) into LDS
//    V[xi][tile half][ci][16]; the patches of the next chunk are loaded into
//    registers first (their latency hides behind the MFMAs).
//  * GEMMs on v_mfma_f32_16x16x4_f32 (exact fp32 products): a wave owns 16
//    output channels x 16 or 32 tiles for ALL 16 xi, so each lane ends with
//    the 16 xi values of its (channel, tile) pairs in registers and applies
//    A^T M A there -- no LDS round trip for the output transform.  B operand
//    reads V rows 4s + k at pitch 16: the four k-groups hit disjoint bank
//    ranges (conflict-free ds_read_b32); A comes from U as one float4 per
//    (xi, chunk) per lane (U's layout permuted so a lane's 4 k-steps are
//    contiguous).
// Exactness: B^T, A^T entries are 0 / +-1 and G's are 0 / +-1/2 (exact in
// binary); fp32 rounding of the transforms and the 16-term GEMM sums -- the
// GPU test holds it to 1e-5 of the output's max magnitude vs float64.
#include <cstdlib>

#include "common.h"

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int kCIC = 16;  // input channels per chunk (K = 4 MFMA steps of 4)
constexpr int kTRB = 4;   // tile rows per block (8 output rows)

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// wino_pad_ci / wino_pad_co (below) for device code
__device__ __forceinline__ int wino_pad_ci_d(int ci) { return (ci + kCIC - 1) / kCIC * kCIC; }
__device__ __forceinline__ int wino_pad_co_d(int co) { return co == 16 ? 16 : (co + 31) / 32 * 32; }

// One 2 x 2 output tile at dst (row pitch w), clipped to the plane.  add
// (nullable): the same tile of a gradient this result is summed into -- the
// data gradient's other half when the conv's input also feeds a residual add
// (mde_wino_conv_acc): one fp32 add per element, as autograd's accumulation.
__device__ __forceinline__ void store_tile(float* dst, const float* add, int oy, int ox, int h,
                                           int w, float y00, float y01, float y10, float y11) {
  if (add) {
    if (oy < h) {
      if (ox + 1 < w) {
        const float2 a = *reinterpret_cast<const float2*>(add);
        y00 = a.x + y00;
        y01 = a.y + y01;
      } else if (ox < w) {
        y00 = add[0] + y00;
      }
    }
    if (oy + 1 < h) {
      if (ox + 1 < w) {
        const float2 a = *reinterpret_cast<const float2*>(add + w);
        y10 = a.x + y10;
        y11 = a.y + y11;
      } else if (ox < w) {
        y10 = add[w] + y10;
      }
    }
  }
  if (oy < h) {
    if (ox + 1 < w) {
      *reinterpret_cast<float2*>(dst) = make_float2(y00, y01);
    } else if (ox < w) {
      dst[0] = y00;
    }
  }
  if (oy + 1 < h) {
    if (ox + 1 < w) {
      *reinterpret_cast<float2*>(dst + w) = make_float2(y10, y11);
    } else if (ox < w) {
      dst[w] = y10;
    }
  }
}

// offset of U[xi = 0] for (output channel co, input channel ci) of a conv with
// `nchunks` 16-channel input chunks; xi adds 256 (layout below)
__device__ __forceinline__ int64_t u_offset(int co, int ci, int nchunks) {
  const int chunk = ci / kCIC, s = (ci % kCIC) / 4, k = ci % 4;
  return ((((int64_t)(co / 16) * nchunks + chunk) * 16) * 64 + k * 16 + co % 16) * 4 + s;
}

// U[co / 16][chunk][xi][k][co % 16][s] (ci = 16 chunk + 4 s + k): one float4
// per lane (lane = co % 16 + 16 k) and (xi, chunk) holds its four k-steps, and
// a wave's 64 lanes read one contiguous KB per (xi, chunk): whole cache lines
// (the [co][chunk][xi][k][s] order of round 4 gave every load 16 half-line
// segments, and the texture addresser ran ~79 % busy at 32 channels).  FLIP: the data-gradient filter
// g'[co' = ci][ci' = co] = rot180(g[co][ci]) (co_n / ci_n are the output /
// input channels of the conv being RUN, i.e. swapped for FLIP).
// co_p / ci_p: the padded extents of U (wino_pad_*): padded rows are zeros.
template <bool FLIP>
__global__ void __launch_bounds__(256)
    wino_weight_kernel(const float* __restrict__ g, float* __restrict__ U, int co_n, int ci_n,
                       int co_p, int ci_p) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)co_p * ci_p) return;
  const int co = (int)(t / ci_p), ci = (int)(t % ci_p);
  float w[3][3];
  const bool real = co < co_n && ci < ci_n;
  const float* src = FLIP ? g + ((int64_t)ci * co_n + co) * 9 : g + ((int64_t)co * ci_n + ci) * 9;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      w[r][c] = !real ? 0.f : FLIP ? src[(2 - r) * 3 + (2 - c)] : src[r * 3 + c];
  // G w: rows (w0, (w0+w1+w2)/2, (w0-w1+w2)/2, w2), then the same on columns
  float a[4][3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    a[0][c] = w[0][c];
    a[1][c] = 0.5f * ((w[0][c] + w[1][c]) + w[2][c]);
    a[2][c] = 0.5f * ((w[0][c] - w[1][c]) + w[2][c]);
    a[3][c] = w[2][c];
  }
  float* dst = U + u_offset(co, ci, ci_p / kCIC);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float u[4] = {a[r][0], 0.5f * ((a[r][0] + a[r][1]) + a[r][2]),
                        0.5f * ((a[r][0] - a[r][1]) + a[r][2]), a[r][2]};
#pragma unroll
    for (int c = 0; c < 4; ++c) dst[(4 * r + c) * 256] = u[c];
  }
}

// Both transforms of one filter in one launch (the forward's U and the data
// gradient's flipped U'), one thread per (co, ci) of the FORWARD conv.
__device__ __forceinline__ void wino_g(const float (&w)[3][3], float (&u)[4][4]) {
  float a[4][3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    a[0][c] = w[0][c];
    a[1][c] = 0.5f * ((w[0][c] + w[1][c]) + w[2][c]);
    a[2][c] = 0.5f * ((w[0][c] - w[1][c]) + w[2][c]);
    a[3][c] = w[2][c];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    u[r][0] = a[r][0];
    u[r][1] = 0.5f * ((a[r][0] + a[r][1]) + a[r][2]);
    u[r][2] = 0.5f * ((a[r][0] - a[r][1]) + a[r][2]);
    u[r][3] = a[r][2];
  }
}

// Padded extents: U is (co_pu x ci_pu), U2 (ci_p2 x co_p2) = (padded cin as
// output channels x padded cout as input chunks); a thread per (co, ci) of
// the union, zeros outside the real filter.
__global__ void __launch_bounds__(256)
    wino_weight2_kernel(const float* __restrict__ g, float* __restrict__ U,
                        float* __restrict__ U2, int co_n, int ci_n, int co_pu, int ci_pu,
                        int ci_p2, int co_p2, int co_all, int ci_all) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)co_all * ci_all) return;
  const int co = (int)(t / ci_all), ci = (int)(t % ci_all);
  const bool real = co < co_n && ci < ci_n;
  const float* src = g + ((int64_t)co * ci_n + ci) * 9;
  float w[3][3], wf[3][3], u[4][4];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      w[r][c] = real ? src[r * 3 + c] : 0.f;
      wf[2 - r][2 - c] = w[r][c];
    }
  // forward: row co of the (co_n x ci_n) conv; flipped: row ci of (ci_n x co_n)
  if (co < co_pu && ci < ci_pu) {
    wino_g(w, u);
    float* dst = U + u_offset(co, ci, ci_pu / kCIC);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[(4 * r + c) * 256] = u[r][c];
  }
  if (ci < ci_p2 && co < co_p2) {
    wino_g(wf, u);
    float* dst = U2 + u_offset(ci, co, co_p2 / kCIC);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[(4 * r + c) * 256] = u[r][c];
  }
}

// Every Winograd filter of a forward in ONE launch (mde_wino_weight_table):
// table [rows][8] int64 = {weight, U, U' (0: none), cin, cout, first block,
// 0, 0} of each forward conv (cout x cin), blocks of 256 (co, ci) pairs over
// the union of both padded transforms, as wino_weight2_kernel (same values).
__global__ void __launch_bounds__(256)
    wino_weight_table_kernel(const int64_t* __restrict__ tab, int rows) {
  const int64_t b = blockIdx.x;
  int lo = 0, hi = rows - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[(int64_t)mid * 8 + 5] <= b) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* t = tab + (int64_t)lo * 8;
  const float* g = reinterpret_cast<const float*>(t[0]);
  float* U = reinterpret_cast<float*>(t[1]);
  float* U2 = reinterpret_cast<float*>(t[2]);
  const int ci_n = (int)t[3], co_n = (int)t[4];
  const int co_pu = wino_pad_co_d(co_n), ci_pu = wino_pad_ci_d(ci_n);
  const int ci_p2 = U2 ? wino_pad_co_d(ci_n) : 0, co_p2 = U2 ? wino_pad_ci_d(co_n) : 0;
  const int co_all = co_pu > co_p2 ? co_pu : co_p2, ci_all = ci_pu > ci_p2 ? ci_pu : ci_p2;
  const int64_t e = (b - t[5]) * 256 + threadIdx.x;
  if (e >= (int64_t)co_all * ci_all) return;
  const int co = (int)(e / ci_all), ci = (int)(e % ci_all);
  const bool real = co < co_n && ci < ci_n;
  const float* src = g + ((int64_t)co * ci_n + ci) * 9;
  float w[3][3], wf[3][3], u[4][4];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      w[r][c] = real ? src[r * 3 + c] : 0.f;
      wf[2 - r][2 - c] = w[r][c];
    }
  if (co < co_pu && ci < ci_pu) {
    wino_g(w, u);
    float* dst = U + u_offset(co, ci, ci_pu / kCIC);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[(4 * r + c) * 256] = u[r][c];
  }
  if (U2 && ci < ci_p2 && co < co_p2) {
    wino_g(wf, u);
    float* dst = U2 + u_offset(ci, co, co_p2 / kCIC);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[(4 * r + c) * 256] = u[r][c];
  }
}

// A block: 4 x TCB tiles (8 x 2 TCB output pixels) x CO_B output channels.
// CO_B = 64 (TCB 8): four waves along output channels, each with both 16-tile
// groups; CO_B = 32 (TCB 8): two waves along channels x two along tile groups;
// CO_B = 16 (TCB 16, the decoder's 16 -> 16 convs): one along channels x four.
// STATS: also the following BatchNorm's per-block statistics of y (as the
// direct conv's epilogue: stats[c][total / ncog][4] = (shift, count, s1, s2),
// one record per channel and pixel block; the shift is a sample of the channel).
template <int CO_B, int TCB, bool STATS = false, bool BPRE = false>
__global__ void __launch_bounds__(256, 2)
    wino_f23_kernel(const float* __restrict__ x, const float* __restrict__ U, float* __restrict__ y,
                    int ci_n, int co_n, int h, int w, int bcols, int brows, int ncog, int total,
                    float* __restrict__ stats, int xsplit, const float* __restrict__ add,
                    int nch) {
  constexpr int NTB = kTRB * TCB;      // tiles per block
  constexpr int NG = NTB / 16;         // 16-tile groups (MFMA N tiles)
  constexpr int WCO = CO_B / 16;       // waves along output channels
  constexpr int NTW = NG / (4 / WCO);  // 16-tile groups per wave
  constexpr int PPT = NTB * kCIC / 256;  // (channel, tile) patches per thread and chunk
  static_assert(NTW >= 1 && NTW * (4 / WCO) == NG, "wave tiling");
  // LDS floats per (xi, 16-tile group): [ci][16] + a pad that puts the groups
  // a wave's transform writes at once (2 groups x 2 channels, or 4 groups of
  // one channel) on disjoint banks: 32 / 16 (mod 64)
  constexpr int kVP = kCIC * 16 + (NG == 2 ? 32 : 16);
  __shared__ __attribute__((aligned(16))) float V[16][NG][kVP];

  // XCD-aware block order (blocks b, b + 8, ... share an XCD's L2): logical
  // block l -> (channel group fastest, so the groups reading one input tile
  // share that L2; then tile column, tile row, image).  xsplit > 1 (the
  // weight-heavy wide-Cout convs, where U outweighs the input): the 8 XCDs
  // form (8 / xsplit) tile ranges x xsplit channel-group ranges, so each XCD
  // streams only 1 / xsplit of U (see wino_xsplit).
  const int per = gridDim.x >> 3;
  const int xcd = blockIdx.x & 7, jx = blockIdx.x >> 3;
  int cog, tile;
  if (xsplit == 1) {
    const int l = xcd * per + jx;
    if (l >= total) return;
    cog = l % ncog;
    tile = l / ncog;
  } else {
    const int cpx = ncog / xsplit;  // channel groups per XCD
    const int tpx = per / cpx;      // tiles per XCD
    const int ntiles = total / ncog;
    cog = (xcd % xsplit) * cpx + jx % cpx;
    tile = (xcd / xsplit) * tpx + jx / cpx;
    if (tile >= ntiles) return;
  }
  int rest = tile;
  const int bc = rest % bcols;
  rest /= bcols;
  const int br = rest % brows;
  const int img = rest / brows;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, kq = lane >> 4;
  const int co0 = cog * CO_B + 16 * (wv % WCO);
  const int nt0 = (wv / WCO) * NTW;
  const int64_t hw = (int64_t)h * w;
  const float* xb = x + (int64_t)img * ci_n * hw;
  const int nchunks = nch;  // ci_n rounded up to 16 (its U rows past ci_n are zeros)
  const float* ua = U + ((int64_t)(co0 / 16) * nchunks * 16 * 64 + lane) * 4;

  // Input staging: per chunk, the block's 16 channels x 10 input rows x
  // (2 TCB + 4) columns (global column 2 bc TCB - 2 onward: even, so every
  // float2 is 8-byte aligned and lies wholly inside or outside the plane,
  // w even) are loaded as float2 row segments into registers (the next
  // chunk's while this one multiplies), written to LDS with the padding
  // zeroed, and each thread forms its (channel, tile) 4 x 4 patches from
  // there.  (One dword load per patch element made the texture addresser
  // ~70 % busy and cost 0.8 VMEM instructions per MFMA: SQ / TA counters,
  // profiles/r04_wino_pmc.txt.)
  constexpr int RR = 2 * kTRB + 2;        // input rows of a block
  constexpr int RW2 = TCB + 2;            // float2 per row (2 TCB + 4 columns)
  // LDS pitches for the patch reads (lane = tile: column 2 tc, row 2 tr; the
  // next 32 / 64 lanes the next channel): rows 2 tr at 16-bank steps
  // (2 RWP = 16 or 48 mod 64) and an odd channel pitch, so the 4 row groups of a
  // channel use disjoint even banks and the next channel the odd ones
  constexpr int RWP = 2 * RW2 <= 24 ? 24 : 40;  // 2 RWP = 48 or 16 (mod 64)
  constexpr int CPI = RR * RWP + 1;
  constexpr int RAW = kCIC * RR * RW2;    // float2 per chunk
  constexpr int RPT = (RAW + 255) / 256;  // float2 per thread
  __shared__ float raw[kCIC * CPI];
  const int gr0 = 2 * br * kTRB - 1, gc0 = 2 * bc * TCB - 2;
  float2 rv[RPT];
  auto load = [&](int chunk) {
    const float* src = xb + (int64_t)chunk * kCIC * hw;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int e = tid + 256 * k;
      const int ch = e / (RR * RW2), rem = e - ch * (RR * RW2);
      const int r = rem / RW2, c2 = rem - r * RW2;
      const int gr = gr0 + r, gc = gc0 + 2 * c2;
      const bool ok = e < RAW && gr >= 0 && gr < h && gc >= 0 && gc < w &&
                      chunk * kCIC + ch < ci_n;  // padded input channels read as zeros
      const int64_t off = ok ? (int64_t)(e < RAW ? ch : 0) * hw + (int64_t)gr * w + gc : 0;
      const float2 t = *reinterpret_cast<const float2*>(src + off);
      rv[k] = ok ? t : make_float2(0.f, 0.f);
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int e = tid + 256 * k;
      if (e < RAW) {
        const int ch = e / (RR * RW2), rem = e - ch * (RR * RW2);
        const int r = rem / RW2, c2 = rem - r * RW2;
        float* d = raw + ch * CPI + r * RWP + 2 * c2;
        d[0] = rv[k].x;
        d[1] = rv[k].y;
      }
    }
  };
  // B^T d B into V[xi][16-tile group][ci][16]; patch of tile (tr, tc): raw
  // rows 2 tr .. + 3, columns 2 tc + 1 .. + 4
  auto transform = [&]() {
#pragma unroll
    for (int pp = 0; pp < PPT; ++pp) {
      const int p = tid + 256 * pp, ch = p / NTB, tl = p % NTB;
      const float* q = raw + ch * CPI + 2 * (tl / TCB) * RWP + 2 * (tl % TCB) + 1;
      float d[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[i][j] = q[i * RWP + j];
      float t[4][4];  // B^T d: rows d0 - d2, d1 + d2, d2 - d1, d1 - d3
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[0][j] = d[0][j] - d[2][j];
        t[1][j] = d[1][j] + d[2][j];
        t[2][j] = d[2][j] - d[1][j];
        t[3][j] = d[1][j] - d[3][j];
      }
      float* dst = &V[0][tl >> 4][ch * 16 + (tl & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v[4] = {t[i][0] - t[i][2], t[i][1] + t[i][2], t[i][2] - t[i][1],
                            t[i][1] - t[i][3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[(4 * i + j) * NG * kVP] = v[j];
      }
    }
  };

  f4 acc[16][NTW];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[xi][n] = f4{0.f, 0.f, 0.f, 0.f};

  // A operands (U rows, L2-resident) through a 4-deep register ring: the
  // float4 of step xi is loaded 4 steps (>= 16 MFMAs) ahead, across the chunk
  // boundary too, so the L2 latency is never waited on right after the load
  constexpr int RING = 4;
  f4 ring[RING];
#pragma unroll
  for (int i = 0; i < RING; ++i) ring[i] = *reinterpret_cast<const f4*>(ua + i * 256);
  load(0);
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    __syncthreads();  // the previous chunk's V (and raw) readers are done
    stage();
    __syncthreads();
    if (chunk + 1 < nchunks) load(chunk + 1);
    transform();
    __syncthreads();
    const float* uc = ua + (int64_t)chunk * 4096;
    const float* un = ua + (int64_t)(chunk + 1 < nchunks ? chunk + 1 : chunk) * 4096;
    if constexpr (BPRE) {
      // B operands one xi step ahead in registers: step xi's LDS reads are in
      // flight during step xi - 1's MFMAs instead of waited on at its start
      float b[2][4][NTW];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int n = 0; n < NTW; ++n) b[0][s][n] = V[0][nt0 + n][(4 * s + kq) * 16 + li];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) {
        const f4 a = ring[xi % RING];
        ring[xi % RING] = *reinterpret_cast<const f4*>(
            xi + RING < 16 ? uc + (xi + RING) * 256 : un + (xi + RING - 16) * 256);
        if (xi + 1 < 16) {
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int n = 0; n < NTW; ++n)
              b[(xi + 1) & 1][s][n] = V[xi + 1 < 16 ? xi + 1 : 15][nt0 + n][(4 * s + kq) * 16 + li];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int n = 0; n < NTW; ++n) acc[xi][n] = mfma(a[s], b[xi & 1][s][n], acc[xi][n]);
      }
    } else {
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) {
        const f4 a = ring[xi % RING];
        ring[xi % RING] = *reinterpret_cast<const f4*>(
            xi + RING < 16 ? uc + (xi + RING) * 256 : un + (xi + RING - 16) * 256);
        // keep the load here: the scheduler otherwise sinks it next to its use
        // (register pressure) and every step waits on L2 again
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int n = 0; n < NTW; ++n)
            acc[xi][n] = mfma(a[s], V[xi][nt0 + n][(4 * s + kq) * 16 + li], acc[xi][n]);
      }
    }
  }

  // A^T M A per (channel, tile): lane holds channels co0 + 4 kq + r, tile 16 (nt0 + n) + li
  float* yb = y + (int64_t)img * co_n * hw;
  const float* ab = add ? add + (int64_t)img * co_n * hw : nullptr;
  mde::Sh run[STATS ? 4 : 1];
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    const int tl = 16 * (nt0 + n) + li;
    const int oy = 2 * (br * kTRB + tl / TCB), ox = 2 * (bc * TCB + tl % TCB);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float u0[4], u1[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float m0 = acc[b][n][r], m1 = acc[4 + b][n][r], m2 = acc[8 + b][n][r],
                    m3 = acc[12 + b][n][r];
        u0[b] = (m0 + m1) + m2;
        u1[b] = (m1 - m2) - m3;
      }
      const float y00 = (u0[0] + u0[1]) + u0[2], y01 = (u0[1] - u0[2]) - u0[3];
      const float y10 = (u1[0] + u1[1]) + u1[2], y11 = (u1[1] - u1[2]) - u1[3];
      if constexpr (STATS) {
        const bool ok0 = oy < h && ox < w, ok1 = oy + 1 < h && ox < w;
        if (n == 0)  // the shift: the channel's value at this wave's first tile (li = 0)
          run[r] = {__shfl(ok0 ? y00 : 0.f, lane & 48, 64), 0.f, 0.f, 0.f};
        mde::sh_add(run[r], y00, ok0);
        mde::sh_add(run[r], y01, ok0);
        mde::sh_add(run[r], y10, ok1);
        mde::sh_add(run[r], y11, ok1);
      }
      const int64_t yo = (int64_t)(co0 + 4 * kq + r) * hw + (int64_t)oy * w + ox;
      if (co0 + 4 * kq + r < co_n)  // padded output channels are not stored
        store_tile(yb + yo, ab ? ab + yo : nullptr, oy, ox, h, w, y00, y01, y10, y11);
    }
  }
  if constexpr (STATS) {
    // the 16 lanes of a k-group share its 4 channels: butterfly over li, then
    // the waves holding the same channels (other tile groups) merged in wave
    // order through LDS (V reused once every wave is past its last read)
    constexpr int NWN = 4 / WCO;  // waves per channel set
    __syncthreads();
    float* part = &V[0][0][0];  // [wave][16 channels][4]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mde::Sh a = run[r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) a = mde::sh_xor_sum(a, o);
      if (li == 0) {
        float* p4 = part + (wv * 16 + 4 * kq + r) * 4;
        p4[0] = a.ref;
        p4[1] = a.n;
        p4[2] = a.s1;
        p4[3] = a.s2;
      }
    }
    __syncthreads();
    if (tid < CO_B && cog * CO_B + tid < co_n) {
      const int wc = tid / 16, c16 = tid % 16;  // channel set (wave % WCO), channel within
      mde::Sh a{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NWN; ++k) {
        const float* p4 = part + ((k * WCO + wc) * 16 + c16) * 4;
        a = k == 0 ? mde::Sh{p4[0], p4[1], p4[2], p4[3]}
                   : mde::sh_merge(a, {p4[0], p4[1], p4[2], p4[3]});
      }
      const int G = total / ncog, gb = tile;
      float* o4 = stats + ((int64_t)(cog * CO_B + tid) * G + gb) * 4;
      o4[0] = a.ref;
      o4[1] = a.n;
      o4[2] = a.s1;
      o4[3] = a.s2;
    }
  }
}

// The 32-output-channel block (4 x 8 tiles x 32 channels) with the transform
// positions split across waves instead of the tiles: wave (cg = wv % 2,
// xh = wv / 2) owns channels 16 cg .. + 15, BOTH 16-tile groups and the eight
// positions xi = 8 xh .. + 7 (transform rows 2 xh, 2 xh + 1).  A wave then
// streams only half of its channels' U per chunk (8 whole-line float4 loads
// for its 64 MFMAs, the 64-channel block's ratio; wino_f23_kernel<32, 8>
// loads all 16 and shares them with no one), while its B reads and MFMAs stay
// as many.  A^T M A is linear in M, so each wave applies it to its half (the
// other rows zero) and the two halves are added: a wave hands its partial
// outputs of the tile group it does not store to its partner through LDS and
// stores the group it owns (xh) -- the same statistics layout as the tile
// split.  The halves are summed in a different order than the one-wave
// transform (not bitwise wino_f23_kernel; the float64 tests hold both).
// BPRE as wino_f23_kernel's.
template <bool STATS>
__global__ void __launch_bounds__(256, 2)
    wino_f23x_kernel(const float* __restrict__ x, const float* __restrict__ U, float* __restrict__ y,
                     int ci_n, int co_n, int h, int w, int bcols, int brows, int ncog, int total,
                     float* __restrict__ stats, const float* __restrict__ add) {
  constexpr int CO_B = 32, TCB = 8;
  constexpr int NTB = kTRB * TCB;  // 32 tiles
  constexpr int NG = NTB / 16;     // 2 tile groups, both in every wave
  constexpr int PPT = NTB * kCIC / 256;
  constexpr int kVP = kCIC * 16 + 32;
  __shared__ __attribute__((aligned(16))) float V[16][NG][kVP];

  const int per = gridDim.x >> 3;
  const int xcd = blockIdx.x & 7, jx = blockIdx.x >> 3;
  const int l = xcd * per + jx;
  if (l >= total) return;
  const int cog = l % ncog, tile = l / ncog;
  int rest = tile;
  const int bc = rest % bcols;
  rest /= bcols;
  const int br = rest % brows;
  const int img = rest / brows;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, kq = lane >> 4;
  const int cg = wv & 1, xh = wv >> 1;
  const int co0 = cog * CO_B + 16 * cg;
  const int64_t hw = (int64_t)h * w;
  const float* xb = x + (int64_t)img * ci_n * hw;
  const int nchunks = ci_n / kCIC;
  const float* ua = U + ((int64_t)(co0 / 16) * nchunks * 16 * 64 + lane) * 4 + 8 * xh * 256;

  constexpr int RR = 2 * kTRB + 2;
  constexpr int RW2 = TCB + 2;
  constexpr int RWP = 24;
  constexpr int CPI = RR * RWP + 1;
  constexpr int RAW = kCIC * RR * RW2;
  constexpr int RPT = (RAW + 255) / 256;
  __shared__ float raw[kCIC * CPI];
  const int gr0 = 2 * br * kTRB - 1, gc0 = 2 * bc * TCB - 2;
  float2 rv[RPT];
  auto load = [&](int chunk) {
    const float* src = xb + (int64_t)chunk * kCIC * hw;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int e = tid + 256 * k;
      const int ch = e / (RR * RW2), rem = e - ch * (RR * RW2);
      const int r = rem / RW2, c2 = rem - r * RW2;
      const int gr = gr0 + r, gc = gc0 + 2 * c2;
      const bool ok = e < RAW && gr >= 0 && gr < h && gc >= 0 && gc < w;
      const int64_t off = ok ? (int64_t)(e < RAW ? ch : 0) * hw + (int64_t)gr * w + gc : 0;
      const float2 t = *reinterpret_cast<const float2*>(src + off);
      rv[k] = ok ? t : make_float2(0.f, 0.f);
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int e = tid + 256 * k;
      if (e < RAW) {
        const int ch = e / (RR * RW2), rem = e - ch * (RR * RW2);
        const int r = rem / RW2, c2 = rem - r * RW2;
        float* d = raw + ch * CPI + r * RWP + 2 * c2;
        d[0] = rv[k].x;
        d[1] = rv[k].y;
      }
    }
  };
  auto transform = [&]() {
#pragma unroll
    for (int pp = 0; pp < PPT; ++pp) {
      const int p = tid + 256 * pp, ch = p / NTB, tl = p % NTB;
      const float* q = raw + ch * CPI + 2 * (tl / TCB) * RWP + 2 * (tl % TCB) + 1;
      float d[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[i][j] = q[i * RWP + j];
      float t[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[0][j] = d[0][j] - d[2][j];
        t[1][j] = d[1][j] + d[2][j];
        t[2][j] = d[2][j] - d[1][j];
        t[3][j] = d[1][j] - d[3][j];
      }
      float* dst = &V[0][tl >> 4][ch * 16 + (tl & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v[4] = {t[i][0] - t[i][2], t[i][1] + t[i][2], t[i][2] - t[i][1],
                            t[i][1] - t[i][3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[(4 * i + j) * NG * kVP] = v[j];
      }
    }
  };

  f4 acc[8][NG];  // [position 8 xh + xi][tile group]
#pragma unroll
  for (int xi = 0; xi < 8; ++xi)
#pragma unroll
    for (int n = 0; n < NG; ++n) acc[xi][n] = f4{0.f, 0.f, 0.f, 0.f};

  constexpr int RING = 4;
  f4 ring[RING];
#pragma unroll
  for (int i = 0; i < RING; ++i) ring[i] = *reinterpret_cast<const f4*>(ua + i * 256);
  load(0);
  const int xo = 8 * xh;  // this wave's first transform position
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    __syncthreads();
    stage();
    __syncthreads();
    if (chunk + 1 < nchunks) load(chunk + 1);
    transform();
    __syncthreads();
    const float* uc = ua + (int64_t)chunk * 4096;
    const float* un = ua + (int64_t)(chunk + 1 < nchunks ? chunk + 1 : chunk) * 4096;
    float b[2][4][NG];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int n = 0; n < NG; ++n) b[0][s][n] = V[xo][n][(4 * s + kq) * 16 + li];
#pragma unroll
    for (int xi = 0; xi < 8; ++xi) {
      const f4 a = ring[xi % RING];
      ring[xi % RING] = *reinterpret_cast<const f4*>(
          xi + RING < 8 ? uc + (xi + RING) * 256 : un + (xi + RING - 8) * 256);
      if (xi + 1 < 8) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int n = 0; n < NG; ++n)
            b[(xi + 1) & 1][s][n] = V[xo + (xi + 1 < 8 ? xi + 1 : 7)][n][(4 * s + kq) * 16 + li];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int n = 0; n < NG; ++n) acc[xi][n] = mfma(a[s], b[xi & 1][s][n], acc[xi][n]);
    }
  }

  // partial A^T M A of this wave's rows: row pair (2 xh, 2 xh + 1) of M[4][4];
  // A^T = [1 1 1 0; 0 1 -1 -1] -> u0 gets rows 0, 1, 2 and u1 rows 1, -2, -3
  auto partial = [&](int n, int r, float (&out)[4]) {
    float u0[4], u1[4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const float ma = acc[bb][n][r], mb = acc[4 + bb][n][r];  // rows 2 xh, 2 xh + 1
      if (xh == 0) {  // rows 0, 1
        u0[bb] = ma + mb;
        u1[bb] = mb;
      } else {  // rows 2, 3
        u0[bb] = ma;
        u1[bb] = -ma - mb;
      }
    }
    out[0] = (u0[0] + u0[1]) + u0[2];
    out[1] = (u0[1] - u0[2]) - u0[3];
    out[2] = (u1[0] + u1[1]) + u1[2];
    out[3] = (u1[1] - u1[2]) - u1[3];
  };
  // hand the partner (same channels, other rows) the group it stores
  __syncthreads();  // every wave is past its last V read
  float* xch = &V[0][0][0];  // [cg][group][r][4][64 lanes]
  // (the group index stays a compile-time constant under a wave-uniform
  // branch: an accumulator indexed at run time would live in scratch)
#pragma unroll
  for (int ng = 0; ng < NG; ++ng) {
    if (ng != xh) {  // the group the partner stores
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float o[4];
        partial(ng, r, o);
#pragma unroll
        for (int q = 0; q < 4; ++q) xch[(((cg * 2 + ng) * 4 + r) * 4 + q) * 64 + lane] = o[q];
      }
    }
  }
  __syncthreads();
  float* yb = y + (int64_t)img * co_n * hw;
  const float* ab = add ? add + (int64_t)img * co_n * hw : nullptr;
  const int n = xh;  // the group this wave stores
  const int tl = 16 * n + li;
  const int oy = 2 * (br * kTRB + tl / TCB), ox = 2 * (bc * TCB + tl % TCB);
  mde::Sh run[STATS ? 4 : 1];
  float own[4][4];
#pragma unroll
  for (int ng = 0; ng < NG; ++ng)
    if (ng == xh)
#pragma unroll
      for (int r = 0; r < 4; ++r) partial(ng, r, own[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float* o = own[r];
    const float* pp = xch + ((cg * 2 + n) * 4 + r) * 4 * 64 + lane;
    // rows 0-1 partial + rows 2-3 partial, in that order whichever wave stores
    const float y00 = xh == 0 ? o[0] + pp[0] : pp[0] + o[0];
    const float y01 = xh == 0 ? o[1] + pp[64] : pp[64] + o[1];
    const float y10 = xh == 0 ? o[2] + pp[128] : pp[128] + o[2];
    const float y11 = xh == 0 ? o[3] + pp[192] : pp[192] + o[3];
    if constexpr (STATS) {
      const bool ok0 = oy < h && ox < w, ok1 = oy + 1 < h && ox < w;
      run[r] = {__shfl(ok0 ? y00 : 0.f, lane & 48, 64), 0.f, 0.f, 0.f};
      mde::sh_add(run[r], y00, ok0);
      mde::sh_add(run[r], y01, ok0);
      mde::sh_add(run[r], y10, ok1);
      mde::sh_add(run[r], y11, ok1);
    }
    const int64_t yo = (int64_t)(co0 + 4 * kq + r) * hw + (int64_t)oy * w + ox;
    store_tile(yb + yo, ab ? ab + yo : nullptr, oy, ox, h, w, y00, y01, y10, y11);
  }
  if constexpr (STATS) {
    // as wino_f23_kernel's: butterfly over the 16 tiles, then the two waves
    // holding a channel set (its two tile groups) merged in wave order
    __syncthreads();
    float* part = &V[0][0][0] + 8192;  // past the exchange slots
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mde::Sh a = run[r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) a = mde::sh_xor_sum(a, o);
      if (li == 0) {
        float* p4 = part + (wv * 16 + 4 * kq + r) * 4;
        p4[0] = a.ref;
        p4[1] = a.n;
        p4[2] = a.s1;
        p4[3] = a.s2;
      }
    }
    __syncthreads();
    if (tid < CO_B) {
      const int wc = tid / 16, c16 = tid % 16;
      mde::Sh a{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const float* p4 = part + ((k * 2 + wc) * 16 + c16) * 4;
        a = k == 0 ? mde::Sh{p4[0], p4[1], p4[2], p4[3]}
                   : mde::sh_merge(a, {p4[0], p4[1], p4[2], p4[3]});
      }
      const int G = total / ncog, gb = tile;
      float* o4 = stats + ((int64_t)(cog * CO_B + tid) * G + gb) * 4;
      o4[0] = a.ref;
      o4[1] = a.n;
      o4[2] = a.s1;
      o4[3] = a.s2;
    }
  }
}

// Persistent variant (the activation-heavy convs, xsplit == 1).  The blocks
// of an XCD split its contiguous share of the (channel group, tile block)
// items into runs of `ipb`; a block walks its run with ONE chunk pipeline
// across item boundaries, so the next (item, chunk)'s input rows are in
// flight while this one's transform, its MFMAs and -- at an item's last
// chunk -- its output transform and stores run.  The ISA count of
// wino_f23_kernel showed why: ~1,000 instructions a wave of per-block setup
// (64-bit staging addresses and bounds masks, accumulator zeroing) and ~230
// of epilogue against ~340 per 16-channel chunk, so the 32-channel convs (two
// chunks an item) spent over half their time outside the MFMA loop.  Here a
// thread's staging units are planned once per block; an item costs one
// bounds pass over them (7 offsets), the loads are 32-bit-offset buffer loads
// of the chunk's 16 planes (an out-of-plane unit reads past the buffer:
// zeros, no select), and interior tile blocks store with no per-tile tests.
// Same products, same summation order: bitwise the results of wino_f23_kernel.
template <int CO_B, int TCB, bool STATS = false>
__global__ void __launch_bounds__(256, 2)
    wino_f23p_kernel(const float* __restrict__ x, const float* __restrict__ U, float* __restrict__ y,
                     int ci_n, int co_n, int h, int w, int bcols, int brows, int ncog, int total,
                     float* __restrict__ stats, int per_xcd, int ipb,
                     const float* __restrict__ add) {
  constexpr int NTB = kTRB * TCB;
  constexpr int NG = NTB / 16;
  constexpr int WCO = CO_B / 16;
  constexpr int NTW = NG / (4 / WCO);
  constexpr int PPT = NTB * kCIC / 256;
  static_assert(NTW >= 1 && NTW * (4 / WCO) == NG, "wave tiling");
  constexpr int kVP = kCIC * 16 + (NG == 2 ? 32 : 16);
  __shared__ __attribute__((aligned(16))) float V[16][NG][kVP];
  constexpr int RR = 2 * kTRB + 2;
  constexpr int RW2 = TCB + 2;
  constexpr int RWP = 2 * RW2 <= 24 ? 24 : 40;
  constexpr int CPI = RR * RWP + 1;
  constexpr int RAW = kCIC * RR * RW2;
  constexpr int RPT = (RAW + 255) / 256;
  __shared__ float raw[kCIC * CPI];

  const int xcd = blockIdx.x & 7, jx = blockIdx.x >> 3;
  const int lb = xcd * per_xcd + jx * ipb;
  int le = lb + ipb;
  if (le > (xcd + 1) * per_xcd) le = (xcd + 1) * per_xcd;
  if (le > total) le = total;
  if (lb >= le) return;
  const int nchunks = ci_n / kCIC;
  const int nsteps = (le - lb) * nchunks;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, kq = lane >> 4;
  const int hw = h * w;  // < 2^24 (wino_persistent_ok)

  // a thread's staging units, tile independent: plane offset within the
  // block's window and (row, column) of the window for the bounds pass
  int rel[RPT], rcw[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int e = tid + 256 * k;
    const int ch = e / (RR * RW2), rem = e - ch * (RR * RW2);
    const int r = rem / RW2, c2 = rem - r * RW2;
    rel[k] = ch * hw + r * w + 2 * c2;
    rcw[k] = e < RAW ? (r << 16) | (2 * c2) : 0x7fff0000;  // row 32767: never in the plane
  }
  uint32_t voff[RPT];
  // the bounds pass of an item: byte offsets within the chunk's 16 planes
  auto item_offsets = [&](int gr0, int gc0) {
    const int base = gr0 * w + gc0;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int gr = gr0 + (rcw[k] >> 16), gc = gc0 + (rcw[k] & 0xffff);
      const bool ok = (unsigned)gr < (unsigned)h && (unsigned)gc < (unsigned)w;
      voff[k] = ok ? (uint32_t)(4 * (base + rel[k])) : 0x7ffffff0u;
    }
  };
  using u2v = uint32_t __attribute__((ext_vector_type(2)));
  float2 rv[RPT];
  auto load = [&](int img, int chunk) {
    const uint64_t a = (uint64_t)(x + ((int64_t)img * ci_n + (int64_t)chunk * kCIC) * hw);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, 4 * kCIC * hw, 0x00020000);
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const u2v t = __builtin_bit_cast(u2v, __builtin_amdgcn_raw_buffer_load_b64(R, voff[k], 0, 0));
      rv[k] = make_float2(__uint_as_float(t.x), __uint_as_float(t.y));
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int e = tid + 256 * k;
      if (e < RAW) {
        const int ch = e / (RR * RW2), rem = e - ch * (RR * RW2);
        const int r = rem / RW2, c2 = rem - r * RW2;
        float* d = raw + ch * CPI + r * RWP + 2 * c2;
        d[0] = rv[k].x;
        d[1] = rv[k].y;
      }
    }
  };
  auto transform = [&]() {
#pragma unroll
    for (int pp = 0; pp < PPT; ++pp) {
      const int p = tid + 256 * pp, ch = p / NTB, tl = p % NTB;
      const float* q = raw + ch * CPI + 2 * (tl / TCB) * RWP + 2 * (tl % TCB) + 1;
      float d[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[i][j] = q[i * RWP + j];
      float t[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[0][j] = d[0][j] - d[2][j];
        t[1][j] = d[1][j] + d[2][j];
        t[2][j] = d[2][j] - d[1][j];
        t[3][j] = d[1][j] - d[3][j];
      }
      float* dst = &V[0][tl >> 4][ch * 16 + (tl & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v[4] = {t[i][0] - t[i][2], t[i][1] + t[i][2], t[i][2] - t[i][1],
                            t[i][1] - t[i][3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[(4 * i + j) * NG * kVP] = v[j];
      }
    }
  };
  // item l -> (channel group, image, block row, block column): the order of
  // wino_f23_kernel's logical blocks (channel group fastest)
  auto decode = [&](int l, int& cog, int& img, int& br, int& bc) {
    cog = l % ncog;
    int rest = l / ncog;
    bc = rest % bcols;
    rest /= bcols;
    br = rest % brows;
    img = rest / brows;
  };
  // the lane's U row of a (channel group, chunk): a fixed lane part + a uniform step
  const float* ulane = U + ((int64_t)(wv % WCO) * nchunks * 16 * 64 + lane) * 4;
  auto uptr = [&](int cog, int chunk) {
    return ulane + (int64_t)(cog * (CO_B / 16) * nchunks + chunk) * 4096;
  };

  f4 acc[16][NTW];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[xi][n] = f4{0.f, 0.f, 0.f, 0.f};

  int it = lb, chunk = 0;  // the current step's item and chunk
  int cog, img, br, bc;
  decode(it, cog, img, br, bc);
  item_offsets(2 * br * kTRB - 1, 2 * bc * TCB - 2);
  constexpr int RING = 4;
  f4 ring[RING];
  {
    const float* u0 = uptr(cog, 0);
#pragma unroll
    for (int i = 0; i < RING; ++i) ring[i] = *reinterpret_cast<const f4*>(u0 + i * 256);
  }
  load(img, 0);
  const int nt0 = (wv / WCO) * NTW;
  for (int s = 0; s < nsteps; ++s) {
    __syncthreads();  // the previous step's V (and raw) readers are done
    stage();
    __syncthreads();
    int it_n = it, chunk_n = chunk + 1;
    if (chunk_n == nchunks) {
      chunk_n = 0;
      ++it_n;
    }
    const bool more = s + 1 < nsteps;
    int cog_n = cog, img_n = img, br_n = br, bc_n = bc;
    if (chunk_n == 0) {  // the next item: decode's order, stepped without divisions
      if (++cog_n == ncog) {
        cog_n = 0;
        if (++bc_n == bcols) {
          bc_n = 0;
          if (++br_n == brows) {
            br_n = 0;
            ++img_n;
          }
        }
      }
    }
    if (more) {
      if (chunk_n == 0) item_offsets(2 * br_n * kTRB - 1, 2 * bc_n * TCB - 2);
      load(img_n, chunk_n);
    }
    transform();
    __syncthreads();
    const float* uc = uptr(cog, chunk);
    const float* un = more ? uptr(cog_n, chunk_n) : uc;
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
      const f4 a = ring[xi % RING];
      ring[xi % RING] = *reinterpret_cast<const f4*>(
          xi + RING < 16 ? uc + (xi + RING) * 256 : un + (xi + RING - 16) * 256);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int n = 0; n < NTW; ++n)
          acc[xi][n] = mfma(a[s4], V[xi][nt0 + n][(4 * s4 + kq) * 16 + li], acc[xi][n]);
    }

    if (chunk == nchunks - 1) {  // the item's output transform, stores (+ statistics)
      const int co0 = cog * CO_B + 16 * (wv % WCO);
      float* yb = y + (int64_t)img * co_n * hw;
      const float* ab = add ? add + (int64_t)img * co_n * hw : nullptr;
      // every output pixel of the tile block inside the plane: no per-pixel tests
      const bool inner = 2 * (br + 1) * kTRB <= h && 2 * (bc + 1) * TCB <= w;
      mde::Sh run[STATS ? 4 : 1];
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
        const int tl = 16 * (nt0 + n) + li;
        const int oy = 2 * (br * kTRB + tl / TCB), ox = 2 * (bc * TCB + tl % TCB);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float u0[4], u1[4];
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const float m0 = acc[b][n][r], m1 = acc[4 + b][n][r], m2 = acc[8 + b][n][r],
                        m3 = acc[12 + b][n][r];
            u0[b] = (m0 + m1) + m2;
            u1[b] = (m1 - m2) - m3;
          }
          const float y00 = (u0[0] + u0[1]) + u0[2], y01 = (u0[1] - u0[2]) - u0[3];
          const float y10 = (u1[0] + u1[1]) + u1[2], y11 = (u1[1] - u1[2]) - u1[3];
          if constexpr (STATS) {
            const bool ok0 = oy < h && ox < w, ok1 = oy + 1 < h && ox < w;
            if (n == 0)
              run[r] = {__shfl(ok0 ? y00 : 0.f, lane & 48, 64), 0.f, 0.f, 0.f};
            mde::sh_add(run[r], y00, ok0);
            mde::sh_add(run[r], y01, ok0);
            mde::sh_add(run[r], y10, ok1);
            mde::sh_add(run[r], y11, ok1);
          }
          const int64_t yo = (int64_t)(co0 + 4 * kq + r) * hw + oy * w + ox;
          float* dst = yb + yo;
          if (inner && !ab) {
            *reinterpret_cast<float2*>(dst) = make_float2(y00, y01);
            *reinterpret_cast<float2*>(dst + w) = make_float2(y10, y11);
          } else {
            store_tile(dst, ab ? ab + yo : nullptr, oy, ox, h, w, y00, y01, y10, y11);
          }
        }
      }
      if constexpr (STATS) {
        constexpr int NWN = 4 / WCO;
        __syncthreads();  // every wave is past its last V read of this step
        float* part = &V[0][0][0];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          mde::Sh a = run[r];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) a = mde::sh_xor_sum(a, o);
          if (li == 0) {
            float* p4 = part + (wv * 16 + 4 * kq + r) * 4;
            p4[0] = a.ref;
            p4[1] = a.n;
            p4[2] = a.s1;
            p4[3] = a.s2;
          }
        }
        __syncthreads();
        if (tid < CO_B) {
          const int wc = tid / 16, c16 = tid % 16;
          mde::Sh a{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < NWN; ++k) {
            const float* p4 = part + ((k * WCO + wc) * 16 + c16) * 4;
            a = k == 0 ? mde::Sh{p4[0], p4[1], p4[2], p4[3]}
                       : mde::sh_merge(a, {p4[0], p4[1], p4[2], p4[3]});
          }
          const int G = total / ncog, gb = it / ncog;
          float* o4 = stats + ((int64_t)(cog * CO_B + tid) * G + gb) * 4;
          o4[0] = a.ref;
          o4[1] = a.n;
          o4[2] = a.s1;
          o4[3] = a.s2;
        }
      }
#pragma unroll
      for (int xi = 0; xi < 16; ++xi)
#pragma unroll
        for (int n = 0; n < NTW; ++n) acc[xi][n] = f4{0.f, 0.f, 0.f, 0.f};
    }
    it = it_n;
    chunk = chunk_n;
    cog = cog_n;
    img = img_n;
    br = br_n;
    bc = bc_n;
  }
}

struct WinoGeo {
  int bcols, brows, ncog, co_b;
  int ci_p, co_p;  // padded channel counts (U's extents; padded rows / columns are zeros)
  int64_t total;
};

// Channel padding (round 6, the NewCRF projections the 32 / 16 alignment
// rules sent to MIOpen: proj_x 24 -> 128 and 40 -> 256 and the data
// gradients 128 -> 24, 256 -> 40, 512 -> 112; newcrf_layers.py:384-392):
// input channels to a multiple of 16 (the chunk; the extra planes read as
// zeros), output channels to a multiple of 32 (16 stays 16; the extra
// channels are computed from zero filter rows and not stored).  Taken while
// the padded product stays within 2x the real one.
inline int wino_pad_ci(int64_t ci) { return (int)mde::cdiv(ci, kCIC) * kCIC; }
inline int wino_pad_co(int64_t co) { return co == 16 ? 16 : (int)mde::cdiv(co, 32) * 32; }

inline bool wino_geo(int64_t n, int64_t ci, int64_t co, int64_t h, int64_t w, WinoGeo* g) {
  if (n <= 0 || ci < 1 || co < 1 || h < 1 || w < 2 || ci > 65536 || co > 65536) return false;
  g->ci_p = wino_pad_ci(ci);
  g->co_p = wino_pad_co(co);
  if ((int64_t)g->ci_p * g->co_p > 2 * ci * co) return false;  // padding must not double the work
  if (w % 2) return false;  // float2 output stores at even offsets
  if (n * g->ci_p * h * w >= ((int64_t)1 << 31) || n * g->co_p * h * w >= ((int64_t)1 << 31))
    return false;
  g->co_b = g->co_p % 64 == 0 ? 64 : (g->co_p == 16 ? 16 : 32);
  g->ncog = (int)(g->co_p / g->co_b);
  g->bcols = (int)mde::cdiv(w, g->co_b == 16 ? 32 : 16);
  g->brows = (int)mde::cdiv(h, 2 * kTRB);
  g->total = n * g->ncog * g->bcols * g->brows;
  return g->total < 0x7fffffff;
}

// XCD split of a launch (wino_f23_kernel's xsplit): each XCD's L2 sees every
// block of its share, so with B channel-group ranges x 8 / B tile ranges the
// XCDs together fetch U about 8 / B times and the input about B times
// (bytes: U = 16 cin cout floats, x = n cin h w floats).  B = 1 (the
// activation-heavy DDRNet convs) keeps the original walk; the NewCRF
// projections at 1/16 and 1/32 (Cout 512-1024 on 30x40 / 15x20 planes) are
// weight-heavy.  MDE_WINO_XSPLIT=1/2/4/8 forces one (where Cout allows).
inline int wino_xsplit(int64_t n, int64_t ci, int64_t co, int64_t h, int64_t w,
                       const WinoGeo& g) {
  static const int forced = [] {
    const char* e = std::getenv("MDE_WINO_XSPLIT");
    return e ? std::atoi(e) : 0;
  }();
  const double u = 16.0 * ci * co, x = (double)n * ci * h * w;
  int best = 1;
  double best_b = 8 * u + x;
  for (int b = 2; b <= 8; b *= 2) {
    if (g.ncog % b) break;
    if (forced) {
      if (b == forced) return b;
      continue;
    }
    const double bytes = 8 / b * u + b * x;
    if (bytes < 0.8 * best_b) best = b, best_b = bytes;
  }
  return best;
}

// wino_f23p_kernel (persistent) where it applies: mode 1 (MDE_WINO_P=1 at
// load, mde_wino_mode at run time), or 0 = the one-item-a-block kernel, the
// default: measured per shape at bs 32 (tools/wino_bench.py --modes 0,1,
// profiles/r06_wino_persistent_ab.txt) the persistent kernel is no faster on
// the routed shapes (32 -> 32 @120x160 103.7 -> 102.1 us, @240x320 408 -> 419,
// 64 -> 64 @60x80 72 -> 78, 128 -> 128 @30x40 73 -> 91) and the cfg2 step went
// 982.7 -> 968.1 img/s: the per-block setup it removes was already hidden by
// the CU's second block; the loop itself is bound by the texture addresser
// (16 dwordx4 U loads a wave and chunk).  Only 16 -> 16 gains (994 -> 689 us),
// which stays on the direct kernel (520 us).  Its byte offsets within a
// chunk's 16 planes (64 h w < 2^30, below the out-of-plane offset) and packed
// (row, column) staging units need h * w < 2^24 and h, w < 32767.
int g_wino_mode = [] {
  const char* e = std::getenv("MDE_WINO_P");
  return e && e[0] == '1' ? 1 : 0;
}();

// B operands prefetched one xi step ahead (wino_f23_kernel BPRE): mode bit 2
// of mde_wino_mode, MDE_WINO_BPRE at load (A/B)
int g_wino_bpre = [] {
  const char* e = std::getenv("MDE_WINO_BPRE");
  return e && e[0] == '0' ? 0 : 1;
}();
// the 32-channel blocks on wino_f23x_kernel (positions split across waves):
// mode bit 4, MDE_WINO_X at load
int g_wino_x = [] {
  const char* e = std::getenv("MDE_WINO_X");
  return e && e[0] == '1' ? 1 : 0;
}();

inline bool wino_persistent_ok(int64_t h, int64_t w) {
  return g_wino_mode == 1 && h * w < ((int64_t)1 << 24) && h < 32767 && w < 32767;
}

// items a persistent block walks (MDE_WINO_IPB; 0 = the share of two blocks a CU)
inline int wino_ipb() {
  static const int v = [] {
    const char* e = std::getenv("MDE_WINO_IPB");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

inline int wino_cus() {
  static const int cus = [] {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    return c > 0 ? c : 256;
  }();
  return cus;
}

}  // namespace

extern "C" {

// 1 when the Winograd kernels take a stride-1 / pad-1 3x3 conv of these
// channels and plane (this pass: the conv actually run, i.e. (cout, cin) swapped
// for the data gradient); the caller applies its own size thresholds.
int mde_wino_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype) {
  WinoGeo g;
  return dtype == MDE_F32 && wino_geo(1, cin, cout, h, w, &g) ? 1 : 0;
}

int mde_wino_mode(int mode) {
  const int prev = g_wino_mode | (g_wino_bpre << 1) | (g_wino_x << 2);
  if (mode >= 0 && mode <= 7) {
    g_wino_mode = mode & 1;
    g_wino_bpre = (mode >> 1) & 1;
    g_wino_x = (mode >> 2) & 1;
  }
  return prev;
}

// U of the forward conv (cout x cin) and of its data gradient (cin x cout),
// padded (wino_pad_*): the larger of the two, so one size serves both.
size_t mde_wino_weight_bytes(int64_t cin, int64_t cout) {
  if (cin < 1 || cout < 1) return 0;
  const size_t f = (size_t)wino_pad_co(cout) * (size_t)wino_pad_ci(cin);
  const size_t b = (size_t)wino_pad_co(cin) * (size_t)wino_pad_ci(cout);
  return sizeof(float) * 16 * (f > b ? f : b);
}

// U from the [cout][cin][3][3] filter of the FORWARD conv; flip = 1 gives the
// data-gradient transform (U' for the conv cout -> cin).
int mde_wino_weight(const float* weight, float* u, int64_t cin, int64_t cout, int flip,
                    void* stream) {
  if (!weight || !u || cin < 1 || cout < 1 || cin > 65536 || cout > 65536)
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t pairs = cin * cout;
  // the run conv: cout -> cin for the data gradient
  const int co_r = (int)(flip ? cin : cout), ci_r = (int)(flip ? cout : cin);
  const int co_p = wino_pad_co(co_r), ci_p = wino_pad_ci(ci_r);
  const dim3 grid((unsigned)mde::cdiv((int64_t)co_p * ci_p, 256));
  if (flip)
    MDE_LAUNCH(mde::K_WINO_WEIGHT, 4.0 * pairs * 9 + 64.0 * co_p * ci_p, s,
               wino_weight_kernel<true>, grid, dim3(256), 0, weight, u, co_r, ci_r, co_p, ci_p);
  else
    MDE_LAUNCH(mde::K_WINO_WEIGHT, 4.0 * pairs * 9 + 64.0 * co_p * ci_p, s,
               wino_weight_kernel<false>, grid, dim3(256), 0, weight, u, co_r, ci_r, co_p, ci_p);
  return MDE_OK;
}

// Both transforms at once: u for the forward conv, u_flip for its data
// gradient (as mde_wino_weight with flip = 0 / 1).
int mde_wino_weight2(const float* weight, float* u, float* u_flip, int64_t cin, int64_t cout,
                     void* stream) {
  if (!weight || !u || !u_flip || cin < 1 || cout < 1 || cin > 65536 || cout > 65536)
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t pairs = cin * cout;
  const int co_pu = wino_pad_co(cout), ci_pu = wino_pad_ci(cin);  // forward: cout x cin
  const int ci_p2 = wino_pad_co(cin), co_p2 = wino_pad_ci(cout);  // data gradient: cin x cout
  const int co_all = co_pu > co_p2 ? co_pu : co_p2, ci_all = ci_pu > ci_p2 ? ci_pu : ci_p2;
  MDE_LAUNCH(mde::K_WINO_WEIGHT,
             4.0 * pairs * 9 + 64.0 * ((double)co_pu * ci_pu + (double)ci_p2 * co_p2), s,
             wino_weight2_kernel, dim3((unsigned)mde::cdiv((int64_t)co_all * ci_all, 256)),
             dim3(256), 0, weight, u, u_flip, (int)cout, (int)cin, co_pu, ci_pu, ci_p2, co_p2,
             co_all, ci_all);
  return MDE_OK;
}

// the 256-pair blocks of one table row (mde_wino_weight_table)
int64_t mde_wino_weight_blocks(int64_t cin, int64_t cout, int both) {
  if (cin < 1 || cout < 1 || cin > 65536 || cout > 65536) return 0;
  const int64_t co_pu = wino_pad_co(cout), ci_pu = wino_pad_ci(cin);
  const int64_t ci_p2 = both ? wino_pad_co(cin) : 0, co_p2 = both ? wino_pad_ci(cout) : 0;
  const int64_t co_all = co_pu > co_p2 ? co_pu : co_p2, ci_all = ci_pu > ci_p2 ? ci_pu : ci_p2;
  return mde::cdiv(co_all * ci_all, 256);
}

int mde_wino_weight_table(const int64_t* table, int rows, int64_t blocks, int64_t pairs,
                          void* stream) {
  if (!table || rows <= 0 || blocks <= 0 || blocks > 0x7fffffff || pairs < 0)
    return MDE_ERR_INVALID_ARG;
  MDE_LAUNCH(mde::K_WINO_WEIGHT, 4.0 * 9 * pairs + 128.0 * pairs, (hipStream_t)stream,
             wino_weight_table_kernel, dim3((unsigned)blocks), dim3(256), 0, table, rows);
  return MDE_OK;
}

// y[n][cout][h][w] = conv3x3(x[n][cin][h][w]) (stride 1, pad 1) from U =
// mde_wino_weight(..).  `pass` 0 = forward, 1 = data gradient (timing id only).
}  // extern "C"

namespace {

int wino_launch(const float* x, const float* u, float* y, float* stats, const float* add,
                int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, int pass, int dtype,
                void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !u || !y) return MDE_ERR_INVALID_ARG;
  WinoGeo g;
  if (!wino_geo(n, cin, cout, h, w, &g)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  // the MFMA work the kernel does: 16 MACs per 2 x 2 tile and (cin, cout) pair
  // (the direct conv's 36 / 2.25), so the roofline prices the Winograd GEMMs,
  // not a direct-conv equivalent
  const double flops = 2.0 * 16 * n * (double)((h + 1) / 2) * (double)((w + 1) / 2) *
                       (double)cin * cout;
  // activations in and out, plus the transformed filter U once (the GEMMs'
  // other operand: at 1/32 scale it outweighs the planes)
  const double bytes = 4.0 * n * h * w * (double)(cin + cout) + 64.0 * (double)cin * cout;
  const int xsplit = wino_xsplit(n, g.ci_p, g.co_p, h, w, g);
  const int kid = pass ? mde::K_WINO_DGRAD : mde::K_WINO_FWD;
  // padded channels: the one-block kernel only (it masks the padded loads / stores)
  const bool padded = g.ci_p != cin || g.co_p != cout;
  if (xsplit == 1 && wino_persistent_ok(h, w) && !padded) {
    // persistent blocks: per XCD, its share of the items in runs of ipb
    const int per_xcd = (int)mde::cdiv(g.total, 8);
    int ipb = wino_ipb();
    if (ipb <= 0) ipb = (int)mde::cdiv(per_xcd, 2 * wino_cus() / 8);  // two blocks a CU
    const int pb = (int)mde::cdiv(per_xcd, ipb);
    const dim3 grid((unsigned)(8 * pb)), block(256);
#define MDE_WINOP(CB, TC, ST)                                                                     \
  MDE_LAUNCH_MFMA(kid, bytes, flops, s, (wino_f23p_kernel<CB, TC, ST>), grid, block, 0, x, u, y,  \
                  (int)cin, (int)cout, (int)h, (int)w, g.bcols, g.brows, g.ncog, (int)g.total,   \
                  stats, per_xcd, ipb, add)
    if (stats) {
      if (g.co_b == 64)
        MDE_WINOP(64, 8, true);
      else if (g.co_b == 32)
        MDE_WINOP(32, 8, true);
      else
        MDE_WINOP(16, 16, true);
    } else {
      if (g.co_b == 64)
        MDE_WINOP(64, 8, false);
      else if (g.co_b == 32)
        MDE_WINOP(32, 8, false);
      else
        MDE_WINOP(16, 16, false);
    }
#undef MDE_WINOP
    return MDE_OK;
  }
  int64_t nblk = (g.total + 7) / 8 * 8;
  if (xsplit == 1 && g.co_b == 32 && g_wino_x && !padded) {
    const dim3 grid((unsigned)nblk), block(256);
    if (stats)
      MDE_LAUNCH_MFMA(kid, bytes, flops, s, wino_f23x_kernel<true>, grid, block, 0, x, u, y,
                      (int)cin, (int)cout, (int)h, (int)w, g.bcols, g.brows, g.ncog, (int)g.total,
                      stats, add);
    else
      MDE_LAUNCH_MFMA(kid, bytes, flops, s, wino_f23x_kernel<false>, grid, block, 0, x, u, y,
                      (int)cin, (int)cout, (int)h, (int)w, g.bcols, g.brows, g.ncog, (int)g.total,
                      stats, add);
    return MDE_OK;
  }
  if (xsplit > 1) {
    const int64_t ntiles = g.total / g.ncog, a = 8 / xsplit;
    nblk = 8 * ((ntiles + a - 1) / a) * (g.ncog / xsplit);
  }
  const dim3 grid((unsigned)nblk), block(256);
#define MDE_WINO(CB, TC, ST)                                                                      \
  do {                                                                                            \
    if (g_wino_bpre)                                                                              \
      MDE_LAUNCH_MFMA(kid, bytes, flops, s, (wino_f23_kernel<CB, TC, ST, true>), grid, block, 0,  \
                      x, u, y, (int)cin, (int)cout, (int)h, (int)w, g.bcols, g.brows, g.ncog,     \
                      (int)g.total, stats, xsplit, add, g.ci_p / kCIC);                           \
    else                                                                                          \
      MDE_LAUNCH_MFMA(kid, bytes, flops, s, (wino_f23_kernel<CB, TC, ST, false>), grid, block, 0, \
                      x, u, y, (int)cin, (int)cout, (int)h, (int)w, g.bcols, g.brows, g.ncog,     \
                      (int)g.total, stats, xsplit, add, g.ci_p / kCIC);                           \
  } while (0)
  if (stats) {
    if (g.co_b == 64)
      MDE_WINO(64, 8, true);
    else if (g.co_b == 32)
      MDE_WINO(32, 8, true);
    else
      MDE_WINO(16, 16, true);
  } else {
    if (g.co_b == 64)
      MDE_WINO(64, 8, false);
    else if (g.co_b == 32)
      MDE_WINO(32, 8, false);
    else
      MDE_WINO(16, 16, false);
  }
#undef MDE_WINO
  return MDE_OK;
}

}  // namespace

extern "C" {

int mde_wino_conv_stats(const float* x, const float* u, float* y, float* stats, int64_t n,
                        int64_t cin, int64_t cout, int64_t h, int64_t w, int pass, int dtype,
                        void* stream) {
  return wino_launch(x, u, y, stats, nullptr, n, cin, cout, h, w, pass, dtype, stream);
}

int mde_wino_conv(const float* x, const float* u, float* y, int64_t n, int64_t cin, int64_t cout,
                  int64_t h, int64_t w, int pass, int dtype, void* stream) {
  return wino_launch(x, u, y, nullptr, nullptr, n, cin, cout, h, w, pass, dtype, stream);
}

int mde_wino_conv_acc(const float* x, const float* u, const float* add, float* y, int64_t n,
                      int64_t cin, int64_t cout, int64_t h, int64_t w, int pass, int dtype,
                      void* stream) {
  if (!add) return MDE_ERR_INVALID_ARG;
  return wino_launch(x, u, y, nullptr, add, n, cin, cout, h, w, pass, dtype, stream);
}

// Records per channel of mde_wino_conv_stats (the pixel blocks), or 0.
int mde_wino_stats_blocks(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w) {
  WinoGeo g;
  if (!wino_geo(n, cin, cout, h, w, &g)) return 0;
  return (int)(g.total / g.ncog);
}

}  // extern "C"
