// Stride-2 3x3 convolutions (padding 1, bias-free, NCHW fp32) at DDRNet's
// channel counts: forward and data gradient on v_mfma_f32_32x32x2_f32 (exact
// f32 products, f32 accumulation), with no NCHW <-> NHWC transposes.
//
// Reference call sites (src/GuideDepth/model/DDRNet_23_slim.py): the stem's
// second conv (:232-233, 32 -> 32 at 240x320), the first BasicBlock conv of
// layer2 / layer3 / layer4 (:41-72 with stride 2, built by _make_layer
// :291-309), down3 / down4 (:254-265) and layer5's Bottleneck conv2 (:80).
// MIOpen runs them as Winograd (the 32-channel ones) or as NHWC implicit GEMMs
// behind batched transposes and SubTensorOp fills (tools/conv_kernel_map.py).
//
// Forward: y[n][co][q] = sum_{ci,ky,kx} w[co][ci][ky][kx] x[n][ci][2r+ky-1][2c+kx-1]
// as a GEMM with M = output channels (BM-row tiles), N = BQ output pixels of
// one image (flattened q = r Wo + c, any width), K = (ci, tap) in chunks of 4
// input channels x 9 taps.  A chunk stages the weights [m][36] (pitch 38:
// conflict-free ds_read_b32) and the BAND of input rows under the tile's
// output rows (rows 2 r_first - 1 .. 2 r_last + 1, full width + halo; plane
// pitch odd, row pitch odd, so the two k-lanes of an operand read never share
// a bank).  Wave w stages input channel w of the chunk: R rows of NJ
// 64-element segments per lane, clamped addresses, zero padding applied at
// LDS-store time; the next chunk's loads are in flight during this chunk's
// MFMAs (register prefetch).
//
// Data gradient (the transposed convolution): the four parity classes of gx,
// gx[2m+a][2n+b], each a stride-1 product of gy with the taps that reach it
// (a = 0: ky = 1; a = 1: ky = 0 at gy row m + 1 and ky = 2 at row m; the same
// for columns), so all 9 x co products are useful.  M = input channels,
// N = BQ positions (m, n) of the gy grid, K = (co, class taps); one block keeps
// the four classes' accumulators and writes gx rows 2m and 2m + 1 as float2
// pairs (all of gx is written; odd Hi: the last odd row does not exist).
#include <cstdlib>

#include "common.h"

namespace {

using f16v = float __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma32(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

constexpr int CIC = 4;        // channels per K chunk (= waves per block: wave w stages channel w)
constexpr int KCH = CIC * 9;  // K values per chunk
constexpr int AP = 38;        // A-tile pitch: 38 i mod 64 distinct for i < 32 (38 = 2 x 19)

__device__ __forceinline__ int xcd_logical(int total) {
  const int g = gridDim.x, per = g >> 3;
  const int b = blockIdx.x;
  const int l = (b & 7) * per + (b >> 3);
  return l < total ? l : -1;
}

inline unsigned xcd_grid(int64_t total) { return (unsigned)((total + 7) / 8 * 8); }

// Output rows spanned by BQ consecutive flattened pixels of a Wo-wide plane.
inline int rows_span(int bq, int64_t wo, int64_t ho) {
  int64_t r = (bq - 1 + wo - 1) / wo + 1;
  return (int)(r < ho ? r : ho);
}

// Band staging: channel `c` (this wave's), rows br = 0..R-1 of the band that
// starts at input row `row0`, columns col0 + (lane + 64 j), j < NJ, of a
// plane of h x w (zero outside), pitch xw (elements past xw not stored).
template <int R, int NJ>
struct Band {
  float v[R][NJ];
  uint64_t mrow;  // rows in range
  uint32_t mcol;  // column segments in range (per j)
  __device__ __forceinline__ void load(const float* __restrict__ plane, int h, int w, int row0,
                                       int col0, int xw, int lane) {
    mrow = 0;
    mcol = 0;
    int cols[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cc = lane + 64 * j, gc = col0 + cc;
      mcol |= (cc < xw && gc >= 0 && gc < w) ? 1u << j : 0u;
      cols[j] = clampi(gc, 0, w - 1);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int gr = row0 + r;
      mrow |= (gr >= 0 && gr < h) ? (uint64_t)1 << r : (uint64_t)0;
      const float* src = plane + (int64_t)clampi(gr, 0, h - 1) * w;
#pragma unroll
      for (int j = 0; j < NJ; ++j) v[r][j] = src[cols[j]];
    }
  }
  __device__ __forceinline__ void store(float* sx, int xw, int lane) const {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int cc = lane + 64 * j;
        if (cc < xw) {
          const bool ok = ((mrow >> r) & 1) && ((mcol >> j) & 1u);
          sx[r * xw + cc] = ok ? v[r][j] : 0.f;
        }
      }
  }
};

// ------------------------------------------------------------------ forward
// TW = 0: a tile is BQ consecutive pixels of the flattened output plane and
// the band spans full input rows.  TW > 0: a tile is TH = BQ / TW output rows
// x TW output columns (2D), and the band is 2 TH + 1 input rows x 2 TW + 1
// columns -- far less staging for wide planes (the stem's 240x320 output).
// CI3: the stem's 3 input channels (one chunk, channel 3 of it zero).
template <int BM, int BQ, int MT, int QT, int R, int NJ, int TW = 0, bool CI3 = false>
__global__ void __launch_bounds__(256)
    c3s2_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                    float* __restrict__ y, int ci_n, int co_n, int hi, int wi, int ho, int wo,
                    int xw, int ps, int qtiles, int mtiles, int total) {
  constexpr int WQ = BQ / (32 * QT), WM = BM / (32 * MT);
  static_assert(WQ * WM == 4, "four waves per block");
  static_assert(TW == 0 || BQ % TW == 0, "2D tiles: whole rows of TW");
  constexpr int AV = (BM * KCH / 4 + 255) / 256;  // float4 of weights per thread and chunk
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sX = smem;                 // [CIC][ps]
  float* sA = smem + CIC * ps + (4 - (CIC * ps) % 4) % 4;  // [BM][AP], 16-byte aligned

  const int lb = xcd_logical(total);
  if (lb < 0) return;
  const int mt = lb % mtiles, rest = lb / mtiles;
  const int qt = rest % qtiles, img = rest / qtiles;
  const int m0 = mt * BM, q0 = qt * BQ;
  const int Q = ho * wo;
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WQ, wq = wv % WQ;
  // tile origin (output row r_first, column c_first) and the band origin
  int r_first, c_first;
  if constexpr (TW > 0) {
    const int tcols = (wo + TW - 1) / TW;
    r_first = (qt / tcols) * (BQ / TW);
    c_first = (qt % tcols) * TW;
  } else {
    r_first = q0 / wo;
    c_first = 0;
  }
  const int row0 = 2 * r_first - 1, col0 = 2 * c_first - 1;
  const int64_t hwi = (int64_t)hi * wi;
  const float* xb = x + (int64_t)img * ci_n * hwi;

  // this lane's output pixels (row, column; -1 = none) per pixel tile, and
  // the band offset of their tap (0, 0)
  int prow[QT], pcol[QT], bbase[QT];
#pragma unroll
  for (int y2 = 0; y2 < QT; ++y2) {
    const int i = wq * 32 * QT + 32 * y2 + li;  // pixel index within the tile
    int rq, cq;
    if constexpr (TW > 0) {
      rq = r_first + i / TW;
      cq = c_first + i % TW;
    } else {
      const int q = q0 + i < Q ? q0 + i : Q - 1;
      rq = q / wo;
      cq = q - rq * wo;
    }
    const bool ok = rq < ho && cq < wo && (TW > 0 || q0 + i < Q);
    prow[y2] = ok ? rq : -1;
    pcol[y2] = cq;
    bbase[y2] = 2 * ((ok ? rq : r_first) - r_first) * xw + 2 * ((ok ? cq : c_first) - c_first);
  }
  int koff[KCH / 2];
#pragma unroll
  for (int s = 0; s < KCH / 2; ++s) {
    const int k = 2 * s + h, c = k / 9, t = k % 9;
    koff[s] = c * ps + (t / 3) * xw + t % 3;
  }

  Band<R, NJ> band;
  float4 ra[AV];
  auto load = [&](int ci0) {
    const bool cin_ok = !CI3 || ci0 + wv < ci_n;
    band.load(xb + (int64_t)(cin_ok ? ci0 + wv : 0) * hwi, hi, wi, row0, col0, xw, lane);
    if (!cin_ok) band.mrow = 0;
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int e = tid + 256 * i;  // float4 index over [BM][9 float4]
      const int m = e / 9, f = e - m * 9;
      const bool ok = e < BM * 9;
      if constexpr (CI3) {  // 27 floats per output channel: scalar, masked
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int idx = 4 * f + j, c = idx / 9;
          const bool vok = ok && ci0 + c < ci_n;
          const float t = wt[vok ? ((int64_t)(m0 + m) * ci_n + ci0 + c) * 9 + idx % 9 : 0];
          v[j] = vok ? t : 0.f;
        }
        ra[i] = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        const float* src = wt + ((int64_t)(m0 + (ok ? m : 0)) * ci_n + ci0) * 9 + 4 * f;
        ra[i] = *reinterpret_cast<const float4*>(src);
      }
    }
  };
  auto store = [&]() {
    band.store(sX + wv * ps, xw, lane);
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int e = tid + 256 * i;
      if (e < BM * 9) {
        const int m = e / 9, f = e - m * 9;
        float* d = sA + m * AP + 4 * f;
        *reinterpret_cast<float2*>(d) = make_float2(ra[i].x, ra[i].y);
        *reinterpret_cast<float2*>(d + 2) = make_float2(ra[i].z, ra[i].w);
      }
    }
  };

  f16v acc[MT][QT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < QT; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const float* pa = sA + (wm * 32 * MT + li) * AP + h;
  load(0);
  for (int ci0 = 0; ci0 < ci_n; ci0 += CIC) {
    __syncthreads();
    store();
    __syncthreads();
    if (ci0 + CIC < ci_n) load(ci0 + CIC);
#pragma unroll
    for (int s = 0; s < KCH / 2; ++s) {
      float a[MT], b[QT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = pa[i * 32 * AP + 2 * s];
#pragma unroll
      for (int j = 0; j < QT; ++j) b[j] = sX[bbase[j] + koff[s]];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < QT; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
  }
  float* yb = y + (int64_t)img * co_n * Q;
#pragma unroll
  for (int j = 0; j < QT; ++j) {
    if (prow[j] < 0) continue;
    const int q = prow[j] * wo + pcol[j];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 * MT + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        yb[(int64_t)m * Q + q] = acc[i][j][r];
      }
  }
}

// ------------------------------------------------- stride 1 (wide channels)
// The same band GEMM at stride 1, for DDRNet's 64 / 128 / 256-channel 3x3
// BasicBlock convs (DDRNet_23_slim.py:41-72) that MIOpen runs as Winograd:
// out[n][m][q] = sum_{c,t} A[m][(t, c)] in[n][c][r+ky-1][col+kx-1].  FLIP = the
// data gradient (in = gy, out = gx, A[m = ci][(t, c = co)] = w[co][ci][8 - t]).
// K is tap-major within a chunk (k = 4 t + c): the two k-lanes of an MFMA
// step read channels c, c + 1 of one tap, one plane pitch apart, and the
// plane pitch is 32 (mod 64) words, so the lane halves hit disjoint banks
// while each half reads 32 consecutive pixels.
template <bool FLIP, int BM, int BQ, int MT, int QT, int R, int NJ>
__global__ void __launch_bounds__(256)
    c3s1_kernel(const float* __restrict__ in, const float* __restrict__ wt,
                float* __restrict__ out, int k_n, int m_n, int h, int w, int xw, int ps,
                int qtiles, int mtiles, int total) {
  constexpr int WQ = BQ / (32 * QT), WM = BM / (32 * MT);
  static_assert(WQ * WM == 4, "four waves per block");
  constexpr int AV = (BM * KCH / 4 + 255) / 256;  // float4 of weights per thread and chunk
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sX = smem;             // [CIC][ps]
  float* sA = smem + CIC * ps;  // [BM][AP]

  const int lb = xcd_logical(total);
  if (lb < 0) return;
  const int mt = lb % mtiles, rest = lb / mtiles;
  const int qt = rest % qtiles, img = rest / qtiles;
  const int m0 = mt * BM, q0 = qt * BQ;
  const int Q = h * w;
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, hh = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WQ, wq = wv % WQ;
  const int r_first = q0 / w;
  const int64_t hw = (int64_t)h * w;
  const float* ib = in + (int64_t)img * k_n * hw;

  int bbase[QT];
#pragma unroll
  for (int y2 = 0; y2 < QT; ++y2) {
    int q = q0 + wq * 32 * QT + 32 * y2 + li;
    q = q < Q ? q : Q - 1;
    const int rq = q / w, cq = q - rq * w;
    bbase[y2] = (rq - r_first) * xw + cq + hh * ps;
  }
  int koff[KCH / 2];  // k = 2 s + hh: tap s / 2, channel 2 (s & 1) + hh (hh folded into bbase)
#pragma unroll
  for (int s2 = 0; s2 < KCH / 2; ++s2) {
    const int t = s2 >> 1;
    koff[s2] = 2 * (s2 & 1) * ps + (t / 3) * xw + t % 3;
  }

  Band<R, NJ> band;
  float4 ra[AV];
  auto load = [&](int k0) {
    band.load(ib + (int64_t)(k0 + wv) * hw, h, w, r_first - 1, -1, xw, lane);
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int e = tid + 256 * i;
      const bool ok = e < BM * 9;
      const int ee = ok ? e : 0;
      const float* src;
      if constexpr (FLIP) {  // [c][m][9] = w[k0 + c][m0 + m][t'], BM * 9 contiguous per c
        const int c = ee / (BM * 9 / 4), f = ee - c * (BM * 9 / 4);
        src = wt + ((int64_t)(k0 + c) * m_n + m0) * 9 + 4 * f;
      } else {  // [m][c][9] = w[m0 + m][k0 + c][t], 36 contiguous per m
        const int m = ee / 9, f = ee - m * 9;
        src = wt + ((int64_t)(m0 + m) * k_n + k0) * 9 + 4 * f;
      }
      ra[i] = *reinterpret_cast<const float4*>(src);
    }
  };
  auto store = [&]() {
    band.store(sX + wv * ps, xw, lane);
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int e = tid + 256 * i;
      if (e < BM * 9) {
        const float v[4] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          int m, c, t;
          if constexpr (FLIP) {
            const int c0 = e / (BM * 9 / 4), idx = 4 * (e - c0 * (BM * 9 / 4)) + j;
            c = c0;
            m = idx / 9;
            t = 8 - (idx - m * 9);
          } else {
            const int m0l = e / 9, idx = 4 * (e - m0l * 9) + j;
            m = m0l;
            c = idx / 9;
            t = idx - c * 9;
          }
          sA[m * AP + 4 * t + c] = v[j];
        }
      }
    }
  };

  f16v acc[MT][QT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < QT; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const float* pa = sA + (wm * 32 * MT + li) * AP + hh;
  load(0);
  for (int k0 = 0; k0 < k_n; k0 += CIC) {
    __syncthreads();
    store();
    __syncthreads();
    if (k0 + CIC < k_n) load(k0 + CIC);
#pragma unroll
    for (int s2 = 0; s2 < KCH / 2; ++s2) {
      float a[MT], b[QT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = pa[i * 32 * AP + 2 * s2];
#pragma unroll
      for (int j = 0; j < QT; ++j) b[j] = sX[bbase[j] + koff[s2]];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < QT; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
  }
  float* ob = out + (int64_t)img * m_n * Q;
#pragma unroll
  for (int j = 0; j < QT; ++j) {
    const int q = q0 + wq * 32 * QT + 32 * j + li;
    if (q >= Q) continue;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 * MT + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh;
        ob[(int64_t)m * Q + q] = acc[i][j][r];
      }
  }
}

// ------------------------------------------------------------ data gradient
// Class taps: (a, b) -> list of (ky, kx, dy, dx); dy / dx = gy row / column
// offset (tap 0 of a class-1 axis reads gy at m + 1).
struct Tap {
  int ky, kx, dy, dx;
};
__device__ constexpr int ntaps(int a, int b) { return (a ? 2 : 1) * (b ? 2 : 1); }
__device__ constexpr Tap class_tap(int a, int b, int i) {
  // i enumerates (row tap, column tap) pairs row-major
  const int nb = b ? 2 : 1;
  const int ia = i / nb, ib = i % nb;
  const int ky = a ? (ia == 0 ? 0 : 2) : 1, dy = a ? (ia == 0 ? 1 : 0) : 0;
  const int kx = b ? (ib == 0 ? 0 : 2) : 1, dx = b ? (ib == 0 ? 1 : 0) : 0;
  return Tap{ky, kx, dy, dx};
}

template <int BM, int BQ, int R, int NJ>
__global__ void __launch_bounds__(256)
    c3s2_dgrad_kernel(const float* __restrict__ gy, const float* __restrict__ wt,
                      float* __restrict__ gx, int ci_n, int co_n, int hi, int wi, int ho, int wo,
                      int xw, int ps, int qtiles, int mtiles, int total) {
  constexpr int WQ = BQ / 32, WM = BM / 32;
  static_assert(WQ * WM == 4, "four waves per block, one 32 x 32 tile each");
  constexpr int AV = (BM * KCH + 255) / 256;  // weight floats per thread and chunk
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sX = smem;             // [CIC][ps]: gy band
  float* sA = smem + CIC * ps;  // [BM][AP]: w[co0 + c][ci][t] at [ci][9 c + t]

  const int lb = xcd_logical(total);
  if (lb < 0) return;
  const int mt = lb % mtiles, rest = lb / mtiles;
  const int qt = rest % qtiles, img = rest / qtiles;
  const int m0 = mt * BM, q0 = qt * BQ;
  const int Q = ho * wo;
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WQ, wq = wv % WQ;
  const int r_first = q0 / wo;
  const int64_t hwo = (int64_t)ho * wo;
  const float* gb = gy + (int64_t)img * co_n * hwo;

  int qq = q0 + wq * 32 + li;
  const bool qok = qq < Q;
  qq = qok ? qq : Q - 1;
  const int rq = qq / wo, cq = qq - rq * wo;
  const int bbase = (rq - r_first) * xw + cq;

  Band<R, NJ> band;
  float ra[AV];
  auto load = [&](int co0) {
    band.load(gb + (int64_t)(co0 + wv) * hwo, ho, wo, r_first, 0, xw, lane);
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      // element e over [CIC][BM][9] (contiguous 9-tap rows of w[co][ci])
      const int e = tid + 256 * i;
      const int c = e / (BM * 9), rr = e - c * BM * 9;
      const bool ok = e < BM * KCH;
      ra[i] = wt[ok ? ((int64_t)(co0 + c) * ci_n + m0) * 9 + rr : 0];
    }
  };
  auto store = [&]() {
    band.store(sX + wv * ps, xw, lane);
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int e = tid + 256 * i;
      if (e < BM * KCH) {
        const int c = e / (BM * 9), rr = e - c * BM * 9;
        const int m = rr / 9, t = rr - m * 9;
        sA[m * AP + 9 * c + t] = ra[i];
      }
    }
  };

  f16v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const float* pa = sA + (wm * 32 + li) * AP;
  load(0);
  for (int co0 = 0; co0 < co_n; co0 += CIC) {
    __syncthreads();
    store();
    __syncthreads();
    if (co0 + CIC < co_n) load(co0 + CIC);
    // class (a, b): K = (c, tap i) = c * nt + i, two per MFMA step (lane half h)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int nt = ntaps(a, b);
#pragma unroll
        for (int s = 0; s < 2 * nt; ++s) {  // CIC * nt / 2 steps
          const int k = 2 * s + h, c = k / nt, i = k - c * nt;
          const Tap tp = class_tap(a, b, i);
          const float av = pa[9 * c + 3 * tp.ky + tp.kx];
          const float bv = sX[c * ps + bbase + tp.dy * xw + tp.dx];
          acc[a][b] = mfma32(av, bv, acc[a][b]);
        }
      }
  }
  if (!qok) return;
  const int64_t hwi = (int64_t)hi * wi;
  float* gxb = gx + (int64_t)img * ci_n * hwi;
  const int row = 2 * rq, col = 2 * cq;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    float* d = gxb + (int64_t)m * hwi + (int64_t)row * wi + col;
    *reinterpret_cast<float2*>(d) = make_float2(acc[0][0][r], acc[0][1][r]);
    if (row + 1 < hi) *reinterpret_cast<float2*>(d + wi) = make_float2(acc[1][0][r], acc[1][1][r]);
  }
}

// -------------------------------------------------------------------- plans
struct S2Geo {
  int bm, bq, r, nj, xw, ps, qtiles, mtiles;
  int64_t total;
};

inline int odd_up(int v) { return v | 1; }

// forward: BM (output channels) x BQ (pixels) per block.  Output planes at
// least 128 wide (wo % 32 == 0) take 2D tiles of 4 rows x 32 columns (tw = 32):
// a band of 9 x 65 input elements per channel instead of 5 full rows.
inline bool fwd_geo(int64_t n, int64_t ci, int64_t co, int64_t hi, int64_t wi, S2Geo* g,
                    int* tw) {
  const int64_t ho = (hi - 1) / 2 + 1, wo = (wi - 1) / 2 + 1, Q = ho * wo;
  g->bm = co % 64 == 0 ? 64 : 32;
  if (co % g->bm) return false;
  g->bq = (Q >= 1024 || g->bm == 32) ? 128 : 64;
  *tw = (wo >= 128 && wo % 32 == 0 && g->bq == 128) ? 32 : 0;
  if (*tw) {
    const int th = g->bq / *tw;
    g->r = 2 * th + 1;
    g->xw = 2 * *tw + 1;
    g->qtiles = (int)(mde::cdiv(ho, th) * (wo / *tw));
  } else {
    const int rows = rows_span(g->bq, wo, ho);
    g->r = 2 * rows + 1;
    g->xw = odd_up((int)wi + 2);
    g->qtiles = (int)mde::cdiv(Q, g->bq);
  }
  g->nj = (g->xw + 63) / 64;
  g->ps = odd_up(g->r * g->xw);
  g->mtiles = (int)(co / g->bm);
  g->total = n * g->qtiles * g->mtiles;
  return g->total < 0x7fffffff;
}

// data gradient: BM (input channels) x BQ (gy positions) per block
inline bool dgrad_geo(int64_t n, int64_t ci, int64_t co, int64_t hi, int64_t wi, S2Geo* g) {
  const int64_t ho = (hi - 1) / 2 + 1, wo = (wi - 1) / 2 + 1, Q = ho * wo;
  g->bm = ci % 64 == 0 ? 64 : 32;
  if (ci % g->bm) return false;
  g->bq = g->bm == 64 ? 64 : 128;
  const int rows = rows_span(g->bq, wo, ho);
  g->r = rows + 1;
  g->xw = odd_up((int)wo + 1);
  g->nj = (g->xw + 63) / 64;
  g->ps = odd_up(g->r * g->xw);
  g->qtiles = (int)mde::cdiv(Q, g->bq);
  g->mtiles = (int)(ci / g->bm);
  g->total = n * g->qtiles * g->mtiles;
  return g->total < 0x7fffffff;
}

// stride 1: BM output channels (of this pass) x BQ pixels; plane pitch = 32 (mod 64)
inline bool s1_geo_at(int64_t n, int64_t m_ch, int64_t h, int64_t w, int bm, int bq, S2Geo* g) {
  const int64_t Q = h * w;
  if (m_ch % bm) return false;
  g->bm = bm;
  g->bq = bq;
  const int rows = rows_span(g->bq, w, h);
  g->r = rows + 2;
  g->xw = (int)w + 2;
  g->nj = (g->xw + 63) / 64;
  g->ps = 0;
  g->qtiles = (int)mde::cdiv(Q, g->bq);
  g->mtiles = (int)(m_ch / g->bm);
  g->total = n * g->qtiles * g->mtiles;
  return g->total < 0x7fffffff;
}

// baseline tile: BM 64 (32 for 32-channel outputs) x BQ 128 (64 on planes < 1024)
inline bool s1_geo(int64_t n, int64_t m_ch, int64_t h, int64_t w, S2Geo* g) {
  const int bm = m_ch % 64 == 0 ? 64 : 32;
  const int bq = (h * w >= 1024 || bm == 32) ? 128 : 64;
  return s1_geo_at(n, m_ch, h, w, bm, bq, g);
}

inline int pitch32(int v) { return (v + 31) / 64 * 64 + 32; }  // >= v, = 32 (mod 64)

inline bool s2_shape_ok(int64_t n, int64_t ci, int64_t co, int64_t hi, int64_t wi) {
  return n > 0 && (ci == 3 || (ci >= 32 && ci % 32 == 0)) && co >= 32 && co % 32 == 0 &&
         hi >= 2 && wi >= 2 && wi % 2 == 0 && n * ci * hi * wi < ((int64_t)1 << 31) &&
         n * co * hi * wi < ((int64_t)1 << 31);
}

// The (R, NJ) instantiations: the DDRNet planes (wi 320 / 160 / 80 / 40 / 20)
// plus the generic fallbacks below them.
// (BM, BQ, MT, QT, R, NJ, TW, CI3)
#define MDE_S2_FWD_GEOS(X)              \
  X(32, 128, 1, 1, 5, 6, 0, false)      \
  X(64, 128, 2, 1, 7, 3, 0, false)      \
  X(64, 128, 2, 1, 11, 2, 0, false)     \
  X(64, 64, 1, 1, 11, 1, 0, false)      \
  X(64, 64, 1, 1, 17, 1, 0, false)      \
  X(32, 128, 1, 1, 9, 2, 32, false)     \
  X(64, 128, 2, 1, 9, 2, 32, false)     \
  X(32, 128, 1, 1, 9, 2, 32, true)
#define MDE_S2_DGRAD_GEOS(X) \
  X(32, 128, 3, 3)           \
  X(64, 64, 3, 3)            \
  X(32, 128, 4, 2)           \
  X(64, 64, 4, 2)            \
  X(64, 64, 6, 1)            \
  X(64, 64, 9, 1)

// (BM, BQ, MT, QT, R, NJ); the 2 x 2 wave tiles (four MFMAs per k-step on two
// A and two B reads) are taken when they still give >= 512 blocks
#define MDE_S1_GEOS(X)     \
  X(32, 128, 1, 1, 4, 3)   \
  X(64, 128, 2, 1, 5, 2)   \
  X(64, 128, 2, 1, 7, 1)   \
  X(64, 64, 1, 1, 7, 1)    \
  X(64, 64, 1, 1, 10, 1)   \
  X(64, 128, 2, 1, 4, 3)   \
  X(32, 256, 1, 2, 5, 3)   \
  X(64, 256, 2, 2, 7, 2)   \
  X(64, 256, 2, 2, 5, 3)   \
  X(128, 128, 2, 2, 7, 1)  \
  X(128, 128, 2, 2, 4, 3)  \
  X(128, 128, 2, 2, 5, 2)

template <bool FLIP>
int launch_s1(const float* in, const float* wt, float* out, int64_t n, int64_t k_ch,
              int64_t m_ch, int64_t h, int64_t w, int kid, double bytes, double flops,
              hipStream_t s) {
  S2Geo g;
  static const int pref = [] {  // MDE_C3W_TILE=0: the baseline tile only (A/B)
    const char* e = std::getenv("MDE_C3W_TILE");
    return e ? std::atoi(e) : 1;
  }();
  bool big = false;
  if (pref) {
    const int cand[3][2] = {{128, 128}, {64, 256}, {32, 256}};
    for (const auto& c : cand) {
      if (s1_geo_at(n, m_ch, h, w, c[0], c[1], &g) && g.total >= 512) {
#define MDE_MATCH(BM, BQ, MT, QT, R, NJ) \
  if (!big && g.bm == BM && g.bq == BQ && g.r <= R && g.nj == NJ) big = true;
        MDE_S1_GEOS(MDE_MATCH)
#undef MDE_MATCH
        if (big) break;
      }
    }
  }
  if (!big && !s1_geo(n, m_ch, h, w, &g)) return MDE_ERR_UNSUPPORTED;
  const dim3 grid(xcd_grid(g.total)), block(256);
#define MDE_GO(BM, BQ, MT, QT, R, NJ)                                                             \
  if (g.bm == BM && g.bq == BQ && g.r <= R && g.nj == NJ) {                                     \
    const int ps = pitch32(R * g.xw);                                                             \
    const size_t smem = sizeof(float) * ((size_t)CIC * ps + (size_t)BM * AP);                     \
    MDE_LAUNCH_MFMA(kid, bytes, flops, s, (c3s1_kernel<FLIP, BM, BQ, MT, QT, R, NJ>), grid, block,  \
                    smem, in, wt, out, (int)k_ch, (int)m_ch, (int)h, (int)w, g.xw, ps, g.qtiles, \
                    g.mtiles, (int)g.total);                                                      \
    return MDE_OK;                                                                                \
  }
  MDE_S1_GEOS(MDE_GO)
#undef MDE_GO
  return MDE_ERR_UNSUPPORTED;
}

inline bool s1_supported(int64_t m_ch, int64_t k_ch, int64_t h, int64_t w) {
  S2Geo g;
  if (k_ch < 32 || m_ch < 32 || k_ch % 32 || m_ch % 32 || h < 1 || w < 1 ||
      !s1_geo(1, m_ch, h, w, &g))
    return false;
#define MDE_MATCH(BM, BQ, MT, QT, R, NJ) \
  if (g.bm == BM && g.bq == BQ && g.r <= R && g.nj == NJ) return true;
  MDE_S1_GEOS(MDE_MATCH)
#undef MDE_MATCH
  return false;
}

}  // namespace

extern "C" {

int mde_conv3x3_wide_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int pass,
                               int dtype) {
  if (dtype != MDE_F32) return 0;
  if (pass == 0) return s1_supported(cout, cin, h, w) ? 1 : 0;
  if (pass == 1) return s1_supported(cin, cout, h, w) ? 1 : 0;
  return 0;
}

int mde_conv3x3_wide_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t cin,
                         int64_t cout, int64_t h, int64_t w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !weight || !y || n <= 0) return MDE_ERR_INVALID_ARG;
  if (!s1_supported(cout, cin, h, w) || n * (cin > cout ? cin : cout) * h * w >= ((int64_t)1 << 31))
    return MDE_ERR_UNSUPPORTED;
  const double flops = 2.0 * 9 * n * h * w * (double)cin * cout;
  const double bytes = 4.0 * n * h * w * (double)(cin + cout);
  return launch_s1<false>((const float*)x, weight, (float*)y, n, cin, cout, h, w, mde::K_C3W_FWD,
                          bytes, flops, (hipStream_t)stream);
}

int mde_conv3x3_wide_bwd_data(const void* gy, const float* weight, void* gx, int64_t n,
                              int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype,
                              void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !weight || !gx || n <= 0) return MDE_ERR_INVALID_ARG;
  if (!s1_supported(cin, cout, h, w) || n * (cin > cout ? cin : cout) * h * w >= ((int64_t)1 << 31))
    return MDE_ERR_UNSUPPORTED;
  const double flops = 2.0 * 9 * n * h * w * (double)cin * cout;
  const double bytes = 4.0 * n * h * w * (double)(cin + cout);
  return launch_s1<true>((const float*)gy, weight, (float*)gx, n, cout, cin, h, w,
                         mde::K_C3W_DGRAD, bytes, flops, (hipStream_t)stream);
}


// Measured against MIOpen at bs 32 (tools/c1_bench.py, profiles/r04_c1_bench.txt):
// the band kernels win on the planes of >= 256 output pixels (forward) and
// >= 1024 gy pixels (data gradient); the 15x20 -> 8x10 and 30x40 -> 15x20
// data gradients (one or two waves per SIMD over a long K loop) lose, so the
// queries send those to MIOpen.
int mde_conv3x3s2_fwd_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype) {
  S2Geo g;
  int tw = 0;
  if (dtype != MDE_F32 || !s2_shape_ok(1, cin, cout, h, w) || !fwd_geo(1, cin, cout, h, w, &g, &tw))
    return 0;
  if (((h - 1) / 2 + 1) * ((w - 1) / 2 + 1) < 256) return 0;
  const bool ci3 = cin == 3;
#define MDE_MATCH(BM, BQ, MT, QT, R, NJ, TW, C3) \
  if (g.bm == BM && g.bq == BQ && g.r <= R && g.nj == NJ && tw == TW && ci3 == C3) return 1;
  MDE_S2_FWD_GEOS(MDE_MATCH)
#undef MDE_MATCH
  return 0;
}

int mde_conv3x3s2_dgrad_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype) {
  S2Geo g;
  if (dtype != MDE_F32 || !s2_shape_ok(1, cin, cout, h, w) || !dgrad_geo(1, cin, cout, h, w, &g))
    return 0;
  if (((h - 1) / 2 + 1) * ((w - 1) / 2 + 1) < 1024) return 0;
#define MDE_MATCH(BM, BQ, R, NJ) \
  if (g.bm == BM && g.bq == BQ && g.r <= R && g.nj == NJ) return 1;
  MDE_S2_DGRAD_GEOS(MDE_MATCH)
#undef MDE_MATCH
  return 0;
}

int mde_conv3x3s2_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t cin,
                      int64_t cout, int64_t h, int64_t w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !weight || !y) return MDE_ERR_INVALID_ARG;
  S2Geo g;
  int tw = 0;
  if (!s2_shape_ok(n, cin, cout, h, w) || !fwd_geo(n, cin, cout, h, w, &g, &tw))
    return MDE_ERR_UNSUPPORTED;
  const bool ci3 = cin == 3;
  hipStream_t s = (hipStream_t)stream;
  const int64_t ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const double flops = 2.0 * 9 * n * ho * wo * (double)cin * cout;
  const double bytes = 4.0 * n * ((double)cin * h * w + (double)cout * ho * wo);
  const dim3 grid(xcd_grid(g.total)), block(256);
#define MDE_GO(BM, BQ, MT, QT, R, NJ, TW, C3)                                                     \
  if (g.bm == BM && g.bq == BQ && g.r <= R && g.nj == NJ && tw == TW && ci3 == C3) {            \
    const int ps = odd_up(R * g.xw); /* the template's R rows per staged plane */                \
    const size_t smem = sizeof(float) * ((size_t)CIC * ps + 4 + (size_t)BM * AP);                 \
    MDE_LAUNCH_MFMA(mde::K_C3S2_FWD, bytes, flops, s,                                             \
                    (c3s2_fwd_kernel<BM, BQ, MT, QT, R, NJ, TW, C3>), grid, block, smem,          \
                    (const float*)x, weight, (float*)y, (int)cin, (int)cout, (int)h, (int)w,      \
                    (int)ho, (int)wo, g.xw, ps, g.qtiles, g.mtiles, (int)g.total);                \
    return MDE_OK;                                                                                \
  }
  MDE_S2_FWD_GEOS(MDE_GO)
#undef MDE_GO
  return MDE_ERR_UNSUPPORTED;
}

int mde_conv3x3s2_bwd_data(const void* gy, const float* weight, void* gx, int64_t n, int64_t cin,
                           int64_t cout, int64_t h, int64_t w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !weight || !gx) return MDE_ERR_INVALID_ARG;
  S2Geo g;
  if (!s2_shape_ok(n, cin, cout, h, w) || !dgrad_geo(n, cin, cout, h, w, &g))
    return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int64_t ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const double flops = 2.0 * 9 * n * ho * wo * (double)cin * cout;
  const double bytes = 4.0 * n * ((double)cin * h * w + (double)cout * ho * wo);
  const dim3 grid(xcd_grid(g.total)), block(256);
#define MDE_GO(BM, BQ, R, NJ)                                                                     \
  if (g.bm == BM && g.bq == BQ && g.r <= R && g.nj == NJ) {                                     \
    const int ps = odd_up(R * g.xw);                                                              \
    const size_t smem = sizeof(float) * ((size_t)CIC * ps + (size_t)BM * AP);                     \
    MDE_LAUNCH_MFMA(mde::K_C3S2_DGRAD, bytes, flops, s, (c3s2_dgrad_kernel<BM, BQ, R, NJ>), grid, \
                    block, smem, (const float*)gy, weight, (float*)gx, (int)cin, (int)cout,       \
                    (int)h, (int)w, (int)ho, (int)wo, g.xw, ps, g.qtiles, g.mtiles,               \
                    (int)g.total);                                                                \
    return MDE_OK;                                                                                \
  }
  MDE_S2_DGRAD_GEOS(MDE_GO)
#undef MDE_GO
  return MDE_ERR_UNSUPPORTED;
}

}  // extern "C"
