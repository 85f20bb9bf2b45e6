// 1x1 convolutions at DDRNet's wide channel counts (NCHW fp32, bias-free,
// stride 1 or 2) on v_mfma_f32_32x32x2_f32 (exact f32 products, f32
// accumulation), with no NCHW <-> NHWC transposes.
//
// Reference call sites (src/GuideDepth/model/DDRNet_23_slim.py): the
// Bottleneck's conv1 / conv3 (:79,84), the residual downsample of every stage
// (:294-296, stride 2 for layer2/3/4/5), compression3 / compression4
// (:245,250), DAPPM's scale0 / shortcut / compression and the pooled branches
// (:121-171).  MIOpen runs these (and their gradients) as NHWC implicit GEMMs
// behind batched transposes and SubTensorOp zero fills (~1.6 ms of the cfg2
// step, tools/conv_kernel_map.py); here every pass is one NCHW kernel.
//
// Channel mix (forward, and the data gradient with the transposed weight):
//   out[n][m][q] = sum_k A[m][k] in[n][k][q']      A = W (fwd) or W^T (dgrad)
// M = output channels, N = pixels of one image, K = input channels, as
// 128 x 128 (or 64 / 32 x 128) block tiles; K in chunks of 32 staged in LDS
// (A rows [m][k], pitch 34 words; B rows [k][q], pitch BQ + 32): every MFMA
// operand is one conflict-free ds_read_b32.  Stride 2: the forward gathers
// the even input pixels (q' = 2r W + 2c); the data gradient writes gx at the
// even positions and zeros at the others (the 1x1 / s2 conv's gradient there).
//
// Weight gradient: G[co][ci] = sum_{n,q} gy[n][co][q] x[n][ci][q'], an outer
// product over all pixels: block tiles of (co, ci), the pixel range split
// over blocks (split-K), per-block partials in a slab summed in block order
// by a second kernel (deterministic, no atomics).
#include <cstdlib>

#include "common.h"

namespace {

using f16v = float __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma32(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

constexpr int KC = 32;   // K values staged per chunk
constexpr int KCP = 34;  // LDS pitch of a [row][k] tile: 34 i mod 64 distinct for i < 32

// Blocks b and b + 8 share an XCD (round-robin placement): logical block
// order with consecutive ids on one XCD, so the tiles that share an input
// chunk (consecutive logical ids) go through the same L2.  `total` logical
// blocks; the grid is rounded up to a multiple of 8.
__device__ __forceinline__ int xcd_logical(int total) {
  const int g = gridDim.x, per = g >> 3;
  const int b = blockIdx.x;
  const int l = (b & 7) * per + (b >> 3);
  return l < total ? l : -1;
}

inline unsigned xcd_grid(int64_t total) { return (unsigned)((total + 7) / 8 * 8); }

// q / d for 0 <= q < 2^22, 1 <= d < 2^10, with d's float reciprocal: the
// float quotient is within one of the true one, fixed by one compare each way
// (a 32-bit integer division is a ~30-instruction sequence on the VALU).
__device__ __forceinline__ int fdiv(int q, int d, float inv) {
  int r = (int)((float)q * inv);
  r -= r * d > q ? 1 : 0;
  r += (r + 1) * d <= q ? 1 : 0;
  return r;
}

// ------------------------------------------------------------- channel mix
// BM x BQ block tile, wave tile (32 MT) x (32 QT), 4 waves.
// SIN = 2: input pixel of q is (2 (q / wo), 2 (q % wo)) of a hin x win plane.
// SOUT = 2: output value of q goes to (2 r, 2 c) of an hout x wout plane
// (wout even), zeros to (2r, 2c+1), (2r+1, 2c), (2r+1, 2c+1).
// TRANSA: A[m][k] = wt[k * M + m] (the data gradient: W is [K = co][M = ci]).
// PAD: K or M not a multiple of 32 (MobileNetV3's 16 / 24 / 40 / 72 / 80 /
// 112 / 120 / 184 / 200 / 240 / 480-channel 1x1 convs, multiples of 8): loads
// past K / M are zeros (never issued), rows past M are not stored.
template <int BM, int BQ, int MT, int QT, int SIN, int SOUT, bool TRANSA, bool PAD = false>
__global__ void __launch_bounds__(256)
    cm_kernel(const float* __restrict__ in, const float* __restrict__ wt, float* __restrict__ out,
              int K, int M, int hin, int win, int wo, int Q, int hout, int wout, int qtiles,
              int mtiles, int total) {
  constexpr int WQ = BQ / (32 * QT), WM = BM / (32 * MT);
  static_assert(WQ * WM == 4, "four waves per block");
  constexpr int BQP = BQ + 32;
  constexpr int AV = BM * KC / 1024;  // float4 of A per thread and chunk
  constexpr int BV = KC * BQ / 1024;  // float4 of B per thread and chunk
  static_assert(AV >= 1 && BV >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) float sA[BM * KCP];
  __shared__ __attribute__((aligned(16))) float sB[KC * BQP];

  const int lb = xcd_logical(total);
  if (lb < 0) return;
  const int mt = lb % mtiles, rest = lb / mtiles;
  const int qt = rest % qtiles, img = rest / qtiles;
  const int m0 = mt * BM, q0 = qt * BQ;
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WQ, wq = wv % WQ;
  const int64_t hwin = (int64_t)hin * win;
  const float* inb = in + (int64_t)img * K * hwin;
  const float inv_wo = 1.f / (float)wo;

  float4 ra[AV], rb[BV];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int e = 4 * (tid + 256 * i);
      if constexpr (TRANSA) {
        const int k = e / BM, m = e % BM;
        // (K, M multiples of 4: a float4 is all in or all out)
        const bool ok = !PAD || (k0 + k < K && m0 + m < M);
        const float4 t = *reinterpret_cast<const float4*>(wt + (ok ? (int64_t)(k0 + k) * M + m0 + m : 0));
        ra[i] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        const int m = e / KC, k = e % KC;
        const bool ok = !PAD || (k0 + k < K && m0 + m < M);
        const float4 t = *reinterpret_cast<const float4*>(wt + (ok ? (int64_t)(m0 + m) * K + k0 + k : 0));
        ra[i] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int e = 4 * (tid + 256 * i);
      const int k = e / BQ, q0e = q0 + e % BQ;
      const bool kok = !PAD || k0 + k < K;
      const float* src = inb + (int64_t)(kok ? k0 + k : 0) * hwin;
      const int q = kok ? q0e : Q;  // a channel past K: every element out of range (zeros)
      if constexpr (SIN == 1) {
        // Q % 4 == 0: a float4 is all in or all out; out-of-range loads a
        // real element (q = 0) and is zeroed at store time
        const float4 t = *reinterpret_cast<const float4*>(src + (q < Q ? q : 0));
        rb[i] = q < Q ? t : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int qq = q + j, r = fdiv(qq < Q ? qq : 0, wo, inv_wo), c = (qq < Q ? qq : 0) - r * wo;
          const float t = src[qq < Q ? (int64_t)(2 * r) * win + 2 * c : 0];
          v[j] = qq < Q ? t : 0.f;
        }
        rb[i] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int e = 4 * (tid + 256 * i);
      if constexpr (TRANSA) {
        const int k = e / BM, m = e % BM;
        sA[(m + 0) * KCP + k] = ra[i].x;
        sA[(m + 1) * KCP + k] = ra[i].y;
        sA[(m + 2) * KCP + k] = ra[i].z;
        sA[(m + 3) * KCP + k] = ra[i].w;
      } else {
        const int m = e / KC, k = e % KC;
        *reinterpret_cast<float2*>(sA + m * KCP + k) = make_float2(ra[i].x, ra[i].y);
        *reinterpret_cast<float2*>(sA + m * KCP + k + 2) = make_float2(ra[i].z, ra[i].w);
      }
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int e = 4 * (tid + 256 * i);
      const int k = e / BQ, q = e % BQ;
      *reinterpret_cast<float4*>(sB + k * BQP + q) = rb[i];
    }
  };

  f16v acc[MT][QT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < QT; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const float* pa = sA + (wm * 32 * MT + li) * KCP + h;
  const float* pb = sB + h * BQP + wq * 32 * QT + li;
  load(0);
  for (int k0 = 0; k0 < K; k0 += KC) {
    __syncthreads();  // the previous chunk's operands are consumed
    store();
    __syncthreads();
    if (k0 + KC < K) load(k0 + KC);
#pragma unroll
    for (int s = 0; s < KC / 2; ++s) {
      float a[MT], b[QT];
#pragma unroll
      for (int x = 0; x < MT; ++x) a[x] = pa[x * 32 * KCP + 2 * s];
#pragma unroll
      for (int y = 0; y < QT; ++y) b[y] = pb[2 * s * BQP + y * 32];
#pragma unroll
      for (int x = 0; x < MT; ++x)
#pragma unroll
        for (int y = 0; y < QT; ++y) acc[x][y] = mfma32(a[x], b[y], acc[x][y]);
    }
  }

  // D: lane column = pixel (li), rows = channels (r & 3) + 8 (r >> 2) + 4 h
  float* ob = out + (int64_t)img * M * hout * wout;
#pragma unroll
  for (int y = 0; y < QT; ++y) {
    const int q = q0 + wq * 32 * QT + 32 * y + li;
    if (q >= Q) continue;
    int64_t po = q;
    int rr = 0, cc = 0;
    if constexpr (SOUT == 2) {
      rr = fdiv(q, wo, inv_wo);
      cc = q - rr * wo;
      po = (int64_t)(2 * rr) * wout + 2 * cc;
    }
#pragma unroll
    for (int x = 0; x < MT; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 * MT + 32 * x + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (PAD && m >= M) continue;
        float* dst = ob + (int64_t)m * hout * wout + po;
        if constexpr (SOUT == 1) {
          *dst = acc[x][y][r];
        } else {
          *reinterpret_cast<float2*>(dst) = make_float2(acc[x][y][r], 0.f);
          if (2 * rr + 1 < hout) *reinterpret_cast<float2*>(dst + wout) = make_float2(0.f, 0.f);
        }
      }
  }
}

// ----------------------------------------------------------- weight gradient
// G[co][ci] partial over pixel chunks [c_begin, c_end) of the N*Q pixels
// (chunks of 32): block tile BCO x BCI, wave tile (32 MT) x (32 NT).
template <int BCO, int BCI, int MT, int NT, int SIN>
__global__ void __launch_bounds__(256)
    c1_wgrad_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                    float* __restrict__ part, int CO, int CI, int Q, int hin, int win, int wo,
                    int64_t npix, int nchunks, int ksplit, int cotiles, int citiles, int total) {
  constexpr int WN = BCI / (32 * NT), WMv = BCO / (32 * MT);
  static_assert(WN * WMv == 4, "four waves per block");
  constexpr int AV = BCO * KC / 1024, BV = BCI * KC / 1024;
  static_assert(AV >= 1 && BV >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) float sA[BCO * KCP];
  __shared__ __attribute__((aligned(16))) float sB[BCI * KCP];
  const int lb = xcd_logical(total);
  if (lb < 0) return;
  const int ntile = cotiles * citiles;
  const int tile = lb % ntile, ks = lb / ntile;
  const int cot = tile % cotiles, cit = tile / cotiles;
  const int co0 = cot * BCO, ci0 = cit * BCI;
  const int c_begin = (int)((int64_t)nchunks * ks / ksplit);
  const int c_end = (int)((int64_t)nchunks * (ks + 1) / ksplit);
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WN, wn = wv % WN;
  const int64_t hwin = (int64_t)hin * win;

  const float inv_wo = 1.f / (float)wo;
  float4 ra[AV], rb[BV];
  // chunk = KC consecutive pixels of the n * Q flattened pixels (Q >= KC, so a
  // chunk touches at most two images): image / offset of its first pixel by
  // one wave-uniform division, each float4 (4 pixels of one image, Q % 4 == 0)
  // wraps into the next image at most once
  auto load = [&](int chunk) {
    const int p0 = chunk * KC;
    const int n0 = p0 / Q, q0 = p0 - n0 * Q;
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int e = 4 * (tid + 256 * i);
      const int row = e / KC, k = e % KC;
      const bool wrap = q0 + k >= Q;
      const int n = n0 + (wrap ? 1 : 0), q = q0 + k - (wrap ? Q : 0);
      const bool ok = p0 + k < npix && co0 + row < CO;  // rows past CO: a 128-row tile over 64
      const int cr = co0 + row < CO ? co0 + row : CO - 1;
      const float4 t = *reinterpret_cast<const float4*>(
          gy + ((ok ? n : 0) * CO + cr) * Q + (ok ? q : 0));
      ra[i] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int e = 4 * (tid + 256 * i);
      const int row = e / KC, k = e % KC;
      const bool wrap = q0 + k >= Q;
      const int n = n0 + (wrap ? 1 : 0), q = q0 + k - (wrap ? Q : 0);
      const bool ok = p0 + k < npix && ci0 + row < CI;
      const int cr = ci0 + row < CI ? ci0 + row : CI - 1;
      const float* src = x + (int64_t)((ok ? n : 0) * CI + cr) * hwin;
      if constexpr (SIN == 1) {
        const float4 t = *reinterpret_cast<const float4*>(src + (ok ? q : 0));
        rb[i] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        float v[4];
        const int qb = ok ? q : 0;
        const int r = fdiv(qb, wo, inv_wo);
        int c = qb - r * wo, rr = r;
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // wo % 4 need not hold: step along the row
          const float t = src[(2 * rr) * win + 2 * c];
          v[j] = ok ? t : 0.f;
          if (++c == wo) {
            c = 0;
            ++rr;
          }
        }
        rb[i] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      const int e = 4 * (tid + 256 * i);
      const int row = e / KC, k = e % KC;
      *reinterpret_cast<float2*>(sA + row * KCP + k) = make_float2(ra[i].x, ra[i].y);
      *reinterpret_cast<float2*>(sA + row * KCP + k + 2) = make_float2(ra[i].z, ra[i].w);
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
      const int e = 4 * (tid + 256 * i);
      const int row = e / KC, k = e % KC;
      *reinterpret_cast<float2*>(sB + row * KCP + k) = make_float2(rb[i].x, rb[i].y);
      *reinterpret_cast<float2*>(sB + row * KCP + k + 2) = make_float2(rb[i].z, rb[i].w);
    }
  };

  f16v acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const float* pa = sA + (wm * 32 * MT + li) * KCP + h;
  const float* pb = sB + (wn * 32 * NT + li) * KCP + h;
  if (c_begin < c_end) load(c_begin);
  for (int c = c_begin; c < c_end; ++c) {
    __syncthreads();
    store();
    __syncthreads();
    if (c + 1 < c_end) load(c + 1);
#pragma unroll
    for (int s = 0; s < KC / 2; ++s) {
      float a[MT], b[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = pa[i * 32 * KCP + 2 * s];
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = pb[j * 32 * KCP + 2 * s];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
  }
  // D: lane column = ci (li), rows = co (r & 3) + 8 (r >> 2) + 4 h
  float* pp = part + (int64_t)ks * CO * CI;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm * 32 * MT + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int ci = ci0 + wn * 32 * NT + 32 * j + li;
        if (co < CO && ci < CI) pp[(int64_t)co * CI + ci] = acc[i][j][r];
      }
}

// gw[e] = sum_s part[s][e] in a fixed order (E % 4 == 0): a block owns 64
// float4 columns; its 16 waves sum the slabs s = w, w + 16, ... (lane = column,
// four loads in flight), then wave 0 adds the 16 wave sums in wave order.
__global__ void __launch_bounds__(1024)
    c1_wreduce_kernel(const float* __restrict__ part, float* __restrict__ gw, int64_t E, int ks) {
  __shared__ float4 red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t e4 = (int64_t)blockIdx.x * 64 + lane;
  const bool ok = 4 * e4 < E;
  const float4* p4 = reinterpret_cast<const float4*>(part);
  const int64_t E4 = E / 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  int s = wv;
  for (; s + 48 < ks; s += 64) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ok ? p4[(int64_t)(s + 16 * u) * E4 + e4] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a.x += v[u].x;
      a.y += v[u].y;
      a.z += v[u].z;
      a.w += v[u].w;
    }
  }
  for (; s < ks; s += 16) {
    const float4 v = ok ? p4[(int64_t)s * E4 + e4] : make_float4(0.f, 0.f, 0.f, 0.f);
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    a.w += v.w;
  }
  red[wv][lane] = a;
  __syncthreads();
  if (wv == 0 && ok) {
    float4 t = red[0][lane];
    for (int k = 1; k < 16; ++k) {
      const float4 b = red[k][lane];
      t.x += b.x;
      t.y += b.y;
      t.z += b.z;
      t.w += b.w;
    }
    reinterpret_cast<float4*>(gw)[e4] = t;
  }
}

// ------------------------------------------- weight gradient, small channel counts
// G[co][ci] for stride-1 convs whose whole (co, ci) block is a few 16 x 16
// MFMA tiles (MobileNetV3's expand / project 1x1s: 16..120 channels,
// mobilenetv3.py LARGE) -- HBM-bound, where the 128 x 32 tiles of
// c1_wgrad_kernel multiplied up to 4x padding and re-staged gy rows.  No LDS
// staging: wave = a 16 * MT x 16 * NT block of G over chunks of 16 pixels of
// one image (Q % 16 == 0); lane (l16, g4) loads 4 consecutive pixels of gy row
// co = 16 i + l16 and of x row ci = 16 j + l16 as float4 (16 rows x 64 B per
// load) and feeds them to v_mfma_f32_16x16x4_f32 k-step by k-step (MFMA k =
// g4 at step s <-> pixel 4 g4 + s, the same map on both operands).  The 4
// waves of a block sum through LDS in a fixed order into one partial row per
// block; c1_wreduce_kernel sums the rows in a fixed order.
using f4v = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma16(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int MT, int NT>
__global__ void __launch_bounds__(256)
    c1_wgrad_small_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                          float* __restrict__ part, int CO, int CI, int Q, int64_t nchunks,
                          int64_t per_block, int groups_ci) {
  __shared__ f4v red[3][MT * NT][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, l16 = lane & 15, g4 = lane >> 4;
  const int gco = blockIdx.y / groups_ci, gci = blockIdx.y - gco * groups_ci;
  const int co0 = gco * 16 * MT, ci0 = gci * 16 * NT;
  const int64_t c0 = (int64_t)blockIdx.x * per_block;
  const int64_t c1 = c0 + per_block < nchunks ? c0 + per_block : nchunks;
  f4v acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  // rows past CO / CI read row 0 (a real address) and are zeroed
  bool aok[MT], bok[NT];
  int64_t aoff[MT], boff[NT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int co = co0 + 16 * i + l16;
    aok[i] = co < CO;
    aoff[i] = (int64_t)(aok[i] ? co : 0) * Q;
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int ci = ci0 + 16 * j + l16;
    bok[j] = ci < CI;
    boff[j] = (int64_t)(bok[j] ? ci : 0) * Q;
  }
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
  for (int64_t c = c0 + wv; c < c1; c += 4) {
    const int64_t p0 = c * 16;
    const int64_t img = p0 / Q;
    const int64_t q = p0 - img * Q + 4 * g4;
    const float* gb = gy + img * CO * Q + q;
    const float* xb = x + img * CI * Q + q;
    float4 a[MT], b[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const float4 t = *reinterpret_cast<const float4*>(gb + aoff[i]);
      a[i] = aok[i] ? t : z;
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float4 t = *reinterpret_cast<const float4*>(xb + boff[j]);
      b[j] = bok[j] ? t : z;
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[i][j] = mfma16(a[i].x, b[j].x, acc[i][j]);
        acc[i][j] = mfma16(a[i].y, b[j].y, acc[i][j]);
        acc[i][j] = mfma16(a[i].z, b[j].z, acc[i][j]);
        acc[i][j] = mfma16(a[i].w, b[j].w, acc[i][j]);
      }
  }
  if (wv > 0) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) red[wv - 1][i * NT + j][lane] = acc[i][j];
  }
  __syncthreads();
  if (wv != 0) return;
  float* out = part + (int64_t)blockIdx.x * CO * CI;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      f4v t = acc[i][j];
#pragma unroll
      for (int k = 0; k < 3; ++k) t += red[k][i * NT + j][lane];  // waves in order
      const int ci = ci0 + 16 * j + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + 16 * i + 4 * g4 + r;  // D[4 g4 + r][l16]
        if (co < CO && ci < CI) out[(int64_t)co * CI + ci] = t[r];
      }
    }
}

// ------------------------------------------------- small-channel channel mix
// MobileNetV3's stride-1 expand / project convs (16 -> 64, 64 -> 24, 24 -> 72,
// 72 -> 40, 40 -> 120, ... on 240x320 .. 60x80 planes) and their data
// gradients: K and M <= 128, so cm_kernel's 32-row K chunks and 32..128-row M
// tiles are mostly padding and its LDS staging of the pixel tile buys no
// reuse.  Here one wave owns 64 consecutive pixels of one image and every
// output channel: lane (l16, g4) loads the float4 in[k0 + g4][q0 + 4 l16 ..
// + 3] (16 lanes read one 256-byte row segment), element t of it is the B
// operand of pixel tile t (pixels 4 l16 + t), so the four accumulators of one
// channel tile hold four consecutive pixels per lane and every output row is
// one float4 store per lane.  A (the M x K weight, zero-padded to 16 MT rows)
// sits in LDS as [k][m], pitch P with P mod 64 in {16, 48} (the four k rows of
// one read land in distinct banks).  Accumulation order over k is fixed.
template <int MT, bool TRANSA>
__global__ void __launch_bounds__(256)
    c1_mix_small_kernel(const float* __restrict__ in, const float* __restrict__ wt,
                        float* __restrict__ out, int K, int M, int Q, int qchunks,
                        int64_t total) {
  constexpr int P = 16 * MT + (MT % 2 == 0 ? 16 : 0);
  extern __shared__ float sw[];  // K x P
  for (int e = threadIdx.x; e < K * P; e += 256) {
    const int k = e / P, m = e - k * P;
    float v = 0.f;
    if (m < M) v = TRANSA ? wt[(int64_t)k * M + m] : wt[(int64_t)m * K + k];
    sw[e] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, l16 = lane & 15, g4 = lane >> 4;
  const int64_t c = (int64_t)blockIdx.x * 4 + wv;
  if (c >= total) return;
  const int64_t img = c / qchunks;
  const int q = (int)(c - img * qchunks) * 64 + 4 * l16;
  const bool qok = q < Q;  // Q % 4 == 0: a float4 is all in or all out
  const float* xb = in + img * K * Q + (qok ? q : 0);
  f4v acc[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int k0 = 0; k0 < K; k0 += 32) {
    // (f4v, not float4: a select between float4 temporaries goes to scratch)
    f4v b[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int k = k0 + 4 * s + g4;  // K % 8 == 0: the step is all in or all out
      const bool ok = qok && k0 + 4 * s < K;
      const f4v t = *reinterpret_cast<const f4v*>(xb + (ok ? (int64_t)k * Q : 0));
      b[s] = ok ? t : f4v{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (k0 + 4 * s < K) {
        const float* pa = sw + (k0 + 4 * s + g4) * P + l16;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const float a = pa[16 * i];
          acc[i][0] = mfma16(a, b[s][0], acc[i][0]);
          acc[i][1] = mfma16(a, b[s][1], acc[i][1]);
          acc[i][2] = mfma16(a, b[s][2], acc[i][2]);
          acc[i][3] = mfma16(a, b[s][3], acc[i][3]);
        }
      }
    }
  }
  if (!qok) return;
  float* ob = out + img * M * Q + q;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * i + 4 * g4 + r;  // D[4 g4 + r][l16]
      if (m < M)
        *reinterpret_cast<float4*>(ob + (int64_t)m * Q) =
            make_float4(acc[i][0][r], acc[i][1][r], acc[i][2][r], acc[i][3][r]);
    }
}

inline bool c1_mix_small_on() {
  static const bool on = [] {
    const char* e = std::getenv("MDE_C1_MIX_SMALL");
    return !(e && e[0] == '0');
  }();
  return on;
}

// c1_mix_small_kernel's M tiles for an (M, K) channel mix, or 0: stride 1,
// M, K <= 128 off the 32 grid (DDRNet's 32-multiples keep cm_kernel), the
// padded weight <= 32 KB of LDS.
inline int mix_small_mt(int64_t M, int64_t K) {
  if (!c1_mix_small_on() || M > 128 || K > 128 || (M % 32 == 0 && K % 32 == 0)) return 0;
  const int mt = (int)mde::cdiv(M, 16);
  const int p = 16 * mt + (mt % 2 == 0 ? 16 : 0);
  return K * p <= 8192 ? mt : 0;
}

template <bool TRANSA>
int launch_mix_small(int mt, const float* in, const float* wt, float* out, int64_t n, int64_t K,
                     int64_t M, int64_t Q, int kid, double bytes, double flops, hipStream_t s) {
  const int64_t qchunks = mde::cdiv(Q, 64), total = n * qchunks;
  const dim3 grid((unsigned)mde::cdiv(total, 4)), block(256);
  const size_t lds = sizeof(float) * (size_t)K * (16 * mt + (mt % 2 == 0 ? 16 : 0));
#define MDE_MIX(MTv)                                                                           \
  case MTv:                                                                                    \
    MDE_LAUNCH_MFMA(kid, bytes, flops, s, (c1_mix_small_kernel<MTv, TRANSA>), grid, block, lds, \
                    in, wt, out, (int)K, (int)M, (int)Q, (int)qchunks, total);                 \
    return MDE_OK;
  switch (mt) {
    MDE_MIX(1)
    MDE_MIX(2)
    MDE_MIX(3)
    MDE_MIX(4)
    MDE_MIX(5)
    MDE_MIX(6)
    MDE_MIX(7)
    MDE_MIX(8)
    default:
      return MDE_ERR_UNSUPPORTED;
  }
#undef MDE_MIX
}

struct SmallWg {
  int mt, nt, groups_ci, groups;
  int64_t nchunks, per_block, blocks;
};

inline bool c1_small_on() {
  static const bool on = [] {
    const char* e = std::getenv("MDE_C1_SMALL");
    return !(e && e[0] == '0');
  }();
  return on;
}

// the small-channel path: stride 1, Q % 16 == 0, at most 8 MFMA tiles a wave
// and 3 wave groups (co / ci up to ~128 x 48)
inline bool small_plan(int64_t n, int64_t ci, int64_t co, int64_t q, SmallWg* p) {
  if (!c1_small_on() || q % 16) return false;
  if (ci % 32 == 0 && co % 32 == 0) return false;  // the 32-grid shapes keep c1_wgrad_kernel
  const int co16 = (int)mde::cdiv(co, 16), ci16 = (int)mde::cdiv(ci, 16);
  if (co16 * ci16 > 24) return false;
  // wave tile MT x NT (MT * NT <= 8, MT, NT in {1, 2, 4, 8}) covering the
  // most of (co16, ci16) with the fewest groups
  int bm = 0, bn = 0, best = 1 << 30;
  for (int mt : {1, 2, 4, 8})
    for (int nt : {1, 2, 4, 8}) {
      if (mt * nt > 8) continue;
      const int g = (int)(mde::cdiv(co16, mt) * mde::cdiv(ci16, nt));
      const int waste = g * mt * nt;  // tiles computed
      if (g <= 3 && waste < best) {
        best = waste;
        bm = mt;
        bn = nt;
      }
    }
  if (!bm) return false;
  p->mt = bm;
  p->nt = bn;
  p->groups_ci = (int)mde::cdiv(ci16, bn);
  p->groups = (int)mde::cdiv(co16, bm) * p->groups_ci;
  p->nchunks = n * q / 16;
  int64_t blocks = 512 / p->groups;  // one partial row a block, summed by c1_wreduce_kernel
  if (blocks > p->nchunks / 4) blocks = p->nchunks / 4 > 1 ? p->nchunks / 4 : 1;
  p->per_block = mde::cdiv(p->nchunks, blocks);
  p->blocks = mde::cdiv(p->nchunks, p->per_block);
  return true;
}

inline size_t small_ws_bytes(const SmallWg& p, int64_t ci, int64_t co) {
  return sizeof(float) * (size_t)(p.blocks * ci * co);
}

// ------------------------------------------------------------------- plans
inline bool c1_shape_ok(int64_t n, int64_t ci, int64_t co, int64_t h, int64_t w, int stride) {
  if (n <= 0 || h <= 0 || w <= 0 || (stride != 1 && stride != 2)) return false;
  // multiples of 8 (padded to 32 in the kernels, PAD), >= 16
  if (ci % 8 || co % 8 || ci < 16 || co < 16) return false;
  const int64_t ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  if ((ho * wo) % 4) return false;
  if (stride == 2 && w % 2) return false;  // gx rows written as (value, 0) pairs
  return n * ci * h * w < (int64_t)1 << 31 && n * co * ho * wo < (int64_t)1 << 31 &&
         ho * wo >= KC && ho < (1 << 12) && wo < (1 << 10);
}

// M-tile of the channel mix: 128 when M % 128 == 0, else 64, else 32.
inline int cm_bm(int64_t m) { return m % 128 == 0 ? 128 : (m % 64 == 0 ? 64 : 32); }

template <int SIN, int SOUT, bool TRANSA>
int launch_cm(const float* in, const float* wt, float* out, int64_t n, int64_t K, int64_t M,
              int64_t hin, int64_t win, int64_t ho, int64_t wo, int64_t hout, int64_t wout,
              int kid, double bytes, double flops, hipStream_t s) {
  const int64_t Q = ho * wo;
  const int bm = cm_bm(M);
  constexpr int BQ = 128;
  const int64_t qtiles = mde::cdiv(Q, BQ), mtiles = mde::cdiv(M, bm);
  const int64_t total = n * qtiles * mtiles;
  if (total > 0x7fffffff) return MDE_ERR_INVALID_ARG;
  const dim3 grid(xcd_grid(total)), block(256);
  const bool pad = K % KC || M % bm;
#define MDE_CM(BMv, MTv, QTv)                                                                     \
  do {                                                                                            \
    if (pad)                                                                                      \
      MDE_LAUNCH_MFMA(kid, bytes, flops, s,                                                       \
                      (cm_kernel<BMv, BQ, MTv, QTv, SIN, SOUT, TRANSA, true>), grid, block, 0,    \
                      in, wt, out, (int)K, (int)M, (int)hin, (int)win, (int)wo, (int)Q,           \
                      (int)hout, (int)wout, (int)qtiles, (int)mtiles, (int)total);                \
    else                                                                                          \
      MDE_LAUNCH_MFMA(kid, bytes, flops, s, (cm_kernel<BMv, BQ, MTv, QTv, SIN, SOUT, TRANSA>),    \
                      grid, block, 0, in, wt, out, (int)K, (int)M, (int)hin, (int)win, (int)wo,   \
                      (int)Q, (int)hout, (int)wout, (int)qtiles, (int)mtiles, (int)total);        \
  } while (0)
  if (bm == 128)
    MDE_CM(128, 2, 2);
  else if (bm == 64)
    MDE_CM(64, 2, 1);
  else
    MDE_CM(32, 1, 1);
#undef MDE_CM
  return MDE_OK;
}

struct WgPlan {
  int bco, bci, cotiles, citiles, ksplit, nchunks;
  int64_t npix;
};

inline WgPlan wg_plan(int64_t n, int64_t ci, int64_t co, int64_t ho, int64_t wo) {
  // block tiles with four 32-multiple wave tiles: 128x128, 128x64, 64x128,
  // 64x64, and 128x32 / 32x128 (the 32-channel side; the other side padded
  // to 128 rows and masked when it is 64)
  WgPlan p;
  const int a = co % 128 == 0 ? 128 : (co % 64 == 0 ? 64 : 32);
  const int b = ci % 128 == 0 ? 128 : (ci % 64 == 0 ? 64 : 32);
  if (b == 32) {
    p.bco = 128;
    p.bci = 32;
  } else if (a == 32) {
    p.bco = 32;
    p.bci = 128;
  } else {
    p.bco = a;
    p.bci = b;
  }
  p.cotiles = (int)mde::cdiv(co, p.bco);
  p.citiles = (int)mde::cdiv(ci, p.bci);
  p.npix = n * ho * wo;
  p.nchunks = (int)mde::cdiv(p.npix, KC);
  const int tiles = p.cotiles * p.citiles;
  // ~512 blocks (two per CU), at least 8 chunks per block, slab <= 64 MB
  int ks = (int)mde::cdiv(512, tiles);
  if (ks > p.nchunks / 8) ks = p.nchunks / 8;
  const int64_t cap = ((int64_t)16 << 20) / (ci * co);
  if (ks > cap) ks = (int)cap;
  p.ksplit = ks < 1 ? 1 : ks;
  return p;
}

}  // namespace

extern "C" {

int mde_conv1x1_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int stride,
                          int dtype) {
  return dtype == MDE_F32 && c1_shape_ok(1, cin, cout, h, w, stride) ? 1 : 0;
}

int mde_conv1x1_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t cin,
                    int64_t cout, int64_t h, int64_t w, int stride, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !weight || !y) return MDE_ERR_INVALID_ARG;
  if (!c1_shape_ok(n, cin, cout, h, w, stride)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int64_t ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  const double flops = 2.0 * n * ho * wo * (double)cin * cout;
  const double bytes = 4.0 * n * (double)ho * wo * (cin + cout);
  if (stride == 1) {
    if (const int mt = mix_small_mt(cout, cin))
      return launch_mix_small<false>(mt, (const float*)x, weight, (float*)y, n, cin, cout, ho * wo,
                                     mde::K_C1_FWD, bytes, flops, s);
    return launch_cm<1, 1, false>((const float*)x, weight, (float*)y, n, cin, cout, h, w, ho, wo,
                                  ho, wo, mde::K_C1_FWD, bytes, flops, s);
  }
  return launch_cm<2, 1, false>((const float*)x, weight, (float*)y, n, cin, cout, h, w, ho, wo,
                                ho, wo, mde::K_C1_FWD, bytes, flops, s);
}

int mde_conv1x1_bwd_data(const void* gy, const float* weight, void* gx, int64_t n, int64_t cin,
                         int64_t cout, int64_t h, int64_t w, int stride, int dtype,
                         void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !weight || !gx) return MDE_ERR_INVALID_ARG;
  if (!c1_shape_ok(n, cin, cout, h, w, stride)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int64_t ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  const double flops = 2.0 * n * ho * wo * (double)cin * cout;
  const double bytes = 4.0 * n * ((double)ho * wo * cout + (double)h * w * cin);
  // GEMM K = cout (gy's channels), M = cin; gy is a ho x wo plane
  if (stride == 1) {
    if (const int mt = mix_small_mt(cin, cout))
      return launch_mix_small<true>(mt, (const float*)gy, weight, (float*)gx, n, cout, cin, ho * wo,
                                    mde::K_C1_DGRAD, bytes, flops, s);
    return launch_cm<1, 1, true>((const float*)gy, weight, (float*)gx, n, cout, cin, ho, wo, ho,
                                 wo, h, w, mde::K_C1_DGRAD, bytes, flops, s);
  }
  return launch_cm<1, 2, true>((const float*)gy, weight, (float*)gx, n, cout, cin, ho, wo, ho, wo,
                               h, w, mde::K_C1_DGRAD, bytes, flops, s);
}

size_t mde_conv1x1_wgrad_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                                   int stride, int dtype) {
  if (dtype != MDE_F32 || !c1_shape_ok(n, cin, cout, h, w, stride)) return 0;
  const int64_t ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  SmallWg sp;
  if (stride == 1 && small_plan(n, cin, cout, ho * wo, &sp)) return small_ws_bytes(sp, cin, cout);
  const WgPlan p = wg_plan(n, cin, cout, ho, wo);
  return sizeof(float) * (size_t)p.ksplit * (size_t)(cin * cout);
}

int mde_conv1x1_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t cin,
                      int64_t cout, int64_t h, int64_t w, int stride, void* workspace, int dtype,
                      void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !x || !gweight || !workspace) return MDE_ERR_INVALID_ARG;
  if (!c1_shape_ok(n, cin, cout, h, w, stride)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int64_t ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  SmallWg sp;
  if (stride == 1 && small_plan(n, cin, cout, ho * wo, &sp)) {
    const double flops = 2.0 * n * ho * wo * (double)cin * cout;
    const double bytes = 4.0 * n * (double)ho * wo * (cin + cout);
    float* part = (float*)workspace;
    const int64_t E = cin * cout;
    const dim3 grid((unsigned)sp.blocks, (unsigned)sp.groups);
#define MDE_WGS(MTv, NTv)                                                                          \
  if (sp.mt == MTv && sp.nt == NTv)                                                                \
    MDE_LAUNCH_MFMA(mde::K_C1_WGRAD, bytes, flops, s, (c1_wgrad_small_kernel<MTv, NTv>), grid,     \
                    dim3(256), 0, (const float*)gy, (const float*)x, part, (int)cout, (int)cin,    \
                    (int)(ho * wo), sp.nchunks, sp.per_block, sp.groups_ci);
    MDE_WGS(1, 1) else MDE_WGS(1, 2) else MDE_WGS(1, 4) else MDE_WGS(1, 8)
    else MDE_WGS(2, 1) else MDE_WGS(2, 2) else MDE_WGS(2, 4)
    else MDE_WGS(4, 1) else MDE_WGS(4, 2) else MDE_WGS(8, 1) else return MDE_ERR_UNSUPPORTED;
#undef MDE_WGS
    MDE_LAUNCH(mde::K_C1_WREDUCE, 4.0 * E * (sp.blocks + 1), s, c1_wreduce_kernel,
               dim3((unsigned)mde::cdiv(E / 4, 64)), dim3(1024), 0, (const float*)part, gweight, E,
               (int)sp.blocks);
    return MDE_OK;
  }
  const WgPlan p = wg_plan(n, cin, cout, ho, wo);
  const int64_t total = (int64_t)p.cotiles * p.citiles * p.ksplit;
  const dim3 grid(xcd_grid(total)), block(256);
  const double flops = 2.0 * n * ho * wo * (double)cin * cout;
  const double bytes = 4.0 * n * (double)ho * wo * (cin + cout);
  float* part = (float*)workspace;
  const int Q = (int)(ho * wo);
#define MDE_WG(BCO, BCI, MTv, NTv, SINv)                                                          \
  MDE_LAUNCH_MFMA(mde::K_C1_WGRAD, bytes, flops, s, (c1_wgrad_kernel<BCO, BCI, MTv, NTv, SINv>), \
                  grid, block, 0, (const float*)gy, (const float*)x, part, (int)cout, (int)cin, Q, \
                  (int)h, (int)w, (int)wo, p.npix, p.nchunks, p.ksplit, p.cotiles, p.citiles,     \
                  (int)total)
#define MDE_WG_S(SINv)                       \
  do {                                       \
    if (p.bco == 128 && p.bci == 128)        \
      MDE_WG(128, 128, 2, 2, SINv);          \
    else if (p.bco == 128 && p.bci == 64)    \
      MDE_WG(128, 64, 2, 1, SINv);           \
    else if (p.bco == 64 && p.bci == 128)    \
      MDE_WG(64, 128, 1, 2, SINv);           \
    else if (p.bco == 64 && p.bci == 64)     \
      MDE_WG(64, 64, 1, 1, SINv);            \
    else if (p.bci == 32)                    \
      MDE_WG(128, 32, 1, 1, SINv);           \
    else                                     \
      MDE_WG(32, 128, 1, 1, SINv);           \
  } while (0)
  if (stride == 1)
    MDE_WG_S(1);
  else
    MDE_WG_S(2);
#undef MDE_WG_S
#undef MDE_WG
  const int64_t E = cin * cout;
  MDE_LAUNCH(mde::K_C1_WREDUCE, 4.0 * E * (p.ksplit + 1), s, c1_wreduce_kernel,
             dim3((unsigned)mde::cdiv(E / 4, 64)), dim3(1024), 0, part, gweight, E, p.ksplit);
  return MDE_OK;
}

}  // extern "C"
