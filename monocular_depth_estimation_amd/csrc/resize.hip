// Bilinear and nearest resizes (NCHW; bilinear on fp32 or bf16 storage, fp32
// arithmetic) for gfx950.
//
// Index math follows ATen's area_pixel_compute_source_index /
// nearest_neighbor_compute_source_index so the sampled pixels and the
// interpolation weights are the ones the reference's F.interpolate calls use
// (src/GuideDepth/model/GuideDepth.py:46-55, DDRNet_23_slim.py:182-191,
// 332-351).  Products are written with __fmul_rn/__fadd_rn so hipcc cannot
// contract them into FMAs: a contracted source index could floor to a
// different pixel than the reference near integer boundaries.
//
// Backward is a gather: every input pixel sums the output gradients whose
// stencil touches it, so there are no atomics and gx is written exactly once.
#include <cmath>
#include <cstdlib>

#include "common.h"

namespace {

struct Lin {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ float src_index(float scale, int dst, int align) {
  if (align) return __fmul_rn(scale, (float)dst);
  float s = __fadd_rn(__fmul_rn(scale, __fadd_rn((float)dst, 0.5f)), -0.5f);
  return s < 0.f ? 0.f : s;
}

__device__ __forceinline__ Lin lin_index(float scale, int dst, int in_size,
                                         int align) {
  const float s = src_index(scale, dst, align);
  int i0 = (int)s;  // s >= 0, so truncation is floor
  if (i0 > in_size - 1) i0 = in_size - 1;
  const int i1 = i0 + (i0 < in_size - 1 ? 1 : 0);
  float l1 = __fadd_rn(s, -(float)i0);
  l1 = fminf(fmaxf(l1, 0.f), 1.f);
  return {i0, i1, __fadd_rn(1.f, -l1), l1};
}

// l0 a + l1 b with the rounding pinned (one product, one fused multiply-add):
// the fp32 and bf16-storage instantiations of a kernel must not let the
// compiler contract the sum differently (bf16 results == rounded fp32 ones).
__device__ __forceinline__ float lerp2(const Lin& L, float a, float b) {
  return __fmaf_rn(L.l1, b, __fmul_rn(L.l0, a));
}
__device__ __forceinline__ float madd(float w, float v, float acc) { return __fmaf_rn(w, v, acc); }

// Weight with which output index `o` reads input index `i` along one axis.
__device__ __forceinline__ float lin_weight(float scale, int o, int i,
                                            int in_size, int align) {
  const Lin L = lin_index(scale, o, in_size, align);
  float w = 0.f;
  if (L.i0 == i) w += L.l0;
  if (L.i1 == i) w += L.l1;
  return w;
}

// Output-index window that can read input index i (generic ratios).
__device__ __forceinline__ void lin_window(float scale, int i, int out_size,
                                           int* lo, int* hi) {
  if (!(scale > 0.f)) {
    *lo = 0;
    *hi = out_size - 1;
    return;
  }
  const int a = (int)floorf(((float)i - 1.f) / scale) - 2;
  const int b = (int)ceilf(((float)i + 2.f) / scale) + 1;
  *lo = a < 0 ? 0 : a;
  *hi = b > out_size - 1 ? out_size - 1 : b;
}

// Forward, generic ratio: each thread produces VEC consecutive outputs of
// kFwdRows consecutive output rows of one plane.  The column indices and
// weights (W) are computed once per thread, the row ones (H) once per row;
// the decomposition of the thread index is 32-bit (the host checks that the
// thread count fits).  Input rows are gathered (L1 / L2 hits: a row feeds
// many outputs at upsampling ratios); output rows leave as VEC-wide stores.
constexpr int kFwdRows = 4;

template <int VEC, typename T>
__global__ void __launch_bounds__(256)
    bilinear_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int total, int hi, int wi,
                        int ho, int wo, float sh, float sw, int align) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int chunks = (wo + VEC - 1) / VEC;
  const int groups = (ho + kFwdRows - 1) / kFwdRows;
  const int ch = t % chunks;
  const int rg = t / chunks;
  const int plane = rg / groups;
  const int oh0 = (rg - plane * groups) * kFwdRows;
  Lin W[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    const int ow = ch * VEC + k;
    W[k] = lin_index(sw, ow < wo ? ow : wo - 1, wi, align);
  }
  const T* xp = x + (int64_t)plane * hi * wi;
#pragma unroll
  for (int r = 0; r < kFwdRows; ++r) {
    const int oh = oh0 + r;
    if (oh >= ho) break;
    const Lin H = lin_index(sh, oh, hi, align);
    const T* r0 = xp + (int64_t)H.i0 * wi;
    const T* r1 = xp + (int64_t)H.i1 * wi;
    float v[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k)
      v[k] = lerp2(H, lerp2(W[k], mde::ld1(r0 + W[k].i0), mde::ld1(r0 + W[k].i1)),
                   lerp2(W[k], mde::ld1(r1 + W[k].i0), mde::ld1(r1 + W[k].i1)));
    T* out = y + ((int64_t)plane * ho + oh) * wo + ch * VEC;
    if (VEC == 4 && ch * VEC + 4 <= wo) {
      mde::st4(out, make_float4(v[0], v[1], v[2], v[3]));
    } else {
#pragma unroll
      for (int k = 0; k < VEC; ++k)
        if (ch * VEC + k < wo) mde::st1(out + k, v[k]);
    }
  }
}

inline int64_t fwd_threads(int64_t planes, int64_t ho, int64_t wo, int vec) {
  return planes * mde::cdiv(ho, kFwdRows) * mde::cdiv(wo, vec);
}

// Exact x2 (align_corners=False, scale 0.5, out = 2*in).  With ATen's
// source-index clamp the x2 stencil is a 2-tap filter with clamped indices:
//   out[2i]   = 0.25 x[max(i-1,0)]  + 0.75 x[i]
//   out[2i+1] = 0.75 x[i] + 0.25 x[min(i+1,in-1)]
// per axis (rows of horizontally interpolated columns, as ATen orders it),
// and its adjoint is the 4-tap filter (0.25 0.75 0.75 0.25) over output
// indices 2i-1..2i+2, again clamped.  One thread owns one input column and
// slides down RS rows, so every input (fwd) / output-gradient (bwd) row is
// read once per thread and every result is written once, coalesced.
constexpr int kX2Rows = 8;   // rows per thread
constexpr int kX2Warps = 4;  // threadIdx.y

template <typename T>
__device__ __forceinline__ float2 x2_hrow(const T* row, int j, int wi) {
  const float l = mde::ld1(row + (j > 0 ? j - 1 : 0));
  const float c = mde::ld1(row + j);
  const float r = mde::ld1(row + (j < wi - 1 ? j + 1 : wi - 1));
  return make_float2(0.25f * l + 0.75f * c, 0.75f * c + 0.25f * r);
}

template <typename T>
__global__ void __launch_bounds__(64 * kX2Warps)
    bilinear_fwd_x2_kernel(const T* __restrict__ x, T* __restrict__ y, int hi, int wi) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  const int i0 = (blockIdx.y * kX2Warps + threadIdx.y) * kX2Rows;
  if (j >= wi || i0 >= hi) return;
  const int64_t plane = blockIdx.z;
  const T* xp = x + plane * hi * (int64_t)wi;
  const int wo = 2 * wi;
  T* yp = y + plane * (2 * hi) * (int64_t)wo + 2 * j;
  float2 prev = x2_hrow(xp + (int64_t)(i0 > 0 ? i0 - 1 : 0) * wi, j, wi);
  float2 cur = x2_hrow(xp + (int64_t)i0 * wi, j, wi);
  const int i1 = i0 + kX2Rows < hi ? i0 + kX2Rows : hi;
  for (int i = i0; i < i1; ++i) {
    const float2 nxt = x2_hrow(xp + (int64_t)(i < hi - 1 ? i + 1 : hi - 1) * wi, j, wi);
    mde::st2(yp + (int64_t)(2 * i) * wo,
             make_float2(0.25f * prev.x + 0.75f * cur.x, 0.25f * prev.y + 0.75f * cur.y));
    mde::st2(yp + (int64_t)(2 * i + 1) * wo,
             make_float2(0.75f * cur.x + 0.25f * nxt.x, 0.75f * cur.y + 0.25f * nxt.y));
    prev = cur;
    cur = nxt;
  }
}

// Forward with two input columns per thread (wi even): one float2 of each
// input row (+ the neighbours from the adjacent lanes by wave shuffles)
// gives four consecutive outputs of two output rows, written as float4.
template <typename T>
__global__ void __launch_bounds__(64 * kX2Warps)
    bilinear_fwd_x2_pair_kernel(const T* __restrict__ x, T* __restrict__ y, int hi, int wi) {
  const int lane = threadIdx.x;
  const int j0 = 2 * (blockIdx.x * 64 + lane);
  const int i0 = (blockIdx.y * kX2Warps + threadIdx.y) * kX2Rows;
  if (i0 >= hi) return;  // uniform per wave
  const bool ok = j0 < wi;
  const int jc = ok ? j0 : 0;
  const int64_t plane = blockIdx.z;
  const T* xp = x + plane * hi * (int64_t)wi;
  const int wo = 2 * wi;
  T* yp = y + plane * (2 * hi) * (int64_t)wo + 2 * jc;
  // horizontally interpolated input row r: outputs 2j0 .. 2j0+3
  auto hrow = [&](int r) {
    r = r < 0 ? 0 : (r > hi - 1 ? hi - 1 : r);
    const T* row = xp + (int64_t)r * wi;
    const float2 c = mde::ld2(row + jc);
    float l = __shfl_up(c.y, 1, 64), rr = __shfl_down(c.x, 1, 64);
    if (lane == 0) l = mde::ld1(row + (jc > 0 ? jc - 1 : 0));
    if (lane == 63 || jc + 2 >= wi) rr = mde::ld1(row + (jc + 2 < wi ? jc + 2 : wi - 1));
    return make_float4(0.25f * l + 0.75f * c.x, 0.75f * c.x + 0.25f * c.y,
                       0.25f * c.x + 0.75f * c.y, 0.75f * c.y + 0.25f * rr);
  };
  float4 prev = hrow(i0 - 1), cur = hrow(i0);
#pragma unroll
  for (int k = 0; k < kX2Rows; ++k) {
    const int i = i0 + k;
    if (i >= hi) break;  // uniform per wave
    const float4 nxt = hrow(i + 1);
    if (ok) {
      mde::st4(yp + (int64_t)(2 * i) * wo,
               make_float4(0.25f * prev.x + 0.75f * cur.x, 0.25f * prev.y + 0.75f * cur.y,
                           0.25f * prev.z + 0.75f * cur.z, 0.25f * prev.w + 0.75f * cur.w));
      mde::st4(yp + (int64_t)(2 * i + 1) * wo,
               make_float4(0.75f * cur.x + 0.25f * nxt.x, 0.75f * cur.y + 0.25f * nxt.y,
                           0.75f * cur.z + 0.25f * nxt.z, 0.75f * cur.w + 0.25f * nxt.w));
    }
    prev = cur;
    cur = nxt;
  }
}

// 4-tap adjoint filter of one output-gradient row at input column j.
template <typename T>
__device__ __forceinline__ float x2_hgrad(const T* row, int j, int wo) {
  const float2 m = mde::ld2(row + 2 * j);
  const float l = mde::ld1(row + (2 * j > 0 ? 2 * j - 1 : 0));
  const float r = mde::ld1(row + (2 * j + 2 < wo ? 2 * j + 2 : wo - 1));
  return 0.25f * l + 0.75f * m.x + 0.75f * m.y + 0.25f * r;
}

template <typename T>
__global__ void __launch_bounds__(64 * kX2Warps)
    bilinear_bwd_x2_kernel(const T* __restrict__ gy, T* __restrict__ gx, int hi, int wi) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  const int i0 = (blockIdx.y * kX2Warps + threadIdx.y) * kX2Rows;
  if (j >= wi || i0 >= hi) return;
  const int64_t plane = blockIdx.z;
  const int ho = 2 * hi, wo = 2 * wi;
  const T* gp = gy + plane * ho * (int64_t)wo;
  T* xp = gx + plane * hi * (int64_t)wi + j;
  auto hrow = [&](int o) {
    o = o < 0 ? 0 : (o > ho - 1 ? ho - 1 : o);
    return x2_hgrad(gp + (int64_t)o * wo, j, wo);
  };
  float a = hrow(2 * i0 - 1), b = hrow(2 * i0);
  const int i1 = i0 + kX2Rows < hi ? i0 + kX2Rows : hi;
  for (int i = i0; i < i1; ++i) {
    const float c = hrow(2 * i + 1), d = hrow(2 * i + 2);
    mde::st1(xp + (int64_t)i * wi, 0.25f * a + 0.75f * b + 0.75f * c + 0.25f * d);
    a = c;
    b = d;
  }
}

// Same adjoint, two input columns per thread (wi even): one float4 of each
// output-gradient row (columns 2j .. 2j+3) feeds both columns, the two
// neighbours 2j-1 / 2j+4 come from the adjacent lanes' float4 (wave shuffles;
// loads only at the wave's edges), results leave as float2 -- 1 load + 1/2
// store instruction per output row and column pair instead of 3 + 1 per
// column.  Rows are processed in a fully unrolled kX2Rows window so the
// loads of successive rows are all in flight together.
// TWO: the output feeds two consumers whose gradients gy and gy2 arrive
// separately (the guided-upsampling block's feature_conv and skip fusion,
// modules.py:89,100): summed on load, so autograd's accumulation pass (read
// both, write the sum, read it again here) never runs.
template <bool TWO = false, typename T = float>
__global__ void __launch_bounds__(64 * kX2Warps)
    bilinear_bwd_x2_pair_kernel(const T* __restrict__ gy, T* __restrict__ gx, int hi, int wi,
                                const T* __restrict__ gy2 = nullptr) {
  const int lane = threadIdx.x;
  const int j0 = 2 * (blockIdx.x * 64 + lane);  // input columns j0, j0 + 1
  const int i0 = (blockIdx.y * kX2Warps + threadIdx.y) * kX2Rows;
  if (i0 >= hi) return;  // uniform per wave
  const bool ok = j0 < wi;
  const int jc = ok ? j0 : 0;
  const int64_t plane = blockIdx.z;
  const int ho = 2 * hi, wo = 2 * wi;
  const T* gp = gy + plane * ho * (int64_t)wo;
  const T* gp2 = TWO ? gy2 + plane * ho * (int64_t)wo : nullptr;
  T* xp = gx + plane * hi * (int64_t)wi + jc;
  // pair-filtered row o: (gx-column j0 part, gx-column j0+1 part)
  auto hrow = [&](int o) {
    o = o < 0 ? 0 : (o > ho - 1 ? ho - 1 : o);
    const T* row = gp + (int64_t)o * wo;
    const T* row2 = TWO ? gp2 + (int64_t)o * wo : nullptr;
    float4 v = mde::ld4(row + 2 * jc);
    if (TWO) {
      const float4 v2 = mde::ld4(row2 + 2 * jc);
      v.x += v2.x; v.y += v2.y; v.z += v2.z; v.w += v2.w;
    }
    float l = __shfl_up(v.w, 1, 64), r = __shfl_down(v.x, 1, 64);
    if (lane == 0) {
      const int e = 2 * jc > 0 ? 2 * jc - 1 : 0;
      l = TWO ? mde::ld1(row + e) + mde::ld1(row2 + e) : mde::ld1(row + e);
    }
    if (lane == 63 || 2 * jc + 4 >= wo) {
      const int e = 2 * jc + 4 < wo ? 2 * jc + 4 : wo - 1;
      r = TWO ? mde::ld1(row + e) + mde::ld1(row2 + e) : mde::ld1(row + e);
    }
    return make_float2(0.25f * l + 0.75f * v.x + 0.75f * v.y + 0.25f * v.z,
                       0.25f * v.y + 0.75f * v.z + 0.75f * v.w + 0.25f * r);
  };
  float2 a = hrow(2 * i0 - 1), b = hrow(2 * i0);
#pragma unroll
  for (int k = 0; k < kX2Rows; ++k) {
    const int i = i0 + k;
    if (i >= hi) break;  // uniform per wave
    const float2 c = hrow(2 * i + 1), d = hrow(2 * i + 2);
    if (ok)
      mde::st2(xp + (int64_t)i * wi,
               make_float2(0.25f * a.x + 0.75f * b.x + 0.75f * c.x + 0.25f * d.x,
                           0.25f * a.y + 0.75f * b.y + 0.75f * c.y + 0.25f * d.y));
    a = c;
    b = d;
  }
}

// bf16 storage (cfg3 autocast), four input columns per lane (wi % 4 == 0): a
// lane's loads and stores are 8 / 16 bytes, as the fp32 pair kernels' are, so
// halving the element size halves the instructions per byte instead of the
// bytes per instruction.  Same filters, same fp32 arithmetic order as the
// pair kernels (bit-exact with them on the same values, rounded on store).
__device__ __forceinline__ void ld8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void ld8(const mde::bf16* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8(mde::bf16* p, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    w[k] = (uint32_t)mde::f2bf(v[2 * k]) | ((uint32_t)mde::f2bf(v[2 * k + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// Flat lane mapping: thread t -> (plane, band of kX2Rows input rows, column
// quad q), quads fastest, so a wave is fully used whatever wi is (20 quads per
// row at wi = 80).  Neighbour columns come from the adjacent lanes by wave
// shuffles, except at a row's first / last quad and the wave's edge lanes,
// which load them (clamped).  Every lane runs all kX2Rows rows (rows past the
// plane are clamped and not stored) so the shuffles never sit in divergent
// control flow.
struct QuadMap {
  int64_t total;  // planes * bands * quads
  int q, quads, i0;
  int64_t plane;
  bool live;
};

__device__ __forceinline__ QuadMap quad_map(int64_t planes, int hi, int wi) {
  QuadMap m;
  m.quads = wi >> 2;
  const int bands = (hi + kX2Rows - 1) / kX2Rows;
  m.total = planes * bands * (int64_t)m.quads;
  int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  m.live = t < m.total;
  if (!m.live) t = m.total - 1;
  m.q = (int)(t % m.quads);
  const int64_t r = t / m.quads;
  m.i0 = (int)(r % bands) * kX2Rows;
  m.plane = r / bands;
  return m;
}

template <typename T>
__global__ void __launch_bounds__(256)
    bilinear_fwd_x2_quad_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t planes,
                                int hi, int wi) {
  const int lane = threadIdx.x & 63;
  const QuadMap m = quad_map(planes, hi, wi);
  const int jc = 4 * m.q;
  const T* xp = x + m.plane * hi * (int64_t)wi;
  const int wo = 2 * wi;
  T* yp = y + m.plane * (2 * hi) * (int64_t)wo + 2 * jc;
  // Neighbour columns jc - 1 / jc + 4 (clamped).  bf16: plain loads by every
  // lane -- no lane shuffles and no branch around a load, so no wait inside
  // the unrolled rows (a conditional edge load made the compiler wait for
  // every load in flight; 16x240x320 backward 104 -> 77 us).  fp32: from the
  // adjacent lanes by shuffles, loads at the wave / row edges only (plain
  // loads measured 3-7 % slower there: twice the bytes per extra load).
  constexpr bool kPlain = sizeof(T) == 2;
  const bool ledge = lane == 0 || m.q == 0, redge = lane == 63 || m.q == m.quads - 1;
  const int el = jc > 0 ? jc - 1 : 0, er = jc + 4 < wi ? jc + 4 : wi - 1;
  // horizontally interpolated input row r: outputs 2jc .. 2jc+7
  auto hrow = [&](int r, float* o) {
    r = r < 0 ? 0 : (r > hi - 1 ? hi - 1 : r);
    const T* row = xp + (int64_t)r * wi;
    const float4 c = mde::ld4(row + jc);
    float l, rr;
    if constexpr (kPlain) {
      l = mde::ld1(row + el);
      rr = mde::ld1(row + er);
    } else {
      l = __shfl_up(c.w, 1, 64);
      rr = __shfl_down(c.x, 1, 64);
      if (ledge) l = mde::ld1(row + el);
      if (redge) rr = mde::ld1(row + er);
    }
    const float v[6] = {l, c.x, c.y, c.z, c.w, rr};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[2 * k] = 0.25f * v[k] + 0.75f * v[k + 1];
      o[2 * k + 1] = 0.75f * v[k + 1] + 0.25f * v[k + 2];
    }
  };
  float prev[8], cur[8];
  hrow(m.i0 - 1, prev);
  hrow(m.i0, cur);
#pragma unroll
  for (int k = 0; k < kX2Rows; ++k) {
    const int i = m.i0 + k;
    float nxt[8], a[8], b[8];
    hrow(i + 1, nxt);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      a[q] = 0.25f * prev[q] + 0.75f * cur[q];
      b[q] = 0.75f * cur[q] + 0.25f * nxt[q];
    }
    if (m.live && i < hi) {
      st8(yp + (int64_t)(2 * i) * wo, a);
      st8(yp + (int64_t)(2 * i + 1) * wo, b);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      prev[q] = cur[q];
      cur[q] = nxt[q];
    }
  }
}

template <bool TWO, typename T>
__global__ void __launch_bounds__(256)
    bilinear_bwd_x2_quad_kernel(const T* __restrict__ gy, T* __restrict__ gx, int64_t planes,
                                int hi, int wi, const T* __restrict__ gy2) {
  const int lane = threadIdx.x & 63;
  const QuadMap m = quad_map(planes, hi, wi);
  const int jc = 4 * m.q;  // input columns jc .. jc + 3
  const int ho = 2 * hi, wo = 2 * wi;
  const T* gp = gy + m.plane * ho * (int64_t)wo;
  const T* gp2 = TWO ? gy2 + m.plane * ho * (int64_t)wo : nullptr;
  T* xp = gx + m.plane * hi * (int64_t)wi + jc;
  // neighbour columns 2jc - 1 / 2jc + 8 (clamped): as in the forward, plain
  // loads by every lane for bf16, shuffles + edge loads for fp32
  constexpr bool kPlain = sizeof(T) == 2;
  const bool ledge = lane == 0 || m.q == 0, redge = lane == 63 || m.q == m.quads - 1;
  const int el = 2 * jc > 0 ? 2 * jc - 1 : 0, er = 2 * jc + 8 < wo ? 2 * jc + 8 : wo - 1;
  // column-filtered gradient row o for input columns jc .. jc+3
  auto hrow = [&](int o, float* h) {
    o = o < 0 ? 0 : (o > ho - 1 ? ho - 1 : o);
    const T* row = gp + (int64_t)o * wo;
    const T* row2 = TWO ? gp2 + (int64_t)o * wo : nullptr;
    float v[10];  // output-gradient columns 2jc - 1 .. 2jc + 8
    ld8(row + 2 * jc, v + 1);
    if (TWO) {
      float v2[8];
      ld8(row2 + 2 * jc, v2);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q + 1] += v2[q];
    }
    if constexpr (kPlain) {
      v[0] = mde::ld1(row + el);
      v[9] = mde::ld1(row + er);
      if (TWO) {
        v[0] += mde::ld1(row2 + el);
        v[9] += mde::ld1(row2 + er);
      }
    } else {
      float l = __shfl_up(v[8], 1, 64), r = __shfl_down(v[1], 1, 64);
      if (ledge) l = TWO ? mde::ld1(row + el) + mde::ld1(row2 + el) : mde::ld1(row + el);
      if (redge) r = TWO ? mde::ld1(row + er) + mde::ld1(row2 + er) : mde::ld1(row + er);
      v[0] = l;
      v[9] = r;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      h[k] = 0.25f * v[2 * k] + 0.75f * v[2 * k + 1] + 0.75f * v[2 * k + 2] + 0.25f * v[2 * k + 3];
  };
  float a[4], b[4];
  hrow(2 * m.i0 - 1, a);
  hrow(2 * m.i0, b);
#pragma unroll
  for (int k = 0; k < kX2Rows; ++k) {
    const int i = m.i0 + k;
    float c[4], d[4];
    hrow(2 * i + 1, c);
    hrow(2 * i + 2, d);
    if (m.live && i < hi)
      mde::st4(xp + (int64_t)i * wi,
               make_float4(0.25f * a[0] + 0.75f * b[0] + 0.75f * c[0] + 0.25f * d[0],
                           0.25f * a[1] + 0.75f * b[1] + 0.75f * c[1] + 0.25f * d[1],
                           0.25f * a[2] + 0.75f * b[2] + 0.75f * c[2] + 0.25f * d[2],
                           0.25f * a[3] + 0.75f * b[3] + 0.75f * c[3] + 0.25f * d[3]));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a[q] = c[q];
      b[q] = d[q];
    }
  }
}

// fp32 x2 on the quad kernels: the backward by default (kbench at the decoder
// shapes: 34 / 92 / 166 -> 32 / 81 / 164 us); the forward stays on the pair
// kernel (quad 34 / 112 / 215 vs 35 / 94 / 171 us: its 32-byte-per-lane row
// stores are slower).  MDE_X2_QUAD = 0 (pair kernels only) / 2 (quad for both)
// for A/B runs.
inline int quad_f32() {
  static const int mode = [] {
    const char* e = getenv("MDE_X2_QUAD");
    return e ? atoi(e) : 1;
  }();
  return mode;
}

inline dim3 quad_grid(int64_t planes, int64_t hi, int64_t wi) {
  return dim3((unsigned)mde::cdiv(planes * mde::cdiv(hi, kX2Rows) * (wi / 4), 256));
}

// Exact integer ratio S = 4 or 8 (align_corners=False, scale 1/S): the
// MobileNetV3-NewCRF head upsample (model_mobileV3_large_newCRFs.py:55-58,124,
// 1 x 120x160 -> 480x640).  One lane owns input column j of one plane and a
// band of kXsRows input rows.  Forward: each input row is interpolated
// horizontally once into the lane's S output columns (S/4 float4s); every
// output row r then mixes the two input rows lin_index(r) names (ATen's order:
// rows of horizontally interpolated columns), written as S/4 float4 stores
// per lane -- coalesced rows.  Backward (the adjoint, a gather): the lane reads
// the S gradient columns it owns as float4s per output row, gets the S/2 halo
// columns on either side from the neighbouring lanes by wave shuffles (loads
// only at wave edges), forms the column-adjoint sum with its 2S exact weights
// (lin_weight, so the clamped edges are exact) and adds it into the (at most
// two) band rows lin_index(r) names.  All rows of a band are unrolled so their
// loads are in flight together.  gy rows at band edges are read by two bands
// (S of every S*kXsRows + S rows, served by L2).
constexpr int kXsRows = 4;   // input rows per lane

// Flat lane mapping: thread t -> (plane, band of kXsRows input rows, column j),
// columns fastest, so narrow planes (DDRNet's 15 x 20 -> 60 x 80: 20 columns)
// still fill every lane of a wave instead of 20 of 64.
struct XsMap {
  int64_t plane;
  int ib, j;
  bool live;
};

__device__ __forceinline__ XsMap xs_map(int64_t planes, int hi, int wi) {
  const int bands = (hi + kXsRows - 1) / kXsRows;
  const int64_t total = planes * bands * (int64_t)wi;
  int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  XsMap m;
  m.live = t < total;
  if (!m.live) t = total - 1;
  m.j = (int)(t % wi);
  const int64_t r = t / wi;
  m.ib = (int)(r % bands) * kXsRows;
  m.plane = r / bands;
  return m;
}

template <int S, typename T>
__global__ void __launch_bounds__(256)
    bilinear_fwd_xs_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t planes, int hi,
                           int wi) {
  const XsMap m = xs_map(planes, hi, wi);
  const int i0 = m.ib, jc = m.j;
  const bool ok = m.live;
  const int64_t plane = m.plane;
  const T* xp = x + plane * hi * (int64_t)wi;
  const int wo = S * wi, ho = S * hi;
  const float sc = 1.f / S;
  // this lane's S output columns: input columns and weights (exact ATen math)
  Lin W[S];
#pragma unroll
  for (int q = 0; q < S; ++q) W[q] = lin_index(sc, S * jc + q, wi, 0);
  auto hrow = [&](int r, float* o) {
    r = r < 0 ? 0 : (r > hi - 1 ? hi - 1 : r);
    const T* row = xp + (int64_t)r * wi;
#pragma unroll
    for (int q = 0; q < S; ++q) o[q] = lerp2(W[q], mde::ld1(row + W[q].i0), mde::ld1(row + W[q].i1));
  };
  float rows[kXsRows + 2][S];
#pragma unroll
  for (int k = 0; k < kXsRows + 2; ++k) hrow(i0 - 1 + k, rows[k]);
  T* yp = y + plane * ho * (int64_t)wo + S * jc;
#pragma unroll
  for (int k = 0; k < kXsRows; ++k) {
    const int i = i0 + k;
#pragma unroll
    for (int q = 0; q < S; ++q) {
      const int r = S * i + q;
      // interior: rows (i-1, i) for q < S/2, (i, i+1) after; at the plane
      // edges lin_index clamps onto the same row, which rows[] also holds
      // (hrow clamps), so the static pick gives ATen's value there too
      const Lin H = lin_index(sc, r, hi, 0);
      const float* a = rows[q < S / 2 ? k : k + 1];
      const float* b = rows[q < S / 2 ? k + 1 : k + 2];
      float o[S];
#pragma unroll
      for (int c = 0; c < S; ++c) o[c] = lerp2(H, a[c], b[c]);
      if (ok && i < hi) {
#pragma unroll
        for (int c = 0; c < S; c += 4)
          mde::st4(yp + (int64_t)r * wo + c, make_float4(o[c], o[c + 1], o[c + 2], o[c + 3]));
      }
    }
  }
}

template <int S, typename T>
__global__ void __launch_bounds__(256)
    bilinear_bwd_xs_kernel(const T* __restrict__ gy, T* __restrict__ gx, int64_t planes, int hi,
                           int wi) {
  constexpr int HALF = S / 2;
  const XsMap m = xs_map(planes, hi, wi);
  const int ib = m.ib, j = m.j, jc = m.j;
  const bool ok = m.live;
  const int64_t plane = m.plane;
  const int wo = S * wi, ho = S * hi;
  const float sc = 1.f / S;
  const T* gp = gy + plane * ho * (int64_t)wo;
  // weights of output columns S*j - HALF .. S*j + S + HALF - 1 for input column j
  float wc[2 * S];
#pragma unroll
  for (int k = 0; k < 2 * S; ++k) {
    const int c = S * jc - HALF + k;
    wc[k] = (c >= 0 && c < wo) ? lin_weight(sc, c, jc, wi, 0) : 0.f;
  }
  float acc[kXsRows];
#pragma unroll
  for (int k = 0; k < kXsRows; ++k) acc[k] = 0.f;
  constexpr int NR = S * kXsRows + S;  // output rows S*ib - HALF .. S*(ib+R) + HALF - 1
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    // rows outside the plane (band edges) are clamped and weighted 0: no
    // branch splits the unrolled rows, so all their loads are in flight at once
    const int rq = S * ib - HALF + k;
    const bool rv = rq >= 0 && rq < ho;
    const int r = rq < 0 ? 0 : (rq > ho - 1 ? ho - 1 : rq);
    const T* row = gp + (int64_t)r * wo;
    float v[S];
#pragma unroll
    for (int c = 0; c < S; c += 4) {
      const float4 t = mde::ld4(row + S * jc + c);
      v[c] = t.x; v[c + 1] = t.y; v[c + 2] = t.z; v[c + 3] = t.w;
    }
    float s = 0.f;
#pragma unroll
    for (int h = 0; h < HALF; ++h) {
      // halo columns: plain loads at clamped addresses by every lane (a
      // column outside the plane has weight 0) -- no shuffles, no selects,
      // nothing hipcc could turn into a branch around a load
      const int cl = S * jc - HALF + h, cr = S * jc + S + h;
      s = madd(wc[h], mde::ld1(row + (cl >= 0 ? cl : 0)), s);
      s = madd(wc[S + HALF + h], mde::ld1(row + (cr < wo ? cr : wo - 1)), s);
    }
#pragma unroll
    for (int c = 0; c < S; ++c) s = madd(wc[HALF + c], v[c], s);
    s = rv ? s : 0.f;
    const Lin H = lin_index(sc, r, hi, 0);
#pragma unroll
    for (int b = 0; b < kXsRows; ++b) {
      float wgt = 0.f;
      if (H.i0 == ib + b) wgt += H.l0;
      if (H.i1 == ib + b) wgt += H.l1;
      acc[b] = madd(wgt, s, acc[b]);
    }
  }
  if (!ok) return;
  T* out = gx + (plane * hi + ib) * (int64_t)wi + j;
#pragma unroll
  for (int b = 0; b < kXsRows; ++b)
    if (ib + b < hi) mde::st1(out + (int64_t)b * wi, acc[b]);
}

inline dim3 xs_grid(int64_t planes, int64_t hi, int64_t wi) {
  return dim3((unsigned)mde::cdiv(planes * mde::cdiv(hi, kXsRows) * wi, 256));
}

// Integer upsampling ratio handled by the xS kernels (4 or 8), else 0.
int xs_ratio(int64_t hi, int64_t wi, int64_t ho, int64_t wo, float sh, float sw, int align,
             int64_t planes) {
  if (align || planes > 65535) return 0;
  for (int r : {4, 8})
    if (ho == r * hi && wo == r * wi && sh == 1.f / r && sw == 1.f / r) return r;
  return 0;
}

inline dim3 x2_grid(int64_t planes, int64_t hi, int64_t wi) {
  return dim3((unsigned)mde::cdiv(wi, 64), (unsigned)mde::cdiv(hi, kX2Rows * kX2Warps),
              (unsigned)planes);
}

// Backward, generic ratio, one plane per block in LDS (the DDRNet resizes of
// tiny maps, e.g. 8x10 -> 60x80 and 15x20 -> 60x80: every output-gradient
// plane fits).  The adjoint is separable: t[o][j] = sum_p Wc[p,j] gy[o][p]
// (column pass, gy staged once), then gx[i][j] = sum_o Wr[o,i] t[o][j].  The
// per-axis weights come from tables built once per block over the candidate
// windows (exact ATen source-index math, zero-padded to kw / kh entries).
constexpr int kPlaneMax = 12288;  // floats of gy (and of t) per block

template <typename T>
__global__ void __launch_bounds__(256)
    bilinear_bwd_plane_kernel(const T* __restrict__ gy, T* __restrict__ gx,
                              int hi, int wi, int ho, int wo, float sh, float sw,
                              int align, int kh, int kw) {
  extern __shared__ float lds[];
  float* sg = lds;                    // [ho][wo]
  float* st = sg + ho * wo;           // [ho][wi]
  float* cw = st + ho * wi;           // [wi][kw]
  float* rw = cw + wi * kw;           // [hi][kh]
  int* clo = (int*)(rw + hi * kh);    // [wi]
  int* rlo = clo + wi;                // [hi]
  int* cfirst = rlo + hi;             // [wi] first nonzero tap of column j's window
  int* ccnt = cfirst + wi;            // [wi] taps from there to the last nonzero one
  int* rfirst = ccnt + wi;            // [hi]
  int* rcnt = rfirst + hi;            // [hi]
  const int tid = threadIdx.x;
  const int64_t plane = blockIdx.x;
  const T* g = gy + plane * ho * (int64_t)wo;
  const int np = ho * wo;
  for (int e = tid; e < np; e += 256) sg[e] = mde::ld1(g + e);
  for (int e = tid; e < wi * kw; e += 256) {
    const int j = e / kw, k = e % kw;
    int lo, hi_;
    lin_window(sw, j, wo, &lo, &hi_);
    if (k == 0) clo[j] = lo;
    cw[e] = lo + k <= hi_ ? lin_weight(sw, lo + k, j, wi, align) : 0.f;
  }
  for (int e = tid; e < hi * kh; e += 256) {
    const int i = e / kh, k = e % kh;
    int lo, hi_;
    lin_window(sh, i, ho, &lo, &hi_);
    if (k == 0) rlo[i] = lo;
    rw[e] = lo + k <= hi_ ? lin_weight(sh, lo + k, i, hi, align) : 0.f;
  }
  __syncthreads();
  // tight windows: lin_window is conservative (~3/scale + 6 taps, about twice
  // the ~2/scale + 2 that carry weight); the passes below visit only the taps
  // between the first and last nonzero weight (zeros inside add exact +0)
  for (int e = tid; e < wi + hi; e += 256) {
    const bool col = e < wi;
    const int idx = col ? e : e - wi, kk = col ? kw : kh;
    const float* wt = col ? cw + idx * kw : rw + idx * kh;
    int f = kk, l = -1;
    for (int k = 0; k < kk; ++k)
      if (wt[k] != 0.f) {
        f = k < f ? k : f;
        l = k;
      }
    if (l < 0) f = 0;
    (col ? cfirst : rfirst)[idx] = f;
    (col ? ccnt : rcnt)[idx] = l - f + 1;
  }
  __syncthreads();
  for (int e = tid; e < ho * wi; e += 256) {
    const int o = e / wi, j = e % wi;
    const float* row = sg + o * wo;
    const int f = cfirst[j], cnt = ccnt[j];
    const float* wc = cw + j * kw + f;
    const int lo = clo[j] + f;
    float acc = 0.f;
    for (int k = 0; k < cnt; ++k) acc = madd(wc[k], row[min(lo + k, wo - 1)], acc);
    st[e] = acc;
  }
  __syncthreads();
  T* out = gx + plane * hi * (int64_t)wi;
  for (int e = tid; e < hi * wi; e += 256) {
    const int i = e / wi, j = e % wi;
    const int f = rfirst[i], cnt = rcnt[i];
    const float* wr = rw + i * kh + f;
    const int lo = rlo[i] + f;
    float acc = 0.f;
    for (int k = 0; k < cnt; ++k) acc = madd(wr[k], st[min(lo + k, ho - 1) * wi + j], acc);
    mde::st1(out + e, acc);
  }
}

// Backward, generic ratio, banded: one thread owns input column j of a band
// of kBandRows input rows of one plane.  Its column weights over the
// output-column window (<= kColWin entries, zero-padded) are computed once
// and kept in registers; the thread then streams the output-gradient rows
// that can touch the band, forms the column-adjoint sum of each row once and
// adds it into the (at most two) band rows that row's stencil reads.  Used
// when the column window fits kColWin (upsampling up to ~8.7x, e.g. the
// DDRNet 8x10 -> 60x80 and 15x20 -> 60x80 resizes); wider windows take the
// per-pixel kernel below.
constexpr int kBandRows = 4;
constexpr int kColWin = 32;

template <typename T>
__global__ void __launch_bounds__(256)
    bilinear_bwd_band_kernel(const T* __restrict__ gy, T* __restrict__ gx,
                             int64_t planes, int hi, int wi, int ho, int wo,
                             float sh, float sw, int align) {
  const int bands = (hi + kBandRows - 1) / kBandRows;
  const int64_t total = planes * bands * (int64_t)wi;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % wi);
    const int64_t r = t / wi;
    const int ib = (int)(r % bands) * kBandRows;
    const int64_t plane = r / bands;
    int clo, chi;
    lin_window(sw, j, wo, &clo, &chi);
    float cw[kColWin];
#pragma unroll
    for (int k = 0; k < kColWin; ++k)
      cw[k] = clo + k <= chi ? lin_weight(sw, clo + k, j, wi, align) : 0.f;
    const int ilast = ib + kBandRows - 1 < hi ? ib + kBandRows - 1 : hi - 1;
    int rlo, rhi, unused;
    lin_window(sh, ib, ho, &rlo, &unused);
    lin_window(sh, ilast, ho, &unused, &rhi);
    const T* g = gy + plane * ho * (int64_t)wo;
    float acc[kBandRows];
#pragma unroll
    for (int b = 0; b < kBandRows; ++b) acc[b] = 0.f;
    for (int o = rlo; o <= rhi; ++o) {
      const Lin H = lin_index(sh, o, hi, align);
      const int d0 = H.i0 - ib, d1 = H.i1 - ib;
      if ((unsigned)d0 >= (unsigned)kBandRows && (unsigned)d1 >= (unsigned)kBandRows)
        continue;
      const T* grow = g + (int64_t)o * wo;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < kColWin; ++k) {
        const int p = clo + k < wo - 1 ? clo + k : wo - 1;
        s = madd(cw[k], mde::ld1(grow + p), s);
      }
#pragma unroll
      for (int b = 0; b < kBandRows; ++b) {
        float wgt = 0.f;
        if (d0 == b) wgt += H.l0;
        if (d1 == b) wgt += H.l1;
        acc[b] = madd(wgt, s, acc[b]);
      }
    }
    T* out = gx + (plane * hi + ib) * (int64_t)wi + j;
#pragma unroll
    for (int b = 0; b < kBandRows; ++b)
      if (ib + b < hi) mde::st1(out + (int64_t)b * wi, acc[b]);
  }
}

// Backward, generic ratio: candidate windows per axis, exact weights.
template <typename T>
__global__ void __launch_bounds__(256)
    bilinear_bwd_kernel(const T* __restrict__ gy, T* __restrict__ gx,
                        int64_t planes, int hi, int wi, int ho, int wo,
                        float sh, float sw, int align) {
  const int64_t total = planes * hi * (int64_t)wi;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % wi);
    const int64_t r = t / wi;
    const int i = (int)(r % hi);
    const int64_t plane = r / hi;
    int rlo, rhi, clo, chi;
    lin_window(sh, i, ho, &rlo, &rhi);
    lin_window(sw, j, wo, &clo, &chi);
    const T* g = gy + plane * ho * (int64_t)wo;
    float acc = 0.f;
    for (int o = rlo; o <= rhi; ++o) {
      const float wr = lin_weight(sh, o, i, hi, align);
      if (wr == 0.f) continue;
      const T* grow = g + (int64_t)o * wo;
      for (int p = clo; p <= chi; ++p) {
        const float wc = lin_weight(sw, p, j, wi, align);
        if (wc != 0.f) acc = madd(__fmul_rn(wr, wc), mde::ld1(grow + p), acc);
      }
    }
    mde::st1(gx + t, acc);
  }
}

__device__ __forceinline__ int nearest_src(float scale, int dst, int in_size) {
  const int s = (int)floorf(__fmul_rn((float)dst, scale));
  return s < in_size - 1 ? s : in_size - 1;
}

__global__ void __launch_bounds__(256)
    nearest_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                       int64_t planes, int hi, int wi, int ho, int wo,
                       float sh, float sw) {
  const int64_t total = planes * ho * (int64_t)wo;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int ow = (int)(t % wo);
    const int64_t r = t / wo;
    const int oh = (int)(r % ho);
    const int64_t plane = r / ho;
    y[t] = x[(plane * hi + nearest_src(sh, oh, hi)) * (int64_t)wi +
             nearest_src(sw, ow, wi)];
  }
}

__global__ void __launch_bounds__(256)
    nearest_bwd_kernel(const float* __restrict__ gy, float* __restrict__ gx,
                       int64_t planes, int hi, int wi, int ho, int wo,
                       float sh, float sw) {
  const int64_t total = planes * hi * (int64_t)wi;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % wi);
    const int64_t r = t / wi;
    const int i = (int)(r % hi);
    const int64_t plane = r / hi;
    // outputs o with floor(o*scale) == i lie in [i/scale - 1, (i+1)/scale + 1]
    int rlo = sh > 0.f ? (int)floorf((float)i / sh) - 1 : 0;
    int rhi = sh > 0.f ? (int)ceilf((float)(i + 1) / sh) + 1 : ho - 1;
    int clo = sw > 0.f ? (int)floorf((float)j / sw) - 1 : 0;
    int chi = sw > 0.f ? (int)ceilf((float)(j + 1) / sw) + 1 : wo - 1;
    rlo = rlo < 0 ? 0 : rlo;
    clo = clo < 0 ? 0 : clo;
    rhi = rhi > ho - 1 ? ho - 1 : rhi;
    chi = chi > wo - 1 ? wo - 1 : chi;
    const float* g = gy + plane * ho * (int64_t)wo;
    float acc = 0.f;
    for (int o = rlo; o <= rhi; ++o) {
      if (nearest_src(sh, o, hi) != i) continue;
      for (int p = clo; p <= chi; ++p)
        if (nearest_src(sw, p, wi) == j) acc += g[(int64_t)o * wo + p];
    }
    gx[t] = acc;
  }
}

// The guide pyramid (GuideDepth.py:46-47): nearest x0.5 and x0.25 of the
// same image in one pass.  ATen's nearest source index at these scale factors
// is floor(dst * 2.0) = 2 dst and floor(dst * 4.0) = 4 dst, so
//   half[r][c] = x[2r][2c],   quarter[r][c] = x[4r][4c] = half[2r][2c].
// One lane reads 8 consecutive pixels of an even input row (two float4; odd
// rows are never fetched) and writes 4 half-resolution pixels (float4) and,
// on rows 4k, 2 quarter-resolution pixels (float2).  Lanes run fastest along
// the row, so every wave reads and writes contiguous bytes.  Needs w % 8 == 0
// and h % 4 == 0 (the 640 x 480 input); the host falls back to two
// nearest_fwd launches otherwise.
__global__ void __launch_bounds__(256)
    nearest_pyramid_kernel(const float* __restrict__ x, float* __restrict__ half,
                           float* __restrict__ quarter, int64_t planes, int h, int w) {
  const int ho = h >> 1, wo = w >> 1, wq = w >> 2, quads = w >> 3;
  const int64_t total = planes * ho * (int64_t)quads;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(t % quads);
    const int64_t pr = t / quads;  // plane * ho + r
    const int r = (int)(pr % ho);
    const int64_t plane = pr / ho;
    const float* src = x + (plane * h + 2 * r) * (int64_t)w + 8 * q;
    const float4 a = *reinterpret_cast<const float4*>(src);
    const float4 b = *reinterpret_cast<const float4*>(src + 4);
    *reinterpret_cast<float4*>(half + pr * wo + 4 * q) = make_float4(a.x, a.z, b.x, b.z);
    if ((r & 1) == 0)
      *reinterpret_cast<float2*>(quarter + (plane * (h >> 2) + (r >> 1)) * (int64_t)wq + 2 * q) =
          make_float2(a.x, b.x);
  }
}

inline int grid_for(int64_t work) {
  const int64_t b = mde::cdiv(work, 256);
  return (int)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

// Candidate-window length of lin_window along an axis (<= 3/scale + 6).
int win_len(float scale, int64_t out_size) {
  if (!(scale > 0.f)) return (int)out_size;
  const double k = std::ceil(3.0 / scale) + 6.0;
  return (int)(k < (double)out_size ? k : (double)out_size);
}

bool plane_fits(int64_t hi, int64_t wi, int64_t ho, int64_t wo, float sh, float sw) {
  if (!(sh > 0.f) || !(sw > 0.f) || ho * wo > kPlaneMax || ho * wi > kPlaneMax) return false;
  const int64_t kh = win_len(sh, ho), kw = win_len(sw, wo);
  return (ho * wo + ho * wi + wi * kw + hi * kh + 3 * (wi + hi)) * 4 <= 64 * 1024;
}

bool dims_ok(int64_t n, int64_t c, int64_t hi, int64_t wi, int64_t ho,
             int64_t wo) {
  return n > 0 && c > 0 && hi > 0 && wi > 0 && ho > 0 && wo > 0 &&
         hi < (1 << 30) && wi < (1 << 30) && ho < (1 << 30) && wo < (1 << 30);
}

}  // namespace

namespace {

// Forward dispatch, one storage type: the exact x2 / x4 / x8 kernels, else
// the generic one.  fp32 x2: the pair kernel (quad only under MDE_X2_QUAD=2,
// see quad_f32); bf16 x2: the quad kernel (lane loads / stores of 8 / 16
// bytes, as the fp32 pair kernel's).
template <typename T>
int bilinear_fwd_t(const T* x, T* y, int64_t n, int64_t c, int64_t hi, int64_t wi, int64_t ho,
                    int64_t wo, float scale_h, float scale_w, int align_corners, hipStream_t s) {
  constexpr bool kBf = sizeof(T) == 2;
  const double bytes = (double)sizeof(T) * n * c * (double)(hi * wi + ho * wo);
  const bool x2 = !align_corners && scale_h == 0.5f && scale_w == 0.5f &&
                  ho == 2 * hi && wo == 2 * wi && n * c <= 65535;
  // The pair kernel (two columns per lane) wins when it keeps at least as many lanes
  // busy as the one-column kernel: 64-lane rows of wi/2 pairs vs of wi columns.
  const bool pair = x2 && wi % 2 == 0 &&
                    mde::cdiv(wi, 64) >= 2 * mde::cdiv(wi / 2, 64);
  const int xs = xs_ratio(hi, wi, ho, wo, scale_h, scale_w, align_corners, n * c);
  if (xs == 4) {
    MDE_LAUNCH(mde::K_BILINEAR_FWD, bytes, s, (bilinear_fwd_xs_kernel<4, T>),
               xs_grid(n * c, hi, wi), dim3(256), 0, x, y, n * c, (int)hi, (int)wi);
  } else if (xs == 8) {
    MDE_LAUNCH(mde::K_BILINEAR_FWD, bytes, s, (bilinear_fwd_xs_kernel<8, T>),
               xs_grid(n * c, hi, wi), dim3(256), 0, x, y, n * c, (int)hi, (int)wi);
  } else if (x2 && wi % 4 == 0 && (kBf || quad_f32() > 1)) {
    MDE_LAUNCH(mde::K_BILINEAR_FWD, bytes, s, bilinear_fwd_x2_quad_kernel<T>,
               quad_grid(n * c, hi, wi), dim3(256), 0, x, y, n * c, (int)hi, (int)wi);
  } else if (pair || (kBf && x2 && wi % 2 == 0)) {
    MDE_LAUNCH(mde::K_BILINEAR_FWD, bytes, s, bilinear_fwd_x2_pair_kernel<T>,
               x2_grid(n * c, hi, wi / 2), dim3(64, kX2Warps), 0, x, y, (int)hi, (int)wi);
  } else if (x2) {
    MDE_LAUNCH(mde::K_BILINEAR_FWD, bytes, s, bilinear_fwd_x2_kernel<T>, x2_grid(n * c, hi, wi),
               dim3(64, kX2Warps), 0, x, y, (int)hi, (int)wi);
  } else {
    const int vec = wo % 4 == 0 ? 4 : 1;
    const int64_t threads = fwd_threads(n * c, ho, wo, vec);
    if (threads > INT32_MAX - 256) return MDE_ERR_UNSUPPORTED;
    const dim3 grid((unsigned)mde::cdiv(threads, 256));
    if (vec == 4)
      MDE_LAUNCH(mde::K_BILINEAR_FWD, bytes, s, (bilinear_fwd_kernel<4, T>), grid, dim3(256), 0, x,
                 y, (int)threads, (int)hi, (int)wi, (int)ho, (int)wo, scale_h, scale_w,
                 align_corners);
    else
      MDE_LAUNCH(mde::K_BILINEAR_FWD, bytes, s, (bilinear_fwd_kernel<1, T>), grid, dim3(256), 0, x,
                 y, (int)threads, (int)hi, (int)wi, (int)ho, (int)wo, scale_h, scale_w,
                 align_corners);
  }
  return MDE_OK;
}

template <typename T>
int bilinear_bwd_t(const T* gy, T* gx, int64_t n, int64_t c, int64_t hi, int64_t wi, int64_t ho,
                    int64_t wo, float scale_h, float scale_w, int align_corners, hipStream_t s) {
  constexpr bool kBf = sizeof(T) == 2;
  const int64_t planes = n * c;
  const double bytes = (double)sizeof(T) * n * c * (double)(hi * wi + ho * wo);
  const bool x2 = !align_corners && scale_h == 0.5f && scale_w == 0.5f &&
                  ho == 2 * hi && wo == 2 * wi && planes <= 65535;
  const int xs = xs_ratio(hi, wi, ho, wo, scale_h, scale_w, align_corners, planes);
  if (xs == 4) {
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, (bilinear_bwd_xs_kernel<4, T>),
               xs_grid(planes, hi, wi), dim3(256), 0, gy, gx, planes, (int)hi, (int)wi);
  } else if (xs == 8) {
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, (bilinear_bwd_xs_kernel<8, T>),
               xs_grid(planes, hi, wi), dim3(256), 0, gy, gx, planes, (int)hi, (int)wi);
  } else if (x2 && wi % 4 == 0 && (kBf || quad_f32() > 0)) {
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, (bilinear_bwd_x2_quad_kernel<false, T>),
               quad_grid(planes, hi, wi), dim3(256), 0, gy, gx, planes, (int)hi, (int)wi,
               (const T*)nullptr);
  } else if (x2 && wi % 2 == 0) {
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, (bilinear_bwd_x2_pair_kernel<false, T>),
               x2_grid(planes, hi, wi / 2), dim3(64, kX2Warps), 0, gy, gx, (int)hi, (int)wi,
               (const T*)nullptr);
  } else if (x2) {
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, bilinear_bwd_x2_kernel<T>, x2_grid(planes, hi, wi),
               dim3(64, kX2Warps), 0, gy, gx, (int)hi, (int)wi);
  } else if (plane_fits(hi, wi, ho, wo, scale_h, scale_w)) {
    const int kh = win_len(scale_h, ho), kw = win_len(scale_w, wo);
    const size_t lds = sizeof(float) * ((size_t)ho * wo + (size_t)ho * wi + (size_t)wi * kw +
                                        (size_t)hi * kh + 3 * (wi + hi));
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, bilinear_bwd_plane_kernel<T>, dim3((unsigned)planes),
               dim3(256), lds, gy, gx, (int)hi, (int)wi, (int)ho, (int)wo, scale_h, scale_w,
               align_corners, kh, kw);
  } else if (scale_w > 0.f && 3.0 / scale_w + 6.0 <= kColWin) {
    const int64_t bands = mde::cdiv(hi, kBandRows);
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, bilinear_bwd_band_kernel<T>,
               dim3(grid_for(planes * bands * wi)), dim3(256), 0, gy, gx, planes, (int)hi,
               (int)wi, (int)ho, (int)wo, scale_h, scale_w, align_corners);
  } else {
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, bilinear_bwd_kernel<T>,
               dim3(grid_for(planes * hi * wi)), dim3(256), 0, gy, gx, planes, (int)hi, (int)wi,
               (int)ho, (int)wo, scale_h, scale_w, align_corners);
  }
  return MDE_OK;
}

}  // namespace

extern "C" {

int mde_bilinear_fwd(const void* x, void* y, int64_t n, int64_t c, int64_t hi,
                     int64_t wi, int64_t ho, int64_t wo, float scale_h,
                     float scale_w, int align_corners, int dtype,
                     void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  if (!x || !y || !dims_ok(n, c, hi, wi, ho, wo)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MDE_BF16)
    return bilinear_fwd_t((const mde::bf16*)x, (mde::bf16*)y, n, c, hi, wi, ho, wo, scale_h,
                          scale_w, align_corners, s);
  return bilinear_fwd_t((const float*)x, (float*)y, n, c, hi, wi, ho, wo, scale_h, scale_w,
                        align_corners, s);
}

int mde_bilinear_bwd(const void* gy, void* gx, int64_t n, int64_t c,
                     int64_t hi, int64_t wi, int64_t ho, int64_t wo,
                     float scale_h, float scale_w, int align_corners,
                     int dtype, void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  if (!gy || !gx || !dims_ok(n, c, hi, wi, ho, wo)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MDE_BF16)
    return bilinear_bwd_t((const mde::bf16*)gy, (mde::bf16*)gx, n, c, hi, wi, ho, wo, scale_h,
                          scale_w, align_corners, s);
  return bilinear_bwd_t((const float*)gy, (float*)gx, n, c, hi, wi, ho, wo, scale_h, scale_w,
                        align_corners, s);
}

static bool x2_pair(int64_t planes, int64_t hi, int64_t wi, int64_t ho, int64_t wo, float scale_h,
                    float scale_w, int align_corners) {
  return !align_corners && scale_h == 0.5f && scale_w == 0.5f && ho == 2 * hi && wo == 2 * wi &&
         planes <= 65535 && wi % 2 == 0 &&
         xs_ratio(hi, wi, ho, wo, scale_h, scale_w, align_corners, planes) == 0;
}

int mde_bilinear_bwd2_supported(int64_t n, int64_t c, int64_t hi, int64_t wi, int64_t ho,
                                int64_t wo, float scale_h, float scale_w, int align_corners) {
  return dims_ok(n, c, hi, wi, ho, wo) &&
         x2_pair(n * c, hi, wi, ho, wo, scale_h, scale_w, align_corners);
}

int mde_bilinear_bwd2(const void* gy, const void* gy2, void* gx, int64_t n, int64_t c,
                      int64_t hi, int64_t wi, int64_t ho, int64_t wo, float scale_h,
                      float scale_w, int align_corners, int dtype, void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  if (!gy || !gy2 || !gx || !dims_ok(n, c, hi, wi, ho, wo)) return MDE_ERR_INVALID_ARG;
  if (!x2_pair(n * c, hi, wi, ho, wo, scale_h, scale_w, align_corners))
    return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const double bytes = 4.0 * n * c * (double)(hi * wi + 2 * ho * wo);
  if (dtype == MDE_BF16) {
    using B = mde::bf16;
    if (wi % 4 == 0) {
      MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes / 2, s, (bilinear_bwd_x2_quad_kernel<true, B>),
                 quad_grid(n * c, hi, wi), dim3(256), 0, (const B*)gy, (B*)gx, n * c, (int)hi,
                 (int)wi, (const B*)gy2);
      return MDE_OK;
    }
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes / 2, s, (bilinear_bwd_x2_pair_kernel<true, B>),
               x2_grid(n * c, hi, wi / 2), dim3(64, kX2Warps), 0, (const B*)gy, (B*)gx, (int)hi,
               (int)wi, (const B*)gy2);
    return MDE_OK;
  }
  if (wi % 4 == 0 && quad_f32() > 0) {
    MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, (bilinear_bwd_x2_quad_kernel<true, float>),
               quad_grid(n * c, hi, wi), dim3(256), 0, (const float*)gy, (float*)gx, n * c,
               (int)hi, (int)wi, (const float*)gy2);
    return MDE_OK;
  }
  MDE_LAUNCH(mde::K_BILINEAR_BWD, bytes, s, (bilinear_bwd_x2_pair_kernel<true, float>),
             x2_grid(n * c, hi, wi / 2), dim3(64, kX2Warps), 0, (const float*)gy, (float*)gx,
             (int)hi, (int)wi, (const float*)gy2);
  return MDE_OK;
}

int mde_nearest_fwd(const void* x, void* y, int64_t n, int64_t c, int64_t hi,
                    int64_t wi, int64_t ho, int64_t wo, float scale_h,
                    float scale_w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !y || !dims_ok(n, c, hi, wi, ho, wo)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const double bytes = 8.0 * n * c * (double)(ho * wo);
  MDE_LAUNCH(mde::K_NEAREST_FWD, bytes, s, nearest_fwd_kernel,
             dim3(grid_for(n * c * ho * wo)), dim3(256), 0, (const float*)x,
             (float*)y, n * c, (int)hi, (int)wi, (int)ho, (int)wo, scale_h,
             scale_w);
  return MDE_OK;
}

int mde_nearest_pyramid_supported(int64_t n, int64_t c, int64_t h, int64_t w) {
  return n > 0 && c > 0 && h >= 4 && w >= 8 && h % 4 == 0 && w % 8 == 0 && h < (1 << 30) &&
         w < (1 << 30);
}

int mde_nearest_pyramid(const void* x, void* half, void* quarter, int64_t n, int64_t c, int64_t h,
                        int64_t w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !half || !quarter) return MDE_ERR_INVALID_ARG;
  if (!mde_nearest_pyramid_supported(n, c, h, w)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  // algorithmic bytes of the two nearest_fwd calls it replaces (read + write
  // of every output element)
  const double bytes = 8.0 * n * c * (double)((h / 2) * (w / 2) + (h / 4) * (w / 4));
  MDE_LAUNCH(mde::K_NEAREST_FWD, bytes, s, nearest_pyramid_kernel,
             dim3(grid_for(n * c * (h / 2) * (w / 8))), dim3(256), 0, (const float*)x,
             (float*)half, (float*)quarter, n * c, (int)h, (int)w);
  return MDE_OK;
}

int mde_nearest_bwd(const void* gy, void* gx, int64_t n, int64_t c, int64_t hi,
                    int64_t wi, int64_t ho, int64_t wo, float scale_h,
                    float scale_w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !gx || !dims_ok(n, c, hi, wi, ho, wo)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const double bytes = 4.0 * n * c * (double)(hi * wi + ho * wo);
  MDE_LAUNCH(mde::K_NEAREST_BWD, bytes, s, nearest_bwd_kernel,
             dim3(grid_for(n * c * hi * wi)), dim3(256), 0, (const float*)gy,
             (float*)gx, n * c, (int)hi, (int)wi, (int)ho, (int)wo, scale_h,
             scale_w);
  return MDE_OK;
}

}  // extern "C"
