// Depthwise convolution (groups == channels, square k3/k5, stride 1/2, zero
// padding, no bias), NCHW fp32: MobileNetV3-Large's 15 depthwise stages
// (torchvision mobilenet_v3_large().features[1..15].block[*][0], used at
// src/model_mobileV3_large_newCRFs.py:165,178-182).
//
// All three kernels are LDS-tiled over one (image, channel) plane: a block
// owns a 16x64 tile (4 waves, each lane a column and 4 rows), stages the
// input window it needs (tile + halo, zero-filled outside the plane) with
// coalesced row reads, and keeps the plane's k*k taps in registers.
//   fwd       y[oy,ox]  = sum_t w[t] x[oy*s-p+ky, ox*s-p+kx]
//   bwd data  gx[iy,ix] = sum over taps with (iy+p-ky) % s == 0 of
//                         w[t] gy[(iy+p-ky)/s, (ix+p-kx)/s]   (input-space tile)
//   bwd wgt   gw[c,t]   = sum_{n,oy,ox} gy x(...)  -> per-tile partials
//                         (register accumulators, wave shuffles, fixed order)
//                         then one block per channel sums its partials in a
//                         fixed order: deterministic, no atomics.
// Algorithmic HBM bytes: fwd 4(|x| + |y|), bwd data 4(|gy| + |gx|),
// bwd weight 4(|gy| + |x|).

#include "common.h"

namespace mde {
namespace {

constexpr int kTW = 64;   // tile width (one wave of columns)
constexpr int kTH = 16;   // tile height (4 waves x 4 rows)
constexpr int kR = 4;     // rows per thread

struct DwShape {
  int64_t c, h, w, ho, wo;
  int pad;
};

template <int K, int S>
__global__ void __launch_bounds__(256)
    dw_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                  float* __restrict__ y, DwShape d) {
  constexpr int IH = (kTH - 1) * S + K, IW = (kTW - 1) * S + K;
  __shared__ float tile[IH][IW];
  const int64_t plane = blockIdx.z;
  const int64_t ch = plane % d.c;
  const int64_t oy0 = (int64_t)blockIdx.y * kTH, ox0 = (int64_t)blockIdx.x * kTW;
  const int64_t iy0 = oy0 * S - d.pad, ix0 = ox0 * S - d.pad;
  const float* xp = x + plane * d.h * d.w;
  for (int i = threadIdx.x; i < IH * IW; i += 256) {
    const int r = i / IW, col = i - r * IW;
    const int64_t iy = iy0 + r, ix = ix0 + col;
    tile[r][col] = (iy >= 0 && iy < d.h && ix >= 0 && ix < d.w) ? xp[iy * d.w + ix] : 0.f;
  }
  float wk[K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) wk[t] = wt[ch * K * K + t];
  __syncthreads();
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t ox = ox0 + tx;
  if (ox >= d.wo) return;
  float* yp = y + plane * d.ho * d.wo;
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int ly = ty * kR + r;
    const int64_t oy = oy0 + ly;
    if (oy >= d.ho) break;
    float acc = 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
      for (int kx = 0; kx < K; ++kx)
        acc = fmaf(tile[ly * S + ky][tx * S + kx], wk[ky * K + kx], acc);
    yp[oy * d.wo + ox] = acc;
  }
}

__host__ __device__ constexpr int floor_div(int64_t a, int b) {
  return (int)(a >= 0 ? a / b : -((-a + b - 1) / b));
}

template <int K, int S>
__global__ void __launch_bounds__(256)
    dw_bwd_data_kernel(const float* __restrict__ gy, const float* __restrict__ wt,
                       float* __restrict__ gx, DwShape d) {
  // gy rows/cols a 16x64 input tile can reach
  constexpr int GH = (kTH + K + S - 3) / S + 1, GW = (kTW + K + S - 3) / S + 1;
  __shared__ float tile[GH][GW];
  const int64_t plane = blockIdx.z;
  const int64_t ch = plane % d.c;
  const int64_t iy0 = (int64_t)blockIdx.y * kTH, ix0 = (int64_t)blockIdx.x * kTW;
  const int64_t oy_lo = floor_div(iy0 + d.pad - (K - 1), S);
  const int64_t ox_lo = floor_div(ix0 + d.pad - (K - 1), S);
  const float* gp = gy + plane * d.ho * d.wo;
  for (int i = threadIdx.x; i < GH * GW; i += 256) {
    const int r = i / GW, col = i - r * GW;
    const int64_t oy = oy_lo + r, ox = ox_lo + col;
    tile[r][col] = (oy >= 0 && oy < d.ho && ox >= 0 && ox < d.wo) ? gp[oy * d.wo + ox] : 0.f;
  }
  float wk[K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) wk[t] = wt[ch * K * K + t];
  __syncthreads();
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t ix = ix0 + tx;
  if (ix >= d.w) return;
  float* xp = gx + plane * d.h * d.w;
  const int64_t relx0 = ix + d.pad - ox_lo * S;  // >= K-1
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int64_t iy = iy0 + ty * kR + r;
    if (iy >= d.h) break;
    const int64_t rely0 = iy + d.pad - oy_lo * S;
    float acc = 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int64_t ry = rely0 - ky;
      if (S > 1 && (ry % S) != 0) continue;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int64_t rx = relx0 - kx;
        if (S > 1 && (rx % S) != 0) continue;
        acc = fmaf(tile[ry / S][rx / S], wk[ky * K + kx], acc);
      }
    }
    xp[iy * d.w + ix] = acc;
  }
}

// Per-tile partial sums of the weight gradient: part[(ch * P + p) * K*K + t],
// p = (image, tile_y, tile_x) in row-major order.
template <int K, int S>
__global__ void __launch_bounds__(256)
    dw_bwd_weight_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                         float* __restrict__ part, DwShape d, int64_t n) {
  constexpr int IH = (kTH - 1) * S + K, IW = (kTW - 1) * S + K;
  __shared__ float tile[IH][IW];
  __shared__ float red[4][K * K];
  const int64_t plane = blockIdx.z;
  const int64_t ch = plane % d.c, img = plane / d.c;
  const int64_t oy0 = (int64_t)blockIdx.y * kTH, ox0 = (int64_t)blockIdx.x * kTW;
  const int64_t iy0 = oy0 * S - d.pad, ix0 = ox0 * S - d.pad;
  const float* xp = x + plane * d.h * d.w;
  for (int i = threadIdx.x; i < IH * IW; i += 256) {
    const int r = i / IW, col = i - r * IW;
    const int64_t iy = iy0 + r, ix = ix0 + col;
    tile[r][col] = (iy >= 0 && iy < d.h && ix >= 0 && ix < d.w) ? xp[iy * d.w + ix] : 0.f;
  }
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t ox = ox0 + tx;
  const float* gp = gy + plane * d.ho * d.wo;
  float g[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int64_t oy = oy0 + ty * kR + r;
    g[r] = (ox < d.wo && oy < d.ho) ? gp[oy * d.wo + ox] : 0.f;
  }
  __syncthreads();
  float acc[K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) acc[t] = 0.f;
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int ly = ty * kR + r;
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
      for (int kx = 0; kx < K; ++kx)
        acc[ky * K + kx] = fmaf(g[r], tile[ly * S + ky][tx * S + kx], acc[ky * K + kx]);
  }
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < K * K; ++t) {
    const float v = wave_sum(acc[t]);
    if (lane == 0) red[ty][t] = v;
  }
  __syncthreads();
  if (threadIdx.x < K * K) {
    const int t = threadIdx.x;
    const int64_t tiles = (int64_t)gridDim.x * gridDim.y;
    const int64_t p = img * tiles + (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    const int64_t P = n * tiles;
    part[(ch * P + p) * K * K + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
  }
}

// One block per channel: gw[ch, t] = sum_p part[ch, p, t] (fixed order).
template <int K>
__global__ void __launch_bounds__(256)
    dw_wreduce_kernel(const float* __restrict__ part, float* __restrict__ gw, int64_t P) {
  __shared__ float red[4][K * K];
  const int64_t ch = blockIdx.x;
  const float* pp = part + ch * P * K * K;
  float acc[K * K];
#pragma unroll
  for (int t = 0; t < K * K; ++t) acc[t] = 0.f;
  for (int64_t p = threadIdx.x; p < P; p += 256)
#pragma unroll
    for (int t = 0; t < K * K; ++t) acc[t] += pp[p * K * K + t];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < K * K; ++t) {
    const float v = wave_sum(acc[t]);
    if (lane == 0) red[wid][t] = v;
  }
  __syncthreads();
  if (threadIdx.x < K * K) {
    const int t = threadIdx.x;
    gw[ch * K * K + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
  }
}

bool dw_ok(int64_t n, int64_t c, int64_t h, int64_t w, int64_t k, int64_t stride,
           int64_t pad) {
  return n > 0 && c > 0 && h > 0 && w > 0 && (k == 3 || k == 5) &&
         (stride == 1 || stride == 2) && pad >= 0 && pad < k && n * c <= 65535 &&
         (h + 2 * pad - k) >= 0 && (w + 2 * pad - k) >= 0;
}

DwShape make_shape(int64_t c, int64_t h, int64_t w, int64_t k, int64_t s, int64_t pad) {
  DwShape d;
  d.c = c;
  d.h = h;
  d.w = w;
  d.ho = (h + 2 * pad - k) / s + 1;
  d.wo = (w + 2 * pad - k) / s + 1;
  d.pad = (int)pad;
  return d;
}

template <int K, int S>
int launch_fwd(const float* x, const float* wt, float* y, int64_t n, const DwShape& d,
               hipStream_t st) {
  const dim3 grid((unsigned)cdiv(d.wo, kTW), (unsigned)cdiv(d.ho, kTH), (unsigned)(n * d.c));
  const double bytes = 4.0 * n * d.c * (d.h * d.w + d.ho * d.wo);
  MDE_LAUNCH(K_DW_FWD, bytes, st, (dw_fwd_kernel<K, S>), grid, dim3(256), 0, x, wt, y, d);
  return 0;
}

template <int K, int S>
int launch_bwd(const float* gy, const float* x, const float* wt, float* gx, float* gw,
               float* part, int64_t n, const DwShape& d, hipStream_t st) {
  if (gx) {
    const dim3 grid((unsigned)cdiv(d.w, kTW), (unsigned)cdiv(d.h, kTH), (unsigned)(n * d.c));
    const double bytes = 4.0 * n * d.c * (d.h * d.w + d.ho * d.wo);
    MDE_LAUNCH(K_DW_BWD_DATA, bytes, st, (dw_bwd_data_kernel<K, S>), grid, dim3(256), 0, gy,
               wt, gx, d);
  }
  if (gw) {
    const dim3 grid((unsigned)cdiv(d.wo, kTW), (unsigned)cdiv(d.ho, kTH), (unsigned)(n * d.c));
    const double bytes = 4.0 * n * d.c * (d.h * d.w + d.ho * d.wo);
    MDE_LAUNCH(K_DW_BWD_WEIGHT, bytes, st, (dw_bwd_weight_kernel<K, S>), grid, dim3(256), 0,
               gy, x, part, d, n);
    const int64_t P = n * (int64_t)grid.x * grid.y;
    MDE_LAUNCH(K_DW_WREDUCE, 4.0 * d.c * P * K * K, st, dw_wreduce_kernel<K>,
               dim3((unsigned)d.c), dim3(256), 0, part, gw, P);
  }
  return 0;
}

}  // namespace
}  // namespace mde

using namespace mde;

extern "C" {

size_t mde_dwconv_workspace(int64_t n, int64_t c, int64_t h, int64_t w, int64_t k,
                            int64_t stride, int64_t pad) {
  if (!dw_ok(n, c, h, w, k, stride, pad)) return 0;
  const DwShape d = make_shape(c, h, w, k, stride, pad);
  return (size_t)(4 * c * n * cdiv(d.wo, kTW) * cdiv(d.ho, kTH) * k * k);
}

int mde_dwconv_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t c,
                   int64_t h, int64_t w, int64_t k, int64_t stride, int64_t pad, int dtype,
                   void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !weight || !y || !dw_ok(n, c, h, w, k, stride, pad)) return MDE_ERR_INVALID_ARG;
  const DwShape d = make_shape(c, h, w, k, stride, pad);
  hipStream_t st = (hipStream_t)stream;
  const float* xp = (const float*)x;
  float* yp = (float*)y;
  if (k == 3 && stride == 1) return launch_fwd<3, 1>(xp, weight, yp, n, d, st);
  if (k == 3 && stride == 2) return launch_fwd<3, 2>(xp, weight, yp, n, d, st);
  if (k == 5 && stride == 1) return launch_fwd<5, 1>(xp, weight, yp, n, d, st);
  return launch_fwd<5, 2>(xp, weight, yp, n, d, st);
}

int mde_dwconv_bwd(const void* gy, const void* x, const float* weight, void* gx, float* gweight,
                   int64_t n, int64_t c, int64_t h, int64_t w, int64_t k, int64_t stride,
                   int64_t pad, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !dw_ok(n, c, h, w, k, stride, pad) || (gx && !weight) ||
      (gweight && (!x || !workspace)))
    return MDE_ERR_INVALID_ARG;
  const DwShape d = make_shape(c, h, w, k, stride, pad);
  hipStream_t st = (hipStream_t)stream;
  const float* g = (const float*)gy;
  const float* xp = (const float*)x;
  float* gxp = (float*)gx;
  float* part = (float*)workspace;
  if (k == 3 && stride == 1) return launch_bwd<3, 1>(g, xp, weight, gxp, gweight, part, n, d, st);
  if (k == 3 && stride == 2) return launch_bwd<3, 2>(g, xp, weight, gxp, gweight, part, n, d, st);
  if (k == 5 && stride == 1) return launch_bwd<5, 1>(g, xp, weight, gxp, gweight, part, n, d, st);
  return launch_bwd<5, 2>(g, xp, weight, gxp, gweight, part, n, d, st);
}

}  // extern "C"
