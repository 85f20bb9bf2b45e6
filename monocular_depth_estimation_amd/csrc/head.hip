// 3x3 / stride-1 / pad-1 convolution with ONE output channel, NCHW fp32: the
// NewCRF decoder's depth head (src/model_mobileV3_large_newCRFs.py
// Decoder.conv1, nn.Conv2d(128, 1, 3, padding=1) at 120 x 160, bs 16), which
// MIOpen ran as Winograd F(2,3) / F(3,2) launches at ~0.6 ms a step for a
// pass that reads one 157 MB tensor.  All three passes are HBM-bound VALU
// work (9 C MACs a pixel; no GEMM shape worth an MFMA: one output channel):
//
//   forward    y[n][p]       = b + sum_c sum_t w[c][t] x[n][c][p + t]
//   data grad  gx[n][c][p]   = sum_t w[c][t] gy[n][p - t]
//   weight     gw[c][t]      = sum_{n,p} gy[n][p] x[n][c][p + t]
//
// A thread owns 4 consecutive pixels of a row (float4 loads of the centre,
// scalar loads of the two halo columns; zero padding by masks), so a wave
// streams whole rows.  The weight gradient sums per (channel, row slice)
// block in a fixed tree, then head_wreduce_kernel adds the slices in order:
// every pass is bitwise reproducible (no atomics).
#include "common.h"

namespace {

// x row r of a plane (zeros outside [0, h) x [0, w)): the 6 values of columns
// q0 - 1 .. q0 + 4 (q0 % 4 == 0, w % 4 == 0)
__device__ __forceinline__ void row6(const float* __restrict__ plane, int r, int q0, int h, int w,
                                     float (&v)[6]) {
  if (r < 0 || r >= h) {
#pragma unroll
    for (int i = 0; i < 6; ++i) v[i] = 0.f;
    return;
  }
  const float* row = plane + (int64_t)r * w;
  const float4 c = *reinterpret_cast<const float4*>(row + q0);
  v[0] = q0 > 0 ? row[q0 - 1] : 0.f;
  v[1] = c.x;
  v[2] = c.y;
  v[3] = c.z;
  v[4] = c.w;
  v[5] = q0 + 4 < w ? row[q0 + 4] : 0.f;
}

// block = 64 pixel quads x 4 channel groups (wave g sums channels g, g + 4,
// ...): 4x the threads of one-quad-per-thread (the 128-channel loop per
// thread left a 300-block grid latency-bound at 1.3 TB/s); the four partial
// sums combine through LDS in a fixed order
__global__ void __launch_bounds__(256)
    head_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                    const float* __restrict__ bias, float* __restrict__ y, int n, int c, int h,
                    int w) {
  __shared__ float4 red[4][64];
  const int w4 = w >> 2, qd = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * 64 + qd;
  const bool live = t < (int64_t)n * h * w4;
  const int64_t tc = live ? t : 0;
  const int q0 = 4 * (int)(tc % w4);
  const int64_t rt = tc / w4;
  const int r = (int)(rt % h), img = (int)(rt / h);
  const int64_t hw = (int64_t)h * w;
  const float* xb = x + (int64_t)img * c * hw;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (live) {
#pragma unroll 2
    for (int ch = grp; ch < c; ch += 4) {
      const float* plane = xb + ch * hw;
      const float* wc = wt + ch * 9;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        float v[6];
        row6(plane, r + dy - 1, q0, h, w, v);
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const float k = wc[dy * 3 + dx];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = fmaf(k, v[j + dx], acc[j]);
        }
      }
    }
  }
  red[grp][qd] = make_float4(acc[0], acc[1], acc[2], acc[3]);
  __syncthreads();
  if (grp != 0 || !live) return;
  const float b = bias ? bias[0] : 0.f;
  float4 s = red[0][qd];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const float4 o = red[k][qd];
    s.x += o.x;
    s.y += o.y;
    s.z += o.z;
    s.w += o.w;
  }
  *reinterpret_cast<float4*>(y + (int64_t)img * hw + (int64_t)r * w + q0) =
      make_float4(s.x + b, s.y + b, s.z + b, s.w + b);
}

// gx for channels [blockIdx.y * kDgC, + kDgC): the gy neighbourhood once, then
// 9 MACs a pixel and channel (the flipped taps)
constexpr int kDgC = 32;

__global__ void __launch_bounds__(256)
    head_dgrad_kernel(const float* __restrict__ gy, const float* __restrict__ wt,
                      float* __restrict__ gx, int n, int c, int h, int w) {
  const int w4 = w >> 2;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)n * h * w4) return;
  const int q0 = 4 * (int)(t % w4);
  const int64_t rt = t / w4;
  const int r = (int)(rt % h), img = (int)(rt / h);
  const int64_t hw = (int64_t)h * w;
  const float* g = gy + (int64_t)img * hw;
  float v[3][6];  // gy rows r + 1, r, r - 1 (tap dy reads row r + 1 - dy)
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) row6(g, r + 1 - dy, q0, h, w, v[dy]);
  const int c0 = blockIdx.y * kDgC, c1 = c0 + kDgC < c ? c0 + kDgC : c;
  float* out = gx + ((int64_t)img * c + c0) * hw + (int64_t)r * w + q0;
  for (int ch = c0; ch < c1; ++ch, out += hw) {
    const float* wc = wt + ch * 9;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const float k = wc[dy * 3 + dx];
        // gx[p] += w[t] gy[p - t + 1]: column q0 + j - dx + 1 -> v index j + 2 - dx
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = fmaf(k, v[dy][j + 2 - dx], acc[j]);
      }
    *reinterpret_cast<float4*>(out) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

// weight-gradient partials: block (c, s) over rows [s R, s R + R) of the
// n * h image rows, 9 sums a thread, a fixed tree over the block
constexpr int kWgRows = 60;  // image rows a block sums

__global__ void __launch_bounds__(256)
    head_wgrad_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                      float* __restrict__ part, int n, int c, int h, int w) {
  __shared__ float red[9][256];
  const int ch = blockIdx.x, s = blockIdx.y, tid = threadIdx.x;
  const int w4 = w >> 2;
  const int64_t hw = (int64_t)h * w;
  const int64_t rows = (int64_t)n * h;
  const int64_t r0 = (int64_t)s * kWgRows, r1 = r0 + kWgRows < rows ? r0 + kWgRows : rows;
  float acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = 0.f;
  for (int64_t e = r0 * w4 + tid; e < r1 * w4; e += 256) {
    const int q0 = 4 * (int)(e % w4);
    const int64_t rr = e / w4;
    const int r = (int)(rr % h), img = (int)(rr / h);
    const float4 g = *reinterpret_cast<const float4*>(gy + (int64_t)img * hw + (int64_t)r * w + q0);
    const float* plane = x + ((int64_t)img * c + ch) * hw;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      float v[6];
      row6(plane, r + dy - 1, q0, h, w, v);
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        float a = acc[dy * 3 + dx];
        a = fmaf(g.x, v[dx], a);
        a = fmaf(g.y, v[dx + 1], a);
        a = fmaf(g.z, v[dx + 2], a);
        a = fmaf(g.w, v[dx + 3], a);
        acc[dy * 3 + dx] = a;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) red[k][tid] = acc[k];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) {
#pragma unroll
      for (int k = 0; k < 9; ++k) red[k][tid] += red[k][tid + st];
    }
    __syncthreads();
  }
  if (tid < 9) part[((int64_t)ch * gridDim.y + s) * 9 + tid] = red[tid][0];
}

// gw[c][t] = sum over the slices, in order (one thread per (c, t))
__global__ void __launch_bounds__(256)
    head_wreduce_kernel(const float* __restrict__ part, int c, int slices, float* __restrict__ gw) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= c * 9) return;
  const int ch = e / 9, k = e - ch * 9;
  float s = 0.f;
  for (int i = 0; i < slices; ++i) s += part[((int64_t)ch * slices + i) * 9 + k];
  gw[e] = s;
}

bool head_ok(int64_t n, int64_t c, int64_t h, int64_t w) {
  return n > 0 && c > 0 && h > 0 && w > 0 && w % 4 == 0 && c <= 65535 &&
         n * c * h * w < (1LL << 31) && mde::cdiv(n * h, kWgRows) <= 65535;
}

}  // namespace

extern "C" {

int mde_head_conv_supported(int64_t n, int64_t c, int64_t h, int64_t w) {
  return head_ok(n, c, h, w) ? 1 : 0;
}

int mde_head_conv_fwd(const void* x, const float* weight, const float* bias, void* y, int64_t n,
                      int64_t c, int64_t h, int64_t w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !weight || !y || !head_ok(n, c, h, w)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t threads = n * h * (w / 4);
  const double bytes = 4.0 * (double)n * h * w * (c + 1);
  MDE_LAUNCH(mde::K_HEAD_FWD, bytes, s, head_fwd_kernel, dim3((unsigned)mde::cdiv(threads, 64)),
             dim3(256), 0, (const float*)x, weight, bias, (float*)y, (int)n, (int)c, (int)h,
             (int)w);
  return MDE_OK;
}

int mde_head_conv_dgrad(const void* gy, const float* weight, void* gx, int64_t n, int64_t c,
                        int64_t h, int64_t w, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !weight || !gx || !head_ok(n, c, h, w)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t threads = n * h * (w / 4);
  const double bytes = 4.0 * (double)n * h * w * (c + 1);
  MDE_LAUNCH(mde::K_HEAD_DGRAD, bytes, s, head_dgrad_kernel,
             dim3((unsigned)mde::cdiv(threads, 256), (unsigned)mde::cdiv(c, kDgC)), dim3(256), 0,
             (const float*)gy, weight, (float*)gx, (int)n, (int)c, (int)h, (int)w);
  return MDE_OK;
}

size_t mde_head_conv_wgrad_workspace(int64_t n, int64_t c, int64_t h, int64_t w) {
  if (!head_ok(n, c, h, w)) return 0;
  return sizeof(float) * (size_t)(c * mde::cdiv(n * h, kWgRows) * 9);
}

int mde_head_conv_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t c,
                        int64_t h, int64_t w, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !x || !gweight || !workspace || !head_ok(n, c, h, w)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int slices = (int)mde::cdiv(n * h, kWgRows);
  const double bytes = 4.0 * (double)n * h * w * (c + 1);
  float* part = (float*)workspace;
  MDE_LAUNCH(mde::K_HEAD_WGRAD, bytes, s, head_wgrad_kernel, dim3((unsigned)c, (unsigned)slices),
             dim3(256), 0, (const float*)gy, (const float*)x, part, (int)n, (int)c, (int)h, (int)w);
  MDE_LAUNCH(mde::K_HEAD_WGRAD, 4.0 * (double)c * slices * 9, s, head_wreduce_kernel,
             dim3((unsigned)mde::cdiv(c * 9, 256)), dim3(256), 0, (const float*)part, (int)c,
             slices, gweight);
  return MDE_OK;
}

}  // extern "C"
