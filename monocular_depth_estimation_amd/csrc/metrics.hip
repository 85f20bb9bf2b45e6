// Depth-evaluation error sums on the GPU.
//
// Replaces the per-batch host path of src/test.py:96-124 -- pred / gt copied
// to numpy, pred clamped (test.py:105-108), masked by the evaluation range
// and the Eigen crop (test.py:110-117), then utils.compute_errors
// (src/utils.py:45-66) -- and GuideDepth's FastDepth Result.evaluate
// (src/GuideDepth/metrics.py:41-62).  Every metric of both is a function of
// these sums over the selected pixels, accumulated here in double:
//   0 count                     5 sum (ln g - ln p)^2       10 sum |g - p|
//   1 sum [max(g/p,p/g) < 1.25] 6 sum |g - p| / g           11 sum (log10 p - log10 g)^2
//   2 ... < 1.25^2              7 sum (g - p)^2 / g         12 sum |1/p - 1/g|
//   3 ... < 1.25^3              8 sum (ln p - ln g)         13 sum (1/p - 1/g)^2
//   4 sum (g - p)^2             9 sum |log10 p - log10 g|   14, 15 unused (0)
// Per-pixel terms are formed in fp32 as numpy does on the reference's float32
// arrays; only the accumulation is wider.  One block per kRows image rows
// writes a partial; one block sums the partials in a fixed order
// (deterministic).  Algorithmic HBM bytes: 4(|pred| + |gt|).

#include <cmath>

#include "common.h"

namespace {

constexpr int kSums = 16;
constexpr int kUsed = 14;
constexpr int kRows = 8;

struct EvalArgs {
  int64_t n, h, w;
  float lo, hi;
  int mode;            // bit 0: clamp pred + range-mask gt; bit 1: crop
  int c0, c1, c2, c3;  // crop rows [c0, c1), cols [c2, c3)
};

__device__ __forceinline__ double block_sum_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256)
    eval_partial_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                        EvalArgs A, double* __restrict__ part) {
  __shared__ double red[4];
  double s[kUsed];
#pragma unroll
  for (int i = 0; i < kUsed; ++i) s[i] = 0.0;
  const int64_t rows = A.n * A.h;
  const int64_t r0 = (int64_t)blockIdx.x * kRows;
  for (int64_t rr = r0; rr < r0 + kRows && rr < rows; ++rr) {
    const int y = (int)(rr % A.h);
    if ((A.mode & 2) && (y < A.c0 || y >= A.c1)) continue;
    const float* pr = pred + rr * A.w;
    const float* gr = gt + rr * A.w;
    for (int x = threadIdx.x; x < A.w; x += 256) {
      if ((A.mode & 2) && (x < A.c2 || x >= A.c3)) continue;
      float p = pr[x];
      const float g = gr[x];
      if (A.mode & 1) {
        if (p < A.lo) p = A.lo;
        if (p > A.hi) p = A.hi;
        if (isnan(p)) p = A.lo;
        if (!(g > A.lo && g < A.hi)) continue;
      }
      const float th = fmaxf(g / p, p / g);
      const float d = g - p;
      const float lp = logf(p), lg = logf(g);
      const float l10 = log10f(p) - log10f(g);
      const float ip = 1.f / p - 1.f / g;
      s[0] += 1.0;
      s[1] += th < 1.25f ? 1.0 : 0.0;
      s[2] += th < 1.25f * 1.25f ? 1.0 : 0.0;
      s[3] += th < 1.25f * 1.25f * 1.25f ? 1.0 : 0.0;
      s[4] += (double)(d * d);
      s[5] += (double)((lg - lp) * (lg - lp));
      s[6] += (double)(fabsf(d) / g);
      s[7] += (double)(d * d / g);
      s[8] += (double)(lp - lg);
      s[9] += (double)fabsf(l10);
      s[10] += (double)fabsf(d);
      s[11] += (double)(l10 * l10);
      s[12] += (double)fabsf(ip);
      s[13] += (double)(ip * ip);
    }
  }
  double* o = part + (int64_t)blockIdx.x * kSums;
#pragma unroll
  for (int i = 0; i < kUsed; ++i) {
    const double t = block_sum_d(s[i], red);
    if (threadIdx.x == 0) o[i] = t;
  }
  if (threadIdx.x < kSums - kUsed) o[kUsed + threadIdx.x] = 0.0;
}

// One block: out[i] = sum_b part[b, i] in a fixed order.
__global__ void __launch_bounds__(256)
    eval_final_kernel(const double* __restrict__ part, int64_t blocks, double* __restrict__ out) {
  __shared__ double red[4];
  for (int i = 0; i < kSums; ++i) {
    double v = 0.0;
    for (int64_t b = threadIdx.x; b < blocks; b += 256) v += part[b * kSums + i];
    const double t = block_sum_d(v, red);
    if (threadIdx.x == 0) out[i] = t;
  }
}

int64_t eval_blocks(int64_t n, int64_t h) { return mde::cdiv(n * h, kRows); }

}  // namespace

extern "C" {

size_t mde_eval_workspace(int64_t n, int64_t h, int64_t w) {
  if (n <= 0 || h <= 0 || w <= 0) return 0;
  return (size_t)(sizeof(double) * kSums * eval_blocks(n, h));
}

int mde_eval_sums(const void* pred, const void* gt, int64_t n, int64_t h, int64_t w,
                  float min_depth, float max_depth, int mode, const int32_t* crop,
                  void* workspace, double* sums, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!pred || !gt || !workspace || !sums || n <= 0 || h <= 0 || w <= 0 || mode < 0 ||
      mode > 3 || ((mode & 2) && !crop) || n * h >= ((int64_t)1 << 31) ||
      w >= ((int64_t)1 << 30))
    return MDE_ERR_INVALID_ARG;
  EvalArgs A{n, h, w, min_depth, max_depth, mode, 0, (int)h, 0, (int)w};
  if (mode & 2) {
    A.c0 = crop[0];
    A.c1 = crop[1];
    A.c2 = crop[2];
    A.c3 = crop[3];
  }
  hipStream_t st = (hipStream_t)stream;
  const int64_t blocks = eval_blocks(n, h);
  double* part = (double*)workspace;
  MDE_LAUNCH(mde::K_EVAL, 8.0 * n * h * w, st, eval_partial_kernel, dim3((unsigned)blocks),
             dim3(256), 0, (const float*)pred, (const float*)gt, A, part);
  MDE_LAUNCH(mde::K_EVAL_FINAL, 8.0 * kSums * blocks, st, eval_final_kernel, dim3(1), dim3(256),
             0, part, blocks, sums);
  return MDE_OK;
}

}  // extern "C"
