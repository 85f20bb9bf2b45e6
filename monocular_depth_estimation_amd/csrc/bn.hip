// BatchNorm2d (NCHW, fp32) with fused activation and residual for gfx950.
//
// Replaces nn.BatchNorm2d (+ the ReLU / residual add that follows it) at the
// 73 BN sites of GuideDepth: src/GuideDepth/model/modules.py:43-49,53-59,68-74
// and src/GuideDepth/model/DDRNet_23_slim.py:46-49,80-86,119-172,201-203,
// 231-235,244-265,294-298.  MIOpen's spatial BN was 88 of 153 ms of a
// 640x480 bs=32 train step (profiles/r01_*), ~10% of HBM bandwidth.
//
//   y = act(x * scale[c] + shift[c] (+ r))      scale = gamma*invstd,
//                                               shift = beta - mean*scale
// Training: batch mean / biased variance over (N,H,W) per channel, running
// stats updated with momentum and the unbiased variance, num_batches_tracked
// += 1 — nn.BatchNorm2d semantics.  Eval: running statistics.
//
// Forward  = stats (per-slice shifted sums) -> final (per channel, double)
//            -> apply (streaming).            HBM: 2 reads + 1 write of x.
// Backward = reduce (sum dy', sum dy'(x-mean)) -> final -> apply, where
//            dy' = dy * [act'] is recomputed from x (and r) — y is never
//            stored.                          HBM: 4 reads + 1 write.
// All reductions are two-level with fixed order: deterministic.
#include <cmath>

#include "common.h"

namespace {

constexpr int kTarget = 2048;     // blocks to aim for per reduction launch
constexpr int kMinSlice = 4096;   // elements per slice at least

struct Geo {
  int64_t c, hw, total;  // total = n * hw elements per channel
  int slices;
  int64_t slice_len;     // multiple of 4 when hw % 4 == 0
};

Geo geometry(int64_t n, int64_t c, int64_t hw) {
  Geo g;
  g.c = c;
  g.hw = hw;
  g.total = n * hw;
  int64_t s = mde::cdiv(kTarget, c);
  const int64_t by_size = mde::cdiv(g.total, kMinSlice);
  if (s > by_size) s = by_size;
  if (s < 1) s = 1;
  if (s > 1024) s = 1024;
  g.slices = (int)s;
  int64_t len = mde::cdiv(g.total, s);
  if (hw % 4 == 0) len = mde::cdiv(len, 4) * 4;
  g.slice_len = len;
  return g;
}

__device__ __forceinline__ float act_fn(float v, int act) {
  return act == 1 ? fmaxf(v, 0.f) : v;
}

// Per-channel scale/shift from (gamma, beta, mean, invstd).
__device__ __forceinline__ void coeffs(const float* gamma, const float* beta,
                                       const float* mean, const float* invstd,
                                       int64_t c, float* sc, float* sh) {
  const float s = gamma[c] * invstd[c];
  *sc = s;
  *sh = beta[c] - mean[c] * s;
}

// part[(c * slices + s) * 2 + {0,1}] = sum(x - ref), sum((x - ref)^2)
template <bool VEC>
__global__ void __launch_bounds__(256)
    bn_stats_kernel(const float* __restrict__ x, int64_t c, int64_t hw,
                    int64_t total, int64_t slice_len, int slices,
                    float* __restrict__ part) {
  __shared__ float red[4];
  const int64_t ch = blockIdx.y;
  const int s = blockIdx.x;
  const int64_t i0 = s * slice_len;
  const int64_t i1 = i0 + slice_len < total ? i0 + slice_len : total;
  const float* xc = x + ch * hw;
  const float ref = xc[0];  // shift for the variance (cancellation guard)
  const int64_t chw = c * hw;
  float s1 = 0.f, s2 = 0.f;
  if (VEC) {
    for (int64_t i = i0 + 4 * threadIdx.x; i < i1; i += 4 * 256) {
      const int64_t nn = i / hw, p = i - nn * hw;
      const float4 v = *reinterpret_cast<const float4*>(xc + nn * chw + p);
      const float a = v.x - ref, b = v.y - ref, cc = v.z - ref, d = v.w - ref;
      s1 += (a + b) + (cc + d);
      s2 += (a * a + b * b) + (cc * cc + d * d);
    }
  } else {
    for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
      const int64_t nn = i / hw, p = i - nn * hw;
      const float a = xc[nn * chw + p] - ref;
      s1 += a;
      s2 += a * a;
    }
  }
  const float t1 = mde::block_sum256(s1, red);
  const float t2 = mde::block_sum256(s2, red);
  if (threadIdx.x == 0) {
    float* o = part + (ch * slices + s) * 2;
    o[0] = t1;
    o[1] = t2;
  }
}

// Training: combine slices (double), write mean/invstd, update running stats.
__global__ void __launch_bounds__(256)
    bn_fwd_final_kernel(const float* __restrict__ x, int64_t c, int64_t hw,
                        int64_t total, int slices, const float* __restrict__ part,
                        float momentum, float eps, float* __restrict__ rmean,
                        float* __restrict__ rvar, int64_t* __restrict__ nbt,
                        float* __restrict__ mean, float* __restrict__ invstd) {
  const int64_t ch = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (ch == 0 && nbt) nbt[0] += 1;
  if (ch >= c) return;
  double a = 0.0, b = 0.0;
  const float* p = part + ch * slices * 2;
  for (int s = 0; s < slices; ++s) {
    a += (double)p[2 * s];
    b += (double)p[2 * s + 1];
  }
  const double n = (double)total;
  const double ref = (double)x[ch * hw];
  const double dm = a / n;
  double var = b / n - dm * dm;
  if (var < 0.0) var = 0.0;
  const double m = ref + dm;
  mean[ch] = (float)m;
  invstd[ch] = (float)(1.0 / std::sqrt(var + (double)eps));
  if (rmean) {
    const double unb = total > 1 ? var * n / (n - 1.0) : var;
    rmean[ch] = (float)((1.0 - momentum) * (double)rmean[ch] + momentum * m);
    rvar[ch] = (float)((1.0 - momentum) * (double)rvar[ch] + momentum * unb);
  }
}

// Eval: mean/invstd from the running statistics.
__global__ void __launch_bounds__(256)
    bn_eval_final_kernel(int64_t c, const float* __restrict__ rmean,
                         const float* __restrict__ rvar, float eps,
                         float* __restrict__ mean, float* __restrict__ invstd) {
  const int64_t ch = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (ch >= c) return;
  mean[ch] = rmean[ch];
  invstd[ch] = 1.f / sqrtf(rvar[ch] + eps);
}

// y = act(x * scale + shift (+ r)); one block row of planes, float4 lanes.
template <bool VEC>
__global__ void __launch_bounds__(256)
    bn_apply_kernel(const float* __restrict__ x, const float* __restrict__ r,
                    const float* __restrict__ gamma, const float* __restrict__ beta,
                    const float* __restrict__ mean, const float* __restrict__ invstd,
                    float* __restrict__ y, int64_t planes, int64_t c, int64_t hw,
                    int act) {
  if (VEC) {
    const int64_t hw4 = hw >> 2, total = planes * hw4;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      const int64_t plane = t / hw4;
      float sc, sh;
      coeffs(gamma, beta, mean, invstd, plane % c, &sc, &sh);
      float4 v = reinterpret_cast<const float4*>(x)[t];
      v.x = v.x * sc + sh;
      v.y = v.y * sc + sh;
      v.z = v.z * sc + sh;
      v.w = v.w * sc + sh;
      if (r) {
        const float4 q = reinterpret_cast<const float4*>(r)[t];
        v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
      }
      v.x = act_fn(v.x, act); v.y = act_fn(v.y, act);
      v.z = act_fn(v.z, act); v.w = act_fn(v.w, act);
      reinterpret_cast<float4*>(y)[t] = v;
    }
  } else {
    const int64_t total = planes * hw;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      float sc, sh;
      coeffs(gamma, beta, mean, invstd, (t / hw) % c, &sc, &sh);
      float v = x[t] * sc + sh;
      if (r) v += r[t];
      y[t] = act_fn(v, act);
    }
  }
}

// dy' = dy * [pre-activation > 0] for relu, recomputed exactly as the forward.
__device__ __forceinline__ float dy_eff(float g, float xv, float rv, float sc,
                                        float sh, int act) {
  if (act != 1) return g;
  const float pre = xv * sc + sh + rv;
  return pre > 0.f ? g : 0.f;
}

// part[(c*slices+s)*2] = sum dy', sum dy' * (x - mean)
template <bool VEC>
__global__ void __launch_bounds__(256)
    bn_bwd_reduce_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                         const float* __restrict__ r,
                         const float* __restrict__ gamma, const float* __restrict__ beta,
                         const float* __restrict__ mean, const float* __restrict__ invstd,
                         int64_t c, int64_t hw, int64_t total, int64_t slice_len,
                         int slices, int act, float* __restrict__ part) {
  __shared__ float red[4];
  const int64_t ch = blockIdx.y;
  const int s = blockIdx.x;
  const int64_t i0 = s * slice_len;
  const int64_t i1 = i0 + slice_len < total ? i0 + slice_len : total;
  float sc, sh;
  coeffs(gamma, beta, mean, invstd, ch, &sc, &sh);
  const float mu = mean[ch];
  const int64_t chw = c * hw;
  const int64_t base = ch * hw;
  float s1 = 0.f, s2 = 0.f;
  if (VEC) {
    for (int64_t i = i0 + 4 * threadIdx.x; i < i1; i += 4 * 256) {
      const int64_t nn = i / hw, p = i - nn * hw;
      const int64_t off = base + nn * chw + p;
      const float4 g = *reinterpret_cast<const float4*>(gy + off);
      const float4 v = *reinterpret_cast<const float4*>(x + off);
      float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r) q = *reinterpret_cast<const float4*>(r + off);
      const float a = dy_eff(g.x, v.x, q.x, sc, sh, act);
      const float b = dy_eff(g.y, v.y, q.y, sc, sh, act);
      const float cc = dy_eff(g.z, v.z, q.z, sc, sh, act);
      const float d = dy_eff(g.w, v.w, q.w, sc, sh, act);
      s1 += (a + b) + (cc + d);
      s2 += (a * (v.x - mu) + b * (v.y - mu)) + (cc * (v.z - mu) + d * (v.w - mu));
    }
  } else {
    for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
      const int64_t nn = i / hw, p = i - nn * hw;
      const int64_t off = base + nn * chw + p;
      const float v = x[off];
      const float a = dy_eff(gy[off], v, r ? r[off] : 0.f, sc, sh, act);
      s1 += a;
      s2 += a * (v - mu);
    }
  }
  const float t1 = mde::block_sum256(s1, red);
  const float t2 = mde::block_sum256(s2, red);
  if (threadIdx.x == 0) {
    float* o = part + (ch * slices + s) * 2;
    o[0] = t1;
    o[1] = t2;
  }
}

// ggamma = invstd * sum dy'(x-mean), gbeta = sum dy'; dx = A dy' + B x + D.
__global__ void __launch_bounds__(256)
    bn_bwd_final_kernel(int64_t c, int64_t total, int slices,
                        const float* __restrict__ part, const float* __restrict__ gamma,
                        const float* __restrict__ mean, const float* __restrict__ invstd,
                        int training, float* __restrict__ ggamma,
                        float* __restrict__ gbeta, float* __restrict__ coef) {
  const int64_t ch = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (ch >= c) return;
  double a = 0.0, b = 0.0;
  const float* p = part + ch * slices * 2;
  for (int s = 0; s < slices; ++s) {
    a += (double)p[2 * s];
    b += (double)p[2 * s + 1];
  }
  const double is = (double)invstd[ch];
  const double scale = (double)gamma[ch] * is;
  if (ggamma) ggamma[ch] = (float)(b * is);
  if (gbeta) gbeta[ch] = (float)a;
  double A = scale, B = 0.0, D = 0.0;
  if (training) {
    const double n = (double)total;
    B = -scale * is * is * b / n;
    D = -scale * a / n - B * (double)mean[ch];
  }
  coef[3 * ch] = (float)A;
  coef[3 * ch + 1] = (float)B;
  coef[3 * ch + 2] = (float)D;
}

template <bool VEC>
__global__ void __launch_bounds__(256)
    bn_bwd_apply_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                        const float* __restrict__ r,
                        const float* __restrict__ gamma, const float* __restrict__ beta,
                        const float* __restrict__ mean, const float* __restrict__ invstd,
                        const float* __restrict__ coef, float* __restrict__ gx,
                        float* __restrict__ gr, int64_t planes, int64_t c, int64_t hw,
                        int act) {
  if (VEC) {
    const int64_t hw4 = hw >> 2, total = planes * hw4;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      const int64_t ch = (t / hw4) % c;
      float sc, sh;
      coeffs(gamma, beta, mean, invstd, ch, &sc, &sh);
      const float A = coef[3 * ch], B = coef[3 * ch + 1], D = coef[3 * ch + 2];
      const float4 g = reinterpret_cast<const float4*>(gy)[t];
      const float4 v = reinterpret_cast<const float4*>(x)[t];
      float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r) q = reinterpret_cast<const float4*>(r)[t];
      const float4 e = make_float4(dy_eff(g.x, v.x, q.x, sc, sh, act),
                                   dy_eff(g.y, v.y, q.y, sc, sh, act),
                                   dy_eff(g.z, v.z, q.z, sc, sh, act),
                                   dy_eff(g.w, v.w, q.w, sc, sh, act));
      reinterpret_cast<float4*>(gx)[t] =
          make_float4(A * e.x + B * v.x + D, A * e.y + B * v.y + D,
                      A * e.z + B * v.z + D, A * e.w + B * v.w + D);
      if (gr) reinterpret_cast<float4*>(gr)[t] = e;
    }
  } else {
    const int64_t total = planes * hw;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      const int64_t ch = (t / hw) % c;
      float sc, sh;
      coeffs(gamma, beta, mean, invstd, ch, &sc, &sh);
      const float v = x[t];
      const float e = dy_eff(gy[t], v, r ? r[t] : 0.f, sc, sh, act);
      gx[t] = coef[3 * ch] * e + coef[3 * ch + 1] * v + coef[3 * ch + 2];
      if (gr) gr[t] = e;
    }
  }
}

inline int stream_grid(int64_t work) {
  const int64_t b = mde::cdiv(work, 256);
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

inline size_t round16(size_t v) { return (v + 15) & ~size_t(15); }

bool args_ok(int64_t n, int64_t c, int64_t h, int64_t w) {
  return n > 0 && c > 0 && h > 0 && w > 0 && c <= 65535 &&
         n * h * w < ((int64_t)1 << 40);
}

}  // namespace

extern "C" {

size_t mde_batchnorm_workspace(int64_t n, int64_t c, int64_t h, int64_t w) {
  const Geo g = geometry(n, c, h * w);
  return round16(sizeof(float) * 2 * (size_t)c * g.slices) +
         round16(sizeof(float) * 3 * (size_t)c);
}

int mde_batchnorm_fwd_train(const void* x, const float* gamma, const float* beta,
                            float* running_mean, float* running_var,
                            int64_t* num_batches_tracked, float momentum,
                            float eps, const void* residual, void* y,
                            float* save_mean, float* save_invstd, int64_t n,
                            int64_t c, int64_t h, int64_t w, int act,
                            void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !gamma || !beta || !y || !save_mean || !save_invstd || !workspace ||
      (!running_mean != !running_var) || act < 0 || act > 1 || !args_ok(n, c, h, w))
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t hw = h * w;
  const Geo g = geometry(n, c, hw);
  float* part = (float*)workspace;
  const bool vec = hw % 4 == 0;
  const double bytes = 4.0 * n * c * (double)hw;
  if (vec) {
    MDE_LAUNCH(mde::K_BN_STATS, bytes, s, bn_stats_kernel<true>,
               dim3(g.slices, (unsigned)c), dim3(256), 0, (const float*)x, c, hw,
               g.total, g.slice_len, g.slices, part);
  } else {
    MDE_LAUNCH(mde::K_BN_STATS, bytes, s, bn_stats_kernel<false>,
               dim3(g.slices, (unsigned)c), dim3(256), 0, (const float*)x, c, hw,
               g.total, g.slice_len, g.slices, part);
  }
  MDE_LAUNCH(mde::K_BN_FINAL, 8.0 * c * g.slices, s, bn_fwd_final_kernel,
             dim3((unsigned)mde::cdiv(c, 256)), dim3(256), 0, (const float*)x, c,
             hw, g.total, g.slices, (const float*)part, momentum, eps,
             running_mean, running_var, num_batches_tracked, save_mean,
             save_invstd);
  const double abytes = bytes * (residual ? 3.0 : 2.0);
  if (vec) {
    MDE_LAUNCH(mde::K_BN_APPLY, abytes, s, bn_apply_kernel<true>,
               dim3(stream_grid(n * c * hw / 4)), dim3(256), 0, (const float*)x,
               (const float*)residual, gamma, beta, (const float*)save_mean,
               (const float*)save_invstd, (float*)y, n * c, c, hw, act);
  } else {
    MDE_LAUNCH(mde::K_BN_APPLY, abytes, s, bn_apply_kernel<false>,
               dim3(stream_grid(n * c * hw)), dim3(256), 0, (const float*)x,
               (const float*)residual, gamma, beta, (const float*)save_mean,
               (const float*)save_invstd, (float*)y, n * c, c, hw, act);
  }
  return MDE_OK;
}

int mde_batchnorm_fwd_eval(const void* x, const float* gamma, const float* beta,
                           const float* running_mean, const float* running_var,
                           float eps, const void* residual, void* y,
                           float* save_mean, float* save_invstd, int64_t n,
                           int64_t c, int64_t h, int64_t w, int act, int dtype,
                           void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !gamma || !beta || !running_mean || !running_var || !y ||
      !save_mean || !save_invstd || act < 0 || act > 1 || !args_ok(n, c, h, w))
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t hw = h * w;
  MDE_LAUNCH(mde::K_BN_FINAL, 16.0 * c, s, bn_eval_final_kernel,
             dim3((unsigned)mde::cdiv(c, 256)), dim3(256), 0, c, running_mean,
             running_var, eps, save_mean, save_invstd);
  const double abytes = 4.0 * n * c * (double)hw * (residual ? 3.0 : 2.0);
  if (hw % 4 == 0) {
    MDE_LAUNCH(mde::K_BN_APPLY, abytes, s, bn_apply_kernel<true>,
               dim3(stream_grid(n * c * hw / 4)), dim3(256), 0, (const float*)x,
               (const float*)residual, gamma, beta, (const float*)save_mean,
               (const float*)save_invstd, (float*)y, n * c, c, hw, act);
  } else {
    MDE_LAUNCH(mde::K_BN_APPLY, abytes, s, bn_apply_kernel<false>,
               dim3(stream_grid(n * c * hw)), dim3(256), 0, (const float*)x,
               (const float*)residual, gamma, beta, (const float*)save_mean,
               (const float*)save_invstd, (float*)y, n * c, c, hw, act);
  }
  return MDE_OK;
}

int mde_batchnorm_bwd(const void* gy, const void* x, const void* residual,
                      const float* gamma, const float* beta, const float* mean,
                      const float* invstd, int training, void* gx,
                      void* gresidual, float* ggamma, float* gbeta, int64_t n,
                      int64_t c, int64_t h, int64_t w, int act,
                      void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !x || !gamma || !beta || !mean || !invstd || !gx || !workspace ||
      act < 0 || act > 1 || !args_ok(n, c, h, w) || (gresidual && !residual && act))
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t hw = h * w;
  const Geo g = geometry(n, c, hw);
  float* part = (float*)workspace;
  float* coef = (float*)((char*)workspace + round16(sizeof(float) * 2 * (size_t)c * g.slices));
  const bool vec = hw % 4 == 0;
  const double big = 4.0 * n * c * (double)hw;
  const double rb = residual && act ? big : 0.0;
  if (vec) {
    MDE_LAUNCH(mde::K_BN_BWD_REDUCE, 2.0 * big + rb, s, bn_bwd_reduce_kernel<true>,
               dim3(g.slices, (unsigned)c), dim3(256), 0, (const float*)gy,
               (const float*)x, act ? (const float*)residual : nullptr, gamma,
               beta, mean, invstd, c, hw, g.total, g.slice_len, g.slices, act,
               part);
  } else {
    MDE_LAUNCH(mde::K_BN_BWD_REDUCE, 2.0 * big + rb, s, bn_bwd_reduce_kernel<false>,
               dim3(g.slices, (unsigned)c), dim3(256), 0, (const float*)gy,
               (const float*)x, act ? (const float*)residual : nullptr, gamma,
               beta, mean, invstd, c, hw, g.total, g.slice_len, g.slices, act,
               part);
  }
  MDE_LAUNCH(mde::K_BN_BWD_FINAL, 8.0 * c * g.slices, s, bn_bwd_final_kernel,
             dim3((unsigned)mde::cdiv(c, 256)), dim3(256), 0, c, g.total,
             g.slices, (const float*)part, gamma, mean, invstd, training,
             ggamma, gbeta, coef);
  const double abytes = 3.0 * big + rb + (gresidual ? big : 0.0);
  if (vec) {
    MDE_LAUNCH(mde::K_BN_BWD_APPLY, abytes, s, bn_bwd_apply_kernel<true>,
               dim3(stream_grid(n * c * hw / 4)), dim3(256), 0, (const float*)gy,
               (const float*)x, act ? (const float*)residual : nullptr, gamma,
               beta, mean, invstd, (const float*)coef, (float*)gx,
               (float*)gresidual, n * c, c, hw, act);
  } else {
    MDE_LAUNCH(mde::K_BN_BWD_APPLY, abytes, s, bn_bwd_apply_kernel<false>,
               dim3(stream_grid(n * c * hw)), dim3(256), 0, (const float*)gy,
               (const float*)x, act ? (const float*)residual : nullptr, gamma,
               beta, mean, invstd, (const float*)coef, (float*)gx,
               (float*)gresidual, n * c, c, hw, act);
  }
  return MDE_OK;
}

}  // extern "C"
