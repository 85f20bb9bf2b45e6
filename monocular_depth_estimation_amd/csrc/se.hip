// Squeeze-excitation over a fused channel concatenation (NCHW, fp32).
//
// Reference: torch.cat([x, y], 1) (src/GuideDepth/model/modules.py:90) feeding
// SELayer.forward (modules.py:21-25): mean over H,W -> Linear(C,C/r) -> ReLU
// -> Linear(C/r,C) -> Sigmoid -> x * s.  The concatenation is never
// materialised: channel ch < ca reads xa, otherwise xb.
//
// Forward  = squeeze (per-plane partial sums, deterministic two-level
//            reduction) -> fc (one block per sample) -> scale (streaming).
// Backward = dot (partial sums of g*x) -> fc backward (per sample) ->
//            weight gradients (sum over samples in fixed order) -> apply.
//
// The gated variant (mde_se_gate_*) adds the fc biases and the hardsigmoid
// gate of torchvision's SqueezeExcitation (MobileNetV3-Large blocks 4-6 and
// 11-15: avgpool -> fc1 (+b1) -> ReLU -> fc2 (+b2) -> hardsigmoid -> scale).
#include "common.h"

namespace {

constexpr int kChunk = 16384;  // elements of one plane reduced by one block

template <typename T>
__device__ __forceinline__ const T* plane_ptr(const T* xa, int64_t ca, const T* xb, int64_t cb,
                                              int64_t nidx, int64_t ch, int64_t hw) {
  return ch < ca ? xa + (nidx * ca + ch) * hw
                 : xb + (nidx * cb + (ch - ca)) * hw;
}

// part[plane * chunks + k] = sum of chunk k of plane of x (MODE 0), of g*x
// (MODE 1) or of u = relu(sc*x + sh) (MODE 2: the input is the raw output of
// the conv before a BatchNorm + ReLU; sc / sh = the BN coefficients).
enum { kSum = 0, kDot = 1, kBnRelu = 2 };

__device__ __forceinline__ float bnrelu(float v, float sc, float sh) {
  return fmaxf(fmaf(v, sc, sh), 0.f);
}

template <int MODE, typename T = float>
__global__ void __launch_bounds__(256)
    se_partial_kernel(const T* __restrict__ g, const T* __restrict__ xa,
                      int64_t ca, const T* __restrict__ xb, int64_t cb,
                      int64_t hw, int chunks, float* __restrict__ part,
                      const float* __restrict__ scale = nullptr,
                      const float* __restrict__ shift = nullptr) {
  __shared__ float red[4];
  const int64_t c = ca + cb;
  const int64_t plane = blockIdx.y;
  const int64_t nidx = plane / c, ch = plane % c;
  const T* x = plane_ptr(xa, ca, xb, cb, nidx, ch, hw);
  const T* gp = MODE == kDot ? g + plane * hw : nullptr;
  const float sc = MODE == kBnRelu ? scale[ch] : 0.f, sh = MODE == kBnRelu ? shift[ch] : 0.f;
  const int64_t beg = (int64_t)blockIdx.x * kChunk;
  const int64_t end = beg + kChunk < hw ? beg + kChunk : hw;
  float acc = 0.f;
  if ((hw & 3) == 0) {
    for (int64_t i = beg + 4 * threadIdx.x; i < end; i += 4 * 256) {
      float4 v = mde::ld4(x + i);
      if (MODE == kDot) {
        const float4 q = mde::ld4(gp + i);
        acc += (v.x * q.x + v.y * q.y) + (v.z * q.z + v.w * q.w);
      } else {
        if (MODE == kBnRelu) {
          v.x = bnrelu(v.x, sc, sh); v.y = bnrelu(v.y, sc, sh);
          v.z = bnrelu(v.z, sc, sh); v.w = bnrelu(v.w, sc, sh);
        }
        acc += (v.x + v.y) + (v.z + v.w);
      }
    }
  } else {
    for (int64_t i = beg + threadIdx.x; i < end; i += 256) {
      const float xv = mde::ld1(x + i);
      acc += MODE == kDot ? xv * mde::ld1(gp + i) : (MODE == kBnRelu ? bnrelu(xv, sc, sh) : xv);
    }
  }
  const float tot = mde::block_sum256(acc, red);
  if (threadIdx.x == 0) part[plane * chunks + blockIdx.x] = tot;
}

// One block per sample: mean -> hidden = relu(W1 m) -> s = sigmoid(W2 h).
__device__ __forceinline__ float gate_fn(float z, int gate) {
  // 0: sigmoid; 1: hardsigmoid = clamp(z / 6 + 1/2, 0, 1) (ATen: x <= -3 -> 0, x >= 3 -> 1)
  if (gate == 0) return 1.f / (1.f + expf(-z));
  return z <= -3.f ? 0.f : (z >= 3.f ? 1.f : z / 6.f + 0.5f);
}

// The per-sample FCs are GEMVs; each runs as its own kernel over a grid of
// (sample, 16 outputs) blocks of 16 waves, one wave per output, so the
// weight rows stream with many loads in flight instead of one serial chain.
constexpr int kOutPerBlock = 16;

// hidden[n, j] = relu(W1[j] . mean[n] + b1[j]); block (n, 0) also writes mean.
__global__ void __launch_bounds__(1024)
    se_fc1_kernel(const float* __restrict__ part, int chunks, int c, int cr,
                  float inv_hw, const float* __restrict__ w1,
                  const float* __restrict__ b1, float* __restrict__ hidden,
                  float* __restrict__ mean) {
  extern __shared__ float m[];  // [c]
  const int nidx = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int ch = threadIdx.x; ch < c; ch += blockDim.x) {
    const float* p = part + ((int64_t)nidx * c + ch) * chunks;
    float acc = 0.f;
    for (int k = 0; k < chunks; ++k) acc += p[k];
    m[ch] = acc * inv_hw;
    if (blockIdx.y == 0) mean[(int64_t)nidx * c + ch] = m[ch];
  }
  __syncthreads();
  const int j = blockIdx.y * kOutPerBlock + wid;
  if (j >= cr) return;
  const float* wr = w1 + (int64_t)j * c;
  float acc = 0.f;
  for (int ch = lane; ch < c; ch += 64) acc += wr[ch] * m[ch];
  acc = mde::wave_sum(acc);
  if (b1) acc += b1[j];
  if (lane == 0) hidden[(int64_t)nidx * cr + j] = acc > 0.f ? acc : 0.f;
}

// s[n, ch] = gate(W2[ch] . hidden[n] + b2[ch])
__global__ void __launch_bounds__(1024)
    se_fc2_kernel(int c, int cr, const float* __restrict__ w2,
                  const float* __restrict__ b2, int gate,
                  const float* __restrict__ hidden, float* __restrict__ s) {
  extern __shared__ float hdn[];  // [cr]
  const int nidx = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int j = threadIdx.x; j < cr; j += blockDim.x) hdn[j] = hidden[(int64_t)nidx * cr + j];
  __syncthreads();
  const int ch = blockIdx.y * kOutPerBlock + wid;
  if (ch >= c) return;
  const float* wr = w2 + (int64_t)ch * cr;
  float z = 0.f;
  for (int j = lane; j < cr; j += 64) z += wr[j] * hdn[j];
  z = mde::wave_sum(z);
  if (b2) z += b2[ch];
  if (lane == 0) s[(int64_t)nidx * c + ch] = gate_fn(z, gate);
}

// out[plane, i] = x[plane, i] * s[plane]  (cat fused: plane -> xa or xb);
// BNR: out = s[plane] * relu(sc * x + sh) (x = the BatchNorm's raw input).
template <bool BNR, typename T = float>
__global__ void __launch_bounds__(256)
    se_scale_kernel(const T* __restrict__ xa, int64_t ca,
                    const T* __restrict__ xb, int64_t cb, int64_t hw,
                    int64_t planes, const float* __restrict__ s,
                    T* __restrict__ out, const float* __restrict__ scale = nullptr,
                    const float* __restrict__ shift = nullptr) {
  const int64_t c = ca + cb;
  if ((hw & 3) == 0) {
    const int64_t hw4 = hw >> 2;
    const int64_t total = planes * hw4;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      const int64_t plane = t / hw4, i = (t - plane * hw4) << 2;
      const int64_t ch = plane % c;
      const T* x = plane_ptr(xa, ca, xb, cb, plane / c, ch, hw);
      const float sc = s[plane];
      float4 v = mde::ld4(x + i);
      if (BNR) {
        const float a = scale[ch], b = shift[ch];
        v.x = bnrelu(v.x, a, b); v.y = bnrelu(v.y, a, b);
        v.z = bnrelu(v.z, a, b); v.w = bnrelu(v.w, a, b);
      }
      v.x *= sc; v.y *= sc; v.z *= sc; v.w *= sc;
      mde::st4(out + plane * hw + i, v);
    }
  } else {
    const int64_t total = planes * hw;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      const int64_t plane = t / hw, i = t - plane * hw;
      const int64_t ch = plane % c;
      const T* x = plane_ptr(xa, ca, xb, cb, plane / c, ch, hw);
      const float xv = mde::ld1(x + i);
      const float v = BNR ? bnrelu(xv, scale[ch], shift[ch]) : xv;
      mde::st1(out + t, v * s[plane]);
    }
  }
}

// Per-sample backward through the gate / W2 / relu / W1, three GEMV kernels:
//   dz = ds * gate'(z)  (ds = sum g*x; sigmoid: s(1-s); hardsigmoid: 1/6 on
//        (-3, 3), z recomputed from the hidden)
//   dh = (h > 0) W2^T dz;   dm = W1^T dh
__global__ void __launch_bounds__(1024)
    se_bfc1_kernel(const float* __restrict__ part, int chunks, int c, int cr,
                   const float* __restrict__ w2, const float* __restrict__ b2, int gate,
                   const float* __restrict__ s, const float* __restrict__ hidden,
                   float* __restrict__ dz) {
  extern __shared__ float hh[];  // [cr]
  const int nidx = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (gate == 1) {
    for (int j = threadIdx.x; j < cr; j += blockDim.x) hh[j] = hidden[(int64_t)nidx * cr + j];
    __syncthreads();
  }
  const int ch = blockIdx.y * kOutPerBlock + wid;
  if (ch >= c) return;
  const float* p = part + ((int64_t)nidx * c + ch) * chunks;
  float ds = 0.f;
  for (int k = lane; k < chunks; k += 64) ds += p[k];
  ds = mde::wave_sum(ds);
  float v;
  if (gate == 0) {
    const float sv = s[(int64_t)nidx * c + ch];
    v = ds * (sv * (1.f - sv));
  } else {
    const float* wr = w2 + (int64_t)ch * cr;
    float zz = 0.f;
    for (int j = lane; j < cr; j += 64) zz += wr[j] * hh[j];
    zz = mde::wave_sum(zz);
    if (b2) zz += b2[ch];
    v = (zz > -3.f && zz < 3.f) ? ds / 6.f : 0.f;
  }
  if (lane == 0) dz[(int64_t)nidx * c + ch] = v;
}

__global__ void __launch_bounds__(1024)
    se_bfc2_kernel(int c, int cr, const float* __restrict__ w2,
                   const float* __restrict__ hidden, const float* __restrict__ dz,
                   float* __restrict__ dh) {
  extern __shared__ float z[];  // [c]
  const int nidx = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int ch = threadIdx.x; ch < c; ch += blockDim.x) z[ch] = dz[(int64_t)nidx * c + ch];
  __syncthreads();
  const int j = blockIdx.y * kOutPerBlock + wid;
  if (j >= cr) return;
  float acc = 0.f;
  for (int ch = lane; ch < c; ch += 64) acc += w2[(int64_t)ch * cr + j] * z[ch];
  acc = mde::wave_sum(acc);
  if (lane == 0) dh[(int64_t)nidx * cr + j] = hidden[(int64_t)nidx * cr + j] > 0.f ? acc : 0.f;
}

// gw2[ch, j] = sum_n dz[n,ch] h[n,j];  gw1[j, ch] = sum_n dh[n,j] m[n,ch];
// gb2[ch] = sum_n dz[n,ch];  gb1[j] = sum_n dh[n,j]  (bias gradients nullable)
__device__ __forceinline__ void se_wgrad_body(int64_t t, int n, int c, int cr,
                                              const float* __restrict__ dz,
                                              const float* __restrict__ dh,
                                              const float* __restrict__ hidden,
                                              const float* __restrict__ mean,
                                              float* __restrict__ gw1, float* __restrict__ gw2,
                                              float* __restrict__ gb1, float* __restrict__ gb2) {
  const int64_t pairs = (int64_t)c * cr;
  if (gb2 && t < c) {
    float acc = 0.f;
    for (int k = 0; k < n; ++k) acc += dz[(int64_t)k * c + t];
    gb2[t] = acc;
  }
  if (gb1 && t < cr) {
    float acc = 0.f;
    for (int k = 0; k < n; ++k) acc += dh[(int64_t)k * cr + t];
    gb1[t] = acc;
  }
  if (t < pairs) {
    const int ch = (int)(t / cr), j = (int)(t % cr);
    float acc = 0.f;
    for (int k = 0; k < n; ++k)
      acc += dz[(int64_t)k * c + ch] * hidden[(int64_t)k * cr + j];
    gw2[t] = acc;  // row-major [c, cr]
  } else if (t < 2 * pairs) {
    const int64_t u = t - pairs;
    const int j = (int)(u / c), ch = (int)(u % c);
    float acc = 0.f;
    for (int k = 0; k < n; ++k)
      acc += dh[(int64_t)k * cr + j] * mean[(int64_t)k * c + ch];
    gw1[u] = acc;  // row-major [cr, c]
  }
}

// dm = W1^T dh (the squeeze-mean gradient) and the FC weight / bias gradients
// in one launch: blocks [0, n * ny) are se_bfc3 blocks (sample, 16-channel
// group), the rest grid-stride the se_wgrad pairs (1024 threads each).  Both
// only read dz / dh, so the roles are independent.  Was two launches.
__global__ void __launch_bounds__(1024)
    se_bfc3w_kernel(int n, int ny, int c, int cr, const float* __restrict__ w1,
                    const float* __restrict__ dz, const float* __restrict__ dh,
                    const float* __restrict__ hidden, const float* __restrict__ mean,
                    float* __restrict__ dm, float* __restrict__ gw1, float* __restrict__ gw2,
                    float* __restrict__ gb1, float* __restrict__ gb2) {
  extern __shared__ float hh[];  // [cr]
  const int nb3 = n * ny;
  if ((int)blockIdx.x >= nb3) {
    se_wgrad_body((int64_t)(blockIdx.x - nb3) * blockDim.x + threadIdx.x, n, c, cr, dz, dh, hidden,
                  mean, gw1, gw2, gb1, gb2);
    return;
  }
  const int nidx = blockIdx.x / ny, gy = blockIdx.x % ny;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int j = threadIdx.x; j < cr; j += blockDim.x) hh[j] = dh[(int64_t)nidx * cr + j];
  __syncthreads();
  const int ch = gy * kOutPerBlock + wid;
  if (ch >= c) return;
  float acc = 0.f;
  for (int j = lane; j < cr; j += 64) acc += w1[(int64_t)j * c + ch] * hh[j];
  acc = mde::wave_sum(acc);
  if (lane == 0) dm[(int64_t)nidx * c + ch] = acc;
}

// gx = g * s + dm / hw, written to gxa / gxb (either may be null).
__global__ void __launch_bounds__(256)
    se_apply_kernel(const float* __restrict__ g, int64_t ca, int64_t cb,
                    int64_t hw, int64_t planes, const float* __restrict__ s,
                    const float* __restrict__ dm, float inv_hw,
                    float* __restrict__ gxa, float* __restrict__ gxb) {
  const int64_t c = ca + cb;
  if ((hw & 3) == 0) {
    const int64_t hw4 = hw >> 2;
    const int64_t total = planes * hw4;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      const int64_t plane = t / hw4, i = (t - plane * hw4) << 2;
      const int64_t nidx = plane / c, ch = plane % c;
      float* dst = ch < ca ? (gxa ? gxa + (nidx * ca + ch) * hw : nullptr)
                           : (gxb ? gxb + (nidx * cb + ch - ca) * hw : nullptr);
      if (!dst) continue;
      const float sc = s[plane], add = dm[plane] * inv_hw;
      const float4 q = *reinterpret_cast<const float4*>(g + plane * hw + i);
      *reinterpret_cast<float4*>(dst + i) =
          make_float4(q.x * sc + add, q.y * sc + add, q.z * sc + add,
                      q.w * sc + add);
    }
  } else {
    const int64_t total = planes * hw;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      const int64_t plane = t / hw, i = t - plane * hw;
      const int64_t nidx = plane / c, ch = plane % c;
      float* dst = ch < ca ? (gxa ? gxa + (nidx * ca + ch) * hw : nullptr)
                           : (gxb ? gxb + (nidx * cb + ch - ca) * hw : nullptr);
      if (dst) dst[i] = g[t] * s[plane] + dm[plane] * inv_hw;
    }
  }
}

// ---- SE over BatchNorm + ReLU outputs (the guided-upsampling blocks: the
// two branches' last BN + ReLU, their concatenation and the SE layer in one
// op; modules.py:49-59,87-91).  With z = sc*y + sh (BN of the raw conv
// output y), u = relu(z), out = s * u:
//   du = s*g + dm/HW (dm: the gradient of the squeeze mean), dz = [z > 0] du,
//   and the BatchNorm backward needs S1 = sum dz, S2 = sum dz*(y - mean) per
//   channel.  Both are linear in per-(sample, channel) sums of one pass:
//   A = sum g*m, B = sum m, C = sum g*m*(y - mean), D = sum m*(y - mean),
//   E = sum g*u (= the SE gradient dot) with m = [z > 0].
template <typename T = float>
__global__ void __launch_bounds__(256)
    sebn_bwd_reduce_kernel(const T* __restrict__ g, const T* __restrict__ ya, int64_t ca,
                           const T* __restrict__ yb, int64_t cb, int64_t hw, int chunks,
                           const float* __restrict__ scale, const float* __restrict__ shift,
                           const float* __restrict__ mean, float* __restrict__ part_e,
                           float* __restrict__ part4) {
  __shared__ float red[4];
  const int64_t c = ca + cb;
  const int64_t plane = blockIdx.y;
  const int64_t nidx = plane / c, ch = plane % c;
  const T* y = plane_ptr(ya, ca, yb, cb, nidx, ch, hw);
  const T* gp = g + plane * hw;
  const float sc = scale[ch], sh = shift[ch], mu = mean[ch];
  const int64_t beg = (int64_t)blockIdx.x * kChunk;
  const int64_t end = beg + kChunk < hw ? beg + kChunk : hw;
  float A = 0.f, B = 0.f, C = 0.f, D = 0.f, E = 0.f;
  auto one = [&](float yv, float gv) {
    const float z = fmaf(yv, sc, sh);
    if (z > 0.f) {
      const float d = yv - mu;
      A += gv;
      B += 1.f;
      C += gv * d;
      D += d;
      E += gv * z;
    }
  };
  if ((hw & 3) == 0) {
    for (int64_t i = beg + 4 * threadIdx.x; i < end; i += 4 * 256) {
      const float4 v = mde::ld4(y + i);
      const float4 q = mde::ld4(gp + i);
      one(v.x, q.x); one(v.y, q.y); one(v.z, q.z); one(v.w, q.w);
    }
  } else {
    for (int64_t i = beg + threadIdx.x; i < end; i += 256) one(mde::ld1(y + i), mde::ld1(gp + i));
  }
  A = mde::block_sum256(A, red);
  B = mde::block_sum256(B, red);
  C = mde::block_sum256(C, red);
  D = mde::block_sum256(D, red);
  E = mde::block_sum256(E, red);
  if (threadIdx.x == 0) {
    const int64_t k = plane * chunks + blockIdx.x;
    part_e[k] = E;
    float* o = part4 + 4 * k;
    o[0] = A; o[1] = B; o[2] = C; o[3] = D;
  }
}

// Per channel (one block each): S1, S2 in double over (sample, chunk)
// partials -> the BN parameter gradients and the apply constants coef[ch] =
// (R, T) with gy = m (P g + Q) + R + T (y - mean), P = sc s, Q = sc dm / HW
// (per sample).  Fixed per-thread order and a fixed tree: deterministic.
// One launch for the SE-over-BN backward's tail (was three: se_bfc3, se_wgrad,
// the combine): blocks [0, c) are per-channel combine blocks that first form
// their channel's squeeze-mean gradients dm[:, ch] = W1[:, ch] . dh[n, :]
// (wave per sample, the se_bfc3 summation order) into LDS and dm; blocks
// [c, c + wg) run the FC weight / bias gradients.
constexpr int kMaxSeN = 256;  // samples the combine blocks hold dm for in LDS at once

__global__ void __launch_bounds__(256)
    sebn_bwd_combine_kernel(const float* __restrict__ part4, int chunks, int64_t n, int64_t c,
                            int64_t hw, const float* __restrict__ s, float* __restrict__ dm,
                            const float* __restrict__ scale, const float* __restrict__ invstd,
                            int training, float* __restrict__ ggamma, float* __restrict__ gbeta,
                            float* __restrict__ coef, int cr, const float* __restrict__ w1,
                            const float* __restrict__ dz, const float* __restrict__ dh,
                            const float* __restrict__ hidden, const float* __restrict__ mean,
                            float* __restrict__ gw1, float* __restrict__ gw2) {
  __shared__ double red[2][4];
  __shared__ float dms[kMaxSeN];
  if ((int64_t)blockIdx.x >= c) {
    se_wgrad_body((int64_t)(blockIdx.x - c) * blockDim.x + threadIdx.x, (int)n, (int)c, cr, dz, dh,
                  hidden, mean, gw1, gw2, nullptr, nullptr);
    return;
  }
  const int64_t ch = blockIdx.x;
  const double inv_hw = 1.0 / (double)hw;
  double s1 = 0.0, s2 = 0.0;
  // samples in groups of kMaxSeN (one group, the whole batch, up to 256)
  for (int64_t n0 = 0; n0 < n; n0 += kMaxSeN) {
    const int64_t nb = n - n0 < kMaxSeN ? n - n0 : kMaxSeN;
    if (n0 > 0) __syncthreads();  // the previous group's dms readers are done
    {
      const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
      for (int64_t k = wid; k < nb; k += 4) {
        const int64_t nn = n0 + k;
        float acc = 0.f;
        for (int j = lane; j < cr; j += 64) acc += w1[(int64_t)j * c + ch] * dh[nn * cr + j];
        acc = mde::wave_sum(acc);
        if (lane == 0) {
          dms[k] = acc;
          dm[nn * c + ch] = acc;
        }
      }
    }
    __syncthreads();
    for (int64_t i = threadIdx.x; i < nb * chunks; i += 256) {
      const int64_t plane = (n0 + i / chunks) * c + ch;
      const float* p = part4 + 4 * (plane * chunks + i % chunks);
      const double sv = s[plane], q = (double)dms[i / chunks] * inv_hw;
      s1 += sv * (double)p[0] + q * (double)p[1];
      s2 += sv * (double)p[2] + q * (double)p[3];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = s1;
    red[1][wid] = s2;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  s1 = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  s2 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  const double is = invstd[ch], sc = scale[ch], cnt = (double)n * (double)hw;
  if (ggamma) ggamma[ch] = (float)(is * s2);
  if (gbeta) gbeta[ch] = (float)s1;
  coef[2 * ch] = training ? (float)(-sc * s1 / cnt) : 0.f;
  coef[2 * ch + 1] = training ? (float)(-sc * is * is * s2 / cnt) : 0.f;
}

template <typename T = float>
__global__ void __launch_bounds__(256)
    sebn_bwd_apply_kernel(const T* __restrict__ g, const T* __restrict__ ya, int64_t ca,
                          const T* __restrict__ yb, int64_t cb, int64_t hw, int64_t planes,
                          const float* __restrict__ s, const float* __restrict__ dm, float inv_hw,
                          const float* __restrict__ scale, const float* __restrict__ shift,
                          const float* __restrict__ mean, const float* __restrict__ coef,
                          T* __restrict__ gya, T* __restrict__ gyb) {
  const int64_t c = ca + cb;
  auto one = [](float yv, float gv, float sc, float sh, float P, float Q, float R, float Tc,
                float mu) {
    const float z = fmaf(yv, sc, sh);
    return (z > 0.f ? fmaf(P, gv, Q) : 0.f) + fmaf(Tc, yv - mu, R);
  };
  if ((hw & 3) == 0) {
    const int64_t hw4 = hw >> 2;
    const int64_t total = planes * hw4;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      const int64_t plane = t / hw4, i = (t - plane * hw4) << 2;
      const int64_t nidx = plane / c, ch = plane % c;
      const T* y = plane_ptr(ya, ca, yb, cb, nidx, ch, hw);
      T* dst = ch < ca ? gya + (nidx * ca + ch) * hw : gyb + (nidx * cb + ch - ca) * hw;
      const float sc = scale[ch], sh = shift[ch], mu = mean[ch];
      const float P = sc * s[plane], Q = sc * dm[plane] * inv_hw;
      const float R = coef[2 * ch], Tc = coef[2 * ch + 1];
      const float4 v = mde::ld4(y + i);
      const float4 q = mde::ld4(g + plane * hw + i);
      mde::st4(dst + i, make_float4(one(v.x, q.x, sc, sh, P, Q, R, Tc, mu),
                                    one(v.y, q.y, sc, sh, P, Q, R, Tc, mu),
                                    one(v.z, q.z, sc, sh, P, Q, R, Tc, mu),
                                    one(v.w, q.w, sc, sh, P, Q, R, Tc, mu)));
    }
  } else {
    const int64_t total = planes * hw;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
      const int64_t plane = t / hw, i = t - plane * hw;
      const int64_t nidx = plane / c, ch = plane % c;
      const T* y = plane_ptr(ya, ca, yb, cb, nidx, ch, hw);
      T* dst = ch < ca ? gya + (nidx * ca + ch) * hw : gyb + (nidx * cb + ch - ca) * hw;
      const float sc = scale[ch];
      mde::st1(dst + i, one(mde::ld1(y + i), mde::ld1(g + t), sc, shift[ch], sc * s[plane],
                            sc * dm[plane] * inv_hw, coef[2 * ch], coef[2 * ch + 1], mean[ch]));
    }
  }
}

inline int stream_grid(int64_t work) {
  const int64_t b = mde::cdiv(work, 256);
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

struct SeWs;
int se_bfc(const SeWs& ws, int chunks, int64_t n, int64_t c, int64_t cr, const float* w1,
           const float* w2, const float* b2, int gate, const float* s, const float* hidden,
           const float* mean, float* gw1, float* gw2, float* gb1, float* gb2, hipStream_t st,
           bool tail = false);

struct SeWs {
  float* part;
  float* dz;
  float* dh;
  float* dm;
  float* part4;
  float* coef;
};

inline int64_t se_chunks(int64_t hw) { return mde::cdiv(hw, kChunk); }

inline size_t round16(size_t b) { return (b + 15) & ~size_t(15); }

SeWs se_carve(void* ws, int64_t n, int64_t c, int64_t cr, int64_t hw) {
  char* p = (char*)ws;
  SeWs r;
  r.part = (float*)p;
  p += round16(sizeof(float) * n * c * se_chunks(hw));
  r.dz = (float*)p;
  p += round16(sizeof(float) * n * c);
  r.dh = (float*)p;
  p += round16(sizeof(float) * n * cr);
  r.dm = (float*)p;
  p += round16(sizeof(float) * n * c);
  r.part4 = (float*)p;  // SE-over-BN backward only (mde_se_bn_workspace)
  p += round16(sizeof(float) * 4 * n * c * se_chunks(hw));
  r.coef = (float*)p;
  return r;
}

// The per-sample FC backward + weight gradients: three launches (dz, dh,
// then dm with the weight gradients), two when `tail` (the SE-over-BN combine
// launch takes dm and the weight gradients).  (A one-block fused variant was
// measured at 156 us per SE layer vs 42 us for four launches: a single block
// serialises the n*c partial-sum reductions.)
int se_bfc(const SeWs& ws, int chunks, int64_t n, int64_t c, int64_t cr, const float* w1,
           const float* w2, const float* b2, int gate, const float* s, const float* hidden,
           const float* mean, float* gw1, float* gw2, float* gb1, float* gb2, hipStream_t st,
           bool tail) {
  MDE_LAUNCH(mde::K_SE_BWD_FC, 4.0 * (c * cr + 3.0 * n * c), st, se_bfc1_kernel,
             dim3((unsigned)n, (unsigned)mde::cdiv(c, kOutPerBlock)), dim3(1024),
             sizeof(float) * cr, ws.part, chunks, (int)c, (int)cr, w2, b2, gate, s, hidden,
             ws.dz);
  MDE_LAUNCH(mde::K_SE_BWD_FC, 4.0 * (c * cr + n * (c + 2.0 * cr)), st, se_bfc2_kernel,
             dim3((unsigned)n, (unsigned)mde::cdiv(cr, kOutPerBlock)), dim3(1024),
             sizeof(float) * c, (int)c, (int)cr, w2, hidden, ws.dz, ws.dh);
  if (tail) return MDE_OK;  // the SE-over-BN combine launch does dm and the weight gradients
  const int ny = (int)mde::cdiv(c, kOutPerBlock);
  MDE_LAUNCH(mde::K_SE_BWD_FC, 4.0 * (3.0 * c * cr + n * (3.0 * c + 3.0 * cr)), st,
             se_bfc3w_kernel,
             dim3((unsigned)(n * ny + mde::cdiv(2 * c * cr, 1024))), dim3(1024),
             sizeof(float) * cr, (int)n, ny, (int)c, (int)cr, w1, ws.dz, ws.dh, hidden, mean,
             ws.dm, gw1, gw2, gb1, gb2);
  return MDE_OK;
}

}  // namespace

extern "C" {

size_t mde_se_workspace(int64_t n, int64_t c, int64_t cr, int64_t h,
                        int64_t w) {
  const int64_t hw = h * w;
  return round16(sizeof(float) * n * c * se_chunks(hw)) +
         round16(sizeof(float) * n * c) + round16(sizeof(float) * n * cr) +
         round16(sizeof(float) * n * c);
}

int mde_se_gate_fwd(const void* xa, int64_t ca, const void* xb, int64_t cb,
                    const float* w1, const float* b1, const float* w2, const float* b2,
                    int64_t cr, int gate, void* out, float* s, float* hidden, float* mean,
                    int64_t n, int64_t h, int64_t w, void* workspace, int dtype,
                    void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  const int64_t c = ca + cb, hw = h * w;
  if (gate < 0 || gate > 1) return MDE_ERR_INVALID_ARG;
  if (!xa || ca <= 0 || cb < 0 || (cb > 0 && !xb) || !w1 || !w2 || cr <= 0 ||
      !out || !s || !hidden || !mean || n <= 0 || hw <= 0 || !workspace ||
      c > 4096 || cr > 4096 || n > 65535)
    return MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  SeWs ws = se_carve(workspace, n, c, cr, hw);
  const int chunks = (int)se_chunks(hw);
  const double big = 4.0 * n * c * (double)hw;
  MDE_LAUNCH(mde::K_SE_SQUEEZE, big, st, (se_partial_kernel<kSum, float>),
             dim3(chunks, (unsigned)(n * c)), dim3(256), 0, nullptr,
             (const float*)xa, ca, (const float*)xb, cb, hw, chunks, ws.part);
  MDE_LAUNCH(mde::K_SE_FC, 4.0 * (c * cr + 2.0 * n * c), st, se_fc1_kernel,
             dim3((unsigned)n, (unsigned)mde::cdiv(cr, kOutPerBlock)), dim3(1024),
             sizeof(float) * c, ws.part, chunks, (int)c, (int)cr, 1.f / (float)hw, w1, b1,
             hidden, mean);
  MDE_LAUNCH(mde::K_SE_FC, 4.0 * (c * cr + 2.0 * n * c), st, se_fc2_kernel,
             dim3((unsigned)n, (unsigned)mde::cdiv(c, kOutPerBlock)), dim3(1024),
             sizeof(float) * cr, (int)c, (int)cr, w2, b2, gate, hidden, s);
  MDE_LAUNCH(mde::K_SE_SCALE, 2.0 * big, st, (se_scale_kernel<false, float>),
             dim3(stream_grid(n * c * hw / 4)), dim3(256), 0,
             (const float*)xa, ca, (const float*)xb, cb, hw, n * c, s,
             (float*)out);
  return MDE_OK;
}

int mde_se_gate_bwd(const void* gout, const void* xa, int64_t ca, const void* xb,
                    int64_t cb, const float* w1, const float* w2, const float* b2,
                    int64_t cr, int gate, const float* s, const float* hidden,
                    const float* mean, void* gxa, void* gxb, float* gw1, float* gb1,
                    float* gw2, float* gb2, int64_t n, int64_t h, int64_t w,
                    void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  const int64_t c = ca + cb, hw = h * w;
  if (gate < 0 || gate > 1) return MDE_ERR_INVALID_ARG;
  if (!gout || !xa || ca <= 0 || cb < 0 || (cb > 0 && !xb) || !w1 || !w2 ||
      cr <= 0 || !s || !hidden || !mean || !gw1 || !gw2 || n <= 0 ||
      hw <= 0 || !workspace || c > 4096 || cr > 4096 || n > 65535)
    return MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  SeWs ws = se_carve(workspace, n, c, cr, hw);
  const int chunks = (int)se_chunks(hw);
  const double big = 4.0 * n * c * (double)hw;
  MDE_LAUNCH(mde::K_SE_BWD_DOT, 2.0 * big, st, (se_partial_kernel<kDot, float>),
             dim3(chunks, (unsigned)(n * c)), dim3(256), 0,
             (const float*)gout, (const float*)xa, ca, (const float*)xb, cb,
             hw, chunks, ws.part);
  const int fcs = se_bfc(ws, chunks, n, c, cr, w1, w2, b2, gate, s, hidden, mean, gw1, gw2, gb1,
                         gb2, st);
  if (fcs) return fcs;
  if (gxa || gxb) {
    MDE_LAUNCH(mde::K_SE_BWD_APPLY, 2.0 * big, st, se_apply_kernel,
               dim3(stream_grid(n * c * hw / 4)), dim3(256), 0,
               (const float*)gout, ca, cb, hw, n * c, s, ws.dm,
               1.f / (float)hw, (float*)gxa, (float*)gxb);
  }
  return MDE_OK;
}

int mde_se_fwd(const void* xa, int64_t ca, const void* xb, int64_t cb,
               const float* w1, const float* w2, int64_t cr, void* out,
               float* s, float* hidden, float* mean, int64_t n, int64_t h,
               int64_t w, void* workspace, int dtype, void* stream) {
  return mde_se_gate_fwd(xa, ca, xb, cb, w1, nullptr, w2, nullptr, cr, 0, out, s, hidden,
                         mean, n, h, w, workspace, dtype, stream);
}

int mde_se_bwd(const void* gout, const void* xa, int64_t ca, const void* xb,
               int64_t cb, const float* w1, const float* w2, int64_t cr,
               const float* s, const float* hidden, const float* mean,
               void* gxa, void* gxb, float* gw1, float* gw2, int64_t n,
               int64_t h, int64_t w, void* workspace, int dtype, void* stream) {
  return mde_se_gate_bwd(gout, xa, ca, xb, cb, w1, w2, nullptr, cr, 0, s, hidden, mean, gxa,
                         gxb, gw1, nullptr, gw2, nullptr, n, h, w, workspace, dtype, stream);
}

size_t mde_se_bn_workspace(int64_t n, int64_t c, int64_t cr, int64_t h, int64_t w) {
  return mde_se_workspace(n, c, cr, h, w) + round16(sizeof(float) * 4 * n * c * se_chunks(h * w)) +
         round16(sizeof(float) * 2 * c);
}

}  // extern "C"

// mde_se_bn_fwd / _bwd on storage type T (fp32, or bf16 under autocast: y, out,
// gout, gy in T; coefficients, the SE vector, FC weights and sums fp32).
template <typename T>
static int se_bn_fwd_t(const void* ya, int64_t ca, const void* yb, int64_t cb, const float* scale,
                       const float* shift, const float* w1, const float* w2, int64_t cr, void* out,
                       float* s, float* hidden, float* mean, int64_t n, int64_t hw,
                       void* workspace, hipStream_t st) {
  const int64_t c = ca + cb;
  SeWs ws = se_carve(workspace, n, c, cr, hw);
  const int chunks = (int)se_chunks(hw);
  const double big = (double)sizeof(T) * n * c * (double)hw;
  MDE_LAUNCH(mde::K_SE_SQUEEZE, big, st, (se_partial_kernel<kBnRelu, T>),
             dim3(chunks, (unsigned)(n * c)), dim3(256), 0, nullptr, (const T*)ya, ca,
             (const T*)yb, cb, hw, chunks, ws.part, scale, shift);
  MDE_LAUNCH(mde::K_SE_FC, 4.0 * (c * cr + 2.0 * n * c), st, se_fc1_kernel,
             dim3((unsigned)n, (unsigned)mde::cdiv(cr, kOutPerBlock)), dim3(1024),
             sizeof(float) * c, ws.part, chunks, (int)c, (int)cr, 1.f / (float)hw, w1, nullptr,
             hidden, mean);
  MDE_LAUNCH(mde::K_SE_FC, 4.0 * (c * cr + 2.0 * n * c), st, se_fc2_kernel,
             dim3((unsigned)n, (unsigned)mde::cdiv(c, kOutPerBlock)), dim3(1024),
             sizeof(float) * cr, (int)c, (int)cr, w2, nullptr, 0, hidden, s);
  MDE_LAUNCH(mde::K_SE_SCALE, 2.0 * big, st, (se_scale_kernel<true, T>),
             dim3(stream_grid(n * c * hw / 4)), dim3(256), 0, (const T*)ya, ca, (const T*)yb, cb,
             hw, n * c, s, (T*)out, scale, shift);
  return MDE_OK;
}

template <typename T>
static int se_bn_bwd_t(const void* gout, const void* ya, int64_t ca, const void* yb, int64_t cb,
                       const float* scale, const float* shift, const float* bn_mean,
                       const float* bn_invstd, int training, const float* w1, const float* w2,
                       int64_t cr, const float* s, const float* hidden, const float* mean,
                       void* gya, void* gyb, float* ggamma, float* gbeta, float* gw1, float* gw2,
                       int64_t n, int64_t hw, void* workspace, hipStream_t st) {
  const int64_t c = ca + cb;
  SeWs ws = se_carve(workspace, n, c, cr, hw);
  const int chunks = (int)se_chunks(hw);
  const double big = (double)sizeof(T) * n * c * (double)hw;
  MDE_LAUNCH(mde::K_SE_BWD_DOT, 2.0 * big, st, sebn_bwd_reduce_kernel<T>,
             dim3(chunks, (unsigned)(n * c)), dim3(256), 0, (const T*)gout, (const T*)ya, ca,
             (const T*)yb, cb, hw, chunks, scale, shift, bn_mean, ws.part, ws.part4);
  const int fcs = se_bfc(ws, chunks, n, c, cr, w1, w2, nullptr, 0, s, hidden, mean, gw1, gw2,
                         nullptr, nullptr, st, true);
  if (fcs) return fcs;
  MDE_LAUNCH(mde::K_SE_BWD_FC, 16.0 * n * c * chunks + 4.0 * (3.0 * c * cr + n * (3.0 * c + 3.0 * cr)),
             st, sebn_bwd_combine_kernel,
             dim3((unsigned)(c + mde::cdiv(2 * c * cr, 256))), dim3(256), 0, ws.part4, chunks, n, c,
             hw, s, ws.dm, scale, bn_invstd, training, ggamma, gbeta, ws.coef, (int)cr, w1, ws.dz,
             ws.dh, hidden, mean, gw1, gw2);
  MDE_LAUNCH(mde::K_SE_BWD_APPLY, 3.0 * big, st, sebn_bwd_apply_kernel<T>,
             dim3(stream_grid(n * c * hw / 4)), dim3(256), 0, (const T*)gout, (const T*)ya, ca,
             (const T*)yb, cb, hw, n * c, s, ws.dm, 1.f / (float)hw, scale, shift, bn_mean,
             ws.coef, (T*)gya, (T*)gyb);
  return MDE_OK;
}

extern "C" {

// SELayer(cat([relu(bn_a(ya)), relu(bn_b(yb))])) from the BatchNorms' raw
// inputs: scale / shift [ca + cb] are the two BNs' per-channel coefficients
// (mde_batchnorm_fwd_coef*), concatenated.  The squeeze reads y once, the
// scale pass writes out = s * relu(scale * y + shift); the BN + ReLU outputs
// and their concatenation are never materialised.
int mde_se_bn_fwd(const void* ya, int64_t ca, const void* yb, int64_t cb, const float* scale,
                  const float* shift, const float* w1, const float* w2, int64_t cr, void* out,
                  float* s, float* hidden, float* mean, int64_t n, int64_t h, int64_t w,
                  void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  const int64_t c = ca + cb, hw = h * w;
  if (!ya || ca <= 0 || cb < 0 || (cb > 0 && !yb) || !scale || !shift || !w1 || !w2 ||
      cr <= 0 || !out || !s || !hidden || !mean || n <= 0 || hw <= 0 || !workspace ||
      c > 4096 || cr > 4096 || n > 65535 || n * c > 65535)
    return MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  return dtype == MDE_BF16
             ? se_bn_fwd_t<mde::bf16>(ya, ca, yb, cb, scale, shift, w1, w2, cr, out, s, hidden,
                                      mean, n, hw, workspace, st)
             : se_bn_fwd_t<float>(ya, ca, yb, cb, scale, shift, w1, w2, cr, out, s, hidden, mean,
                                  n, hw, workspace, st);
}

// Backward of mde_se_bn_fwd through the SE layer, the ReLUs and both
// BatchNorms (training: batch statistics, save_mean / save_invstd of the raw
// input; eval: running statistics, no mean / variance terms): one reduction
// pass over (gout, y), the per-sample FC backward, a per-channel combine in
// double, and one apply pass writing gya / gyb = d/dy.  ggamma / gbeta are
// concatenated [ca + cb] like scale / shift.
int mde_se_bn_bwd(const void* gout, const void* ya, int64_t ca, const void* yb, int64_t cb,
                  const float* scale, const float* shift, const float* bn_mean,
                  const float* bn_invstd, int training, const float* w1, const float* w2,
                  int64_t cr, const float* s, const float* hidden, const float* mean, void* gya,
                  void* gyb, float* ggamma, float* gbeta, float* gw1, float* gw2, int64_t n,
                  int64_t h, int64_t w, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  const int64_t c = ca + cb, hw = h * w;
  if (!gout || !ya || ca <= 0 || cb < 0 || (cb > 0 && (!yb || !gyb)) || !gya || !scale ||
      !shift || !bn_mean || !bn_invstd || !w1 || !w2 || cr <= 0 || !s || !hidden || !mean ||
      !gw1 || !gw2 || n <= 0 || hw <= 0 || !workspace || c > 4096 || cr > 4096 ||
      n > 65535 || n * c > 65535)
    return MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  return dtype == MDE_BF16
             ? se_bn_bwd_t<mde::bf16>(gout, ya, ca, yb, cb, scale, shift, bn_mean, bn_invstd,
                                      training, w1, w2, cr, s, hidden, mean, gya, gyb, ggamma,
                                      gbeta, gw1, gw2, n, hw, workspace, st)
             : se_bn_bwd_t<float>(gout, ya, ca, yb, cb, scale, shift, bn_mean, bn_invstd,
                                  training, w1, w2, cr, s, hidden, mean, gya, gyb, ggamma, gbeta,
                                  gw1, gw2, n, hw, workspace, st);
}

}  // extern "C"
