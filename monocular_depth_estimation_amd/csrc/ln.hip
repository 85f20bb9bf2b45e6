// LayerNorm over the channel axis of token-major [rows, C] fp32 tensors and
// the NCHW <-> token-major transposes around it: the NewCRF decoder's
// norm1 / norm2 / norm_crf (src/newcrf_layers.py:197,212,233,419-434 —
// nn.LayerNorm(C), eps 1e-5) and the x.flatten(2).transpose(1, 2) /
// permute(0, 3, 1, 2).contiguous() / v.permute(0, 2, 3, 1) copies
// (:230,425-434).
//
// LayerNorm: one wave per token row, C/64 values per lane held in registers
// (float2/float4 vector loads), two-pass mean/variance from registers, so a
// row is read once.  Backward recomputes x_hat from the saved mean/rstd and
// writes per-block partial sums of the gamma/beta gradients (each block owns
// a fixed range of rows); a column kernel sums them in a fixed order —
// deterministic, no atomics.
// Transpose: 64x64 tiles through LDS (padded rows), coalesced on both sides.
// Algorithmic HBM bytes: LN fwd 8 per element (+8 per row), LN bwd 12 per
// element, transpose 8 per element.

#include <cstdlib>

#include "common.h"

namespace mde {
namespace {

constexpr int64_t kMaxBlocksBwd = 1024;

// backward blocks: about 1024, each owning a contiguous range of >= 4 rows
// (one per wave), so small token counts still fill the chip
int64_t bwd_blocks(int64_t rows) {
  const int64_t b = cdiv(rows, 4);
  return b < kMaxBlocksBwd ? b : kMaxBlocksBwd;
}

template <int VPL>
struct RowIO {
  // lane's VPL values: float4 chunks at 4*lane + 256*j (VPL % 4 == 0), a float2
  // at 2*lane (VPL == 2), else scalars at lane + 64*j.
  __device__ static void load(const float* p, float* v) {
    const int lane = threadIdx.x & 63;
    if constexpr (VPL == 2) {
      const float2 a = reinterpret_cast<const float2*>(p)[lane];
      v[0] = a.x;
      v[1] = a.y;
    } else if constexpr (VPL % 4 != 0) {
#pragma unroll
      for (int j = 0; j < VPL; ++j) v[j] = p[lane + 64 * j];
    } else {
#pragma unroll
      for (int j = 0; j < VPL / 4; ++j) {
        const float4 a = reinterpret_cast<const float4*>(p)[lane + 64 * j];
        v[4 * j] = a.x;
        v[4 * j + 1] = a.y;
        v[4 * j + 2] = a.z;
        v[4 * j + 3] = a.w;
      }
    }
  }
  __device__ static void store(float* p, const float* v) {
    const int lane = threadIdx.x & 63;
    if constexpr (VPL == 2) {
      reinterpret_cast<float2*>(p)[lane] = make_float2(v[0], v[1]);
    } else if constexpr (VPL % 4 != 0) {
#pragma unroll
      for (int j = 0; j < VPL; ++j) p[lane + 64 * j] = v[j];
    } else {
#pragma unroll
      for (int j = 0; j < VPL / 4; ++j)
        reinterpret_cast<float4*>(p)[lane + 64 * j] =
            make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
    }
  }
  // channel index of value i of this lane
  __device__ static int chan(int i) {
    const int lane = threadIdx.x & 63;
    if constexpr (VPL == 2) return 2 * lane + i;
    if constexpr (VPL % 4 != 0) return lane + 64 * i;
    return 4 * (lane + 64 * (i / 4)) + (i & 3);
  }
};

// ADD: the residual add in front of the norm (CRFBlock's `x + attn(..)` /
// `x + mlp(..)` followed by the next LayerNorm, newcrf_layers.py:229-257):
// s = x + r is written AND normalised from registers (one pass instead of an
// add pass and a norm pass).
template <int VPL, bool ADD = false>
__global__ void __launch_bounds__(256)
    ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                  const float* __restrict__ beta, float* __restrict__ y,
                  float* __restrict__ mean_out, float* __restrict__ rstd_out, int64_t rows,
                  float eps, const float* __restrict__ r = nullptr, float* __restrict__ sum = nullptr) {
  constexpr int C = 64 * VPL;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[VPL], g[VPL], b[VPL];
  RowIO<VPL>::load(x + row * C, v);
  if constexpr (ADD) {
    float a[VPL];
    RowIO<VPL>::load(r + row * C, a);
#pragma unroll
    for (int i = 0; i < VPL; ++i) v[i] += a[i];
    RowIO<VPL>::store(sum + row * C, v);
  }
  RowIO<VPL>::load(gamma, g);
  RowIO<VPL>::load(beta, b);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += v[i];
  const float mu = wave_sum(s) * (1.f / C);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const float d = v[i] - mu;
    q = fmaf(d, d, q);
  }
  const float rs = rsqrtf(wave_sum(q) * (1.f / C) + eps);
#pragma unroll
  for (int i = 0; i < VPL; ++i) v[i] = fmaf((v[i] - mu) * rs, g[i], b[i]);
  RowIO<VPL>::store(y + row * C, v);
  if ((threadIdx.x & 63) == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rs;
  }
}

// gx = rstd * (gy*g - mean(gy*g) - x_hat * mean(gy*g*x_hat)); partial
// gamma/beta gradients of this block's rows into part[blk][2][C].
// RES: + gres (the gradient the normalised sum's residual branch carries,
// added in the epilogue instead of by a separate accumulation pass).
template <int VPL, bool RES = false>
__global__ void __launch_bounds__(256)
    ln_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                  const float* __restrict__ gamma, const float* __restrict__ mean,
                  const float* __restrict__ rstd, float* __restrict__ gx,
                  float* __restrict__ part, int64_t rows, int64_t rows_per_blk,
                  const float* __restrict__ gres = nullptr) {
  constexpr int C = 64 * VPL;
  __shared__ float red[4][2][C];
  const int wid = threadIdx.x >> 6;
  float g[VPL], pg[VPL], pb[VPL];
  RowIO<VPL>::load(gamma, g);
#pragma unroll
  for (int i = 0; i < VPL; ++i) pg[i] = pb[i] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = r0 + rows_per_blk < rows ? r0 + rows_per_blk : rows;
  for (int64_t row = r0 + wid; row < r1; row += 4) {
    float v[VPL], d[VPL];
    RowIO<VPL>::load(x + row * C, v);
    RowIO<VPL>::load(gy + row * C, d);
    const float mu = mean[row], rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      v[i] = (v[i] - mu) * rs;  // x_hat
      pg[i] = fmaf(d[i], v[i], pg[i]);
      pb[i] += d[i];
      const float dg = d[i] * g[i];
      s1 += dg;
      s2 = fmaf(dg, v[i], s2);
    }
    s1 = wave_sum(s1) * (1.f / C);
    s2 = wave_sum(s2) * (1.f / C);
#pragma unroll
    for (int i = 0; i < VPL; ++i) d[i] = rs * (d[i] * g[i] - s1 - v[i] * s2);
    if constexpr (RES) {
      // a separate rounded add (no FMA contraction with the product above):
      // bitwise the add autograd's accumulation did
#pragma clang fp contract(off)
      float a[VPL];
      RowIO<VPL>::load(gres + row * C, a);
#pragma unroll
      for (int i = 0; i < VPL; ++i) d[i] = a[i] + d[i];
    }
    RowIO<VPL>::store(gx + row * C, d);
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int ch = RowIO<VPL>::chan(i);
    red[wid][0][ch] = pg[i];
    red[wid][1][ch] = pb[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) {
    const int k = i / C, ch = i - k * C;
    part[((int64_t)blockIdx.x * 2 + k) * C + ch] =
        (red[0][k][ch] + red[1][k][ch]) + (red[2][k][ch] + red[3][k][ch]);
  }
}

// ggamma[ch] / gbeta[ch] = sum over blocks of part: 64 columns per block of
// 16 waves, wave w sums blocks w, w+16, ... (8 loads in flight); the 16 wave
// sums combine in a fixed order.
__global__ void __launch_bounds__(1024)
    ln_wreduce_kernel(const float* __restrict__ part, float* __restrict__ ggamma,
                      float* __restrict__ gbeta, int64_t nblk, int c) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;  // column of the [2][c] partial rows
  float s = 0.f;
  if (i < 2 * c) {
#pragma unroll 8
    for (int64_t b = wid; b < nblk; b += 16) s += part[b * 2 * c + i];
  }
  red[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && i < 2 * c) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    if (i < c) ggamma[i] = t;
    else gbeta[i - c] = t;
  }
}

// y[b][j][i] = x[b][i][j], x: [batch, m, n].
__global__ void __launch_bounds__(256)
    transpose_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t m, int64_t n) {
  __shared__ float t[64][65];
  const int64_t b = blockIdx.z;
  const int64_t i0 = (int64_t)blockIdx.y * 64, j0 = (int64_t)blockIdx.x * 64;
  const float* xp = x + b * m * n;
  float* yp = y + b * m * n;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int64_t i = i0 + r, j = j0 + tx;
    if (i < m && j < n) t[r][tx] = xp[i * n + j];
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int64_t j = j0 + r, i = i0 + tx;
    if (i < m && j < n) yp[j * m + i] = t[tx][r];
  }
}

// The same transpose with 16-byte global accesses (m % 4 == 0, n % 4 == 0:
// every NewCRF token / channel count): a thread moves 4 float4 in and 4
// float4 out per 64 x 64 tile (the scalar kernel: 16 + 16 four-byte
// accesses).  LDS rows of 68 floats: the float4 stores are 16-byte aligned,
// the column reads at most 2-way conflicted.
__global__ void __launch_bounds__(256)
    transpose4_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t m, int64_t n) {
  constexpr int P = 68;
  __shared__ __attribute__((aligned(16))) float t[64 * P];
  const int64_t b = blockIdx.z;
  const int64_t i0 = (int64_t)blockIdx.y * 64, j0 = (int64_t)blockIdx.x * 64;
  const float* xp = x + b * m * n;
  float* yp = y + b * m * n;
  const int c4 = threadIdx.x & 15, rr = threadIdx.x >> 4;  // float4 column, row within 16
  float4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // all four loads in flight
    const int64_t i = i0 + rr + 16 * k, j = j0 + 4 * c4;
    v[k] = i < m && j < n ? *reinterpret_cast<const float4*>(xp + i * n + j)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) *reinterpret_cast<float4*>(t + (rr + 16 * k) * P + 4 * c4) = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int jr = rr + 16 * k;  // y row j0 + jr, columns i0 + 4 c4 .. + 3
    const int64_t j = j0 + jr, i = i0 + 4 * c4;
    const float4 o = make_float4(t[(4 * c4) * P + jr], t[(4 * c4 + 1) * P + jr],
                                 t[(4 * c4 + 2) * P + jr], t[(4 * c4 + 3) * P + jr]);
    if (i < m && j < n) *reinterpret_cast<float4*>(yp + j * m + i) = o;
  }
}

template <int VPL>
int ln_fwd_launch(const float* x, const float* g, const float* b, float* y, float* mu,
                  float* rs, int64_t rows, float eps, hipStream_t st, const float* r = nullptr,
                  float* sum = nullptr) {
  if (r) {
    const double bytes = 16.0 * rows * 64 * VPL + 8.0 * rows;  // x, r read; s, y written
    MDE_LAUNCH(K_LN_FWD, bytes, st, (ln_fwd_kernel<VPL, true>), dim3((unsigned)cdiv(rows, 4)),
               dim3(256), 0, x, g, b, y, mu, rs, rows, eps, r, sum);
    return 0;
  }
  const double bytes = 8.0 * rows * 64 * VPL + 8.0 * rows;
  MDE_LAUNCH(K_LN_FWD, bytes, st, ln_fwd_kernel<VPL>, dim3((unsigned)cdiv(rows, 4)), dim3(256),
             0, x, g, b, y, mu, rs, rows, eps, nullptr, nullptr);
  return 0;
}

template <int VPL>
int ln_bwd_launch(const float* gy, const float* x, const float* g, const float* mu,
                  const float* rs, float* gx, float* gg, float* gb, float* part, int64_t rows,
                  hipStream_t st, const float* gres = nullptr) {
  const int64_t nblk = bwd_blocks(rows);
  if (gres) {
    const double bytes = 16.0 * rows * 64 * VPL + 8.0 * rows;  // + the residual gradient read
    MDE_LAUNCH(K_LN_BWD, bytes, st, (ln_bwd_kernel<VPL, true>), dim3((unsigned)nblk), dim3(256),
               0, gy, x, g, mu, rs, gx, part, rows, cdiv(rows, nblk), gres);
  } else {
    const double bytes = 12.0 * rows * 64 * VPL + 8.0 * rows;
    MDE_LAUNCH(K_LN_BWD, bytes, st, ln_bwd_kernel<VPL>, dim3((unsigned)nblk), dim3(256), 0, gy, x,
               g, mu, rs, gx, part, rows, cdiv(rows, nblk), nullptr);
  }
  const int c = 64 * VPL;
  MDE_LAUNCH(K_LN_WREDUCE, 8.0 * nblk * c, st, ln_wreduce_kernel, dim3((unsigned)cdiv(2 * c, 64)),
             dim3(1024), 0, part, gg, gb, nblk, c);
  return 0;
}

bool ln_ok(int64_t rows, int64_t c) {
  return rows > 0 && rows <= (int64_t)4 * 0x7fffffff && c % 64 == 0 && c >= 64 && c <= 1024;
}

}  // namespace
}  // namespace mde

using namespace mde;

extern "C" {

size_t mde_layernorm_workspace(int64_t rows, int64_t c) {
  if (!ln_ok(rows, c)) return 0;
  return (size_t)(4 * 2 * c * bwd_blocks(rows));
}

int mde_layernorm_add_fwd(const void* x, const void* r, const float* gamma, const float* beta,
                          void* sum, void* y, float* mean, float* rstd, int64_t rows, int64_t c,
                          float eps, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !r || !sum || !gamma || !beta || !y || !mean || !rstd) return MDE_ERR_INVALID_ARG;
  if (!ln_ok(rows, c)) return rows > 0 && c > 1024 && c % 64 == 0 ? MDE_ERR_UNSUPPORTED : MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  const float* xp = (const float*)x;
  const float* rp = (const float*)r;
  float* sp = (float*)sum;
  float* yp = (float*)y;
  switch (c / 64) {
#define MDE_LN_CASE(V) \
  case V: return ln_fwd_launch<V>(xp, gamma, beta, yp, mean, rstd, rows, eps, st, rp, sp);
    MDE_LN_CASE(1) MDE_LN_CASE(2) MDE_LN_CASE(3) MDE_LN_CASE(4) MDE_LN_CASE(5) MDE_LN_CASE(6)
    MDE_LN_CASE(7) MDE_LN_CASE(8) MDE_LN_CASE(9) MDE_LN_CASE(10) MDE_LN_CASE(11)
    MDE_LN_CASE(12) MDE_LN_CASE(13) MDE_LN_CASE(14) MDE_LN_CASE(15) MDE_LN_CASE(16)
#undef MDE_LN_CASE
    default: return MDE_ERR_INVALID_ARG;
  }
}

int mde_layernorm_bwd_res(const void* gy, const void* x, const void* gres, const float* gamma,
                          const float* mean, const float* rstd, void* gx, float* ggamma,
                          float* gbeta, int64_t rows, int64_t c, void* workspace, int dtype,
                          void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !x || !gres || !gamma || !mean || !rstd || !gx || !ggamma || !gbeta || !workspace)
    return MDE_ERR_INVALID_ARG;
  if (!ln_ok(rows, c)) return rows > 0 && c > 1024 && c % 64 == 0 ? MDE_ERR_UNSUPPORTED : MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  const float* g = (const float*)gy;
  const float* xp = (const float*)x;
  const float* rp = (const float*)gres;
  float* gxp = (float*)gx;
  float* part = (float*)workspace;
  switch (c / 64) {
#define MDE_LN_CASE(V) \
  case V: return ln_bwd_launch<V>(g, xp, gamma, mean, rstd, gxp, ggamma, gbeta, part, rows, st, rp);
    MDE_LN_CASE(1) MDE_LN_CASE(2) MDE_LN_CASE(3) MDE_LN_CASE(4) MDE_LN_CASE(5) MDE_LN_CASE(6)
    MDE_LN_CASE(7) MDE_LN_CASE(8) MDE_LN_CASE(9) MDE_LN_CASE(10) MDE_LN_CASE(11)
    MDE_LN_CASE(12) MDE_LN_CASE(13) MDE_LN_CASE(14) MDE_LN_CASE(15) MDE_LN_CASE(16)
#undef MDE_LN_CASE
    default: return MDE_ERR_INVALID_ARG;
  }
}

int mde_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y,
                      float* mean, float* rstd, int64_t rows, int64_t c, float eps, int dtype,
                      void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !gamma || !beta || !y || !mean || !rstd) return MDE_ERR_INVALID_ARG;
  if (!ln_ok(rows, c)) return rows > 0 && c > 1024 && c % 64 == 0 ? MDE_ERR_UNSUPPORTED : MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  const float* xp = (const float*)x;
  float* yp = (float*)y;
  switch (c / 64) {
#define MDE_LN_CASE(V) \
  case V: return ln_fwd_launch<V>(xp, gamma, beta, yp, mean, rstd, rows, eps, st);
    MDE_LN_CASE(1) MDE_LN_CASE(2) MDE_LN_CASE(3) MDE_LN_CASE(4) MDE_LN_CASE(5) MDE_LN_CASE(6)
    MDE_LN_CASE(7) MDE_LN_CASE(8) MDE_LN_CASE(9) MDE_LN_CASE(10) MDE_LN_CASE(11)
    MDE_LN_CASE(12) MDE_LN_CASE(13) MDE_LN_CASE(14) MDE_LN_CASE(15) MDE_LN_CASE(16)
#undef MDE_LN_CASE
    default: return MDE_ERR_INVALID_ARG;
  }
}

int mde_layernorm_bwd(const void* gy, const void* x, const float* gamma, const float* mean,
                      const float* rstd, void* gx, float* ggamma, float* gbeta, int64_t rows,
                      int64_t c, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !x || !gamma || !mean || !rstd || !gx || !ggamma || !gbeta || !workspace)
    return MDE_ERR_INVALID_ARG;
  if (!ln_ok(rows, c)) return rows > 0 && c > 1024 && c % 64 == 0 ? MDE_ERR_UNSUPPORTED : MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  const float* g = (const float*)gy;
  const float* xp = (const float*)x;
  float* gxp = (float*)gx;
  float* part = (float*)workspace;
  switch (c / 64) {
#define MDE_LN_CASE(V) \
  case V: return ln_bwd_launch<V>(g, xp, gamma, mean, rstd, gxp, ggamma, gbeta, part, rows, st);
    MDE_LN_CASE(1) MDE_LN_CASE(2) MDE_LN_CASE(3) MDE_LN_CASE(4) MDE_LN_CASE(5) MDE_LN_CASE(6)
    MDE_LN_CASE(7) MDE_LN_CASE(8) MDE_LN_CASE(9) MDE_LN_CASE(10) MDE_LN_CASE(11)
    MDE_LN_CASE(12) MDE_LN_CASE(13) MDE_LN_CASE(14) MDE_LN_CASE(15) MDE_LN_CASE(16)
#undef MDE_LN_CASE
    default: return MDE_ERR_INVALID_ARG;
  }
}

int mde_transpose(const void* x, void* y, int64_t batch, int64_t m, int64_t n, int dtype,
                  void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !y || batch <= 0 || m <= 0 || n <= 0 || batch > 65535 || cdiv(m, 64) > 65535)
    return MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)cdiv(n, 64), (unsigned)cdiv(m, 64), (unsigned)batch);
  static const bool vec = [] {
    const char* e = std::getenv("MDE_TRANSPOSE4");
    return !(e && e[0] == '0');
  }();
  if (vec && m % 4 == 0 && n % 4 == 0) {
    MDE_LAUNCH(K_TRANSPOSE, 8.0 * batch * m * n, st, transpose4_kernel, grid, dim3(256), 0,
               (const float*)x, (float*)y, m, n);
    return 0;
  }
  MDE_LAUNCH(K_TRANSPOSE, 8.0 * batch * m * n, st, transpose_kernel, grid, dim3(256), 0,
             (const float*)x, (float*)y, m, n);
  return 0;
}

}  // extern "C"
