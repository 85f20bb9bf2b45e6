// Token-major Linear / GELU backward helpers for the NewCRF blocks (fp32).
//
// Reference: Mlp.forward (src/newcrf_layers.py:9-27: fc1 -> nn.GELU() (erf) ->
// fc2) and the qk / proj Linears of WindowAttention (:110-149).  The GEMMs stay
// on hipBLASLt; what PyTorch runs around them in the backward is two more
// passes per Linear over the [T, N] gradient: GELU backward (read dh and the
// saved pre-activation a, write da) and the bias gradient (sum over the T
// tokens, ATen's column reduce).  Here:
//   mde_colsum          gb[n] = sum_t g[t, n]                       (1 read)
//   mde_gelu_bwd_colsum da = dh * gelu'(a), gb[n] = sum_t da[t, n]   (2 reads, 1 write)
// so fc1's bias gradient rides on the GELU backward pass instead of re-reading
// da.  Both reduce in a fixed order -- per-block column partials over a fixed
// token range, then a second kernel sums them (strided per thread, then a
// fixed tree) -- so the results are bitwise reproducible run to run (no
// atomics).
//
// Layout: lane l of a wave owns 4 consecutive columns (float4 loads, 256
// columns = 1 KB per wave row), the block's 4 waves interleave over token rows;
// a block covers a (rows, 256-column) tile.
#include <cmath>

#include "common.h"

namespace {

constexpr int kCols = 256;       // columns per block (64 lanes x 4)
constexpr int kRowsPerBlk = 256;  // token rows per block (each wave: every 4th row)

// GELU'(a) with ATen's erf form (GeluBackwardCUDAKernelImpl, approximate='none'):
// 0.5 (1 + erf(a / sqrt 2)) + a exp(-a^2 / 2) / sqrt(2 pi)
__device__ __forceinline__ float gelu_grad(float a) {
  constexpr float kAlpha = 0.70710678118654752440f;  // M_SQRT1_2
  constexpr float kBeta = 0.39894228040143267794f;   // M_2_SQRTPI * M_SQRT1_2 * 0.5
  const float cdf = 0.5f * (1.f + erff(a * kAlpha));
  const float pdf = expf(-0.5f * a * a) * kBeta;
  return cdf + a * pdf;
}

// part[blockIdx.y][n] = sum over this block's rows of (GELU ? dh * gelu'(a) : g)[t, n];
// GELU also writes da.  n % 4 == 0 is required of the caller (float4 rows).  Each
// wave takes every 4th row of the block's kRowsPerBlk; rows go 8 at a time with
// their loads issued together (clamped row index, masked accumulation) so the
// wave keeps 8 float4 loads in flight instead of one.
constexpr int kUnroll = 8;

template <bool GELU>
__global__ void __launch_bounds__(256)
    colsum_part_kernel(const float* __restrict__ g, const float* __restrict__ a,
                       float* __restrict__ da, int64_t t_rows, int n, float* __restrict__ part) {
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = blockIdx.x * kCols + 4 * lane;
  const bool cok = col < n;
  const int colc = cok ? col : 0;
  const int64_t r0 = (int64_t)blockIdx.y * kRowsPerBlk;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
  for (int i = 0; i < kRowsPerBlk / 4; i += kUnroll) {
    float4 v[kUnroll];
    bool ok[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t r = r0 + wv + 4 * (i + u);
      ok[u] = cok && r < t_rows;
      const int64_t off = (ok[u] ? r : 0) * n + colc;
      v[u] = *reinterpret_cast<const float4*>(g + off);
      if constexpr (GELU) {
        const float4 x = *reinterpret_cast<const float4*>(a + off);
        v[u] = make_float4(v[u].x * gelu_grad(x.x), v[u].y * gelu_grad(x.y),
                           v[u].z * gelu_grad(x.z), v[u].w * gelu_grad(x.w));
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (!ok[u]) continue;
      if constexpr (GELU) {
        const int64_t r = r0 + wv + 4 * (i + u);
        *reinterpret_cast<float4*>(da + r * n + col) = v[u];
      }
      acc.x += v[u].x;
      acc.y += v[u].y;
      acc.z += v[u].z;
      acc.w += v[u].w;
    }
  }
  red[wv][lane] = acc;
  __syncthreads();
  if (wv != 0 || !cok) return;
  float4 s = red[0][lane];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const float4 q = red[k][lane];
    s.x += q.x;
    s.y += q.y;
    s.z += q.z;
    s.w += q.w;
  }
  *reinterpret_cast<float4*>(part + (int64_t)blockIdx.y * n + col) = s;
}

// gb[4j .. 4j+3] = sum over the row blocks b of part[b][4j ..]: one block per 4
// columns, thread t sums rows b = t, t + 256, ... (float4), then a fixed-shape
// tree over the 256 threads -- a fixed order, so bitwise reproducible.
__global__ void __launch_bounds__(256)
    colsum_final_kernel(const float* __restrict__ part, int nblk, int n, float* __restrict__ gb) {
  __shared__ float4 red[256];
  const int t = threadIdx.x, col = 4 * blockIdx.x;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b = t; b < nblk; b += 256) {
    const float4 q = *reinterpret_cast<const float4*>(part + (int64_t)b * n + col);
    s.x += q.x;
    s.y += q.y;
    s.z += q.z;
    s.w += q.w;
  }
  red[t] = s;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      const float4 q = red[t + w];
      float4 r = red[t];
      r.x += q.x;
      r.y += q.y;
      r.z += q.z;
      r.w += q.w;
      red[t] = r;
    }
    __syncthreads();
  }
  if (t == 0) *reinterpret_cast<float4*>(gb + col) = red[0];
}

bool dims_ok(int64_t t_rows, int64_t n) {
  return t_rows > 0 && n > 0 && n % 4 == 0 && n <= (1 << 30) &&
         mde::cdiv(t_rows, kRowsPerBlk) <= 65535;
}

int launch(bool gelu, const float* g, const float* a, float* da, float* gb, int64_t t_rows,
           int64_t n, void* workspace, hipStream_t s) {
  const int nblk = (int)mde::cdiv(t_rows, kRowsPerBlk);
  float* part = (float*)workspace;
  const dim3 grid((unsigned)mde::cdiv(n, kCols), (unsigned)nblk);
  const double bytes = 4.0 * (double)t_rows * n * (gelu ? 3.0 : 1.0);
  if (gelu)
    MDE_LAUNCH(mde::K_MLP_GELU_BWD, bytes, s, colsum_part_kernel<true>, grid, dim3(256), 0, g, a,
               da, t_rows, (int)n, part);
  else
    MDE_LAUNCH(mde::K_COLSUM, bytes, s, colsum_part_kernel<false>, grid, dim3(256), 0, g,
               (const float*)nullptr, (float*)nullptr, t_rows, (int)n, part);
  MDE_LAUNCH(mde::K_COLSUM, 4.0 * (double)nblk * n, s, colsum_final_kernel,
             dim3((unsigned)(n / 4)), dim3(256), 0, (const float*)part, nblk, (int)n, gb);
  return MDE_OK;
}

}  // namespace

extern "C" {

size_t mde_colsum_workspace(int64_t t_rows, int64_t n) {
  if (!dims_ok(t_rows, n)) return 0;
  return sizeof(float) * (size_t)mde::cdiv(t_rows, kRowsPerBlk) * (size_t)n;
}

int mde_colsum(const void* g, float* gb, int64_t t_rows, int64_t n, void* workspace, int dtype,
               void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!g || !gb || !workspace || !dims_ok(t_rows, n)) return MDE_ERR_INVALID_ARG;
  return launch(false, (const float*)g, nullptr, nullptr, gb, t_rows, n, workspace,
                (hipStream_t)stream);
}

int mde_gelu_bwd_colsum(const void* dh, const void* a, void* da, float* gb, int64_t t_rows,
                        int64_t n, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!dh || !a || !da || !gb || !workspace || !dims_ok(t_rows, n)) return MDE_ERR_INVALID_ARG;
  return launch(true, (const float*)dh, (const float*)a, (float*)da, gb, t_rows, n, workspace,
                (hipStream_t)stream);
}

}  // extern "C"
