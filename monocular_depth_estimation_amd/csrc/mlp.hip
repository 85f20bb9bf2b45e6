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
#include <cstdlib>

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

// ---------------------------------------------------------------------------
// Linear weight gradient over tokens, gw[m][n] = sum_t g[t][m] x[t][n] (+ the
// bias gradient gb[m] = sum_t g[t][m] from the same reads): the `g2.t() @ x`
// of the Linear backward, whose reduction runs over all T tokens (16 H W at
// bs 16: 4800 - 307200) into a small [M, N] output.  hipBLASLt runs these at
// 0.25 - 0.35 of the fp32 MFMA peak (the forward GEMMs of the same flops at
// 0.63); here, split-K over token ranges, deterministic:
//
//  * block = 4 waves, a 128 x 128 output tile (wave: 64 x 64 = 4 x 4 tiles of
//    v_mfma_f32_16x16x4_f32), token chunks of 16 rows through double-buffered
//    LDS (A = g[16][128], B = x[16][128], row-major as in HBM: whole 512 B
//    rows, float4 loads, one chunk in flight in registers);
//  * both operands in their natural token-major layout: MFMA tile i of a wave
//    takes output rows m = 4 r + i (r = the MFMA row) so that a lane's four
//    A values -- one per tile -- are one float4 of g's row, likewise B, and
//    the accumulators leave as float4 rows of gw;
//  * blockIdx -> (tile, split) so that the tiles of one token range share an
//    XCD (its L2 serves the g / x re-reads across tiles);
//  * per-split partials [S][M N + M] in the workspace, then lin_wreduce_kernel
//    sums them in split order (fixed order: bitwise reproducible).
constexpr int kWT = 128;  // output tile rows / columns
constexpr int kWK = 16;   // tokens per chunk

using f4v = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int PD>  // chunks in flight from HBM per block: 2 (default) or 1 (MDE_LIN_WGRAD_PD=1)
__global__ void __launch_bounds__(256, 2)
    lin_wgrad_kernel(const float* __restrict__ g, const float* __restrict__ x,
                     float* __restrict__ part, int64_t t_rows, int m, int n, int64_t per_split,
                     int tiles_n, int tiles, int splits, int xcd_map, int bias) {
  __shared__ float4 lds[2][2][kWK][kWT / 4];  // [buffer][g | x][token row][float4 column]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1, l16 = lane & 15, g4 = lane >> 4;
  const int id = blockIdx.x;
  int tile, split;
  if (xcd_map) {  // splits % 8 == 0: the tiles of split s on XCD s % 8
    tile = (id >> 3) % tiles;
    split = (id & 7) + 8 * ((id >> 3) / tiles);
  } else {
    tile = id % tiles;
    split = id / tiles;
  }
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int64_t t0 = (int64_t)split * per_split;
  const int64_t t1 = t0 + per_split < t_rows ? t0 + per_split : t_rows;
  const int nch = t1 > t0 ? (int)((t1 - t0) / kWK) : 0;  // t_rows, per_split: multiples of kWK
  const int lr = tid >> 5, lc = tid & 31;  // loader: float4 (lr, lc) and (lr + 8, lc)
  const float* gp = g + (t0 + lr) * m + (int64_t)tm * kWT + 4 * lc;
  const float* xp = x + (t0 + lr) * n + (int64_t)tn * kWT + 4 * lc;
  // one chunk's loads of this thread, two named register sets (S = 0 / 1;
  // arrays or structs passed by reference here went to scratch)
#define LIN_GLOAD(S, C)                                                         \
  do {                                                                          \
    const float* a_ = gp + (int64_t)(C) * kWK * m;                              \
    const float* b_ = xp + (int64_t)(C) * kWK * n;                              \
    a0_##S = *reinterpret_cast<const float4*>(a_);                              \
    a1_##S = *reinterpret_cast<const float4*>(a_ + 8 * (int64_t)m);             \
    b0_##S = *reinterpret_cast<const float4*>(b_);                              \
    b1_##S = *reinterpret_cast<const float4*>(b_ + 8 * (int64_t)n);             \
  } while (0)
#define LIN_LSTORE(S, BUF)                                                      \
  do {                                                                          \
    lds[BUF][0][lr][lc] = a0_##S;                                               \
    lds[BUF][0][lr + 8][lc] = a1_##S;                                           \
    lds[BUF][1][lr][lc] = b0_##S;                                               \
    lds[BUF][1][lr + 8][lc] = b1_##S;                                           \
  } while (0)
  float4 a0_0, a1_0, b0_0, b1_0, a0_1, a1_1, b0_1, b1_1;
  f4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  float4 bs = make_float4(0.f, 0.f, 0.f, 0.f);  // bias partial: columns 4 l16 + 0..3 of wm's 64
  const bool bias_here = bias && tn == 0 && wn == 0;  // wave-uniform
  auto compute = [&](int buf) {
#pragma unroll
    for (int st = 0; st < kWK / 4; ++st) {
      const float4 a = lds[buf][0][4 * st + g4][wm * 16 + l16];
      const float4 b = lds[buf][1][4 * st + g4][wn * 16 + l16];
      if (bias_here) {
        bs.x += a.x;
        bs.y += a.y;
        bs.z += a.z;
        bs.w += a.w;
      }
      const f4v av{a.x, a.y, a.z, a.w}, bv{b.x, b.y, b.z, b.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
    }
  };
  if constexpr (PD == 2) {
    // chunk c + 2 is loaded while chunk c is multiplied: each load has two
    // chunk periods to land (one was not enough at 2 blocks per CU: the small
    // M x N shapes stream g and x at ~5 TB/s with no reuse)
    if (nch > 0) {
      LIN_GLOAD(0, 0);
      if (nch > 1) LIN_GLOAD(1, 1);
      LIN_LSTORE(0, 0);
    }
    __syncthreads();
#pragma unroll 1
    for (int c = 0; c < nch; c += 2) {
      if (c + 2 < nch) LIN_GLOAD(0, c + 2);
      compute(0);
      if (c + 1 < nch) LIN_LSTORE(1, 1);
      __syncthreads();
      if (c + 1 >= nch) break;  // uniform
      if (c + 3 < nch) LIN_GLOAD(1, c + 3);
      compute(1);
      if (c + 2 < nch) LIN_LSTORE(0, 0);
      __syncthreads();
    }
  } else {
    if (nch > 0) {
      LIN_GLOAD(0, 0);
      LIN_LSTORE(0, 0);
    }
    __syncthreads();
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int buf = c & 1;
      if (c + 1 < nch) LIN_GLOAD(0, c + 1);
      compute(buf);
      if (c + 1 < nch) LIN_LSTORE(0, buf ^ 1);
      __syncthreads();
    }
  }
#undef LIN_GLOAD
#undef LIN_LSTORE
  // lane holds D[4 g4 + r][l16] of tile (i, j): row m = 4 (4 g4 + r) + i, column 4 l16 + j
  float* out = part + (int64_t)split * ((int64_t)m * n + m);
  const int64_t col = (int64_t)tn * kWT + wn * 64 + 4 * l16;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = (int64_t)tm * kWT + wm * 64 + 4 * (4 * g4 + r) + i;
      *reinterpret_cast<float4*>(out + row * n + col) =
          make_float4(acc[i][0][r], acc[i][1][r], acc[i][2][r], acc[i][3][r]);
    }
  if (bias_here) {
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      bs.x += __shfl_xor(bs.x, o, 64);
      bs.y += __shfl_xor(bs.y, o, 64);
      bs.z += __shfl_xor(bs.z, o, 64);
      bs.w += __shfl_xor(bs.w, o, 64);
    }
    if (g4 == 0)
      *reinterpret_cast<float4*>(out + (int64_t)m * n + tm * kWT + wm * 64 + 4 * l16) = bs;
  }
}

// gw / gb = sum over the splits of part[s] (float4 per thread, splits in order)
__global__ void __launch_bounds__(256)
    lin_wreduce_kernel(const float* __restrict__ part, int splits, int64_t mn, int m,
                       float* __restrict__ gw, float* __restrict__ gb) {
  const int64_t e = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  const int64_t stride = mn + m;
  if (e >= (gb ? stride : mn)) return;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int k = 0; k < splits; ++k) {
    const float4 q = mde::ld4_nt(part + (int64_t)k * stride + e);
    s.x += q.x;
    s.y += q.y;
    s.z += q.z;
    s.w += q.w;
  }
  if (e < mn)
    *reinterpret_cast<float4*>(gw + e) = s;
  else
    *reinterpret_cast<float4*>(gb + (e - mn)) = s;
}

int wgrad_pd() {
  static const int pd = [] {
    const char* e = getenv("MDE_LIN_WGRAD_PD");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  return pd;
}

struct WgradPlan {
  int tiles_n, tiles, splits, xcd_map;
  int64_t per_split;
};

bool wgrad_plan(int64_t t_rows, int64_t m, int64_t n, WgradPlan* p) {
  if (t_rows <= 0 || m <= 0 || n <= 0 || t_rows % kWK || m % kWT || n % kWT ||
      t_rows * (m > n ? m : n) >= (1LL << 40) || m * n >= (1LL << 31))
    return false;
  p->tiles_n = (int)(n / kWT);
  p->tiles = (int)(m / kWT) * p->tiles_n;
  // ~512 blocks (2 per CU), >= 32 chunks (512 tokens) per split: fewer,
  // longer splits beat 768 / 1024 blocks (the partials' write + reduce pass
  // grows with the split count; tools/lin_bench.py, profiles/r06_lin_wgrad.txt)
  static const int target = [] {
    const char* e = getenv("MDE_LIN_WGRAD_BLOCKS");
    return e ? atoi(e) : 512;
  }();
  int64_t s = mde::cdiv(target, p->tiles);
  const int64_t smax = t_rows / 512 > 1 ? t_rows / 512 : 1;
  if (s > smax) s = smax;
  if (s >= 8) s = s / 8 * 8;
  int64_t per = mde::cdiv(mde::cdiv(t_rows, s), kWK) * kWK;
  s = mde::cdiv(t_rows, per);
  p->xcd_map = s % 8 == 0;
  p->splits = (int)s;
  p->per_split = per;
  return (int64_t)p->tiles * s < (1LL << 31);
}

// ---------------------------------------------------------------------------
// Per-channel sums of an NCHW tensor, gb[c] = sum_{n, p} g[n][c][p]: a biased
// conv's bias gradient (autograd's grad.sum((0, 2, 3)) behind `y + bias`,
// nn.Conv2d with a bias on the HIP conv path: the NewCRF projections,
// newcrf_layers.py:384-392), which ATen's reduction ran at ~1.3 TB/s.  Block
// (c, s) sums planes [s P, s P + P) of channel c with float4 loads (4 per
// lane in flight), a fixed-shape tree over the block, then chansum_final
// adds the S partials in order: bitwise reproducible.
__global__ void __launch_bounds__(256)
    chansum_part_kernel(const float* __restrict__ g, int64_t n, int c, int64_t hw, int per,
                        float* __restrict__ part) {
  __shared__ float red[256];
  const int ch = blockIdx.x, sp = blockIdx.y, tid = threadIdx.x;
  const int64_t i0 = (int64_t)sp * per, i1 = i0 + per < n ? i0 + per : n;
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
  for (int64_t img = i0; img < i1; ++img) {
    const float* p = g + (img * c + ch) * hw;
    int64_t e = 4 * (int64_t)tid;
    for (; e + 1024 < hw; e += 2048) {
      const float4 u = mde::ld4_nt(p + e), v = mde::ld4_nt(p + e + 1024);
      a0.x += u.x; a0.y += u.y; a0.z += u.z; a0.w += u.w;
      a1.x += v.x; a1.y += v.y; a1.z += v.z; a1.w += v.w;
    }
    if (e < hw) {
      const float4 u = mde::ld4_nt(p + e);
      a0.x += u.x; a0.y += u.y; a0.z += u.z; a0.w += u.w;
    }
  }
  red[tid] = ((a0.x + a0.y) + (a0.z + a0.w)) + ((a1.x + a1.y) + (a1.z + a1.w));
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) part[(int64_t)ch * gridDim.y + sp] = red[0];
}

__global__ void __launch_bounds__(256)
    chansum_final_kernel(const float* __restrict__ part, int c, int splits, float* __restrict__ gb) {
  const int ch = blockIdx.x * 256 + threadIdx.x;
  if (ch >= c) return;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[(int64_t)ch * splits + k];
  gb[ch] = s;
}

inline int chansum_splits(int64_t n, int64_t c) {
  const int64_t s = mde::cdiv(1024, c);  // ~1024 blocks
  return (int)(s < n ? s : n);
}

}  // namespace

extern "C" {

size_t mde_chansum_workspace(int64_t n, int64_t c, int64_t hw) {
  if (n <= 0 || c <= 0 || hw <= 0 || hw % 4 || c > 65535) return 0;
  return sizeof(float) * (size_t)(c * chansum_splits(n, c));
}

int mde_chansum(const void* g, float* gb, int64_t n, int64_t c, int64_t hw, void* workspace,
                int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!g || !gb || !workspace || !mde_chansum_workspace(n, c, hw)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int sp = chansum_splits(n, c);
  const int per = (int)mde::cdiv(n, sp);
  const int used = (int)mde::cdiv(n, per);
  float* part = (float*)workspace;
  MDE_LAUNCH(mde::K_CHANSUM, 4.0 * (double)n * c * hw, s, chansum_part_kernel,
             dim3((unsigned)c, (unsigned)used), dim3(256), 0, (const float*)g, n, (int)c, hw, per,
             part);
  MDE_LAUNCH(mde::K_CHANSUM, 4.0 * (double)c * used, s, chansum_final_kernel,
             dim3((unsigned)mde::cdiv(c, 256)), dim3(256), 0, (const float*)part, (int)c, used, gb);
  return MDE_OK;
}

size_t mde_linear_wgrad_workspace(int64_t t_rows, int64_t m, int64_t n) {
  WgradPlan p;
  if (!wgrad_plan(t_rows, m, n, &p)) return 0;
  return sizeof(float) * (size_t)p.splits * (size_t)(m * n + m);
}

int mde_linear_wgrad(const void* g, const void* x, float* gw, float* gb, int64_t t_rows,
                     int64_t m, int64_t n, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  WgradPlan p;
  if (!g || !x || !gw || !workspace || !wgrad_plan(t_rows, m, n, &p)) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  const double flops = 2.0 * (double)t_rows * m * n;
  const double bytes = 4.0 * ((double)t_rows * (m + n) + (double)m * n);
  const dim3 grid((unsigned)(p.tiles * p.splits));
  if (wgrad_pd() == 1)
    MDE_LAUNCH_MFMA(mde::K_LIN_WGRAD, bytes, flops, s, lin_wgrad_kernel<1>, grid, dim3(256), 0,
                    (const float*)g, (const float*)x, part, t_rows, (int)m, (int)n, p.per_split,
                    p.tiles_n, p.tiles, p.splits, p.xcd_map, gb ? 1 : 0);
  else
    MDE_LAUNCH_MFMA(mde::K_LIN_WGRAD, bytes, flops, s, lin_wgrad_kernel<2>, grid, dim3(256), 0,
                    (const float*)g, (const float*)x, part, t_rows, (int)m, (int)n, p.per_split,
                    p.tiles_n, p.tiles, p.splits, p.xcd_map, gb ? 1 : 0);
  const int64_t len = m * n + (gb ? m : 0);
  MDE_LAUNCH(mde::K_LIN_WREDUCE, 4.0 * (double)p.splits * len + 4.0 * len, s, lin_wreduce_kernel,
             dim3((unsigned)mde::cdiv(len / 4, 256)), dim3(256), 0, (const float*)part, p.splits,
             m * n, (int)m, gw, gb);
  return MDE_OK;
}

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
