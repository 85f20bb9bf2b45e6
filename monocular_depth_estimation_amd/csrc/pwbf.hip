// The BN-ReLU-fused pointwise (1x1) convolution of the guided upsampling
// blocks (src/GuideDepth/model/modules.py:72-73: comb_conv's BatchNorm + ReLU
// feeding the 1x1 reduce / the next block's 1x1) on bf16 activations, with
// bf16 products on v_mfma_f32_16x16x32_bf16 and fp32 accumulation -- what
// autocast hands the reference's 1x1 conv (bf16 input and weight, fp32
// accumulate).  The fp32-product kernels of skip.hip ran these shapes on the
// 16x16x4 fp32 MFMA at 1/16 of the bf16 rate, which at 64 -> 64 was the bound
// (218 us for 236 MB); here every shape is HBM-bound.
//
// Layouts (NCHW, hw % 64 == 0, 64-pixel tiles, one tile per wave at a time):
//  - a "T" load: lane (l16, q4) reads pixels 4 l16 .. +3 (8 bytes) of the 8
//    channel rows 32 k + 8 q4 + j, j = 0..7; sub-tile s of the MFMA's N
//    dimension is pixel 4 l16 + s, so a B fragment (8 channels of one pixel)
//    is two v_perm_b32 per register from those rows, and the D tile gives each
//    lane 4 consecutive pixels of 4 output rows: one 8-byte store per row.
//  - an "R" load: lane (l16, q4) reads pixels 32 kk + 8 q4 .. +7 (16 bytes) of
//    row 16 t + l16: the fragment of a product over pixels (the weight
//    gradient), element j = pixel 8 q4 + j in both operands.
// Forward: y [CO x 64] = W [CO x CI] . S [CI x 64], S = relu(x * sc + sh)
// rounded to bf16 (T loads of x; W rounded to bf16 in registers).
// Backward: gs [CI x 64] = W^T . G (T loads of gy), gW [CO x CI] += G . S^T
// over the tile's pixels (R loads of gy and x); (BNS) the producer BN's two
// backward sums from the gs tile; the next tile's operands are loaded while
// this tile computes (two register sets).
#include "common.h"

namespace {

using mde::bf16;
using bf8v = __bf16 __attribute__((ext_vector_type(8)));
using bf2v = __bf16 __attribute__((ext_vector_type(2)));
using f4v = float __attribute__((ext_vector_type(4)));
using u2v = uint32_t __attribute__((ext_vector_type(2)));
using u4v = uint32_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma_bf(u4v a, u4v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a),
                                                 __builtin_bit_cast(bf8v, b), c, 0, 0, 0);
}

// two fp32 -> packed bf16 (RNE, v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk(float a, float b) {
  return __builtin_bit_cast(uint32_t, bf2v{(__bf16)a, (__bf16)b});
}
__device__ __forceinline__ float lo_f(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

template <typename V>
__device__ __forceinline__ V ld_nt(const bf16* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
}

// B fragment of sub-tile s (pixel 4 l16 + s) from 8 T-loaded rows: element j
// = row j's pixel s.  Raw bf16 bits (no BN): v_perm_b32 pairs.
__device__ __forceinline__ u4v frag_raw(const u2v (&rows)[8], int s) {
  u4v f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t a = (s < 2) ? rows[2 * e].x : rows[2 * e].y;
    const uint32_t b = (s < 2) ? rows[2 * e + 1].x : rows[2 * e + 1].y;
    f[e] = __builtin_amdgcn_perm(b, a, (s & 1) ? 0x07060302u : 0x05040100u);
  }
  return f;
}

__device__ __forceinline__ float pix(const u2v& r, int s) {
  return s == 0 ? lo_f(r.x) : s == 1 ? hi_f(r.x) : s == 2 ? lo_f(r.y) : hi_f(r.y);
}

// The same with the BN + ReLU applied (fp32) before the bf16 rounding.
__device__ __forceinline__ u4v frag_bnr(const u2v (&rows)[8], int s, const float (&sc)[8],
                                        const float (&sh)[8]) {
  u4v f;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    f[e] = pk(fmaxf(fmaf(pix(rows[2 * e], s), sc[2 * e], sh[2 * e]), 0.f),
              fmaxf(fmaf(pix(rows[2 * e + 1], s), sc[2 * e + 1], sh[2 * e + 1]), 0.f));
  return f;
}

// bf16 rounding of a float (RNE), as a float
__device__ __forceinline__ float rbf(float v) { return (float)(__bf16)v; }

// The skip fusion's operand (HAS_D, modules.py:100 `reduce(residual + depth)`
// under autocast): s = bf16(bf16(relu(x * sc + sh)) + d) -- the BN-ReLU output
// and the sum each rounded as autocast's bf16 tensors are.
__device__ __forceinline__ u4v frag_skip(const u2v (&rows)[8], const u2v (&drows)[8], int s,
                                         const float (&sc)[8], const float (&sh)[8]) {
  u4v f;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    f[e] = pk(rbf(fmaxf(fmaf(pix(rows[2 * e], s), sc[2 * e], sh[2 * e]), 0.f)) + pix(drows[2 * e], s),
              rbf(fmaxf(fmaf(pix(rows[2 * e + 1], s), sc[2 * e + 1], sh[2 * e + 1]), 0.f)) +
                  pix(drows[2 * e + 1], s));
  return f;
}

// ----------------------------------------------------------------- forward
// STATS: the output's per-channel shifted sums per block (the layout of
// skip_fwd_mfma_kernel's epilogue: stats[(o * gridDim.x + block) * 4]).
// HAS_D (with BNR): the skip fusion, s = bf16(bf16(relu(bn(x))) + d), plus a
// bias (rounded to bf16 as autocast casts it) -- skip_reduce_bn's forward.
template <int CI, int CO, bool BNR, bool STATS, bool HAS_D = false>
__global__ void __launch_bounds__(256)
    pwbf_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ wt,
                    bf16* __restrict__ y, int64_t n, int64_t hw, const float* __restrict__ isc,
                    const float* __restrict__ ish, float* __restrict__ stats,
                    const bf16* __restrict__ d = nullptr, const float* __restrict__ bias = nullptr) {
  static_assert(!HAS_D || (BNR && !STATS), "skip fusion: BN-ReLU operand, no statistics");
  constexpr int KS = (CI + 31) / 32, OT = (CO + 15) / 16;
  static_assert(CI % 16 == 0 && CO % 8 == 0, "tile shapes");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q4 = lane >> 4;
  // rows this lane T-loads: channel 32 ks + 8 q4 + j (CI = 16: lane groups 2, 3 idle)
  constexpr bool HALF = CI < 32;
  const bool rows_live = !HALF || q4 < 2;
  u4v wa[OT][KS];  // A: W[o = 16 ot + l16][c = 32 ks + 8 q4 + j], bf16
#pragma unroll
  for (int ot = 0; ot < OT; ++ot)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int o = 16 * ot + l16, c = 32 * ks + 8 * q4 + 2 * e;
        const bool ok = o < CO && c < CI;
        wa[ot][ks][e] = pk(ok ? wt[o * CI + c] : 0.f, ok ? wt[o * CI + c + 1] : 0.f);
      }
  float bsc[BNR ? KS : 1][8], bsh[BNR ? KS : 1][8];
  if constexpr (BNR) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 32 * ks + 8 * q4 + j;
        bsc[ks][j] = c < CI ? isc[c] : 0.f;
        bsh[ks][j] = c < CI ? ish[c] : 0.f;
      }
  }
  float rref[STATS ? OT : 1][4], rs1[STATS ? OT : 1][4], rs2[STATS ? OT : 1][4];
#pragma unroll
  for (int ot = 0; ot < (STATS ? OT : 1); ++ot)
#pragma unroll
    for (int i = 0; i < 4; ++i) rref[ot][i] = rs1[ot][i] = rs2[ot][i] = 0.f;
  float bo[HAS_D ? OT : 1][4];  // D rows 16 ot + 4 q4 + i
#pragma unroll
  for (int ot = 0; ot < (HAS_D ? OT : 1); ++ot)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = 16 * ot + 4 * q4 + i;
      bo[ot][i] = HAS_D && bias && o < CO ? rbf(bias[o]) : 0.f;
    }
  int ntile = 0;
  bool first = true;
  const int64_t tpi = hw / 64, tiles = n * tpi, stride = (int64_t)gridDim.x * 4;
  constexpr int KD = HAS_D ? KS : 1;
  struct Raw {
    u2v x[KS][8];
    u2v d[KD][8];
  };
  Raw A, B;
  auto load = [&](int64_t t, Raw& R) {
    if (t >= tiles) t = tiles - 1;  // past the end: a valid tile, unused
    const int64_t nidx = t / tpi, p0 = (t - nidx * tpi) * 64;
    const bf16* xp = x + nidx * CI * hw + p0 + 4 * l16;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        R.x[ks][j] = rows_live ? ld_nt<u2v>(xp + (int64_t)(32 * ks + 8 * q4 + j) * hw) : u2v{0u, 0u};
    if constexpr (HAS_D) {
      const bf16* dp = d + nidx * CI * hw + p0 + 4 * l16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          R.d[ks][j] = rows_live ? ld_nt<u2v>(dp + (int64_t)(32 * ks + 8 * q4 + j) * hw) : u2v{0u, 0u};
    }
  };
  auto compute = [&](int64_t t, const Raw& R) {
    const int64_t nidx = t / tpi, p0 = (t - nidx * tpi) * 64;
    bf16* yp = y + nidx * CO * hw + p0 + 4 * l16;
    u4v bf[KS][4];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        // (idle rows: zero bits, zero BN coefficients and zero weights)
        if constexpr (HAS_D) bf[ks][s] = frag_skip(R.x[ks], R.d[ks], s, bsc[ks], bsh[ks]);
        else if constexpr (BNR) bf[ks][s] = frag_bnr(R.x[ks], s, bsc[ks], bsh[ks]);
        else bf[ks][s] = frag_raw(R.x[ks], s);
      }
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      f4v acc[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if constexpr (HAS_D) acc[s] = f4v{bo[ot][0], bo[ot][1], bo[ot][2], bo[ot][3]};
        else acc[s] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acc[s] = mfma_bf(wa[ot][ks], bf[ks][s], acc[s]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 16 * ot + 4 * q4 + i;
        const u2v u{pk(acc[0][i], acc[1][i]), pk(acc[2][i], acc[3][i])};
        if (o < CO) __builtin_nontemporal_store(u, reinterpret_cast<u2v*>(yp + (int64_t)o * hw));
        if constexpr (STATS) {
          // statistics of the values as stored (bf16-rounded)
          const float vs[4] = {lo_f(u.x), hi_f(u.x), lo_f(u.y), hi_f(u.y)};
          if (first) rref[ot][i] = __shfl(vs[0], lane & 48, 64);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float dv = vs[j] - rref[ot][i];
            rs1[ot][i] += dv;
            rs2[ot][i] = fmaf(dv, dv, rs2[ot][i]);
          }
        }
      }
    }
    first = false;
    ++ntile;
  };
  int64_t t = (int64_t)blockIdx.x * 4 + w;
  if (t < tiles) {
    load(t, A);
    while (true) {
      load(t + stride, B);
      compute(t, A);
      t += stride;
      if (t >= tiles) break;
      load(t + stride, A);
      compute(t, B);
      t += stride;
      if (t >= tiles) break;
    }
  }
  if constexpr (STATS) {
    __shared__ float part[4][CO][4];
#pragma unroll
    for (int ot = 0; ot < OT; ++ot)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        mde::Sh a{rref[ot][i], 4.f * ntile, rs1[ot][i], rs2[ot][i]};
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) a = mde::sh_xor_sum(a, o);
        const int c = 16 * ot + 4 * q4 + i;
        if (l16 == 0 && c < CO) {
          part[w][c][0] = a.ref;
          part[w][c][1] = a.n;
          part[w][c][2] = a.s1;
          part[w][c][3] = a.s2;
        }
      }
    __syncthreads();
    if (threadIdx.x < CO) {
      const int c = threadIdx.x;
      mde::Sh a{part[0][c][0], part[0][c][1], part[0][c][2], part[0][c][3]};
#pragma unroll
      for (int k = 1; k < 4; ++k)
        a = mde::sh_merge(a, {part[k][c][0], part[k][c][1], part[k][c][2], part[k][c][3]});
      float* o4 = stats + ((int64_t)c * gridDim.x + blockIdx.x) * 4;
      o4[0] = a.ref;
      o4[1] = a.n;
      o4[2] = a.s1;
      o4[3] = a.s2;
    }
  }
}

// ---------------------------------------------------------------- backward
template <int CI, int CO, bool BNR, bool BNS, bool HAS_D = false>
struct PwbfRaw {
  static constexpr int MT = CI / 16, OT = (CO + 15) / 16, KO = (CO + 31) / 32;
  u2v gt[KO][8];                // T: gy rows 32 ko + 8 q4 + j, pixels 4 l16 ..
  u4v gr[OT][2];                // R: gy row 16 ot + l16, pixels 32 kk + 8 q4 ..
  u4v sr[MT][2];                // R: x row 16 mt + l16, pixels 32 kk + 8 q4 ..
  u4v dr[HAS_D ? MT : 1][2];    // R: d row 16 mt + l16 (the skip fusion's second input)
  u2v xr[BNS ? MT : 1][4];      // x rows 16 mt + 4 q4 + i, pixels 4 l16 .. (the gs layout)
};

// slab row per block: gW [CO][CI], CO unused bias columns (zeros), (BNS) the
// BN sums [CI][2] -- skip_slab_reduce_kernel<1>'s layout.
// PF: the next tile's operands in a second register set (off at 64 -> 64,
// whose two sets spill).
// HAS_D (with BNR): the skip fusion's backward -- gs is the gradient of s =
// relu(bn(x)) + d (both inputs take it), the weight gradient sees s as the
// forward rounded it, and the slab's bias columns get the row sums of gy.
template <int CI, int CO, bool BNR, bool BNS, bool HAS_D = false, bool PF = (CI * CO < 4096)>
__global__ void __launch_bounds__(256, (CI * CO >= 2048 || (BNS && CI >= 32)) ? 1 : 2)
    pwbf_bwd_kernel(const bf16* __restrict__ g, const bf16* __restrict__ x,
                    const float* __restrict__ wt, bf16* __restrict__ gs, float* __restrict__ slab,
                    int64_t n, int64_t hw, const float* __restrict__ isc,
                    const float* __restrict__ ish, const float* __restrict__ imean,
                    const bf16* __restrict__ d = nullptr) {
  static_assert(!HAS_D || BNR, "skip fusion: BN-ReLU operand");
  using Raw = PwbfRaw<CI, CO, BNR, BNS, HAS_D>;
  constexpr int MT = Raw::MT, OT = Raw::OT, KO = Raw::KO;
  static_assert(CI % 16 == 0 && CO % 8 == 0, "tile shapes");
  static_assert(!BNS || (BNR && CI <= 32), "BN sums: fused BN-ReLU operand, cin <= 32");
  constexpr int ROW = CO * CI + CO + (BNS ? 2 * CI : 0);
  constexpr int SOFF = CO * CI + CO;
  __shared__ float red[4][ROW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q4 = lane >> 4;
  // gy rows this lane T-loads (CO < 32: lane groups past CO idle)
  auto trow_live = [&](int ko) { return 32 * ko + 8 * q4 < CO; };
  u4v wa[MT][KO];  // A of gs = W^T G: W[o = 32 ko + 8 q4 + j][c = 16 mt + l16], bf16
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int ko = 0; ko < KO; ++ko)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 16 * mt + l16, o = 32 * ko + 8 * q4 + 2 * e;
        wa[mt][ko][e] = pk(o < CO ? wt[o * CI + c] : 0.f, o + 1 < CO ? wt[(o + 1) * CI + c] : 0.f);
      }
  f4v gw[OT][MT];
#pragma unroll
  for (int ot = 0; ot < OT; ++ot)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) gw[ot][mt] = f4v{0.f, 0.f, 0.f, 0.f};
  float gbp[HAS_D ? OT : 1] = {};  // row 16 ot + l16 of gy, this lane's pixels
  float bsc[MT], bsh[MT];  // the R-load row's channel 16 mt + l16
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    bsc[mt] = BNR ? isc[16 * mt + l16] : 1.f;
    bsh[mt] = BNR ? ish[16 * mt + l16] : 0.f;
  }
  // BNS: the gs layout's channels' BN coefficients are read from LDS per use
  // (an opaque zero index keeps them there: 3 MT 4 registers saved)
  __shared__ float s_bn[BNS ? 3 : 1][BNS ? CI : 1];
  float es1[BNS ? MT : 1][4], es2[BNS ? MT : 1][4];
  if constexpr (BNS) {
    if (threadIdx.x < CI) {
      s_bn[0][threadIdx.x] = isc[threadIdx.x];
      s_bn[1][threadIdx.x] = ish[threadIdx.x];
      s_bn[2][threadIdx.x] = imean[threadIdx.x];
    }
    __syncthreads();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) es1[mt][i] = es2[mt][i] = 0.f;
  }
  const int64_t tpi = hw / 64, tiles = n * tpi, stride = (int64_t)gridDim.x * 4;
  auto load = [&](int64_t t, Raw& R) {
    if (t >= tiles) t = tiles - 1;  // past the end: a valid tile, unused
    const int64_t nidx = t / tpi, p0 = (t - nidx * tpi) * 64;
    const bf16* gp = g + nidx * CO * hw + p0;
    const bf16* xp = x + nidx * CI * hw + p0;
#pragma unroll
    for (int ko = 0; ko < KO; ++ko)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        R.gt[ko][j] = trow_live(ko) ? *reinterpret_cast<const u2v*>(
                                          gp + (int64_t)(32 * ko + 8 * q4 + j) * hw + 4 * l16)
                                    : u2v{0u, 0u};
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      const int o = 16 * ot + l16;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        R.gr[ot][kk] = o < CO ? *reinterpret_cast<const u4v*>(gp + (int64_t)o * hw + 32 * kk + 8 * q4)
                              : u4v{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        R.sr[mt][kk] = *reinterpret_cast<const u4v*>(xp + (int64_t)(16 * mt + l16) * hw + 32 * kk + 8 * q4);
    if constexpr (HAS_D) {
      const bf16* dp = d + nidx * CI * hw + p0;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          R.dr[mt][kk] = *reinterpret_cast<const u4v*>(dp + (int64_t)(16 * mt + l16) * hw + 32 * kk + 8 * q4);
    }
    if constexpr (BNS) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          R.xr[mt][i] = *reinterpret_cast<const u2v*>(xp + (int64_t)(16 * mt + 4 * q4 + i) * hw + 4 * l16);
    }
  };
  auto compute = [&](int64_t t, const Raw& R) {
    const int64_t nidx = t / tpi, p0 = (t - nidx * tpi) * 64;
    bf16* sp = gs + nidx * CI * hw + p0 + 4 * l16;
    u4v gb[KO][4];
#pragma unroll
    for (int ko = 0; ko < KO; ++ko)
#pragma unroll
      for (int s = 0; s < 4; ++s) gb[ko][s] = frag_raw(R.gt[ko], s);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      f4v acc[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc[s] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ko = 0; ko < KO; ++ko) acc[s] = mfma_bf(wa[mt][ko], gb[ko][s], acc[s]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u2v u{pk(acc[0][i], acc[1][i]), pk(acc[2][i], acc[3][i])};
        __builtin_nontemporal_store(u, reinterpret_cast<u2v*>(sp + (int64_t)(16 * mt + 4 * q4 + i) * hw));
      }
      if constexpr (BNS) {
        int zo = 0;
        asm volatile("" : "+v"(zo));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 16 * mt + 4 * q4 + i + zo;
          const float esc = s_bn[0][c], esh = s_bn[1][c], emu = s_bn[2][c];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float xv = pix(R.xr[mt][i], s);
            const float e = fmaf(xv, esc, esh) > 0.f ? acc[s][i] : 0.f;
            es1[mt][i] += e;
            es2[mt][i] += e * (xv - emu);
          }
        }
      }
    }
    // gW += G . S^T over the tile's 64 pixels (two K = 32 steps)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        u4v sb;
        if constexpr (HAS_D) {  // s as the forward rounded it
          const u4v r = R.sr[mt][kk], dd = R.dr[mt][kk];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sb[e] = pk(rbf(fmaxf(fmaf(lo_f(r[e]), bsc[mt], bsh[mt]), 0.f)) + lo_f(dd[e]),
                       rbf(fmaxf(fmaf(hi_f(r[e]), bsc[mt], bsh[mt]), 0.f)) + hi_f(dd[e]));
        } else if constexpr (BNR) {
          const u4v r = R.sr[mt][kk];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sb[e] = pk(fmaxf(fmaf(lo_f(r[e]), bsc[mt], bsh[mt]), 0.f),
                       fmaxf(fmaf(hi_f(r[e]), bsc[mt], bsh[mt]), 0.f));
        } else {
          sb = R.sr[mt][kk];
        }
#pragma unroll
        for (int ot = 0; ot < OT; ++ot) gw[ot][mt] = mfma_bf(R.gr[ot][kk], sb, gw[ot][mt]);
      }
    }
    if constexpr (HAS_D) {  // the bias gradient: row sums of gy (R layout, fp32)
#pragma unroll
      for (int ot = 0; ot < OT; ++ot)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const u4v q = R.gr[ot][kk];
          gbp[ot] += ((lo_f(q[0]) + hi_f(q[0])) + (lo_f(q[1]) + hi_f(q[1]))) +
                     ((lo_f(q[2]) + hi_f(q[2])) + (lo_f(q[3]) + hi_f(q[3])));
        }
    }
  };
  int64_t t = (int64_t)blockIdx.x * 4 + w;
  if constexpr (!PF) {  // one register set: load, then compute
    Raw A;
    for (; t < tiles; t += stride) {
      load(t, A);
      compute(t, A);
    }
  } else if (t < tiles) {
    Raw A, B;
    load(t, A);
    while (true) {
      load(t + stride, B);
      compute(t, A);
      t += stride;
      if (t >= tiles) break;
      load(t + stride, A);
      compute(t, B);
      t += stride;
      if (t >= tiles) break;
    }
  }
  // gW D layout: o = 16 ot + 4 q4 + i, c = 16 mt + l16
#pragma unroll
  for (int ot = 0; ot < OT; ++ot)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 16 * ot + 4 * q4 + i;
        if (o < CO) red[w][o * CI + 16 * mt + l16] = gw[ot][mt][i];
      }
  if constexpr (BNS) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float a = es1[mt][i], b = es2[mt][i];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          a += __shfl_xor(a, o, 64);
          b += __shfl_xor(b, o, 64);
        }
        if (l16 == 0) {
          const int c = 16 * mt + 4 * q4 + i;
          red[w][SOFF + 2 * c] = a;
          red[w][SOFF + 2 * c + 1] = b;
        }
      }
  }
  if constexpr (HAS_D) {
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      float b = gbp[ot];
      b += __shfl_xor(b, 16, 64);
      b += __shfl_xor(b, 32, 64);
      if (q4 == 0 && 16 * ot + l16 < CO) red[w][CO * CI + 16 * ot + l16] = b;
    }
  }
  __syncthreads();
  float* out = slab + (int64_t)blockIdx.x * ROW;
  for (int i = threadIdx.x; i < ROW; i += 256)
    out[i] = (!HAS_D && i >= CO * CI && i < SOFF) ? 0.f
                                                  : (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

}  // namespace

namespace mde {

#define MDE_PWBF_SHAPES(X) \
  X(16, 8) X(16, 16) X(32, 16) X(32, 32) X(64, 32) X(32, 64) X(16, 32) X(64, 64)

// y = W . relu(x * sc + sh) (sc null: W . x) on bf16 storage; stats (nullable)
// as skip_fwd_mfma_kernel's; grid as the caller sized it (the stats layout).
int pwbf_fwd(const bf16* x, const float* sc, const float* sh, const float* wt, bf16* y,
             float* stats, int64_t n, int64_t cin, int64_t cout, int64_t hw, int blocks,
             hipStream_t s) {
  const double bytes = 2.0 * n * hw * (double)(cin + cout);
  const double flops = 2.0 * n * hw * (double)cin * (double)cout;
#define MDE_PWBF_FWD(A, B)                                                                      \
  if (cin == A && cout == B) {                                                                  \
    if (sc && stats)                                                                            \
      MDE_LAUNCH_MFMA(K_PW_FWD, bytes, flops, s, (pwbf_fwd_kernel<A, B, true, true>),           \
                      dim3(blocks), dim3(256), 0, x, wt, y, n, hw, sc, sh, stats);              \
    else if (stats)                                                                             \
      MDE_LAUNCH_MFMA(K_PW_FWD, bytes, flops, s, (pwbf_fwd_kernel<A, B, false, true>),          \
                      dim3(blocks), dim3(256), 0, x, wt, y, n, hw, sc, sh, stats);              \
    else if (sc)                                                                                \
      MDE_LAUNCH_MFMA(K_PW_FWD, bytes, flops, s, (pwbf_fwd_kernel<A, B, true, false>),          \
                      dim3(blocks), dim3(256), 0, x, wt, y, n, hw, sc, sh, stats);              \
    else                                                                                        \
      MDE_LAUNCH_MFMA(K_PW_FWD, bytes, flops, s, (pwbf_fwd_kernel<A, B, false, false>),         \
                      dim3(blocks), dim3(256), 0, x, wt, y, n, hw, sc, sh, stats);              \
    return MDE_OK;                                                                              \
  }
  MDE_PWBF_SHAPES(MDE_PWBF_FWD)
#undef MDE_PWBF_FWD
  return MDE_ERR_UNSUPPORTED;
}

// gs = W^T gy (through the BN-ReLU operand's gradient), slab rows of gW (and
// with mean: the BN sums); `blocks` slab rows.
int pwbf_bwd(const bf16* gy, const bf16* x, const float* sc, const float* sh, const float* mean,
             const float* wt, bf16* gs, float* slab, int64_t n, int64_t cin, int64_t cout,
             int64_t hw, int blocks, hipStream_t s) {
  const double bytes = 2.0 * n * hw * (double)(cout + 2 * cin);
  const double flops = 4.0 * n * hw * (double)cin * (double)cout;
#define MDE_PWBF_BWD(A, B)                                                                      \
  if (cin == A && cout == B) {                                                                  \
    if (mean) {                                                                                 \
      if constexpr (A <= 32)                                                                    \
        MDE_LAUNCH_MFMA(K_PW_BWD, bytes, flops, s, (pwbf_bwd_kernel<A, B, true, true>),         \
                        dim3(blocks), dim3(256), 0, gy, x, wt, gs, slab, n, hw, sc, sh, mean);  \
      else                                                                                      \
        return MDE_ERR_UNSUPPORTED;                                                             \
    } else if (sc) {                                                                            \
      MDE_LAUNCH_MFMA(K_PW_BWD, bytes, flops, s, (pwbf_bwd_kernel<A, B, true, false>),          \
                      dim3(blocks), dim3(256), 0, gy, x, wt, gs, slab, n, hw, sc, sh, mean);    \
    } else {                                                                                    \
      MDE_LAUNCH_MFMA(K_PW_BWD, bytes, flops, s, (pwbf_bwd_kernel<A, B, false, false>),         \
                      dim3(blocks), dim3(256), 0, gy, x, wt, gs, slab, n, hw, sc, sh, mean);    \
    }                                                                                           \
    return MDE_OK;                                                                              \
  }
  MDE_PWBF_SHAPES(MDE_PWBF_BWD)
#undef MDE_PWBF_BWD
  return MDE_ERR_UNSUPPORTED;
}

// skip_reduce_bn on bf16 storage (64 -> 32, 32 -> 16): out = W . bf16(bf16(
// relu(r * sc + sh)) + d) + bias; the backward's slab rows as skip_slab_reduce
// <0> reads them (gW, gb, [BN sums]).
bool pwbf_skip_ok(int64_t cin, int64_t cout) {
  return (cin == 64 && cout == 32) || (cin == 32 && cout == 16);
}

int pwbf_skip_fwd(const bf16* r, const bf16* d, const float* sc, const float* sh, const float* wt,
                  const float* b, bf16* out, int64_t n, int64_t cin, int64_t cout, int64_t hw,
                  int blocks, hipStream_t s) {
  const double bytes = 2.0 * n * hw * (double)(2 * cin + cout);
  const double flops = 2.0 * n * hw * (double)cin * (double)cout;
  if (cin == 64 && cout == 32)
    MDE_LAUNCH_MFMA(K_SKIP_FWD, bytes, flops, s, (pwbf_fwd_kernel<64, 32, true, false, true>),
                    dim3(blocks), dim3(256), 0, r, wt, out, n, hw, sc, sh, nullptr, d, b);
  else if (cin == 32 && cout == 16)
    MDE_LAUNCH_MFMA(K_SKIP_FWD, bytes, flops, s, (pwbf_fwd_kernel<32, 16, true, false, true>),
                    dim3(blocks), dim3(256), 0, r, wt, out, n, hw, sc, sh, nullptr, d, b);
  else
    return MDE_ERR_UNSUPPORTED;
  return MDE_OK;
}

int pwbf_skip_bwd(const bf16* gy, const bf16* r, const bf16* d, const float* sc, const float* sh,
                  const float* mean, const float* wt, bf16* gs, float* slab, int64_t n,
                  int64_t cin, int64_t cout, int64_t hw, int blocks, hipStream_t s) {
  const double bytes = 2.0 * n * hw * (double)(3 * cin + cout);
  const double flops = 4.0 * n * hw * (double)cin * (double)cout;
  if (cin == 64 && cout == 32 && !mean)
    MDE_LAUNCH_MFMA(K_SKIP_BWD, bytes, flops, s, (pwbf_bwd_kernel<64, 32, true, false, true>),
                    dim3(blocks), dim3(256), 0, gy, r, wt, gs, slab, n, hw, sc, sh, mean, d);
  else if (cin == 32 && cout == 16 && mean)
    MDE_LAUNCH_MFMA(K_SKIP_BWD, bytes, flops, s, (pwbf_bwd_kernel<32, 16, true, true, true>),
                    dim3(blocks), dim3(256), 0, gy, r, wt, gs, slab, n, hw, sc, sh, mean, d);
  else if (cin == 32 && cout == 16)
    MDE_LAUNCH_MFMA(K_SKIP_BWD, bytes, flops, s, (pwbf_bwd_kernel<32, 16, true, false, true>),
                    dim3(blocks), dim3(256), 0, gy, r, wt, gs, slab, n, hw, sc, sh, mean, d);
  else
    return MDE_ERR_UNSUPPORTED;
  return MDE_OK;
}

}  // namespace mde
