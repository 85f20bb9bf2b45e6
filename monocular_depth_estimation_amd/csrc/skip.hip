// Skip fusion of the guided-upsampling block (NCHW, fp32):
//   out[n,o,p] = b[o] + sum_c W[o,c] * (r[n,c,p] + d[n,c,p])
// Reference: `self.reduce(residual + depth)` (src/GuideDepth/model/modules.py:100),
// reduce = nn.Conv2d(in_features, out_features, kernel_size=1) (modules.py:76-78).
// The residual sum is never materialised: forward reads r and d once and
// writes out once; backward re-forms r + d on the fly.
//
// Backward: gs[n,c,p] = sum_o W[o,c] g[n,o,p] (the gradient of both r and d),
// gW = sum_{n,p} g (r+d)^T, gb = sum_{n,p} g.  gW/gb are reduced per block
// into a slab (128-pixel tiles staged in LDS, register-blocked outer products)
// and the slabs are summed in block order by a second kernel, so the result
// is deterministic.
#include "common.h"

namespace {

constexpr int kMaxC = 64;

// BNR (here and in the kernels below): r is the raw input of a BatchNorm +
// ReLU (the comb_conv's last, modules.py:72-73) applied on load,
// s = relu(r * isc[c] + ish[c]) + d, so its output is never written.
template <int CO, int PPT, bool BNR = false, typename T = float>
__global__ void __launch_bounds__(256)
    skip_fwd_kernel(const T* __restrict__ r, const T* __restrict__ d,
                    const float* __restrict__ wt, const float* __restrict__ b,
                    T* __restrict__ out, int64_t n, int cin, int cout,
                    int64_t hw, const float* __restrict__ isc = nullptr,
                    const float* __restrict__ ish = nullptr) {
  __shared__ float sw[kMaxC * kMaxC];
  __shared__ float sb[kMaxC];
  for (int i = threadIdx.x; i < cin * cout; i += blockDim.x) sw[i] = wt[i];
  for (int i = threadIdx.x; i < cout; i += blockDim.x) sb[i] = b[i];
  __syncthreads();
  const int64_t groups = hw / PPT;
  const int64_t total = n * groups;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t nidx = t / groups;
    const int64_t p = (t - nidx * groups) * PPT;
    const T* rp = r + nidx * cin * hw + p;
    const T* dp = d + nidx * cin * hw + p;
    float acc[CO][PPT];
#pragma unroll
    for (int o = 0; o < CO; ++o) {
      const float bo = o < cout ? sb[o] : 0.f;
#pragma unroll
      for (int k = 0; k < PPT; ++k) acc[o][k] = bo;
    }
    for (int c = 0; c < cin; ++c) {
      float s[PPT];
      const float bs = BNR ? isc[c] : 1.f, bh = BNR ? ish[c] : 0.f;
      auto act = [&](float v) { return BNR ? fmaxf(v * bs + bh, 0.f) : v; };
      if (PPT == 4) {
        const float4 a = mde::ld4(rp + c * hw);
        const float4 e = mde::ld4(dp + c * hw);
        s[0] = act(a.x) + e.x; s[1 % PPT] = act(a.y) + e.y;
        s[2 % PPT] = act(a.z) + e.z; s[3 % PPT] = act(a.w) + e.w;
      } else if (PPT == 2) {
        static_assert(PPT != 2 || sizeof(T) == 4, "float2 path is fp32-only");
        const float2 a = *reinterpret_cast<const float2*>(rp + c * hw);
        const float2 e = *reinterpret_cast<const float2*>(dp + c * hw);
        s[0] = act(a.x) + e.x; s[1 % PPT] = act(a.y) + e.y;
      } else {
        s[0] = act(mde::ld1(rp + c * hw)) + mde::ld1(dp + c * hw);
      }
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        if (o < cout) {
          const float wv = sw[o * cin + c];
#pragma unroll
          for (int k = 0; k < PPT; ++k) acc[o][k] += wv * s[k];
        }
      }
    }
    T* op = out + nidx * cout * hw + p;
#pragma unroll
    for (int o = 0; o < CO; ++o) {
      if (o < cout) {
        if (PPT == 4) {
          mde::st4(op + o * hw, make_float4(acc[o][0], acc[o][1 % PPT], acc[o][2 % PPT],
                                           acc[o][3 % PPT]));
        } else if (PPT == 2) {
          *reinterpret_cast<float2*>(op + o * hw) =
              make_float2(acc[o][0], acc[o][1 % PPT]);
        } else {
          mde::st1(op + o * hw, acc[o][0]);
        }
      }
    }
  }
}

constexpr int kTile = 128;  // pixels per LDS tile == threads per block

// FAST: cin == CI and cout == CO exactly; each thread owns an OB x CB block of
// (o, c) pairs for the whole launch.  Otherwise (generic) pairs are strided
// over threads and accumulated in LDS.
template <int CI, int CO, int OB, int CB, bool FAST>
__global__ void __launch_bounds__(kTile)
    skip_bwd_kernel(const float* __restrict__ g, const float* __restrict__ r,
                    const float* __restrict__ d, const float* __restrict__ wt,
                    float* __restrict__ gs, float* __restrict__ slab, int64_t n,
                    int cin, int cout, int64_t hw) {
  extern __shared__ float lds[];
  float* sw = lds;                               // [cout][cin] <= [CO][CI]
  float* gl = sw + CI * CO;                      // [kTile][CO + 1]
  float* sl = gl + kTile * (CO + 1);             // [kTile][CI + 1]
  float* accl = sl + kTile * (CI + 1);           // generic: [cout*cin + cout]
  const int tid = threadIdx.x;
  for (int i = tid; i < cin * cout; i += kTile) sw[i] = wt[i];
  const int npairs = cout * cin;
  if (!FAST)
    for (int i = tid; i < npairs + cout; i += kTile) accl[i] = 0.f;
  // FAST ownership: (ob, cb) block
  constexpr int NCB = CI / CB;
  const int ob = tid / NCB, cb = tid % NCB;
  const bool owner = FAST && ob < CO / OB;
  float acc[OB][CB];
  float accb[OB];
#pragma unroll
  for (int i = 0; i < OB; ++i) {
    accb[i] = 0.f;
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[i][j] = 0.f;
  }
  __syncthreads();

  const int64_t total = n * hw;
  for (int64_t base = (int64_t)blockIdx.x * kTile; base < total;
       base += (int64_t)gridDim.x * kTile) {
    const int64_t q = base + tid;
    float gv[CO];
    if (q < total) {
      const int64_t nidx = q / hw, p = q - nidx * hw;
      const float* gp = g + nidx * cout * hw + p;
#pragma unroll
      for (int o = 0; o < CO; ++o) gv[o] = o < cout ? gp[o * hw] : 0.f;
      const float* rp = r + nidx * cin * hw + p;
      const float* dp = d + nidx * cin * hw + p;
      float* gsp = gs + nidx * cin * hw + p;
      for (int c = 0; c < cin; ++c) {
        const float sv = rp[c * hw] + dp[c * hw];
        sl[tid * (CI + 1) + c] = sv;
        float a = 0.f;
#pragma unroll
        for (int o = 0; o < CO; ++o)
          if (o < cout) a += sw[o * cin + c] * gv[o];
        gsp[c * hw] = a;
      }
    } else {
#pragma unroll
      for (int o = 0; o < CO; ++o) gv[o] = 0.f;
      for (int c = 0; c < cin; ++c) sl[tid * (CI + 1) + c] = 0.f;
    }
#pragma unroll
    for (int o = 0; o < CO; ++o) gl[tid * (CO + 1) + o] = gv[o];
    __syncthreads();
    if (FAST) {
      if (owner) {
        for (int p = 0; p < kTile; ++p) {
          float gg[OB], ss[CB];
#pragma unroll
          for (int i = 0; i < OB; ++i) gg[i] = gl[p * (CO + 1) + ob * OB + i];
#pragma unroll
          for (int j = 0; j < CB; ++j) ss[j] = sl[p * (CI + 1) + cb * CB + j];
#pragma unroll
          for (int i = 0; i < OB; ++i) {
            if (cb == 0) accb[i] += gg[i];
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[i][j] += gg[i] * ss[j];
          }
        }
      }
    } else {
      for (int pr = tid; pr < npairs + cout; pr += kTile) {
        float a = 0.f;
        if (pr < npairs) {
          const int o = pr / cin, c = pr % cin;
          for (int p = 0; p < kTile; ++p)
            a += gl[p * (CO + 1) + o] * sl[p * (CI + 1) + c];
        } else {
          const int o = pr - npairs;
          for (int p = 0; p < kTile; ++p) a += gl[p * (CO + 1) + o];
        }
        accl[pr] += a;
      }
    }
    __syncthreads();
  }

  float* out = slab + (int64_t)blockIdx.x * (npairs + cout);
  if (FAST) {
    if (owner) {
#pragma unroll
      for (int i = 0; i < OB; ++i) {
        const int o = ob * OB + i;
#pragma unroll
        for (int j = 0; j < CB; ++j) out[o * cin + cb * CB + j] = acc[i][j];
        if (cb == 0) out[npairs + o] = accb[i];
      }
    }
  } else {
    for (int pr = tid; pr < npairs + cout; pr += kTile) out[pr] = accl[pr];
  }
}

// cout == 1 (up_3's 16 -> 1 reduce): a thread owns 4 channels of a 4-pixel
// quad (lane % NG = channel group, NG = CI / 4), so its weight-gradient /
// BN-sum accumulators are 4 + 8 registers instead of all channels' (a
// thread-per-quad kernel holding all channels needed 358 registers with the
// BN sums: one wave per SIMD, 537 us at cfg2's up_3).  The one gradient
// channel g is re-read by the NG lanes of a quad (an L1 hit).
// BNR: s = relu(r * isc + ish) + d (see skip_fwd_kernel); BNS (with BNR):
// also that BatchNorm's backward sums sum e, sum e (r - imean[c]) with
// e = gs [r * isc + ish > 0].  Slab row: [CI] weight gradient, [1] bias
// gradient, [2 CI] BN sums.
template <int CI, bool BNR = false, bool BNS = false, typename T = float>
__global__ void __launch_bounds__(256)
    skip_bwd_c1_kernel(const T* __restrict__ g, const T* __restrict__ r,
                       const T* __restrict__ d, const float* __restrict__ wt,
                       T* __restrict__ gs, float* __restrict__ slab, int64_t n, int64_t hw,
                       const float* __restrict__ isc = nullptr,
                       const float* __restrict__ ish = nullptr,
                       const float* __restrict__ imean = nullptr) {
  static_assert(CI % 4 == 0 && (!BNS || BNR), "channel groups of 4; BN sums need BNR");
  constexpr int NG = CI / 4, QPB = 256 / NG;  // channel groups, quads per block pass
  constexpr int ROW = CI + 1 + (BNS ? 2 * CI : 0);
  __shared__ float red[4][ROW];
  const int tid = threadIdx.x, grp = tid % NG, qi = tid / NG;
  float w[4], bs[4], bh[4], mu[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * grp + k;
    w[k] = wt[c];
    bs[k] = BNR ? isc[c] : 1.f;
    bh[k] = BNR ? ish[c] : 0.f;
    mu[k] = BNS ? imean[c] : 0.f;
  }
  float aw[4] = {}, e1[4] = {}, e2[4] = {}, ab = 0.f;
  const int64_t q4 = hw >> 2, total = n * q4;
  for (int64_t t = (int64_t)blockIdx.x * QPB + qi; t < total; t += (int64_t)gridDim.x * QPB) {
    const int64_t nidx = t / q4, p = (t - nidx * q4) << 2;
    const float4 gv = mde::ld4(g + nidx * hw + p);
    if (grp == 0) ab += (gv.x + gv.y) + (gv.z + gv.w);
    const int64_t base = (nidx * CI + 4 * grp) * hw + p;
    float4 a[4], e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] = mde::ld4(r + base + k * hw);
      e[k] = mde::ld4(d + base + k * hw);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      auto act = [&](float v) { return BNR ? fmaxf(v * bs[k] + bh[k], 0.f) : v; };
      const float4 sv = make_float4(act(a[k].x) + e[k].x, act(a[k].y) + e[k].y,
                                    act(a[k].z) + e[k].z, act(a[k].w) + e[k].w);
      aw[k] += (gv.x * sv.x + gv.y * sv.y) + (gv.z * sv.z + gv.w * sv.w);
      const float4 o4 = make_float4(w[k] * gv.x, w[k] * gv.y, w[k] * gv.z, w[k] * gv.w);
      mde::st4(gs + base + k * hw, o4);
      if constexpr (BNS) {
        const float av[4] = {a[k].x, a[k].y, a[k].z, a[k].w}, ov[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float ev = av[j] * bs[k] + bh[k] > 0.f ? ov[j] : 0.f;
          e1[k] += ev;
          e2[k] += ev * (av[j] - mu[k]);
        }
      }
    }
  }
  // lanes of one channel group: lane % NG equal -> butterfly over xor NG .. 32
  auto gsum = [&](float v) {
#pragma unroll
    for (int o = NG; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
  };
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float sw = gsum(aw[k]);
    float s1 = 0.f, s2 = 0.f;
    if constexpr (BNS) {
      s1 = gsum(e1[k]);
      s2 = gsum(e2[k]);
    }
    if (lane < NG) {
      const int c = 4 * lane + k;
      red[wv][c] = sw;
      if constexpr (BNS) {
        red[wv][CI + 1 + 2 * c] = s1;
        red[wv][CI + 1 + 2 * c + 1] = s2;
      }
    }
  }
  const float sb = gsum(ab);  // only group-0 lanes hold bias partials
  if (lane == 0) red[wv][CI] = sb;
  __syncthreads();
  for (int i = tid; i < ROW; i += 256)
    slab[(int64_t)blockIdx.x * ROW + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// MFMA backward for the full-size blocks (64 -> 32 at H/4, 32 -> 16 at H/2;
// hw % 64 == 0).  Each wave walks 64-pixel tiles of one image:
//   gs tile [CI x 64] = W^T [CI x CO] . G [CO x 64]    (K = CO, W^T held in
//       registers as A operands; G read per lane as B, 16 lanes = 64 B rows)
//   gW [CO x CI] += G [CO x 64] . S^T [64 x CI]       (K = pixels with a
//       permuted order: lane group q supplies pixels 16v + 4q .. +3, v = 0..3,
//       so A and B are 4 float4 loads per lane and the four lane groups of a
//       row read 64 contiguous bytes per instruction; S = r + d formed in
//       registers)
//   gb [CO] += row sums of G
// v_mfma_f32_16x16x4_f32 throughout (exact f32 products).  The gW/gb
// accumulators stay in registers for the whole launch and are combined over
// the block's 4 waves in a fixed order into the block's slab row.
using f4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// BNR: the input is r' = relu(r * isc[c] + ish[c]) (a BatchNorm + ReLU fused
// into this conv's operand load; r is the BN input), recomputed for gW; gs is
// then the gradient w.r.t. r' (the BN backward applies the ReLU mask).
// BNS (with BNR): also the BN backward's two reductions, e = gs * [r * isc +
// ish > 0]: sum e and sum e * (r - imean[c]) per channel, from the gs tile in
// registers and r re-read in the gs layout (the same tile the gW part reads,
// an L1 / L2 hit) -- appended to the block's slab row, so the separate BN
// reduce pass over (gs, r) is never run.
// T: storage type of g, r, d, gs (float, or bf16 under autocast; products
// and sums in fp32 either way).
template <int CI, int CO, bool HAS_D, bool BNR = false, bool BNS = false, typename T = float>
__global__ void __launch_bounds__(256, CI * CO >= 4096 ? 1 : 2)  // 64 x 64: W^T + gW need > 256 registers
    skip_bwd_mfma_kernel(const T* __restrict__ g, const T* __restrict__ r,
                         const T* __restrict__ d, const float* __restrict__ wt,
                         T* __restrict__ gs, float* __restrict__ slab, int64_t n,
                         int64_t hw, const float* __restrict__ isc = nullptr,
                         const float* __restrict__ ish = nullptr,
                         const float* __restrict__ imean = nullptr) {
  // CO may be 8: the M tiles of gW = G S^T are then half-empty (rows >= CO
  // are zero operands and are not stored); K of gs = W^T G is CO in steps of 4.
  constexpr int MT = CI / 16, OT = (CO + 15) / 16, KO = CO / 4;
  static_assert(CI % 16 == 0 && CO % 8 == 0, "tile shapes");
  static_assert(!BNS || (BNR && CI <= 32), "BN sums: fused BN-ReLU operand, cin <= 32");
  constexpr int ROW = CO * CI + CO + (BNS ? 2 * CI : 0);  // slab row
  __shared__ float red[4][ROW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q4 = lane >> 4;
  // A operands of gs = W^T G: lane (c = 16mt + l16, o = 4kk + q4) -> W[o][c]
  float wa[MT][KO];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int kk = 0; kk < KO; ++kk) wa[mt][kk] = wt[(4 * kk + q4) * CI + 16 * mt + l16];
  f4 gw[OT][MT];
#pragma unroll
  for (int ot = 0; ot < OT; ++ot)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) gw[ot][mt] = f4{0.f, 0.f, 0.f, 0.f};
  float gbp[OT] = {};
  float bsc[MT], bsh[MT];  // BNR: channel c = 16 mt + l16
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    bsc[mt] = BNR ? isc[16 * mt + l16] : 1.f;
    bsh[mt] = BNR ? ish[16 * mt + l16] : 0.f;
  }
  // BNS: channel 16 mt + 4 q4 + i (the gs layout) coefficients and running
  // sums in registers (cin <= 32: measured faster than LDS-held coefficients
  // with per-tile wave sums; at cin 64 neither beats the separate reduce pass)
  constexpr int SOFF = CO * CI + CO;
  float esc[BNS ? MT : 1][4], esh[BNS ? MT : 1][4], emu[BNS ? MT : 1][4];
  float es1[BNS ? MT : 1][4], es2[BNS ? MT : 1][4];
  if constexpr (BNS) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 16 * mt + 4 * q4 + i;
        esc[mt][i] = isc[c];
        esh[mt][i] = ish[c];
        emu[mt][i] = imean[c];
        es1[mt][i] = 0.f;
        es2[mt][i] = 0.f;
      }
  }
  const int64_t tpi = hw / 64;
  const int64_t tiles = n * tpi;
  for (int64_t t = (int64_t)blockIdx.x * 4 + w; t < tiles; t += (int64_t)gridDim.x * 4) {
    const int64_t nidx = t / tpi, p0 = (t - nidx * tpi) * 64;
    const T* gp = g + nidx * CO * hw + p0;
    const T* rp = r + nidx * CI * hw + p0;
    const T* dp = HAS_D ? d + nidx * CI * hw + p0 : nullptr;
    T* sp = gs ? gs + nidx * CI * hw + p0 : nullptr;
    // gs = W^T G with the forward's permuted pixel order: lane (l16, q4) loads
    // pixels 4*l16 .. 4*l16+3 of G row 4kk + q4 as one float4, component j
    // feeds sub-tile j, and each gs row leaves as one float4 per lane (full
    // 256-byte row segments both ways).
    if (sp) {
      float4 gb[KO];
#pragma unroll
      for (int kk = 0; kk < KO; ++kk)
        gb[kk] = mde::ld4(gp + (4 * kk + q4) * hw + 4 * l16);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f4 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KO; ++kk) {
          acc[0] = mfma4(wa[mt][kk], gb[kk].x, acc[0]);
          acc[1] = mfma4(wa[mt][kk], gb[kk].y, acc[1]);
          acc[2] = mfma4(wa[mt][kk], gb[kk].z, acc[2]);
          acc[3] = mfma4(wa[mt][kk], gb[kk].w, acc[3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          mde::st4_nt(sp + (16 * mt + 4 * q4 + i) * hw + 4 * l16,
                      make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]));
        if constexpr (BNS) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float4 x = mde::ld4(rp + (16 * mt + 4 * q4 + i) * hw + 4 * l16);
            const float xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float e = xv[j] * esc[mt][i] + esh[mt][i] > 0.f ? acc[j][i] : 0.f;
              es1[mt][i] += e;
              es2[mt][i] += e * (xv[j] - emu[mt][i]);
            }
          }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // gW += G S^T over this tile's 64 pixels (lane group q4: pixels 16 q4 ..).
    // Up to 32 output channels the G operands of all M tiles stay in
    // registers and S is read once; beyond, one M tile at a time (S re-read
    // from L2) keeps the kernel out of scratch.
    constexpr int OG = OT <= 2 ? OT : 1;
#pragma unroll
    for (int og = 0; og < OT; og += OG) {
      float ga[OG][16];
#pragma unroll
      for (int oo = 0; oo < OG; ++oo) {
        const int ot = og + oo;
        const int o = 16 * ot + l16;
        if (o < CO) {
          // pixels 16v + 4q4 .. +3: the 4 lane groups of a row read 64
          // contiguous bytes per instruction (same order for S below)
          const T* src = gp + o * hw + 4 * q4;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const float4 x = mde::ld4(src + 16 * v);
            ga[oo][4 * v] = x.x; ga[oo][4 * v + 1] = x.y;
            ga[oo][4 * v + 2] = x.z; ga[oo][4 * v + 3] = x.w;
            gbp[ot] += (x.x + x.y) + (x.z + x.w);
          }
        } else {
#pragma unroll
          for (int k = 0; k < 16; ++k) ga[oo][k] = 0.f;
        }
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const T* ra = rp + (16 * mt + l16) * hw + 4 * q4;
        float sb[16];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          float4 x = mde::ld4(ra + 16 * v);
          if (BNR) {  // BN + ReLU of r, then + d (HAS_D)
            x.x = fmaxf(x.x * bsc[mt] + bsh[mt], 0.f);
            x.y = fmaxf(x.y * bsc[mt] + bsh[mt], 0.f);
            x.z = fmaxf(x.z * bsc[mt] + bsh[mt], 0.f);
            x.w = fmaxf(x.w * bsc[mt] + bsh[mt], 0.f);
          }
          if (HAS_D) {
            const float4 y = mde::ld4(dp + (16 * mt + l16) * hw + 4 * q4 + 16 * v);
            x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
          }
          sb[4 * v] = x.x; sb[4 * v + 1] = x.y; sb[4 * v + 2] = x.z; sb[4 * v + 3] = x.w;
        }
#pragma unroll
        for (int oo = 0; oo < OG; ++oo)
#pragma unroll
          for (int k = 0; k < 16; ++k) gw[og + oo][mt] = mfma4(ga[oo][k], sb[k], gw[og + oo][mt]);
      }
    }
  }
  // gW C layout: o = 16ot + 4 q4 + i, c = 16mt + l16; gb: sum over the 4 lane groups
#pragma unroll
  for (int ot = 0; ot < OT; ++ot) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 16 * ot + 4 * q4 + i;
        if (o < CO) red[w][o * CI + 16 * mt + l16] = gw[ot][mt][i];
      }
    float b = gbp[ot];
    b += __shfl_xor(b, 16, 64);
    b += __shfl_xor(b, 32, 64);
    if (q4 == 0 && 16 * ot + l16 < CO) red[w][CO * CI + 16 * ot + l16] = b;
  }
  if constexpr (BNS) {
    // sum over the 16 lanes (pixel columns) of each lane group, fixed butterfly
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
  __syncthreads();
  float* out = slab + (int64_t)blockIdx.x * ROW;
  for (int i = threadIdx.x; i < ROW; i += 256)
    out[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// The pointwise backward (BN + ReLU operand, optional BNS sums) on bf16
// storage with the NEXT tile's operands in flight during this tile's math:
// the same arithmetic, operand layouts and summation order as
// skip_bwd_mfma_kernel<CI, CO, false, true, BNS, bf16> (so bit-identical
// results), but its tiles ran as 3-4 dependent load -> use round trips at four
// waves per SIMD (SQ counters, tools/gpu_r05j.sh: 60 % of wave time waiting
// on memory).  Here each tile's raw bf16 operands -- G in both lane layouts,
// the input rows for the weight gradient and (BNS) for the BN sums -- are
// loaded one tile ahead into one of two register sets (the loop is unrolled
// by two so both sets have fixed registers), and gs leaves through the
// hardware bf16 conversion.
// T = float (the fp32 step, 16 input channels): the same kernel on float4
// operands (4 pixels a load either way).
template <typename T>
using PwWord = std::conditional_t<std::is_same_v<T, mde::bf16>, uint2, float4>;

template <int CI, int CO, bool BNS, typename T = mde::bf16>
struct PwRaw {
  static constexpr int MT = CI / 16, OT = (CO + 15) / 16, KO = CO / 4;
  static constexpr int OG = OT <= 2 ? OT : 1;
  PwWord<T> gb[KO];               // G rows 4 kk + q4, pixels 4 l16 .. + 3
  PwWord<T> ga[OT][4];            // G rows 16 ot + l16, pixels 16 v + 4 q4 .. + 3
  PwWord<T> sr[MT][4];            // input rows 16 mt + l16, pixels 16 v + 4 q4 ..
  PwWord<T> xr[BNS ? MT : 1][4];  // input rows 16 mt + 4 q4 + i, pixels 4 l16 ..
};

__device__ __forceinline__ float4 unpack_bf4(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ float4 unpack_bf4(float4 u) { return u; }

template <int CI, int CO, bool BNS, typename T = mde::bf16>
__global__ void __launch_bounds__(256, CI * CO >= 4096 ? 1 : 2)
    pw_bwd_pf_kernel(const T* __restrict__ g, const T* __restrict__ r,
                     const float* __restrict__ wt, T* __restrict__ gs,
                     float* __restrict__ slab, int64_t n, int64_t hw,
                     const float* __restrict__ isc, const float* __restrict__ ish,
                     const float* __restrict__ imean) {
  using Raw = PwRaw<CI, CO, BNS, T>;
  using W = PwWord<T>;
  constexpr int MT = Raw::MT, OT = Raw::OT, KO = Raw::KO, OG = Raw::OG;
  static_assert(CI % 16 == 0 && CO % 8 == 0, "tile shapes");
  static_assert(!BNS || CI <= 32, "BN sums: cin <= 32");
  constexpr int ROW = CO * CI + CO + (BNS ? 2 * CI : 0);  // slab row (bias columns unused)
  __shared__ float red[4][ROW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q4 = lane >> 4;
  float wa[MT][KO];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int kk = 0; kk < KO; ++kk) wa[mt][kk] = wt[(4 * kk + q4) * CI + 16 * mt + l16];
  f4 gw[OT][MT];
#pragma unroll
  for (int ot = 0; ot < OT; ++ot)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) gw[ot][mt] = f4{0.f, 0.f, 0.f, 0.f};
  float bsc[MT], bsh[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    bsc[mt] = isc[16 * mt + l16];
    bsh[mt] = ish[16 * mt + l16];
  }
  constexpr int SOFF = CO * CI + CO;
  float esc[BNS ? MT : 1][4], esh[BNS ? MT : 1][4], emu[BNS ? MT : 1][4];
  float es1[BNS ? MT : 1][4], es2[BNS ? MT : 1][4];
  if constexpr (BNS) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 16 * mt + 4 * q4 + i;
        esc[mt][i] = isc[c];
        esh[mt][i] = ish[c];
        emu[mt][i] = imean[c];
        es1[mt][i] = 0.f;
        es2[mt][i] = 0.f;
      }
  }
  const int64_t tpi = hw / 64;
  const int64_t tiles = n * tpi;
  const int64_t stride = (int64_t)gridDim.x * 4;
  // always a valid tile: past the end the last tile is loaded again (unused),
  // so every iteration issues the same loads (straight-line vmcnt counts)
  auto load = [&](int64_t t, Raw& R) {
    if (t >= tiles) t = tiles - 1;
    const int64_t nidx = t / tpi, p0 = (t - nidx * tpi) * 64;
    const T* gp = g + nidx * CO * hw + p0;
    const T* rp = r + nidx * CI * hw + p0;
#pragma unroll
    for (int kk = 0; kk < KO; ++kk)
      R.gb[kk] = *reinterpret_cast<const W*>(gp + (4 * kk + q4) * hw + 4 * l16);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      const int o = 16 * ot + l16 < CO ? 16 * ot + l16 : CO - 1;
#pragma unroll
      for (int v = 0; v < 4; ++v)
        R.ga[ot][v] = *reinterpret_cast<const W*>(gp + o * hw + 4 * q4 + 16 * v);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        R.sr[mt][v] = *reinterpret_cast<const W*>(rp + (16 * mt + l16) * hw + 4 * q4 + 16 * v);
    if constexpr (BNS) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          R.xr[mt][i] = *reinterpret_cast<const W*>(rp + (16 * mt + 4 * q4 + i) * hw + 4 * l16);
    }
  };
  auto compute = [&](int64_t t, const Raw& R) {
    const int64_t nidx = t / tpi, p0 = (t - nidx * tpi) * 64;
    T* sp = gs + nidx * CI * hw + p0;
    float4 gb[KO];
#pragma unroll
    for (int kk = 0; kk < KO; ++kk) gb[kk] = unpack_bf4(R.gb[kk]);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      f4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KO; ++kk) {
        acc[0] = mfma4(wa[mt][kk], gb[kk].x, acc[0]);
        acc[1] = mfma4(wa[mt][kk], gb[kk].y, acc[1]);
        acc[2] = mfma4(wa[mt][kk], gb[kk].z, acc[2]);
        acc[3] = mfma4(wa[mt][kk], gb[kk].w, acc[3]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (std::is_same_v<T, mde::bf16>) {
          using bf2 = __bf16 __attribute__((ext_vector_type(2)));
          const bf2 lo = {(__bf16)acc[0][i], (__bf16)acc[1][i]};
          const bf2 hi = {(__bf16)acc[2][i], (__bf16)acc[3][i]};
          const mde::nt2u u{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
          __builtin_nontemporal_store(u, reinterpret_cast<mde::nt2u*>(sp + (16 * mt + 4 * q4 + i) * hw + 4 * l16));
        } else {
          mde::st4_nt(sp + (16 * mt + 4 * q4 + i) * hw + 4 * l16,
                      make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]));
        }
      }
      if constexpr (BNS) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 x = unpack_bf4(R.xr[mt][i]);
          const float xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float e = xv[j] * esc[mt][i] + esh[mt][i] > 0.f ? acc[j][i] : 0.f;
            es1[mt][i] += e;
            es2[mt][i] += e * (xv[j] - emu[mt][i]);
          }
        }
      }
    }
#pragma unroll
    for (int og = 0; og < OT; og += OG) {
      float ga[OG][16];
#pragma unroll
      for (int oo = 0; oo < OG; ++oo) {
        const int ot = og + oo;
        const bool live = 16 * ot + l16 < CO;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float4 x = unpack_bf4(R.ga[ot][v]);
          ga[oo][4 * v] = live ? x.x : 0.f;
          ga[oo][4 * v + 1] = live ? x.y : 0.f;
          ga[oo][4 * v + 2] = live ? x.z : 0.f;
          ga[oo][4 * v + 3] = live ? x.w : 0.f;
        }
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float sb[16];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float4 x = unpack_bf4(R.sr[mt][v]);
          sb[4 * v] = fmaxf(x.x * bsc[mt] + bsh[mt], 0.f);
          sb[4 * v + 1] = fmaxf(x.y * bsc[mt] + bsh[mt], 0.f);
          sb[4 * v + 2] = fmaxf(x.z * bsc[mt] + bsh[mt], 0.f);
          sb[4 * v + 3] = fmaxf(x.w * bsc[mt] + bsh[mt], 0.f);
        }
#pragma unroll
        for (int oo = 0; oo < OG; ++oo)
#pragma unroll
          for (int k = 0; k < 16; ++k) gw[og + oo][mt] = mfma4(ga[oo][k], sb[k], gw[og + oo][mt]);
      }
    }
  };
  int64_t t = (int64_t)blockIdx.x * 4 + w;
  if (t < tiles) {
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
  // gW C layout: o = 16ot + 4 q4 + i, c = 16mt + l16
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
  __syncthreads();
  float* out = slab + (int64_t)blockIdx.x * ROW;
  for (int i = threadIdx.x; i < ROW; i += 256)
    out[i] = (i >= CO * CI && i < SOFF) ? 0.f : (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// MFMA forward for the full-size blocks (hw % 64 == 0): each wave computes a
// [CO x 64] output tile = W [CO x CI] . S [CI x 64] (+ bias), S = r + d.
// Pixel order is permuted so every access is a full 256-byte row segment:
// lane (l16, q4) loads one float4 = pixels 4*l16 .. 4*l16+3 of channel
// 4kk + q4, and component j of it feeds MFMA sub-tile j (column l16 <->
// pixel 4*l16 + j); the four sub-tiles' accumulators then hold, per lane,
// four consecutive pixels of one output row -- stored as one float4.  W sits
// in registers as the A operands for the whole launch.
// BNR: operand r' = relu(r * isc[c] + ish[c]) (BatchNorm + ReLU of the
// producer fused into the load, so r' is never written to HBM).
// STATS: also the output's per-channel shifted sums over this block's tiles
// -> stats[(o * gridDim.x + block) * 4] = (shift, count, sum (y - shift),
// sum (y - shift)^2): the following BatchNorm's statistics without re-reading
// the output (mde_batchnorm_*_stats).
// T: storage type of r, d, out (float, or bf16 under autocast).
template <int CI, int CO, bool HAS_D, bool BNR = false, bool STATS = false, typename T = float>
__global__ void __launch_bounds__(256)
    skip_fwd_mfma_kernel(const T* __restrict__ r, const T* __restrict__ d,
                         const float* __restrict__ wt, const float* __restrict__ b,
                         T* __restrict__ out, int64_t n, int64_t hw,
                         const float* __restrict__ isc = nullptr,
                         const float* __restrict__ ish = nullptr,
                         float* __restrict__ stats = nullptr, int out_cs = CO) {
  // out_cs: output channels per image (> CO when one launch writes a channel
  // slice of a wider output: the 64 -> 64 pointwise as two 64 -> 32 halves)
  constexpr int OT = (CO + 15) / 16, KC = CI / 4;
  static_assert(CI % 16 == 0 && CO % 8 == 0, "tile shapes");
  // Registers (the 64-input-channel variants ran at one wave per SIMD): the
  // BN scale / shift are read from LDS per use (an opaque index keeps the
  // compiler from hoisting them back into 2 KC registers), the bias exists
  // only with HAS_D (the skip fusion; the pointwise convs have none), and the
  // statistics keep (shift, s1, s2) per channel with one wave-uniform count.
  constexpr bool HB = HAS_D;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q4 = lane >> 4;
  __shared__ float s_bn[BNR ? 2 : 1][BNR ? CI : 1];
  if constexpr (BNR) {
    if (threadIdx.x < CI) {
      s_bn[0][threadIdx.x] = isc[threadIdx.x];
      s_bn[1][threadIdx.x] = ish[threadIdx.x];
    }
    __syncthreads();
  }
  float wa[OT][KC];  // W[o = 16ot + l16][c = 4kk + q4] (0 for o >= CO)
#pragma unroll
  for (int ot = 0; ot < OT; ++ot)
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      const int o = 16 * ot + l16;
      wa[ot][kk] = o < CO ? wt[o * CI + 4 * kk + q4] : 0.f;
    }
  float bo[HB ? OT : 1][4];
#pragma unroll
  for (int ot = 0; ot < (HB ? OT : 1); ++ot)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = 16 * ot + 4 * q4 + i;
      bo[ot][i] = (HB && b && o < CO) ? b[o] : 0.f;
    }
  // channel 16 ot + 4 q4 + i, this lane's pixels: shift, sum d, sum d^2 (every
  // pixel of a tile is valid: hw % 64 == 0, so the count is 4 per tile)
  float rref[STATS ? OT : 1][4], rs1[STATS ? OT : 1][4], rs2[STATS ? OT : 1][4];
#pragma unroll
  for (int ot = 0; ot < (STATS ? OT : 1); ++ot)
#pragma unroll
    for (int i = 0; i < 4; ++i) rref[ot][i] = rs1[ot][i] = rs2[ot][i] = 0.f;
  int ntile = 0;
  bool first = true;  // wave-uniform: the wave's first tile sets the shifts
  const int tpi = (int)(hw / 64);
  const int64_t tiles = n * tpi;
  for (int64_t t = (int64_t)blockIdx.x * 4 + w; t < tiles; t += (int64_t)gridDim.x * 4) {
    const int64_t nidx = t / tpi, p0 = (t - nidx * tpi) * 64;
    const T* rp = r + nidx * CI * hw + p0 + 4 * l16;
    const T* dp = HAS_D ? d + nidx * CI * hw + p0 + 4 * l16 : nullptr;
    T* op = out + nidx * out_cs * hw + p0 + 4 * l16;
    float4 sb[KC];
    int zo = 0;  // opaque 0: the LDS reads below stay in the loop
    asm volatile("" : "+v"(zo));
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      const int64_t off = (int64_t)(4 * kk + q4) * hw;
      float4 v = mde::ld4_nt(rp + off);  // streamed: read once (nontemporal)
      if constexpr (BNR) {  // BN + ReLU of r, then + d (HAS_D)
        const float fsc = s_bn[0][4 * kk + q4 + zo], fsh = s_bn[1][4 * kk + q4 + zo];
        v.x = fmaxf(v.x * fsc + fsh, 0.f);
        v.y = fmaxf(v.y * fsc + fsh, 0.f);
        v.z = fmaxf(v.z * fsc + fsh, 0.f);
        v.w = fmaxf(v.w * fsc + fsh, 0.f);
      }
      if (HAS_D) {
        const float4 e = mde::ld4_nt(dp + off);
        v.x += e.x; v.y += e.y; v.z += e.z; v.w += e.w;
      }
      sb[kk] = v;
    }
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      f4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j] = HB ? f4{bo[ot][0], bo[ot][1], bo[ot][2], bo[ot][3]} : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KC; ++kk) {
        acc[0] = mfma4(wa[ot][kk], sb[kk].x, acc[0]);
        acc[1] = mfma4(wa[ot][kk], sb[kk].y, acc[1]);
        acc[2] = mfma4(wa[ot][kk], sb[kk].z, acc[2]);
        acc[3] = mfma4(wa[ot][kk], sb[kk].w, acc[3]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 16 * ot + 4 * q4 + i;
        if (o < CO)
          mde::st4_nt(op + (int64_t)o * hw, make_float4(acc[0][i], acc[1][i], acc[2][i], acc[3][i]));
        if constexpr (STATS) {
          // statistics of the values as stored (bf16-rounded under autocast)
          float vs[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            vs[j] = sizeof(T) == 2 ? mde::bf2f(mde::f2bf(acc[j][i])) : acc[j][i];
          // one shift per channel and wave: lane l16 = 0's first value, so the
          // 16 lanes of a group sum their (n, s1, s2) plainly at the end
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
  }
  if constexpr (STATS) {
    // the 16 lanes of a lane group share the channels' shifts: plain-sum
    // butterfly, then the 4 waves in order through LDS (re-expressed on wave
    // 0's shift), then one (shift, count, s1, s2) per channel and block
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

// gw[pair] = sum over blocks of slab[block][pair]: one block per pair, fixed
// per-thread order then a fixed tree -> deterministic.  TAG only tells the
// two callers apart in profiles (0: skip fusion, 1: pointwise 1x1 backward).
template <int TAG>
__global__ void __launch_bounds__(256)
    skip_slab_reduce_kernel(const float* __restrict__ slab, int nblocks,
                            int npairs, int cout, float* __restrict__ gw,
                            float* __restrict__ gb, int nextra = 0,
                            float* __restrict__ extra = nullptr) {
  __shared__ float red[4];
  const int t = blockIdx.x;
  const int stride = npairs + cout + nextra;
  float a = 0.f;
  for (int k = threadIdx.x; k < nblocks; k += 256) a += slab[(int64_t)k * stride + t];
  a = mde::block_sum256(a, red);
  if (threadIdx.x == 0) {
    if (t < npairs)
      gw[t] = a;
    else if (t < npairs + cout)
      { if (gb) gb[t - npairs] = a; }
    else
      extra[t - npairs - cout] = a;
  }
}

inline int bwd_blocks(int64_t n, int64_t hw) {
  const int64_t t = mde::cdiv(n * hw, kTile);
  return (int)(t < 1 ? 1 : (t > 1024 ? 1024 : t));
}

template <int CI, int CO, bool FAST>
constexpr size_t bwd_lds() {
  return sizeof(float) * (CI * CO + kTile * (CO + 1) + kTile * (CI + 1) +
                          (FAST ? 0 : CI * CO + CO));
}

}  // namespace

extern "C" {

// bf16 storage (autocast) on the MFMA shapes only: 64 -> 32 and 32 -> 16
// with h*w % 64 == 0 (the full-size decoder blocks); others are fp32-only.
static bool skip_mfma_shape(int64_t cin, int64_t cout, int64_t hw) {
  return hw % 64 == 0 && ((cin == 64 && cout == 32) || (cin == 32 && cout == 16));
}

int mde_skip_reduce_fwd(const void* r, const void* d, const float* wt,
                        const float* b, void* out, int64_t n, int64_t cin,
                        int64_t cout, int64_t h, int64_t w, int dtype,
                        void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  const int64_t hw = h * w;
  if (!r || !d || !wt || !b || !out || n <= 0 || hw <= 0 || cin <= 0 ||
      cout <= 0 || cin > kMaxC || cout > kMaxC)
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MDE_BF16) {
    if (!skip_mfma_shape(cin, cout, hw)) return MDE_ERR_UNSUPPORTED;
    const int64_t blocks = mde::cdiv(n * hw / 64, 4);
    const dim3 g((unsigned)(blocks > 4096 ? 4096 : blocks));
    const double bb = 2.0 * n * hw * (double)(2 * cin + cout);
    using B = mde::bf16;
    if (cin == 64)
      MDE_LAUNCH(mde::K_SKIP_FWD, bb, s, (skip_fwd_mfma_kernel<64, 32, true, false, false, B>), g,
                 dim3(256), 0, (const B*)r, (const B*)d, wt, b, (B*)out, n, hw, nullptr, nullptr,
                 nullptr);
    else
      MDE_LAUNCH(mde::K_SKIP_FWD, bb, s, (skip_fwd_mfma_kernel<32, 16, true, false, false, B>), g,
                 dim3(256), 0, (const B*)r, (const B*)d, wt, b, (B*)out, n, hw, nullptr, nullptr,
                 nullptr);
    return MDE_OK;
  }
  const double bytes = 4.0 * n * hw * (double)(2 * cin + cout);
  auto grid = [&](int ppt) {
    const int64_t blocks = mde::cdiv(n * hw / ppt, 256);
    return dim3((unsigned)(blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks)));
  };
#define SKIP_FWD(CO_, PPT_)                                                  \
  MDE_LAUNCH(mde::K_SKIP_FWD, bytes, s, (skip_fwd_kernel<CO_, PPT_>),        \
             grid(PPT_), dim3(256), 0, (const float*)r, (const float*)d, wt, \
             b, (float*)out, n, (int)cin, (int)cout, hw)
  auto mgrid = [&]() {
    const int64_t blocks = mde::cdiv(n * hw / 64, 4);
    return dim3((unsigned)(blocks > 4096 ? 4096 : blocks));
  };
  if (cin == 64 && cout == 32 && hw % 64 == 0) {
    MDE_LAUNCH(mde::K_SKIP_FWD, bytes, s, (skip_fwd_mfma_kernel<64, 32, true>), mgrid(), dim3(256), 0,
               (const float*)r, (const float*)d, wt, b, (float*)out, n, hw);
  } else if (cin == 32 && cout == 16 && hw % 64 == 0) {
    MDE_LAUNCH(mde::K_SKIP_FWD, bytes, s, (skip_fwd_mfma_kernel<32, 16, true>), mgrid(), dim3(256), 0,
               (const float*)r, (const float*)d, wt, b, (float*)out, n, hw);
  } else if (cout <= 1) {
    if (hw % 4 == 0) SKIP_FWD(1, 4); else SKIP_FWD(1, 1);
  } else if (cout <= 16) {
    if (hw % 4 == 0) SKIP_FWD(16, 4); else SKIP_FWD(16, 1);
  } else if (cout <= 32) {
    if (hw % 2 == 0) SKIP_FWD(32, 2); else SKIP_FWD(32, 1);
  } else {
    SKIP_FWD(64, 1);
  }
#undef SKIP_FWD
  return MDE_OK;
}

size_t mde_skip_reduce_workspace(int64_t n, int64_t cin, int64_t cout,
                                 int64_t h, int64_t w) {
  return sizeof(float) * (size_t)bwd_blocks(n, h * w) *
         (size_t)(cin * cout + cout);
}

int mde_skip_reduce_bwd(const void* gout, const void* r, const void* d,
                        const float* wt, void* gs, float* gw, float* gb,
                        int64_t n, int64_t cin, int64_t cout, int64_t h,
                        int64_t w, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  const int64_t hw = h * w;
  if (!gout || !r || !d || !wt || !gs || !gw || !gb || !workspace || n <= 0 ||
      hw <= 0 || cin <= 0 || cout <= 0 || cin > kMaxC || cout > kMaxC)
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int nb = bwd_blocks(n, hw);
  float* slab = (float*)workspace;
  if (dtype == MDE_BF16) {
    if (!skip_mfma_shape(cin, cout, hw)) return MDE_ERR_UNSUPPORTED;
    const double bb = 2.0 * n * hw * (double)(3 * cin + cout);
    using B = mde::bf16;
    if (cin == 64)
      MDE_LAUNCH(mde::K_SKIP_BWD, bb, s, (skip_bwd_mfma_kernel<64, 32, true, false, false, B>),
                 dim3(nb), dim3(256), 0, (const B*)gout, (const B*)r, (const B*)d, wt, (B*)gs,
                 slab, n, hw, nullptr, nullptr, nullptr);
    else
      MDE_LAUNCH(mde::K_SKIP_BWD, bb, s, (skip_bwd_mfma_kernel<32, 16, true, false, false, B>),
                 dim3(nb), dim3(256), 0, (const B*)gout, (const B*)r, (const B*)d, wt, (B*)gs,
                 slab, n, hw, nullptr, nullptr, nullptr);
    const int stride = (int)(cin * cout + cout);
    MDE_LAUNCH(mde::K_SKIP_BWD_REDUCE, 4.0 * (double)nb * stride, s, skip_slab_reduce_kernel<0>,
               dim3((unsigned)stride), dim3(256), 0, slab, nb, (int)(cin * cout), (int)cout, gw,
               gb, 0, (float*)nullptr);
    return MDE_OK;
  }
  const double bytes = 4.0 * n * hw * (double)(2 * cin + cout + cin);
#define SKIP_BWD(CI_, CO_, OB_, CB_, FAST_)                                   \
  MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s,                                      \
             (skip_bwd_kernel<CI_, CO_, OB_, CB_, FAST_>), dim3(nb),         \
             dim3(kTile), (bwd_lds<CI_, CO_, FAST_>()), (const float*)gout,        \
             (const float*)r, (const float*)d, wt, (float*)gs, slab, n,      \
             (int)cin, (int)cout, hw)
  if (cin == 16 && cout == 1 && hw % 4 == 0) {
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_c1_kernel<16>), dim3(nb),
               dim3(256), 0, (const float*)gout, (const float*)r, (const float*)d,
               wt, (float*)gs, slab, n, hw);
  } else if (cin == 4 && cout == 1 && hw % 4 == 0) {
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_c1_kernel<4>), dim3(nb),
               dim3(256), 0, (const float*)gout, (const float*)r, (const float*)d,
               wt, (float*)gs, slab, n, hw);
  } else if (cin == 64 && cout == 32 && hw % 64 == 0) {
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_mfma_kernel<64, 32, true>), dim3(nb), dim3(256),
               0, (const float*)gout, (const float*)r, (const float*)d, wt, (float*)gs, slab,
               n, hw);
  } else if (cin == 32 && cout == 16 && hw % 64 == 0) {
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_mfma_kernel<32, 16, true>), dim3(nb), dim3(256),
               0, (const float*)gout, (const float*)r, (const float*)d, wt, (float*)gs, slab,
               n, hw);
  } else if (cin == 64 && cout == 32) {
    SKIP_BWD(64, 32, 4, 4, true);
  } else if (cin == 32 && cout == 16) {
    SKIP_BWD(32, 16, 2, 2, true);
  } else if (cin == 16 && cout == 1) {
    SKIP_BWD(16, 1, 1, 1, true);
  } else if (cout <= 16) {
    SKIP_BWD(64, 16, 1, 1, false);
  } else {
    SKIP_BWD(64, 64, 1, 1, false);
  }
#undef SKIP_BWD
  const int stride = (int)(cin * cout + cout);
  MDE_LAUNCH(mde::K_SKIP_BWD_REDUCE, 4.0 * (double)nb * stride, s,
             skip_slab_reduce_kernel<0>, dim3((unsigned)stride), dim3(256), 0, slab,
             nb, (int)(cin * cout), (int)cout, gw, gb);
  return MDE_OK;
}

// ---- skip fusion over the comb_conv's last BatchNorm + ReLU: r is that BN's
// raw input (the 1x1 conv output without its folded bias), in_scale /
// in_shift its coefficients; out = b + W (relu(in_scale r + in_shift) + d).
// Shapes: the MFMA 64 -> 32 / 32 -> 16 (h*w % 64 == 0) and the register
// 16 -> 1 / 4 -> 1 (h*w % 4 == 0) kernels; the backward's BN sums (in_sums
// [cin][2] = sum e, sum e (r - in_mean), e = gs [in_scale r + in_shift > 0],
// for mde_batchnorm_bwd_apply) on all but 64 -> 32.
static bool skip_bn_reg(int64_t cin, int64_t cout, int64_t hw) {
  return hw % 4 == 0 && cout == 1 && (cin == 16 || cin == 4);
}

int mde_skip_reduce_bn_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int sums) {
  const int64_t hw = h * w;
  if (skip_bn_reg(cin, cout, hw)) return 1;
  if (!skip_mfma_shape(cin, cout, hw)) return 0;
  return (!sums || cin <= 32) ? 1 : 0;
}

size_t mde_skip_reduce_bn_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w) {
  return sizeof(float) * (size_t)bwd_blocks(n, h * w) * (size_t)(cin * cout + cout + 2 * cin);
}

}  // extern "C"

// bf16 storage: the bf16-product kernels of pwbf.hip (MDE_PW_BF=0: the
// fp32-product kernels above, for A/B)
static bool pw_bf_on() {
  static const bool on = [] {
    const char* e = std::getenv("MDE_PW_BF");
    return !(e && e[0] == '0');
  }();
  return on;
}

// skip_reduce_bn launches on storage type T (fp32, or bf16 under autocast:
// r, d, out / gout, gs in T; weights, BN coefficients, sums and arithmetic fp32).
template <typename T>
static int skip_bn_fwd_t(const void* r, const void* d, const float* in_scale,
                         const float* in_shift, const float* wt, const float* b, void* out,
                         int64_t n, int64_t cin, int64_t cout, int64_t hw, hipStream_t s) {
  const double bytes = (double)sizeof(T) * n * hw * (double)(2 * cin + cout);
  const T *R = (const T*)r, *D = (const T*)d;
  if (skip_bn_reg(cin, cout, hw)) {
    const int64_t blocks = mde::cdiv(n * hw / 4, 256);
    const dim3 g((unsigned)(blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks)));
    MDE_LAUNCH(mde::K_SKIP_FWD, bytes, s, (skip_fwd_kernel<1, 4, true, T>), g, dim3(256), 0, R, D,
               wt, b, (T*)out, n, (int)cin, (int)cout, hw, in_scale, in_shift);
    return MDE_OK;
  }
  const int64_t blocks = mde::cdiv(n * hw / 64, 4);
  const dim3 g((unsigned)(blocks > 4096 ? 4096 : blocks));
  if constexpr (std::is_same_v<T, mde::bf16>) {
    if (pw_bf_on() && mde::pwbf_skip_ok(cin, cout))  // bf16 products (pwbf.hip)
      return mde::pwbf_skip_fwd(R, D, in_scale, in_shift, wt, b, (mde::bf16*)out, n, cin, cout,
                                hw, (int)g.x, s);
  }
  if (cin == 64)
    MDE_LAUNCH(mde::K_SKIP_FWD, bytes, s, (skip_fwd_mfma_kernel<64, 32, true, true, false, T>), g,
               dim3(256), 0, R, D, wt, b, (T*)out, n, hw, in_scale, in_shift, nullptr);
  else
    MDE_LAUNCH(mde::K_SKIP_FWD, bytes, s, (skip_fwd_mfma_kernel<32, 16, true, true, false, T>), g,
               dim3(256), 0, R, D, wt, b, (T*)out, n, hw, in_scale, in_shift, nullptr);
  return MDE_OK;
}

template <typename T>
static int skip_bn_bwd_t(const void* gout, const void* r, const void* d, const float* in_scale,
                         const float* in_shift, const float* in_mean, const float* wt, void* gs,
                         float* gw, float* gb, float* in_sums, int64_t n, int64_t cin,
                         int64_t cout, int64_t hw, void* workspace, hipStream_t s) {
  const int nb = bwd_blocks(n, hw);
  float* slab = (float*)workspace;
  const double bytes = (double)sizeof(T) * n * hw * (double)(3 * cin + cout);
  const T *G = (const T*)gout, *R = (const T*)r, *D = (const T*)d;
  T* GS = (T*)gs;
  const bool sums = in_sums != nullptr;
  bool done = false;
  if constexpr (std::is_same_v<T, mde::bf16>) {
    if (pw_bf_on() && mde::pwbf_skip_ok(cin, cout)) {  // bf16 products (pwbf.hip)
      const int rc = mde::pwbf_skip_bwd(G, R, D, in_scale, in_shift, sums ? in_mean : nullptr, wt,
                                        GS, slab, n, cin, cout, hw, nb, s);
      if (rc != MDE_OK) return rc;
      done = true;
    }
  }
  if (done) {
  } else if (cin == 16 && sums)
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_c1_kernel<16, true, true, T>), dim3(nb),
               dim3(256), 0, G, R, D, wt, GS, slab, n, hw, in_scale, in_shift, in_mean);
  else if (cin == 16)
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_c1_kernel<16, true, false, T>), dim3(nb),
               dim3(256), 0, G, R, D, wt, GS, slab, n, hw, in_scale, in_shift, in_mean);
  else if (cin == 4 && sums)
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_c1_kernel<4, true, true, T>), dim3(nb),
               dim3(256), 0, G, R, D, wt, GS, slab, n, hw, in_scale, in_shift, in_mean);
  else if (cin == 4)
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_c1_kernel<4, true, false, T>), dim3(nb),
               dim3(256), 0, G, R, D, wt, GS, slab, n, hw, in_scale, in_shift, in_mean);
  else if (cin == 64)
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_mfma_kernel<64, 32, true, true, false, T>),
               dim3(nb), dim3(256), 0, G, R, D, wt, GS, slab, n, hw, in_scale, in_shift, in_mean);
  else if (sums)
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_mfma_kernel<32, 16, true, true, true, T>),
               dim3(nb), dim3(256), 0, G, R, D, wt, GS, slab, n, hw, in_scale, in_shift, in_mean);
  else
    MDE_LAUNCH(mde::K_SKIP_BWD, bytes, s, (skip_bwd_mfma_kernel<32, 16, true, true, false, T>),
               dim3(nb), dim3(256), 0, G, R, D, wt, GS, slab, n, hw, in_scale, in_shift, in_mean);
  const int npairs = (int)(cin * cout);
  const int nextra = sums ? (int)(2 * cin) : 0;
  MDE_LAUNCH(mde::K_SKIP_BWD_REDUCE, 4.0 * (double)nb * (npairs + cout + nextra), s,
             skip_slab_reduce_kernel<0>, dim3((unsigned)(npairs + cout + nextra)), dim3(256), 0, slab,
             nb, npairs, (int)cout, gw, gb, nextra, in_sums);
  return MDE_OK;
}

extern "C" {

int mde_skip_reduce_bn_fwd(const void* r, const void* d, const float* in_scale,
                           const float* in_shift, const float* wt, const float* b, void* out,
                           int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype,
                           void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  const int64_t hw = h * w;
  if (!r || !d || !in_scale || !in_shift || !wt || !b || !out || n <= 0 || hw <= 0)
    return MDE_ERR_INVALID_ARG;
  if (!mde_skip_reduce_bn_supported(cin, cout, h, w, 0)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  return dtype == MDE_BF16
             ? skip_bn_fwd_t<mde::bf16>(r, d, in_scale, in_shift, wt, b, out, n, cin, cout, hw, s)
             : skip_bn_fwd_t<float>(r, d, in_scale, in_shift, wt, b, out, n, cin, cout, hw, s);
}

int mde_skip_reduce_bn_bwd(const void* gout, const void* r, const void* d, const float* in_scale,
                           const float* in_shift, const float* in_mean, const float* wt, void* gs,
                           float* gw, float* gb, float* in_sums, int64_t n, int64_t cin,
                           int64_t cout, int64_t h, int64_t w, void* workspace, int dtype,
                           void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  const int64_t hw = h * w;
  if (!gout || !r || !d || !in_scale || !in_shift || !wt || !gs || !gw || !gb || !workspace ||
      n <= 0 || hw <= 0 || (in_sums && !in_mean))
    return MDE_ERR_INVALID_ARG;
  if (!mde_skip_reduce_bn_supported(cin, cout, h, w, in_sums != nullptr)) return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  return dtype == MDE_BF16
             ? skip_bn_bwd_t<mde::bf16>(gout, r, d, in_scale, in_shift, in_mean, wt, gs, gw, gb,
                                        in_sums, n, cin, cout, hw, workspace, s)
             : skip_bn_bwd_t<float>(gout, r, d, in_scale, in_shift, in_mean, wt, gs, gw, gb,
                                    in_sums, n, cin, cout, hw, workspace, s);
}


// ---------------------------------------------------------------- pointwise
// Bias-free 1x1 convolution (the conv feeding a BatchNorm whose bias is
// folded), the MFMA kernels above with one input.
#define MDE_PW_SHAPES(X) \
  X(16, 8) X(16, 16) X(32, 16) X(32, 32) X(64, 32) X(32, 64) X(16, 32) X(64, 64)

static bool pw_ok(int64_t n, int64_t cin, int64_t cout, int64_t hw) {
  if (n <= 0 || hw <= 0 || hw % 64 != 0) return false;
#define MDE_PW_MATCH(A, B) if (cin == A && cout == B) return true;
  MDE_PW_SHAPES(MDE_PW_MATCH)
#undef MDE_PW_MATCH
  return false;
}

int mde_pointwise_supported(int64_t cin, int64_t cout, int64_t h, int64_t w) {
  return pw_ok(1, cin, cout, h * w) ? 1 : 0;
}

size_t mde_pointwise_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w) {
  // slab rows sized for the BN-sum epilogue too (mde_pointwise_bwd_bn)
  return sizeof(float) * (size_t)bwd_blocks(n, h * w) * (size_t)(cin * cout + cout + 2 * cin);
}

static int pw_fwd_blocks(int64_t n, int64_t hw, bool stats = false) {
  // with the statistics epilogue: fewer, longer blocks (the per-block
  // partials are merged by the BN; ~10 tiles per wave at the cfg2 shapes)
  const int cap = stats ? 1024 : 4096;
  const int64_t blocks = mde::cdiv(n * hw / 64, 4);
  return (int)(blocks > cap ? cap : blocks);
}

}  // extern "C"

template <typename T>
static int pointwise_fwd(const void* x, const float* in_scale, const float* in_shift,
                         const float* wt, void* y, float* stats, int64_t n, int64_t cin,
                         int64_t cout, int64_t h, int64_t w, hipStream_t s) {
  const int64_t hw = h * w;
  if (!x || !wt || !y || (!in_scale != !in_shift)) return MDE_ERR_INVALID_ARG;
  if (!pw_ok(n, cin, cout, hw)) return MDE_ERR_UNSUPPORTED;
  const double bytes = (double)sizeof(T) * n * hw * (double)(cin + cout);
  const dim3 grid((unsigned)pw_fwd_blocks(n, hw, stats != nullptr));
  const T* xi = (const T*)x;
  T* yo = (T*)y;
  if constexpr (std::is_same_v<T, mde::bf16>) {
    if (pw_bf_on())  // bf16 products (pwbf.hip)
      return mde::pwbf_fwd(xi, in_scale, in_shift, wt, yo, stats, n, cin, cout, hw, (int)grid.x, s);
  }
  // 64 -> 64 with the BN operand and the statistics epilogue: two 64 -> 32
  // halves (one launch holding all 64 outputs needs > 256 registers: one wave
  // per SIMD); each half re-reads the input, from L2 mostly
  if (cin == 64 && cout == 64 && in_scale && stats) {
    for (int half = 0; half < 2; ++half)
      MDE_LAUNCH(mde::K_PW_FWD, bytes / 2, s, (skip_fwd_mfma_kernel<64, 32, false, true, true, T>),
                 grid, dim3(256), 0, xi, nullptr, wt + half * 32 * 64, nullptr,
                 yo + half * 32 * hw, n, hw, in_scale, in_shift,
                 stats + (int64_t)half * 32 * grid.x * 4, 64);
    return MDE_OK;
  }
#define MDE_PW_FWD(A, B)                                                                     \
  if (cin == A && cout == B) {                                                               \
    if (in_scale && stats) {                                                                 \
      MDE_LAUNCH(mde::K_PW_FWD, bytes, s, (skip_fwd_mfma_kernel<A, B, false, true, true, T>), \
                 grid, dim3(256), 0, xi, nullptr, wt, nullptr, yo, n, hw, in_scale,          \
                 in_shift, stats);                                                           \
    } else if (stats) {                                                                      \
      MDE_LAUNCH(mde::K_PW_FWD, bytes, s,                                                    \
                 (skip_fwd_mfma_kernel<A, B, false, false, true, T>), grid, dim3(256), 0,    \
                 xi, nullptr, wt, nullptr, yo, n, hw, nullptr, nullptr, stats);              \
    } else if (in_scale) {                                                                   \
      MDE_LAUNCH(mde::K_PW_FWD, bytes, s,                                                    \
                 (skip_fwd_mfma_kernel<A, B, false, true, false, T>), grid, dim3(256), 0,    \
                 xi, nullptr, wt, nullptr, yo, n, hw, in_scale, in_shift, nullptr);          \
    } else {                                                                                 \
      MDE_LAUNCH(mde::K_PW_FWD, bytes, s,                                                    \
                 (skip_fwd_mfma_kernel<A, B, false, false, false, T>), grid, dim3(256), 0,   \
                 xi, nullptr, wt, nullptr, yo, n, hw, nullptr, nullptr, nullptr);            \
    }                                                                                        \
    return MDE_OK;                                                                           \
  }
  MDE_PW_SHAPES(MDE_PW_FWD)
#undef MDE_PW_FWD
  return MDE_ERR_UNSUPPORTED;
}

static bool pw_dtype_ok(int dtype) { return dtype == MDE_F32 || dtype == MDE_BF16; }

extern "C" {

int mde_pointwise_fwd(const void* x, const float* in_scale, const float* in_shift,
                      const float* wt, void* y, int64_t n, int64_t cin, int64_t cout, int64_t h,
                      int64_t w, int dtype, void* stream) {
  if (!pw_dtype_ok(dtype)) return MDE_ERR_UNSUPPORTED;
  return dtype == MDE_BF16
             ? pointwise_fwd<mde::bf16>(x, in_scale, in_shift, wt, y, nullptr, n, cin, cout, h, w,
                                        (hipStream_t)stream)
             : pointwise_fwd<float>(x, in_scale, in_shift, wt, y, nullptr, n, cin, cout, h, w,
                                    (hipStream_t)stream);
}

int mde_pointwise_stats_blocks(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w) {
  if (!pw_ok(n, cin, cout, h * w)) return 0;
  return pw_fwd_blocks(n, h * w, true);
}

int mde_pointwise_fwd_stats(const void* x, const float* in_scale, const float* in_shift,
                            const float* wt, void* y, float* stats, int64_t n, int64_t cin,
                            int64_t cout, int64_t h, int64_t w, int dtype, void* stream) {
  if (!pw_dtype_ok(dtype)) return MDE_ERR_UNSUPPORTED;
  if (!stats) return MDE_ERR_INVALID_ARG;
  return dtype == MDE_BF16
             ? pointwise_fwd<mde::bf16>(x, in_scale, in_shift, wt, y, stats, n, cin, cout, h, w,
                                        (hipStream_t)stream)
             : pointwise_fwd<float>(x, in_scale, in_shift, wt, y, stats, n, cin, cout, h, w,
                                    (hipStream_t)stream);
}

}  // extern "C"

namespace {

// The prefetching backward's shapes: 16 input channels (wider ones spill two
// register sets), and for fp32 operands at most 16 outputs too.
template <int A, int B, typename T>
constexpr bool pw_pf_shape() {
  return A <= 16 && (std::is_same_v<T, mde::bf16> || B <= 16);
}

inline bool pw_pf_on() {
  static const bool on = [] {
    const char* e = std::getenv("MDE_PW_PF");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Pointwise backward; in_mean / in_sums non-null (with in_scale): also the
// producer BatchNorm's backward sums (BNS epilogue), in_sums [cin][2].
template <typename T>
int pointwise_bwd(const void* gy, const void* x, const float* in_scale, const float* in_shift,
                  const float* in_mean, const float* wt, void* gx, float* gw, float* in_sums,
                  int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, void* workspace,
                  hipStream_t s) {
  const int64_t hw = h * w;
  if (!gy || !x || !wt || !gw || !workspace || (!in_scale != !in_shift))
    return MDE_ERR_INVALID_ARG;
  if (!pw_ok(n, cin, cout, hw)) return MDE_ERR_UNSUPPORTED;
  const bool sums = in_sums != nullptr;
  if (sums && (!in_scale || !in_mean || !gx)) return MDE_ERR_INVALID_ARG;
  if (sums && cin > 32) return MDE_ERR_UNSUPPORTED;
  const int nb = bwd_blocks(n, hw);
  float* slab = (float*)workspace;
  const double bytes = (double)sizeof(T) * n * hw * (double)(cout + cin + (gx ? cin : 0));
  const T* gi = (const T*)gy;
  const T* xi = (const T*)x;
  T* go = (T*)gx;
  // bf16 storage with the BN + ReLU operand and gs written, 16 input
  // channels (wider ones spill two register sets): the prefetching kernel
  // (MDE_PW_PF=0: skip_bwd_mfma_kernel)
  const bool pf = go != nullptr && pw_pf_on();
  const bool bfp = std::is_same_v<T, mde::bf16> && go != nullptr && pw_bf_on();
  if (bfp) {  // bf16 products (pwbf.hip)
    const int rc = mde::pwbf_bwd((const mde::bf16*)gy, (const mde::bf16*)x, in_scale, in_shift,
                                 sums ? in_mean : nullptr, wt, (mde::bf16*)gx, slab, n, cin, cout,
                                 hw, nb, s);
    if (rc != MDE_OK) return rc;
  } else {
#define MDE_PW_BWD(A, B)                                                                     \
  if (cin == A && cout == B && pw_pf_shape<A, B, T>() && pf && in_scale) {                   \
    if constexpr (pw_pf_shape<A, B, T>()) {                                                  \
      if (sums) {                                                                            \
        MDE_LAUNCH(mde::K_PW_BWD, bytes, s, (pw_bwd_pf_kernel<A, B, true, T>), dim3(nb),     \
                   dim3(256), 0, gi, xi, wt, go, slab, n, hw, in_scale, in_shift, in_mean);  \
      } else {                                                                               \
        MDE_LAUNCH(mde::K_PW_BWD, bytes, s, (pw_bwd_pf_kernel<A, B, false, T>), dim3(nb),    \
                   dim3(256), 0, gi, xi, wt, go, slab, n, hw, in_scale, in_shift, nullptr);  \
      }                                                                                      \
    }                                                                                        \
  } else if (cin == A && cout == B) {                                                        \
    if (sums) {                                                                              \
      if constexpr (A <= 32)                                                                 \
        MDE_LAUNCH(mde::K_PW_BWD, bytes, s,                                                  \
                   (skip_bwd_mfma_kernel<A, B, false, true, true, T>), dim3(nb), dim3(256),  \
                   0, gi, xi, nullptr, wt, go, slab, n, hw, in_scale, in_shift, in_mean);    \
    } else if (in_scale) {                                                                   \
      MDE_LAUNCH(mde::K_PW_BWD, bytes, s, (skip_bwd_mfma_kernel<A, B, false, true, false, T>), \
                 dim3(nb), dim3(256), 0, gi, xi, nullptr, wt, go, slab, n, hw, in_scale,     \
                 in_shift, nullptr);                                                         \
    } else {                                                                                 \
      MDE_LAUNCH(mde::K_PW_BWD, bytes, s,                                                    \
                 (skip_bwd_mfma_kernel<A, B, false, false, false, T>), dim3(nb), dim3(256),  \
                 0, gi, xi, nullptr, wt, go, slab, n, hw, nullptr, nullptr, nullptr);        \
    }                                                                                        \
  }
  MDE_PW_SHAPES(MDE_PW_BWD)
#undef MDE_PW_BWD
  }
  const int npairs = (int)(cin * cout), nextra = sums ? 2 * (int)cin : 0;
  const int stride = npairs + (int)cout + nextra;
  if (sums) {  // every slab column: gw, (the unused bias columns), the BN sums
    MDE_LAUNCH(mde::K_PW_BWD, 4.0 * (double)nb * stride, s, skip_slab_reduce_kernel<1>,
               dim3((unsigned)stride), dim3(256), 0, slab, nb, npairs, (int)cout, gw,
               (float*)nullptr, nextra, in_sums);
  } else {
    MDE_LAUNCH(mde::K_PW_BWD, 4.0 * (double)nb * stride, s, skip_slab_reduce_kernel<1>,
               dim3((unsigned)npairs), dim3(256), 0, slab, nb, npairs, (int)cout, gw,
               (float*)nullptr, 0, (float*)nullptr);
  }
  return MDE_OK;
}

}  // namespace

extern "C" {

int mde_pointwise_bwd(const void* gy, const void* x, const float* in_scale,
                      const float* in_shift, const float* wt, void* gx, float* gw, int64_t n,
                      int64_t cin, int64_t cout, int64_t h, int64_t w, void* workspace,
                      int dtype, void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  return dtype == MDE_BF16
             ? pointwise_bwd<mde::bf16>(gy, x, in_scale, in_shift, nullptr, wt, gx, gw, nullptr, n,
                                        cin, cout, h, w, workspace, (hipStream_t)stream)
             : pointwise_bwd<float>(gy, x, in_scale, in_shift, nullptr, wt, gx, gw, nullptr, n,
                                    cin, cout, h, w, workspace, (hipStream_t)stream);
}

int mde_pointwise_bwd_bn(const void* gy, const void* x, const float* in_scale,
                         const float* in_shift, const float* in_mean, const float* wt, void* gx,
                         float* gw, float* in_sums, int64_t n, int64_t cin, int64_t cout,
                         int64_t h, int64_t w, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32 && dtype != MDE_BF16) return MDE_ERR_UNSUPPORTED;
  if (!in_scale || !in_shift || !in_mean || !gx || !in_sums) return MDE_ERR_INVALID_ARG;
  return dtype == MDE_BF16
             ? pointwise_bwd<mde::bf16>(gy, x, in_scale, in_shift, in_mean, wt, gx, gw, in_sums,
                                        n, cin, cout, h, w, workspace, (hipStream_t)stream)
             : pointwise_bwd<float>(gy, x, in_scale, in_shift, in_mean, wt, gx, gw, in_sums, n,
                                    cin, cout, h, w, workspace, (hipStream_t)stream);
}

}  // extern "C"
