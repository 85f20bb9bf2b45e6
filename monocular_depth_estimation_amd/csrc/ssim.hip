// DepthNorm + fused SSIM(3x3 box) + L1 loss, forward and gradient in one pass.
//
// Reference:
//   DepthNorm            src/utils.py:7-8 (batch-global min/max, train.py:89)
//   SSIM                 src/loss.py:57-88 (monodepth2 form: ReflectionPad2d(1),
//                        five AvgPool2d(3,1), C1=0.01^2, C2=0.03^2,
//                        mean(clamp((1-S)/2, 0, 1)))
//   nn.L1Loss            src/train.py:53,94
//   loss composition     src/train.py:100 (1.0*ssim + 0.1*l1)
//
// The gradient of mean(clamp((1-S)/2,0,1)) does not depend on the loss value,
// so one streaming pass produces the loss partial sums AND d loss/d pred
// (ssim3_stream_kernel below: column strips x row chunks, separable 3x3 boxes
// from DPP lane shifts and register row rings, no LDS staging).  Loss
// partials go to a per-block slab summed in block order by loss_final_kernel
// (deterministic).
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

constexpr float kC1 = 0.01f * 0.01f;
constexpr float kC2 = 0.03f * 0.03f;

__device__ __forceinline__ int reflect1(int q, int n) {
  if (q < 0) q = -q;
  if (q > n - 1) q = 2 * (n - 1) - q;
  return q < 0 ? 0 : (q > n - 1 ? n - 1 : q);
}


// ---------------------------------------------------------------- min / max
__global__ void __launch_bounds__(256)
    minmax_partial_kernel(const float* __restrict__ x, int64_t numel,
                          float* __restrict__ part) {
  __shared__ float rmn[4], rmx[4];
  float mn = INFINITY, mx = -INFINITY;
  const int64_t n4 = numel >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    mn = fminf(mn, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
    mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       i < numel; i += stride) {
    mn = fminf(mn, x[i]);
    mx = fmaxf(mx, x[i]);
  }
  mn = mde::wave_min(mn);
  mx = mde::wave_max(mx);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    rmn[wid] = mn;
    rmx[wid] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = fminf(fminf(rmn[0], rmn[1]), fminf(rmn[2], rmn[3]));
    part[2 * blockIdx.x + 1] =
        fmaxf(fmaxf(rmx[0], rmx[1]), fmaxf(rmx[2], rmx[3]));
  }
}

__global__ void __launch_bounds__(256)
    minmax_final_kernel(const float* __restrict__ part, int nparts,
                        float* __restrict__ out) {
  __shared__ float rmn[4], rmx[4];
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    mn = fminf(mn, part[2 * i]);
    mx = fmaxf(mx, part[2 * i + 1]);
  }
  mn = mde::wave_min(mn);
  mx = mde::wave_max(mx);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    rmn[wid] = mn;
    rmx[wid] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = fminf(fminf(rmn[0], rmn[1]), fminf(rmn[2], rmn[3]));
    out[1] = fmaxf(fmaxf(rmx[0], rmx[1]), fmaxf(rmx[2], rmx[3]));
  }
}

__global__ void __launch_bounds__(256)
    depthnorm_kernel(const float* __restrict__ x, const float* __restrict__ mm,
                     float* __restrict__ y, int64_t numel) {
  const float mn = mm[0], den = mm[1] - mm[0];
  const int64_t n4 = numel >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    v.x = (v.x - mn) / den;
    v.y = (v.y - mn) / den;
    v.z = (v.z - mn) / den;
    v.w = (v.w - mn) / den;
    reinterpret_cast<float4*>(y)[i] = v;
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       i < numel; i += stride)
    y[i] = (x[i] - mn) / den;
}

// ---------------------------------------------------------------- SSIM + L1
// Streaming kernel: value + gradient in one pass.  A wave owns a strip of kSW = 60 output
// columns (lane l <-> column strip*60 - 2 + l: a 2-column halo each side,
// reflected at the image border) and a chunk of rows, and walks the padded
// rows top to bottom: the 3-wide horizontal sums come from wave shuffles,
// the vertical ones from a 3-row register ring, so every input pixel is read
// once per strip (+2 halo columns of 64) and once per chunk (+4 halo rows).
// The gradient is the transposed box of the per-centre coefficients, done the
// same way one row later; the reflection adds the centre-0 / centre-(n-1)
// coefficients once more to column / row 1 and n-2.  Loss partials: one per
// block (wave order), summed by loss_final_kernel.
constexpr int kSW = 60;  // output columns per strip (64 lanes - 2 x 2 halo)

// Neighbour lanes' values by DPP wave shifts (one VALU op, no LDS round trip):
// lane_prev = value of lane - 1 (0 into lane 0), lane_next = lane + 1 (0 into 63);
// bound_ctrl writes the 0 itself (no move of an `old` operand first).
__device__ __forceinline__ float lane_prev(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float lane_next(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}

template <bool GT>
__global__ void __launch_bounds__(256)
    ssim3_stream_kernel(const float* __restrict__ xp, const float* __restrict__ yp,
                        const float* __restrict__ mm, int h, int w, int strips, int chunks,
                        int chunk_rows, int64_t nwaves, float gs_ssim, float gs_l1,
                        float* __restrict__ part, float* __restrict__ gx,
                        float* __restrict__ gy, int strip_major) {
  __shared__ float red[4];
  constexpr int NC = GT ? 5 : 3;  // coefficient fields
  const int lane = threadIdx.x & 63;
  int64_t lb = blockIdx.x;
  if (strip_major == 2) {
    // XCD swizzle: physical block 8k + x runs on XCD x; give XCD x the
    // contiguous logical range [x per + min(x, rem), ...) so neighbouring
    // logical blocks (adjacent strips) share one XCD's L2
    const int64_t nb = gridDim.x, per = nb / 8, rem = nb % 8;
    const int64_t x = blockIdx.x % 8, kk = blockIdx.x / 8;
    lb = x * per + (x < rem ? x : rem) + kk;
  }
  const int64_t wid = lb * 4 + (threadIdx.x >> 6);
  float lsum = 0.f, l1sum = 0.f;
  if (wid < nwaves) {  // wave-uniform
    // strip_major (1, 2): a block's 4 waves are 4 ADJACENT strips of one chunk, so
    // the 128-B lines two neighbouring strips share (a strip starts 8 B into
    // a line: 64 lanes x 4 B touch 3 lines) come through one CU's L2 instead
    // of two XCDs'; otherwise 4 consecutive chunks of one strip
    int chunk, strip;
    int64_t img;
    if (strip_major) {
      strip = (int)(wid % strips);
      const int64_t rest = wid / strips;
      chunk = (int)(rest % chunks);
      img = rest / chunks;
    } else {
      chunk = (int)(wid % chunks);
      const int64_t rest = wid / chunks;
      strip = (int)(rest % strips);
      img = rest / strips;
    }
    const int q = strip * kSW - 2 + lane;
    const bool qin = q >= 0 && q < w;
    const bool out = lane >= 2 && lane < 2 + kSW && qin;
    const float wl = q == 1 ? 2.f : 1.f, wr = q == w - 2 ? 2.f : 1.f;
    const int64_t base = img * h * w;
    const float* X = xp + base + reflect1(q, w);
    const float* Y = yp + base + reflect1(q, w);
    float tmn = 0.f, tden = 1.f;
    const bool norm = mm != nullptr;
    if (norm) {
      tmn = mm[0];
      tden = mm[1] - mm[0];
    }
    const int g0 = chunk * chunk_rows, g1 = min(h, g0 + chunk_rows);
    const int rs = g0 - 2, re = g1 + 1;  // padded rows walked
    const float inv9 = 1.f / 9.f, k = gs_ssim * -0.5f;
    float hs[3][5] = {};                 // horizontal sums, rows r-2, r-1, r
    float cs[3][NC] = {};                // horizontally summed coefficients, rows p-2..p
    float xr[3] = {}, yr[3] = {};        // inputs, rows r-2..r
    auto load = [&](int r, float& xv, float& yv) {
      const int64_t off = (int64_t)reflect1(r, h) * w;
      xv = X[off];
      const float t = Y[off];
      yv = norm ? (t - tmn) / tden : t;
    };
    auto step = [&](float xv, float yv, int r) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        xr[i] = xr[i + 1];
        yr[i] = yr[i + 1];
#pragma unroll
        for (int f = 0; f < 5; ++f) hs[i][f] = hs[i + 1][f];
      }
      xr[2] = xv;
      yr[2] = yv;
      {
        const float v[5] = {xv, yv, xv * xv, yv * yv, xv * yv};
#pragma unroll
        for (int f = 0; f < 5; ++f)
          hs[2][f] = (lane_prev(v[f]) + v[f]) + lane_next(v[f]);
      }
      if (r < g0) return;  // wave-uniform: the ring is not full yet
      // centre row p = r - 1: statistics, loss, coefficients
      const int p = r - 1;
      const bool valid = qin && p >= 0 && p < h;
      float c[NC];
#pragma unroll
      for (int f = 0; f < NC; ++f) c[f] = 0.f;
      if (valid) {
        float st[5];
#pragma unroll
        for (int f = 0; f < 5; ++f) st[f] = (hs[0][f] + hs[1][f] + hs[2][f]) * inv9;
        const float mx = st[0], my = st[1];
        const float sxx = st[2] - mx * mx, syy = st[3] - my * my;
        const float sxy = st[4] - mx * my;
        const float n1 = 2.f * mx * my + kC1, n2 = 2.f * sxy + kC2;
        const float d1 = mx * mx + my * my + kC1, d2 = sxx + syy + kC2;
        const float D = d1 * d2;
        const float S = (n1 * n2) / D;  // exact division: S(x, x) = 1
        const float fl = (1.f - S) * 0.5f;
        if (out && p < g1 && p >= g0) lsum += fminf(fmaxf(fl, 0.f), 1.f);
        if (fl >= 0.f && fl <= 1.f) {
          // gradient terms with hardware reciprocals (1 ulp; the tests' 1e-4)
          const float rD = __builtin_amdgcn_rcpf(D), rd1 = __builtin_amdgcn_rcpf(d1);
          const float dS_dsx = -S * __builtin_amdgcn_rcpf(d2);  // = dS/dsyy
          const float dS_dsxy = 2.f * n1 * rD;
          const float dS_dmx = 2.f * my * n2 * rD - S * 2.f * mx * rd1;
          c[0] = k * (dS_dmx - 2.f * mx * dS_dsx - my * dS_dsxy);
          c[1] = k * dS_dsx;
          c[2] = k * dS_dsxy;
          if (GT) {
            const float dS_dmy = 2.f * mx * n2 * rD - S * 2.f * my * rd1;
            c[3] = k * (dS_dmy - 2.f * my * dS_dsx - mx * dS_dsxy);
            c[NC - 1] = c[1];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int f = 0; f < NC; ++f) cs[i][f] = cs[i + 1][f];
#pragma unroll
      for (int f = 0; f < NC; ++f)
        cs[2][f] = (wl * lane_prev(c[f]) + c[f]) + wr * lane_next(c[f]);
      // gradient row g = p - 1 from coefficient rows g-1, g, g+1
      const int g = p - 1;
      if (g < g0 || g >= g1) return;  // wave-uniform
      const float vt = g == 1 ? 2.f : 1.f, vb = g == h - 2 ? 2.f : 1.f;
      float sm[NC];
#pragma unroll
      for (int f = 0; f < NC; ++f) sm[f] = (vt * cs[0][f] + cs[1][f]) + vb * cs[2][f];
      if (out) {
        const float x0 = xr[0], y0 = yr[0];
        const float diff = x0 - y0;
        l1sum += fabsf(diff);
        const float sgn = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
        const int64_t off = base + (int64_t)g * w + q;
        if (gx) gx[off] = (sm[0] + 2.f * x0 * sm[1] + y0 * sm[2]) * inv9 + gs_l1 * sgn;
        if (GT && gy) gy[off] = (sm[3] + 2.f * y0 * sm[NC - 1] + x0 * sm[2]) * inv9 - gs_l1 * sgn;
      }
    };
    // rows in groups of 4, the next group's loads issued before this one's math
    float cx[4], cy[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) load(rs + i, cx[i], cy[i]);
    for (int r = rs; r <= re; r += 4) {
      float nx[4], ny[4];
      // the last group's prefetch would read up to 7 rows of the next chunk
      // (HBM traffic for nothing): clamp it to row re, already in cache
#pragma unroll
      for (int i = 0; i < 4; ++i) load(min(r + 4 + i, re), nx[i], ny[i]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (r + i <= re) step(cx[i], cy[i], r + i);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        cx[i] = nx[i];
        cy[i] = ny[i];
      }
    }
  }
  const float ts = mde::block_sum256(lsum, red);
  const float tl = mde::block_sum256(l1sum, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ts;
    part[2 * blockIdx.x + 1] = tl;
  }
}

// Two columns per lane (ssim3_pair_kernel): lane l of a strip holds columns
// c0 = strip * sw - 2 + 2 l and c0 + 1 (lane 0 and lane sw / 2 + 1 are the
// 2-column halos), so the arithmetic runs on packed fp32 pairs
// (v_pk_fma / v_pk_mul / v_pk_add_f32: two outputs per VALU op) and a 3-wide
// horizontal sum costs two DPP lane shifts per two outputs instead of per
// one.  Same algebra, same per-output operation order as ssim3_stream_kernel
// except the horizontal sums' association ((a0 + a1) + prev / next for the
// moments, (prev + a0) + a1 / (a0 + a1) + next for the coefficients) and the
// two divisions (the DepthNorm of the target and S = n / D): a
// reciprocal (hardware rcp; the target's refined once per wave) and one
// residual correction, q = q0 + (n - D q0) r -- packed fp32, 3 operations per
// pair where the IEEE division sequence took ~10 scalar ones per value (the
// kernel is VALU-bound).  The corrected quotient is the correctly rounded one
// except for rare hard cases (then within 1 ulp); an exact quotient of 1 --
// S(x, x) -- comes out exactly 1.
using f2 = __attribute__((ext_vector_type(2))) float;

__device__ __forceinline__ f2 pk(float a, float b) { return f2{a, b}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
// n / d given r ~ 1 / d
__device__ __forceinline__ f2 div2(f2 n, f2 d, f2 r) {
  const f2 q0 = n * r;
  return fma2(fma2(-d, q0, n), r, q0);
}

template <bool GT>
__global__ void __launch_bounds__(256, 3)  // three waves per SIMD (<= 168 VGPRs)
    ssim3_pair_kernel(const float* __restrict__ xp, const float* __restrict__ yp,
                      const float* __restrict__ mm, int h, int w, int sw, int strips, int chunks,
                      int chunk_rows, int64_t nwaves, float gs_ssim, float gs_l1,
                      float* __restrict__ part, float* __restrict__ gx, float* __restrict__ gy) {
  __shared__ float red[4];
  constexpr int NC = GT ? 5 : 3;
  const int lane = threadIdx.x & 63;
  // readfirstlane: the wave index (and the strip, chunk, image and every row
  // index derived from it) is wave-uniform, so the row offsets live in SGPRs
  // and reach the buffer loads as their scalar offset -- no per-row VALU
  // address math (the reflection, a quarter-rate v_mul_lo)
  const int64_t wid =
      (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  float lsum = 0.f, l1sum = 0.f;
  if (wid < nwaves) {  // wave-uniform
    const int strip = (int)(wid % strips);
    const int64_t rest = wid / strips;
    const int chunk = (int)(rest % chunks);
    const int64_t img = rest / chunks;
    const int c0 = strip * sw - 2 + 2 * lane, c1 = c0 + 1;
    const bool in0 = c0 >= 0 && c0 < w, in1 = c1 >= 0 && c1 < w;
    const int lim = strip * sw + sw;  // this strip's output columns: [strip sw, lim)
    const bool out0 = in0 && c0 >= strip * sw && c0 < lim;
    const bool out1 = in1 && c1 >= strip * sw && c1 < lim;
    // coefficient-sum weights: column 1 takes centre 0 twice, column w-2 centre w-1
    const f2 wl = pk(c0 == 1 ? 2.f : 1.f, c1 == 1 ? 2.f : 1.f);
    const f2 wr = pk(c0 == w - 2 ? 2.f : 1.f, c1 == w - 2 ? 2.f : 1.f);
    const int64_t base = img * h * w;
    const int o0 = reflect1(c0, w), o1 = reflect1(c1, w);
    // the image's planes as buffer resources (wave-uniform base, 32-bit lane
    // offsets): no 64-bit address arithmetic per load
    auto rsrc = [&](const float* p) {
      const uint64_t a = (uint64_t)(p + base);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
      return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo),
                                               0, (int)(4 * h * w), 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t XR = rsrc(xp), YR = rsrc(yp);
    float tmn = 0.f, tden = 1.f;
    const bool norm = mm != nullptr;
    if (norm) {
      tmn = mm[0];
      tden = mm[1] - mm[0];
    }
    // 1 / tden, refined once: the per-pixel DepthNorm divisions become div2
    const float r0 = __builtin_amdgcn_rcpf(tden);
    const float rden = fmaf(fmaf(-tden, r0, 1.f), r0, r0);
    const f2 tmn2 = pk(tmn, tmn), tden2 = pk(tden, tden), rden2 = pk(rden, rden);
    const int g0 = chunk * chunk_rows, g1 = min(h, g0 + chunk_rows);
    const int rs = g0 - 2, re = g1 + 1;
    const float inv9 = 1.f / 9.f, k = gs_ssim * -0.5f;
    f2 hs[3][5], cs[3][NC], xr[3], yr[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      xr[i] = yr[i] = pk(0.f, 0.f);
#pragma unroll
      for (int f = 0; f < 5; ++f) hs[i][f] = pk(0.f, 0.f);
#pragma unroll
      for (int f = 0; f < NC; ++f) cs[i][f] = pk(0.f, 0.f);
    }
    // lane column offset (VGPR) + the row's offset (SGPR)
    auto ld = [&](__amdgpu_buffer_rsrc_t R, int col, int rowoff) {
      return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(R, 4 * col, rowoff, 0));
    };
    auto load = [&](int r, f2& xv, f2& yv) {
      const int off = 4 * reflect1(r, h) * w;
      xv = pk(ld(XR, o0, off), ld(XR, o1, off));
      const f2 t = pk(ld(YR, o0, off), ld(YR, o1, off));
      yv = norm ? div2(t - tmn2, tden2, rden2) : t;
    };
    // 3-wide horizontal sums of a column pair: (prev lane's c1) + c0 + c1, c0 + c1 + (next's c0)
    auto hsum = [&](f2 v, f2 wa, f2 wb) {
      const float p = lane_prev(v.y), n = lane_next(v.x);
      return f2{wa.x * p + v.x + wb.x * v.y, wa.y * v.x + v.y + wb.y * n};
    };
    const f2 one2 = pk(1.f, 1.f);
    // one padded row r: PH 0 = horizontal sums only (r < g0), 1 = + the
    // statistics / coefficients of centre row r - 1 (no gradient row yet),
    // 2 = + gradient row r - 2.  No wave-uniform early returns: the main loop
    // runs PH 2 only, so its unrolled body has no joins (no ring moves).
    auto step = [&](auto ph, f2 xv, f2 yv, int r) {
      constexpr int PH = decltype(ph)::value;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        xr[i] = xr[i + 1];
        yr[i] = yr[i + 1];
#pragma unroll
        for (int f = 0; f < 5; ++f) hs[i][f] = hs[i + 1][f];
      }
      xr[2] = xv;
      yr[2] = yv;
      {
        const f2 v[5] = {xv, yv, xv * xv, yv * yv, xv * yv};
        // unweighted: (c0 + c1) + {prev lane's c1, next lane's c0} -- one add,
        // two lane shifts into a register pair, one packed add
#pragma unroll
        for (int f = 0; f < 5; ++f) {
          const float m = v[f].x + v[f].y;
          hs[2][f] = pk(m, m) + pk(lane_prev(v[f].y), lane_next(v[f].x));
        }
      }
      if constexpr (PH >= 1) {
        const int p = r - 1;
        const bool prow = p >= 0 && p < h;
        const bool v0 = in0 && prow, v1 = in1 && prow;
        f2 st[5];
#pragma unroll
        for (int f = 0; f < 5; ++f) st[f] = (hs[0][f] + hs[1][f] + hs[2][f]) * inv9;
        const f2 mx = st[0], my = st[1];
        const f2 sxx = st[2] - mx * mx, syy = st[3] - my * my;
        const f2 sxy = st[4] - mx * my;
        const f2 n1 = 2.f * mx * my + kC1, n2 = 2.f * sxy + kC2;
        const f2 d1 = mx * mx + my * my + kC1, d2 = sxx + syy + kC2;
        const f2 D = d1 * d2;
        const f2 nn = n1 * n2;
        const f2 rD = pk(__builtin_amdgcn_rcpf(D.x), __builtin_amdgcn_rcpf(D.y));
        const f2 S = div2(nn, D, rD);  // corrected quotient: S(x, x) = 1
        const f2 fl = (one2 - S) * 0.5f;
        const float lw = (p < g1 && p >= g0) ? 1.f : 0.f;  // the chunk's own centre rows
        lsum += lw * ((out0 ? fminf(fmaxf(fl.x, 0.f), 1.f) : 0.f) +
                      (out1 ? fminf(fmaxf(fl.y, 0.f), 1.f) : 0.f));
        const bool a0 = v0 && fl.x >= 0.f && fl.x <= 1.f, a1 = v1 && fl.y >= 0.f && fl.y <= 1.f;
        const f2 rd1 = pk(__builtin_amdgcn_rcpf(d1.x), __builtin_amdgcn_rcpf(d1.y));
        const f2 rd2 = pk(__builtin_amdgcn_rcpf(d2.x), __builtin_amdgcn_rcpf(d2.y));
        const f2 dS_dsx = -S * rd2;
        const f2 dS_dsxy = 2.f * n1 * rD;
        const f2 dS_dmx = 2.f * my * n2 * rD - S * 2.f * mx * rd1;
        f2 c[NC];
        c[0] = k * (dS_dmx - 2.f * mx * dS_dsx - my * dS_dsxy);
        c[1] = k * dS_dsx;
        c[2] = k * dS_dsxy;
        if constexpr (GT) {
          const f2 dS_dmy = 2.f * mx * n2 * rD - S * 2.f * my * rd1;
          c[3] = k * (dS_dmy - 2.f * my * dS_dsx - mx * dS_dsxy);
          c[NC - 1] = c[1];
        }
#pragma unroll
        for (int f = 0; f < NC; ++f) c[f] = pk(a0 ? c[f].x : 0.f, a1 ? c[f].y : 0.f);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int f = 0; f < NC; ++f) cs[i][f] = cs[i + 1][f];
#pragma unroll
        for (int f = 0; f < NC; ++f) cs[2][f] = hsum(c[f], wl, wr);
      }
      if constexpr (PH == 2) {
        const int g = r - 2;  // in [g0, g1) for every PH-2 row
        const float vt = g == 1 ? 2.f : 1.f, vb = g == h - 2 ? 2.f : 1.f;
        f2 sm[NC];
#pragma unroll
        for (int f = 0; f < NC; ++f) sm[f] = (vt * cs[0][f] + cs[1][f]) + vb * cs[2][f];
        const f2 x0 = xr[0], y0 = yr[0];
        const f2 diff = x0 - y0;
        const f2 sgn = pk(diff.x > 0.f ? 1.f : (diff.x < 0.f ? -1.f : 0.f),
                          diff.y > 0.f ? 1.f : (diff.y < 0.f ? -1.f : 0.f));
        l1sum += (out0 ? fabsf(diff.x) : 0.f) + (out1 ? fabsf(diff.y) : 0.f);
        const int64_t off = base + (int64_t)g * w + c0;
        {
          const f2 v = (sm[0] + 2.f * x0 * sm[1] + y0 * sm[2]) * inv9 + gs_l1 * sgn;
          if (out0) gx[off] = v.x;
          if (out1) gx[off + 1] = v.y;
        }
        if constexpr (GT) {
          const f2 v = (sm[3] + 2.f * y0 * sm[NC - 1] + x0 * sm[2]) * inv9 - gs_l1 * sgn;
          if (out0) gy[off] = v.x;
          if (out1) gy[off + 1] = v.y;
        }
      }
    };
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    // rows rs .. rs + 3: the rings fill (PH 0, 0, 1, 1); then the chunk's own
    // rows in groups of 6 (a multiple of the 3-row rings: a group leaves them
    // where it found them, so the unrolled body needs no register moves),
    // the next group's loads issued before this one's math (clamped to row re:
    // no rows of the next chunk); the last < 6 rows one by one
    constexpr int GR = 6;
    f2 px[4], py[4], cx[GR], cy[GR];
#pragma unroll
    for (int i = 0; i < 4; ++i) load(rs + i, px[i], py[i]);
#pragma unroll
    for (int i = 0; i < GR; ++i) load(min(rs + 4 + i, re), cx[i], cy[i]);
    step(P0{}, px[0], py[0], rs);
    step(P0{}, px[1], py[1], rs + 1);
    step(P1{}, px[2], py[2], rs + 2);
    step(P1{}, px[3], py[3], rs + 3);
    int r = rs + 4;
    for (; r + GR - 1 <= re; r += GR) {
      f2 nx[GR], ny[GR];
#pragma unroll
      for (int i = 0; i < GR; ++i) load(min(r + GR + i, re), nx[i], ny[i]);
#pragma unroll
      for (int i = 0; i < GR; ++i) step(P2{}, cx[i], cy[i], r + i);
#pragma unroll
      for (int i = 0; i < GR; ++i) {
        cx[i] = nx[i];
        cy[i] = ny[i];
      }
    }
#pragma unroll
    for (int i = 0; i < GR - 1; ++i)
      if (r + i <= re) step(P2{}, cx[i], cy[i], r + i);
  }
  const float ts = mde::block_sum256(lsum, red);
  const float tl = mde::block_sum256(l1sum, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ts;
    part[2 * blockIdx.x + 1] = tl;
  }
}

struct StreamPlan {
  int strips, chunks, chunk_rows, strip_major;
  int64_t nwaves, nblocks;
  int pair_sw;  // > 0: ssim3_pair_kernel with strips of pair_sw output columns
};

// MDE_SSIM_PAIR=0: the one-column-per-lane kernel (A/B)
inline bool ssim_pair() {
  static const bool on = [] {
    const char* e = std::getenv("MDE_SSIM_PAIR");
    return !(e && e[0] == '0');
  }();
  return on;
}

// ~5.5 waves per SIMD (5632) from strips x chunks, chunks of >= 16 rows: at
// 32x480x640, 30-row chunks (4 halo rows each).  The kernel is instruction-
// bound (84-88 us for 2816-8192 waves); fewer, taller chunks cut the halo
// re-reads (PMC: 1.79x algorithmic at 20-row chunks with the old prefetch
// overrun, 1.59x with the overrun clamped).
// pair: plan for ssim3_pair_kernel when it can take the shape (and the
// caller wants the prediction's gradient), else for ssim3_stream_kernel.
inline StreamPlan stream_plan(int64_t b, int64_t h, int64_t w, bool pair) {
  StreamPlan p;
  p.pair_sw = 0;
  if (pair && ssim_pair() && h * w < ((int64_t)1 << 29)) {  // strips of <= 124 columns (62 lane pairs
                                                     // + 2 halo lanes); a plane's bytes < 2^31
    p.strips = (int)mde::cdiv(w, 124);
    p.pair_sw = (int)(mde::cdiv(mde::cdiv(w, p.strips), 2) * 2);
  } else {
    p.strips = (int)mde::cdiv(w, kSW);
  }
  const int64_t per_chunk = b * p.strips;
  static const int64_t target_env = [] {  // MDE_SSIM_WAVES: tuning sweeps only
    const char* e = std::getenv("MDE_SSIM_WAVES");
    return e ? std::atoll(e) : 0;
  }();
  // the pair kernel does twice the work a wave: half the waves, so chunks stay
  // ~32 rows tall (3 halo rows each) at cfg2
  const int64_t target = target_env > 0 ? target_env : (p.pair_sw ? 2816 : 5632);
  int64_t ch = mde::cdiv(target, per_chunk);
  const int64_t maxc = mde::cdiv(h, 16);
  if (ch > maxc) ch = maxc;
  if (ch < 1) ch = 1;
  p.chunk_rows = (int)mde::cdiv(h, ch);
  // the pair kernel steps its chunk's rows in groups of 6: whole groups
  if (p.pair_sw && p.chunk_rows > 6) p.chunk_rows = p.chunk_rows / 6 * 6;
  p.chunks = (int)mde::cdiv(h, p.chunk_rows);
  p.nwaves = per_chunk * p.chunks;
  p.nblocks = mde::cdiv(p.nwaves, 4);
  static const int order = [] {  // MDE_SSIM_ORDER: wave order A/B (tools/gpu_r03d.sh)
    const char* e = std::getenv("MDE_SSIM_ORDER");
    return e ? std::atoi(e) : 0;
  }();
  p.strip_major = order;
  return p;
}

// loss[0] = w_ssim*ssim + w_l1*l1, loss[1] = ssim, loss[2] = l1.
__global__ void __launch_bounds__(256)
    loss_final_kernel(const float* __restrict__ part, int nparts,
                      float inv_numel, float w_ssim, float w_l1,
                      float* __restrict__ loss) {
  __shared__ float red[4];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  const float sa = mde::block_sum256(a, red);
  const float sb = mde::block_sum256(b, red);
  if (threadIdx.x == 0) {
    const float ls = sa * inv_numel, ll = sb * inv_numel;
    loss[0] = w_ssim * ls + w_l1 * ll;
    loss[1] = ls;
    loss[2] = ll;
  }
}

inline int minmax_blocks(int64_t numel) {
  const int64_t b = mde::cdiv(numel / 4 + 1, 256);
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}


}  // namespace

extern "C" {

size_t mde_minmax_workspace(int64_t numel) {
  return sizeof(float) * 2 * (size_t)minmax_blocks(numel);
}

int mde_minmax(const void* x, int64_t numel, float* minmax, void* workspace,
               int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || numel <= 0 || !minmax || !workspace) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int nb = minmax_blocks(numel);
  MDE_LAUNCH(mde::K_MINMAX, 4.0 * numel, s, minmax_partial_kernel, dim3(nb),
             dim3(256), 0, (const float*)x, numel, (float*)workspace);
  MDE_LAUNCH(mde::K_MINMAX_FINAL, 8.0 * nb, s, minmax_final_kernel, dim3(1),
             dim3(256), 0, (const float*)workspace, nb, minmax);
  return MDE_OK;
}

int mde_depthnorm_apply(const void* x, const float* minmax, void* y,
                        int64_t numel, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !y || numel <= 0 || !minmax) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  MDE_LAUNCH(mde::K_DEPTHNORM, 8.0 * numel, s, depthnorm_kernel,
             dim3(minmax_blocks(numel)), dim3(256), 0, (const float*)x,
             minmax, (float*)y, numel);
  return MDE_OK;
}

size_t mde_ssim3_l1_workspace(int64_t b, int64_t h, int64_t w) {
  if (b <= 0 || h <= 0 || w <= 0) return 0;
  const int64_t a = stream_plan(b, h, w, true).nblocks, c = stream_plan(b, h, w, false).nblocks;
  return sizeof(float) * 2 * (size_t)(a > c ? a : c);
}

int mde_ssim3_l1_fwd(const void* pred, const void* target,
                     const float* target_minmax, float w_ssim, float w_l1,
                     float* loss, void* grad_pred, void* grad_target,
                     int64_t b, int64_t h, int64_t w, void* workspace,
                     int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!pred || !target || !loss || !workspace || b <= 0 || h < 2 || w < 2 ||
      h > (1 << 24) || w > (1 << 24))
    return MDE_ERR_INVALID_ARG;
  const StreamPlan sp = stream_plan(b, h, w, grad_pred != nullptr);
  const int64_t nblocks = sp.nblocks;
  if (nblocks > 0x7fffffff) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t numel = b * h * w;
  const float inv = 1.f / (float)numel;
  float* part = (float*)workspace;
  const double bytes =
      4.0 * numel * (2.0 + (grad_pred ? 1.0 : 0.0) + (grad_target ? 1.0 : 0.0));
  if (sp.pair_sw > 0) {
    if (grad_target)
      MDE_LAUNCH(mde::K_SSIM3_L1, bytes, s, ssim3_pair_kernel<true>, dim3((unsigned)nblocks),
                 dim3(256), 0, (const float*)pred, (const float*)target, target_minmax, (int)h,
                 (int)w, sp.pair_sw, sp.strips, sp.chunks, sp.chunk_rows, sp.nwaves, w_ssim * inv,
                 w_l1 * inv, part, (float*)grad_pred, (float*)grad_target);
    else
      MDE_LAUNCH(mde::K_SSIM3_L1, bytes, s, ssim3_pair_kernel<false>, dim3((unsigned)nblocks),
                 dim3(256), 0, (const float*)pred, (const float*)target, target_minmax, (int)h,
                 (int)w, sp.pair_sw, sp.strips, sp.chunks, sp.chunk_rows, sp.nwaves, w_ssim * inv,
                 w_l1 * inv, part, (float*)grad_pred, (float*)nullptr);
  } else if (grad_target) {
    MDE_LAUNCH(mde::K_SSIM3_L1, bytes, s, ssim3_stream_kernel<true>, dim3((unsigned)nblocks),
               dim3(256), 0, (const float*)pred, (const float*)target, target_minmax, (int)h,
               (int)w, sp.strips, sp.chunks, sp.chunk_rows, sp.nwaves, w_ssim * inv, w_l1 * inv,
               part, (float*)grad_pred, (float*)grad_target, sp.strip_major);
  } else {
    MDE_LAUNCH(mde::K_SSIM3_L1, bytes, s, ssim3_stream_kernel<false>, dim3((unsigned)nblocks),
               dim3(256), 0, (const float*)pred, (const float*)target, target_minmax, (int)h,
               (int)w, sp.strips, sp.chunks, sp.chunk_rows, sp.nwaves, w_ssim * inv, w_l1 * inv,
               part, (float*)grad_pred, (float*)nullptr, sp.strip_major);
  }
  MDE_LAUNCH(mde::K_LOSS_FINAL, 8.0 * nblocks, s, loss_final_kernel, dim3(1),
             dim3(256), 0, part, (int)nblocks, inv, w_ssim, w_l1, loss);
  return MDE_OK;
}

}  // extern "C"
