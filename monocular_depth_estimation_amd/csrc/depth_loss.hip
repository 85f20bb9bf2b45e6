// Depth_Loss of GuideDepth (src/GuideDepth/losses.py:15-127), NCHW fp32:
//   alpha * L1 + beta * clamp((1 - SSIM11) * 0.5, 0, 1) + gamma * grad
// SSIM11 (losses.py:41-79): Gaussian window (sigma 1.5) of size
// K = min(11, H, W), ZERO padding 5 (window_size // 2, even when K < 11),
// C1 = (0.01 L)^2, C2 = (0.03 L)^2, L = maxDepth, mean over the map.
// grad (losses.py:82-115): forward differences, last column / row zeroed,
// mean(|gt_dx - p_dx| + |gt_dy - p_dy|).
// Masked mode (beta == gamma == 0, losses.py:26-31): L1 over depth > 0, and
// the loss is that L1 alone (alpha is not applied).
//
// Full window (h, w >= 11, the training shapes): two register-streaming
// kernels, no LDS.  A wave owns a strip of 54 columns (64 lanes, a 5-column
// halo each side) and a chunk of rows and walks its rows top to bottom: the
// 11-tap horizontal Gaussian comes from DPP lane shifts, the vertical one
// from an 11-row register ring, so each input is read once per strip and
// chunk (plus halos).
//   forward  (dloss_fwd_stream_kernel): the five local statistics, SSIM, the
//            loss partial sums (SSIM, L1, gradient term; one record per wave)
//            AND the three per-position gradient coefficients of SSIM
//            (A, B, C below, without the global factor) into the workspace;
//   backward (dloss_bwd_stream_kernel): the clamp gate and scale are global
//            (the SSIM clamp acts on the MEAN), read from the forward's
//            device scalars; d/dx = k * (G*A + 2x G*B + y G*C) + the L1 and
//            gradient-difference terms, G* = the same window, correlated by
//            the same shift + ring scheme.  No statistic is recomputed.
// Small maps (K < 11) keep the LDS-tiled kernels, whose backward recomputes
// the coefficients (dloss_map_kernel<1>) before correlating them.  Masked
// mode is a plain streaming reduction / elementwise pass.
#include <cmath>

#include <cstdlib>

#include "common.h"

namespace {

constexpr int TH = 16, TW = 64, KMAX = 11, PAD = 5;
constexpr int RH = TH + KMAX - 1, RW = TW + KMAX - 1;

struct Win {
  float g[KMAX];
  int k;
};

Win make_window(int64_t h, int64_t w) {
  Win win{};
  int k = 11;
  if (h < k) k = (int)h;
  if (w < k) k = (int)w;
  win.k = k;
  float s = 0.f;
  for (int x = 0; x < k; ++x) {
    const double d = (double)(x - k / 2);
    win.g[x] = (float)std::exp(-(d * d) / (2.0 * 1.5 * 1.5));
    s += win.g[x];
  }
  for (int x = 0; x < k; ++x) win.g[x] /= s;
  return win;
}

// Map-domain statistics for one tile.  MODE 0: loss partial sums.
// MODE 1: gradient coefficients (A, B, C) of each map position -> coef.
template <int MODE>
__global__ void __launch_bounds__(256)
    dloss_map_kernel(const float* __restrict__ pp, const float* __restrict__ tp,
                     int h, int w, int ho, int wo, int tiles_w,
                     int tiles_per_img, Win win, float c1, float c2,
                     int masked, float* __restrict__ part,
                     float* __restrict__ coef, const float* __restrict__ fwd,
                     const float* __restrict__ gout, float beta) {
  __shared__ float sx[RH][RW], sy[RH][RW];
  __shared__ float hs[5][RH][TW];
  __shared__ float red[4];
  const int tid = threadIdx.x;
  const int img = blockIdx.x / tiles_per_img;
  const int tix = blockIdx.x % tiles_per_img;
  const int r0 = (tix / tiles_w) * TH, c0 = (tix % tiles_w) * TW;
  const int K = win.k;
  const float* X = pp + (int64_t)img * h * w;
  const float* Y = tp + (int64_t)img * h * w;

  // map position p reads image rows p-5 .. p-5+K-1 (zero outside)
  const int rh = TH + K - 1, rw = TW + K - 1;
  for (int e = tid; e < rh * rw; e += 256) {
    const int a = e / rw, b = e % rw;
    const int gr = r0 - PAD + a, gc = c0 - PAD + b;
    float xv = 0.f, yv = 0.f;
    if (gr >= 0 && gr < h && gc >= 0 && gc < w) {
      xv = X[(int64_t)gr * w + gc];
      yv = Y[(int64_t)gr * w + gc];
    }
    sx[a][b] = xv;
    sy[a][b] = yv;
  }
  __syncthreads();
  for (int e = tid; e < rh * TW; e += 256) {
    const int a = e / TW, v = e % TW;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
    for (int k = 0; k < K; ++k) {
      const float gk = win.g[k];
      const float xv = sx[a][v + k], yv = sy[a][v + k];
      s0 += gk * xv;
      s1 += gk * yv;
      s2 += gk * (xv * xv);
      s3 += gk * (yv * yv);
      s4 += gk * (xv * yv);
    }
    hs[0][a][v] = s0;
    hs[1][a][v] = s1;
    hs[2][a][v] = s2;
    hs[3][a][v] = s3;
    hs[4][a][v] = s4;
  }
  __syncthreads();

  float kfac = 0.f;
  if (MODE == 1) {
    // d loss / d S_p = gout * beta * (-0.5) * [0 <= (1-M)/2 <= 1] / |map|
    const float m = fwd[4];
    const float f = (1.f - m) * 0.5f;
    const bool act = f >= 0.f && f <= 1.f;
    const float nimg = (float)(gridDim.x / tiles_per_img);
    kfac = act ? gout[0] * beta * -0.5f / ((float)ho * (float)wo * nimg) : 0.f;
  }
  float ssum = 0.f;
  for (int e = tid; e < TH * TW; e += 256) {
    const int i0 = e / TW, j0 = e % TW;
    const int pr = r0 + i0, pc = c0 + j0;
    if (pr >= ho || pc >= wo) continue;
    float q[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const float gk = win.g[k];
#pragma unroll
      for (int z = 0; z < 5; ++z) q[z] += gk * hs[z][i0 + k][j0];
    }
    const float mx = q[0], my = q[1];
    const float sxx = q[2] - mx * mx, syy = q[3] - my * my;
    const float sxy = q[4] - mx * my;
    const float n1 = 2.f * mx * my + c1, n2 = 2.f * sxy + c2;
    const float d1 = mx * mx + my * my + c1, d2 = sxx + syy + c2;
    const float D = d1 * d2;
    const float S = (n1 * n2) / D;
    if (MODE == 0) {
      ssum += S;
    } else {
      const float dS_dsx = -S / d2;
      const float dS_dsxy = 2.f * n1 / D;
      const float dS_dmx = 2.f * my * n2 / D - S * 2.f * mx / d1;
      const int64_t off = (((int64_t)img * ho + pr) * wo + pc);
      const int64_t plane = (int64_t)ho * wo * gridDim.x / tiles_per_img;
      coef[off] = kfac * (dS_dmx - 2.f * mx * dS_dsx - my * dS_dsxy);
      coef[plane + off] = kfac * dS_dsx;
      coef[2 * plane + off] = kfac * dS_dsxy;
    }
  }
  if (MODE == 1) return;

  // image-domain terms on the same tile of pixels (map == image when K == 11;
  // otherwise cover the image with the tiles of the larger of the two grids)
  float l1 = 0.f, gr = 0.f, cnt = 0.f;
  for (int e = tid; e < TH * TW; e += 256) {
    const int i = r0 + e / TW, j = c0 + e % TW;
    if (i >= h || j >= w) continue;
    const int64_t o = (int64_t)i * w + j;
    const float pv = X[o], tv = Y[o];
    if (masked) {
      if (tv > 0.f) {
        l1 += fabsf(pv - tv);
        cnt += 1.f;
      }
    } else {
      l1 += fabsf(pv - tv);
      cnt += 1.f;
      if (j < w - 1) gr += fabsf((Y[o + 1] - tv) - (X[o + 1] - pv));
      if (i < h - 1) gr += fabsf((Y[o + w] - tv) - (X[o + w] - pv));
    }
  }
  const float a0 = mde::block_sum256(ssum, red);
  const float a1 = mde::block_sum256(l1, red);
  const float a2 = mde::block_sum256(gr, red);
  const float a3 = mde::block_sum256(cnt, red);
  if (tid == 0) {
    float* o = part + 4 * (int64_t)blockIdx.x;
    o[0] = a0;
    o[1] = a1;
    o[2] = a2;
    o[3] = a3;
  }
}

__global__ void __launch_bounds__(256)
    dloss_final_kernel(const float* __restrict__ part, int nparts,
                       float inv_numel, float inv_map, float alpha, float beta,
                       float gamma, int masked, float* __restrict__ out) {
  __shared__ float red[4];
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i = threadIdx.x; i < nparts; i += 256)
#pragma unroll
    for (int z = 0; z < 4; ++z) a[z] += part[4 * i + z];
  float s[4];
#pragma unroll
  for (int z = 0; z < 4; ++z) s[z] = mde::block_sum256(a[z], red);
  if (threadIdx.x == 0) {
    if (masked) {
      const float l1 = s[1] / s[3];
      out[0] = l1;
      out[1] = l1;
      out[2] = 0.f;
      out[3] = 0.f;
      out[4] = 0.f;
    } else {
      const float l1 = s[1] * inv_numel;
      const float m = s[0] * inv_map;
      const float ls = fminf(fmaxf((1.f - m) * 0.5f, 0.f), 1.f);
      const float lg = s[2] * inv_numel;
      out[0] = alpha * l1 + beta * ls + gamma * lg;
      out[1] = l1;
      out[2] = ls;
      out[3] = lg;
      out[4] = m;
    }
    out[5] = s[3];
  }
}

__device__ __forceinline__ float sgnf(float v) {
  return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f);
}

// Image-domain gradient: SSIM part by correlating the coefficient maps with
// the window, plus L1 and gradient-difference parts.
__global__ void __launch_bounds__(256)
    dloss_grad_kernel(const float* __restrict__ pp, const float* __restrict__ tp,
                      int h, int w, int ho, int wo, int tiles_w,
                      int tiles_per_img, Win win, int masked, int use_ssim,
                      float alpha, float gamma, const float* __restrict__ coef,
                      int64_t plane, const float* __restrict__ fwd,
                      const float* __restrict__ gout,
                      float* __restrict__ gx) {
  __shared__ float cs[3][RH][RW];
  __shared__ float hs[3][RH][TW];
  const int tid = threadIdx.x;
  const int img = blockIdx.x / tiles_per_img;
  const int tix = blockIdx.x % tiles_per_img;
  const int r0 = (tix / tiles_w) * TH, c0 = (tix % tiles_w) * TW;
  const int K = win.k;
  const float* X = pp + (int64_t)img * h * w;
  const float* Y = tp + (int64_t)img * h * w;
  const float go = gout[0];
  const int rh = TH + K - 1, rw = TW + K - 1;
  if (use_ssim) {
    // image q receives from map positions p in [q + 6 - K, q + 5]
    const int pr0 = r0 + PAD + 1 - K, pc0 = c0 + PAD + 1 - K;
    for (int e = tid; e < rh * rw; e += 256) {
      const int a = e / rw, b = e % rw;
      const int pr = pr0 + a, pc = pc0 + b;
      float v0 = 0.f, v1 = 0.f, v2 = 0.f;
      if (pr >= 0 && pr < ho && pc >= 0 && pc < wo) {
        const int64_t off = ((int64_t)img * ho + pr) * wo + pc;
        v0 = coef[off];
        v1 = coef[plane + off];
        v2 = coef[2 * plane + off];
      }
      cs[0][a][b] = v0;
      cs[1][a][b] = v1;
      cs[2][a][b] = v2;
    }
    __syncthreads();
    // weight of map column pc0 + j + a for image column c0 + j: g[K-1-a]
    for (int e = tid; e < rh * TW; e += 256) {
      const int a = e / TW, v = e % TW;
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
      for (int k = 0; k < K; ++k) {
        const float gk = win.g[K - 1 - k];
        s0 += gk * cs[0][a][v + k];
        s1 += gk * cs[1][a][v + k];
        s2 += gk * cs[2][a][v + k];
      }
      hs[0][a][v] = s0;
      hs[1][a][v] = s1;
      hs[2][a][v] = s2;
    }
    __syncthreads();
  }
  const float inv_n = 1.f / ((float)h * (float)w * (float)(gridDim.x / tiles_per_img));
  const float kl1 = masked ? go / fwd[5] : go * alpha * inv_n;
  const float kg = go * gamma * inv_n;
  for (int e = tid; e < TH * TW; e += 256) {
    const int i0 = e / TW, j0 = e % TW;
    const int i = r0 + i0, j = c0 + j0;
    if (i >= h || j >= w) continue;
    const int64_t o = (int64_t)i * w + j;
    const float pv = X[o], tv = Y[o];
    float g = 0.f;
    if (use_ssim) {
      float SA = 0.f, SB = 0.f, SC = 0.f;
      for (int k = 0; k < K; ++k) {
        const float gk = win.g[K - 1 - k];
        SA += gk * hs[0][i0 + k][j0];
        SB += gk * hs[1][i0 + k][j0];
        SC += gk * hs[2][i0 + k][j0];
      }
      g += SA + 2.f * pv * SB + tv * SC;
    }
    if (masked) {
      if (tv > 0.f) g += kl1 * sgnf(pv - tv);
    } else {
      g += kl1 * sgnf(pv - tv);
      if (gamma != 0.f) {
        // e = gt_d - p_d; d|e|/dp_d = -sgn(e); p_d(j) = p(j+1) - p(j)
        float acc = 0.f;
        if (j < w - 1) acc += sgnf((Y[o + 1] - tv) - (X[o + 1] - pv));
        if (j >= 1) acc -= sgnf((tv - Y[o - 1]) - (pv - X[o - 1]));
        if (i < h - 1) acc += sgnf((Y[o + w] - tv) - (X[o + w] - pv));
        if (i >= 1) acc -= sgnf((tv - Y[o - w]) - (pv - X[o - w]));
        g += kg * acc;
      }
    }
    gx[(int64_t)img * h * w + o] = g;
  }
}

// ------------------------------------------------------------ streaming
constexpr int kSD = 54;  // output columns per strip: 64 lanes - 2 x 5 halo

// value of lane - 1 / lane + 1 (DPP wave shift by one lane; bound_ctrl: the
// lane with no source reads 0, so no zero-initialised destination is needed)
__device__ __forceinline__ float lprev(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float lnext(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}

// base[i] through a 32-bit BYTE offset (i < 2^30, checked on the host): with a
// wave-uniform base the access is one VGPR offset on an SGPR pair, no 64-bit
// address arithmetic per load / store
__device__ __forceinline__ float ldo(const float* base, unsigned i) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + (i << 2));
}
__device__ __forceinline__ void sto(float* base, unsigned i, float v) {
  *reinterpret_cast<float*>(reinterpret_cast<char*>(base) + (i << 2)) = v;
}

// symmetric 11-tap window: c = g[5], k[i] = g[5 - 1 - i] = g[5 + 1 + i]
struct Sym11 {
  float c, k[5];
};

Sym11 sym11(const Win& w) {
  Sym11 s;
  s.c = w.g[5];
  for (int i = 0; i < 5; ++i) s.k[i] = w.g[4 - i];
  return s;
}

// Packed pairs: v_pk_{add,mul,fma}_f32 process two fp32 lanes of a VGPR pair
// per instruction, so the (x, y) and (mu_x, mu_y) / (E x^2, E y^2) filter
// chains run as pairs at twice the scalar VALU rate.
using v2 = float __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2 lprev2(v2 v) { return v2{lprev(v.x), lprev(v.y)}; }
__device__ __forceinline__ v2 lnext2(v2 v) { return v2{lnext(v.x), lnext(v.y)}; }

struct StreamGeo {
  int strips, chunks, chunk_rows;
  int64_t nwaves;
};

StreamGeo stream_geometry(int64_t b, int64_t h, int64_t w) {
  StreamGeo g;
  g.strips = (int)mde::cdiv(w, kSD);
  // ~3 waves per SIMD (measured at 32x480x640: 3072 waves 154.8 us fwd+bwd,
  // 4096 160.2, 6144 164.4); >= 34 rows per chunk (a
  // chunk re-reads 10 halo rows), = 1 (mod 11) so that a chunk streams whole
  // 11-row ring periods (rows + 10 = 0 mod 11): the unrolled period then has
  // no per-row trip guard (only an image's last chunk runs past its rows)
  static const int64_t target = [] {  // MDE_DL_WAVES: tuning sweeps (tools/kbench.py)
    const char* e = std::getenv("MDE_DL_WAVES");
    return e ? std::atoll(e) : 3072;
  }();
  const int64_t want = mde::cdiv(target, b * g.strips);
  int64_t rows = mde::cdiv(h, want < 1 ? 1 : want);
  if (rows < 34) rows = 34;
  rows = (rows + 9) / 11 * 11 + 1;  // next value = 1 (mod 11)
  if (rows > h) rows = h;
  g.chunk_rows = (int)rows;
  g.chunks = (int)mde::cdiv(h, rows);
  g.nwaves = b * g.strips * g.chunks;
  return g;
}

// Forward.  Lane l of a wave <-> column c = strip * 54 - 5 + l; output lanes
// 5..58.  Input rows r0 - 5 .. r1 + 4 of the chunk stream through; after
// row r the map row p = r - 5 is complete (ring slots hold rows p-5..p+5).
template <bool SSIM>
__global__ void __launch_bounds__(256)
    dloss_fwd_stream_kernel(const float* __restrict__ X, const float* __restrict__ Y, int h,
                            int w, int strips, int chunks, int chunk_rows, int64_t nwaves,
                            Sym11 g, float c1, float c2, float* __restrict__ part,
                            float* __restrict__ coef, int64_t plane) {
  const int lane = threadIdx.x & 63;
  // wave-uniform (scalar) indices: per-image bases stay in SGPRs
  const int64_t wid =
      (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (wid >= nwaves) return;
  const int strip = (int)(wid % strips);
  const int chunk = (int)((wid / strips) % chunks);
  const int64_t img = wid / ((int64_t)strips * chunks);
  const int c = strip * kSD - 5 + lane;
  const bool cin = c >= 0 && c < w;
  const bool outl = lane >= 5 && lane < 5 + kSD && c < w;
  const int cc = c < 0 ? 0 : (c >= w ? w - 1 : c);
  const int r0 = chunk * chunk_rows;
  const int r1 = r0 + chunk_rows < h ? r0 + chunk_rows : h;
  // per-image bases (wave-uniform) + 32-bit byte offsets (planes < 2^30)
  const float* Xi = X + img * (int64_t)h * w;
  const float* Yi = Y + img * (int64_t)h * w;
  const int T = (r1 - r0) + 10;  // rows streamed

  v2 r01[11], r23[11];  // ring of horizontally filtered rows: (x, y), (x^2, y^2)
  float r4[11];         // ... and x y
#pragma unroll
  for (int j = 0; j < 11; ++j) {
    r01[j] = v2{0.f, 0.f};
    r23[j] = v2{0.f, 0.f};
    r4[j] = 0.f;
  }
  float ssum = 0.f, l1 = 0.f, gr = 0.f, cnt = 0.f;
  float xp = 0.f, yp = 0.f;  // row r - 1
  // prefetched raw row (clamped address) and its in-range flag: the select
  // happens when the row is consumed, one iteration after the load is issued
  float xn, yn;
  bool okn;
  {
    const int r = r0 - 5;
    const int rc = r < 0 ? 0 : r;
    okn = cin && r >= 0;
    xn = ldo(Xi, (unsigned)(rc * w + cc));
    yn = ldo(Yi, (unsigned)(rc * w + cc));
  }
  // whole 11-row periods (T = 0 mod 11 except in an image's last chunk,
  // whose extra rows are past r1 + 4: no output, clamped loads)
  for (int t0 = 0; t0 < T; t0 += 11) {
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      const int t = t0 + j;
      {
      const int r = r0 - 5 + t;
      const float x = okn ? xn : 0.f, y = okn ? yn : 0.f;
      {  // prefetch row r + 1
        const int rn = r + 1;
        const int rc = rn < 0 ? 0 : (rn >= h ? h - 1 : rn);
        okn = cin && rn >= 0 && rn < h;
        xn = ldo(Xi, (unsigned)(rc * w + cc));
        yn = ldo(Yi, (unsigned)(rc * w + cc));
      }
      // image-domain terms: L1 and the horizontal difference of row r, the
      // vertical difference of row r - 1 (so the row r + 1 load just issued
      // is first needed one iteration later)
      if (r >= r0 && r < r1 && outl) {
        l1 += fabsf(x - y);
        cnt += 1.f;
      }
      const float xr = lnext(x), yr = lnext(y);
      if (r >= r0 && r < r1 && outl && c < w - 1) gr += fabsf((yr - y) - (xr - x));
      if (r - 1 >= r0 && r - 1 < r1 && outl && r < h) gr += fabsf((y - yp) - (x - xp));
      xp = x;
      yp = y;
      if (SSIM) {
        // horizontal 11-tap pass over (x, y): neighbours by DPP shifts, the
        // five statistics as two packed pairs and one scalar
        const v2 cxy = v2{x, y};
        v2 lxy = cxy, rxy = cxy;
        v2 h01 = g.c * cxy;
        v2 h23 = g.c * (cxy * cxy);
        float h4 = g.c * (x * y);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          lxy = lprev2(lxy);
          rxy = lnext2(rxy);
          h01 = g.k[i] * (lxy + rxy) + h01;
          h23 = g.k[i] * (lxy * lxy + rxy * rxy) + h23;
          h4 = fmaf(g.k[i], fmaf(lxy.x, lxy.y, rxy.x * rxy.y), h4);
        }
        r01[j] = h01;
        r23[j] = h23;
        r4[j] = h4;
        if (t >= 10 && r - 5 < r1) {  // map row p = r - 5: ring slot of row p + k - 5 is (j + 1 + k) % 11
          const int p = r - 5;
          v2 q01 = g.c * r01[(j + 6) % 11];
          v2 q23 = g.c * r23[(j + 6) % 11];
          float q4 = g.c * r4[(j + 6) % 11];
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            const int a = (j + 5 - i) % 11, b = (j + 7 + i) % 11;
            q01 = g.k[i] * (r01[a] + r01[b]) + q01;
            q23 = g.k[i] * (r23[a] + r23[b]) + q23;
            q4 = fmaf(g.k[i], r4[a] + r4[b], q4);
          }
          const float mx = q01.x, my = q01.y;
          const float sxx = q23.x - mx * mx, syy = q23.y - my * my;
          const float sxy = q4 - mx * my;
          const float n1 = 2.f * mx * my + c1, n2 = 2.f * sxy + c2;
          const float d1 = mx * mx + my * my + c1, d2 = sxx + syy + c2;
          const float D = d1 * d2;
          // one reciprocal (1 ulp) for the five quotients: 1/d2 = d1/D, 1/d1 = d2/D
          const float iD = __builtin_amdgcn_rcpf(D);
          const float S = (n1 * n2) * iD;
          if (outl) {
            ssum += S;
            if (coef) {
              const float dS_dsx = -S * (d1 * iD);
              const float dS_dsxy = 2.f * n1 * iD;
              const float dS_dmx = 2.f * my * n2 * iD - S * 2.f * mx * (d2 * iD);
              float* co = coef + img * (int64_t)h * w;
              const unsigned off = (unsigned)(p * w + c);
              sto(co, off, dS_dmx - 2.f * mx * dS_dsx - my * dS_dsxy);
              sto(co + plane, off, dS_dsx);
              sto(co + 2 * plane, off, dS_dsxy);
            }
          }
        }
      }
      }
    }
  }
  ssum = mde::wave_sum(ssum);
  l1 = mde::wave_sum(l1);
  gr = mde::wave_sum(gr);
  cnt = mde::wave_sum(cnt);
  if (lane == 0) {
    float* o = part + 4 * wid;
    o[0] = ssum;
    o[1] = l1;
    o[2] = gr;
    o[3] = cnt;
  }
}

// Backward: coefficient rows p = r0 - 5 .. r1 + 4 stream through the ring;
// after row p the image row q = p - 5 has all its window contributions.
template <bool SSIM, bool GRAD>
__global__ void __launch_bounds__(256)
    dloss_bwd_stream_kernel(const float* __restrict__ X, const float* __restrict__ Y, int h,
                            int w, int strips, int chunks, int chunk_rows, int64_t nwaves,
                            Sym11 g, const float* __restrict__ coef, int64_t plane,
                            const float* __restrict__ fwd, const float* __restrict__ gout,
                            float alpha, float beta, float gamma, float inv_n,
                            float* __restrict__ gx) {
  const int lane = threadIdx.x & 63;
  // wave-uniform (scalar) indices: per-image bases stay in SGPRs
  const int64_t wid =
      (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (wid >= nwaves) return;
  const int strip = (int)(wid % strips);
  const int chunk = (int)((wid / strips) % chunks);
  const int64_t img = wid / ((int64_t)strips * chunks);
  const int c = strip * kSD - 5 + lane;
  const bool cin = c >= 0 && c < w;
  const bool outl = lane >= 5 && lane < 5 + kSD && c < w;
  const int cc = c < 0 ? 0 : (c >= w ? w - 1 : c);
  const int r0 = chunk * chunk_rows;
  const int r1 = r0 + chunk_rows < h ? r0 + chunk_rows : h;
  const int64_t base = img * (int64_t)h * w;  // + 32-bit element offsets below
  const float* Xi = X + base;
  const float* Yi = Y + base;
  const float* Ai = coef + base;
  const int T = (r1 - r0) + 10;
  const float go = gout[0];
  float kfac = 0.f;
  if (SSIM) {  // d loss / d S_p = go * beta * (-1/2) * [0 <= (1 - M)/2 <= 1] / |map|
    const float f = (1.f - fwd[4]) * 0.5f;
    kfac = (f >= 0.f && f <= 1.f) ? go * beta * -0.5f * inv_n : 0.f;
  }
  const float kl1 = go * alpha * inv_n, kg = go * gamma * inv_n;

  v2 rab[11];     // ring of horizontally filtered coefficient rows: (A, B)
  float rcr[11];  // ... and C
#pragma unroll
  for (int j = 0; j < 11; ++j) {
    rab[j] = v2{0.f, 0.f};
    rcr[j] = 0.f;
  }
  // Loads use clamped addresses; their in-range flags are applied when the
  // row is consumed (one iteration after the load is issued), so no select
  // makes the wave wait for a load right after issuing it.
  auto load_coef = [&](int p, float& a, float& b, float& cv, bool& ok) {
    const int pc = p < 0 ? 0 : (p >= h ? h - 1 : p);
    ok = cin && p >= 0 && p < h;
    const unsigned o = (unsigned)(pc * w + cc);
    a = ldo(Ai, o);
    b = ldo(Ai + plane, o);
    cv = ldo(Ai + 2 * plane, o);
  };
  auto load_raw = [&](int r, float& x, float& y, bool& ok) {
    const int rc = r < 0 ? 0 : (r >= h ? h - 1 : r);
    ok = cin && r >= 0 && r < h;
    x = ldo(Xi, (unsigned)(rc * w + cc));
    y = ldo(Yi, (unsigned)(rc * w + cc));
  };
  // coefficient rows p (an.., oka) and p + 1 (an2.., oka2) in flight
  float an = 0.f, bn = 0.f, cn = 0.f, an2 = 0.f, bn2 = 0.f, cn2 = 0.f;
  bool oka = false, oka2 = false;
  if (SSIM) {
    load_coef(r0 - 5, an, bn, cn, oka);
    load_coef(r0 - 4, an2, bn2, cn2, oka2);
  }
  // raw rows q (x0, y0) and q + 1 (x1, y1) of the next output q, row q + 2
  // in flight (x2, y2, ok2); eyp = forward row difference of row q - 1
  float x0, y0, x1, y1, x2, y2;
  bool ok0, ok1, ok2;
  load_raw(r0, x0, y0, ok0);
  load_raw(r0 + 1, x1, y1, ok1);
  load_raw(r0 + 2, x2, y2, ok2);
  x0 = ok0 ? x0 : 0.f;
  y0 = ok0 ? y0 : 0.f;
  x1 = ok1 ? x1 : 0.f;
  y1 = ok1 ? y1 : 0.f;
  float eyp = 0.f;  // e_y of row r0 - 1 (only used when r0 >= 1)
  if (GRAD && r0 >= 1) {
    float xm, ym;
    bool okm;
    load_raw(r0 - 1, xm, ym, okm);
    eyp = (y0 - (okm ? ym : 0.f)) - (x0 - (okm ? xm : 0.f));
  }
  // whole 11-row periods (see stream_geometry); rows past r1 + 4 in an
  // image's last chunk produce no output
  for (int t0 = 0; t0 < T; t0 += 11) {
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      const int t = t0 + j;
      {
      if (SSIM) {
        const v2 ab = oka ? v2{an, bn} : v2{0.f, 0.f};
        const float cv = oka ? cn : 0.f;
        an = an2;
        bn = bn2;
        cn = cn2;
        oka = oka2;
        load_coef(r0 - 3 + t, an2, bn2, cn2, oka2);
        v2 l = ab, rr = ab;
        float lc = cv, rc = cv;
        v2 hab = g.c * ab;
        float hc = g.c * cv;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          l = lprev2(l);
          rr = lnext2(rr);
          lc = lprev(lc);
          rc = lnext(rc);
          hab = g.k[i] * (l + rr) + hab;
          hc = fmaf(g.k[i], lc + rc, hc);
        }
        rab[j] = hab;
        rcr[j] = hc;
      }
      if (t >= 10) {  // image row q = p - 5
        const int q = r0 + t - 10;
        float gsum = kl1 * ((x0 > y0) ? 1.f : (x0 < y0 ? -1.f : 0.f));
        if (SSIM) {
          v2 fab = g.c * rab[(j + 6) % 11];
          float fc = g.c * rcr[(j + 6) % 11];
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            const int a = (j + 5 - i) % 11, b = (j + 7 + i) % 11;
            fab = g.k[i] * (rab[a] + rab[b]) + fab;
            fc = fmaf(g.k[i], rcr[a] + rcr[b], fc);
          }
          gsum += kfac * (fab.x + 2.f * x0 * fab.y + y0 * fc);
        }
        float x3, y3;
        bool ok3;
        load_raw(q + 3, x3, y3, ok3);
        if (GRAD) {
          // e = gt_d - p_d (forward differences); dL/dp(j) = kg * (sgn e(j) - sgn e(j-1))
          const float xr = lnext(x0), yr = lnext(y0);
          const float ex = (yr - y0) - (xr - x0);
          const float sx = (c < w - 1) ? ((ex > 0.f) ? 1.f : (ex < 0.f ? -1.f : 0.f)) : 0.f;
          const float sxp = lprev(sx);  // sgn e_x(j - 1); 0 when j - 1 is the column -1
          const float ey = (y1 - y0) - (x1 - x0);
          const float sy = (q < h - 1) ? ((ey > 0.f) ? 1.f : (ey < 0.f ? -1.f : 0.f)) : 0.f;
          const float syp = (q >= 1) ? ((eyp > 0.f) ? 1.f : (eyp < 0.f ? -1.f : 0.f)) : 0.f;
          gsum += kg * ((sx - (c >= 1 ? sxp : 0.f)) + (sy - syp));
          eyp = ey;
        }
        if (outl && q < r1) sto(gx + base, (unsigned)(q * w + c), gsum);
        x0 = x1;
        y0 = y1;
        x1 = ok2 ? x2 : 0.f;
        y1 = ok2 ? y2 : 0.f;
        x2 = x3;
        y2 = y3;
        ok2 = ok3;
      }
      }
    }
  }
}

// Masked mode (beta == gamma == 0): L1 over gt > 0 only; partial record per
// block [0, sum |p - t| over t > 0, 0, count].
__global__ void __launch_bounds__(256)
    dloss_masked_kernel(const float* __restrict__ P, const float* __restrict__ Tg, int64_t n,
                        float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f, k = 0.f;
  const int64_t n4 = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 p = reinterpret_cast<const float4*>(P)[i];
    const float4 t = reinterpret_cast<const float4*>(Tg)[i];
    s += (t.x > 0.f ? fabsf(p.x - t.x) : 0.f) + (t.y > 0.f ? fabsf(p.y - t.y) : 0.f) +
         (t.z > 0.f ? fabsf(p.z - t.z) : 0.f) + (t.w > 0.f ? fabsf(p.w - t.w) : 0.f);
    k += (float)((t.x > 0.f) + (t.y > 0.f) + (t.z > 0.f) + (t.w > 0.f));
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += stride) {
    const float p = P[i], t = Tg[i];
    if (t > 0.f) {
      s += fabsf(p - t);
      k += 1.f;
    }
  }
  const float a = mde::block_sum256(s, red);
  const float b = mde::block_sum256(k, red);
  if (threadIdx.x == 0) {
    float* o = part + 4 * (int64_t)blockIdx.x;
    o[0] = 0.f;
    o[1] = a;
    o[2] = 0.f;
    o[3] = b;
  }
}

__global__ void __launch_bounds__(256)
    dloss_masked_bwd_kernel(const float* __restrict__ P, const float* __restrict__ Tg,
                            int64_t n, const float* __restrict__ fwd,
                            const float* __restrict__ gout, float* __restrict__ gx) {
  const float k = gout[0] / fwd[5];
  const int64_t n4 = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
  auto one = [&](float p, float t) {
    return t > 0.f ? k * ((p > t) ? 1.f : (p < t ? -1.f : 0.f)) : 0.f;
  };
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 p = reinterpret_cast<const float4*>(P)[i];
    const float4 t = reinterpret_cast<const float4*>(Tg)[i];
    reinterpret_cast<float4*>(gx)[i] =
        make_float4(one(p.x, t.x), one(p.y, t.y), one(p.z, t.z), one(p.w, t.w));
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += stride)
    gx[i] = one(P[i], Tg[i]);
}

int masked_blocks(int64_t n) {
  const int64_t b = mde::cdiv(n >> 2, 256 * 4);
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

struct Geo {
  int ho, wo, tiles_w, tiles_per_img;
  int64_t nblocks;
};

Geo geometry(int64_t b, int64_t h, int64_t w, int k) {
  Geo g;
  g.ho = (int)(h + 2 * PAD - k + 1);
  g.wo = (int)(w + 2 * PAD - k + 1);
  const int64_t gh = h > g.ho ? h : g.ho, gw = w > g.wo ? w : g.wo;
  g.tiles_w = (int)mde::cdiv(gw, TW);
  g.tiles_per_img = (int)(mde::cdiv(gh, TH) * g.tiles_w);
  g.nblocks = b * g.tiles_per_img;
  return g;
}

size_t round16(size_t v) { return (v + 15) & ~size_t(15); }

}  // namespace

extern "C" {

// [partial records][3 coefficient planes]; the forward fills the planes
// (full window), the backward reads them: pass the same workspace to both.
static size_t partial_slots(int64_t b, int64_t h, int64_t w) {
  const Win win = make_window(h, w);
  const Geo g = geometry(b, h, w, win.k);
  int64_t slots = g.nblocks;
  if (win.k == KMAX) {
    const int64_t sw = stream_geometry(b, h, w).nwaves;
    if (sw > slots) slots = sw;
  }
  const int64_t mb = masked_blocks(b * h * w);
  return (size_t)(mb > slots ? mb : slots);
}

static size_t coef_offset(int64_t b, int64_t h, int64_t w) {
  return round16(sizeof(float) * 4 * partial_slots(b, h, w));
}

size_t mde_depth_loss_workspace(int64_t b, int64_t h, int64_t w) {
  const Win win = make_window(h, w);
  const Geo g = geometry(b, h, w, win.k);
  return coef_offset(b, h, w) + sizeof(float) * 3 * (size_t)b * g.ho * g.wo;
}

int mde_depth_loss_fwd(const void* pred, const void* gt, float alpha,
                       float beta, float gamma, float max_depth, float* out,
                       int64_t b, int64_t h, int64_t w, void* workspace,
                       int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!pred || !gt || !out || !workspace || b <= 0 || h <= 0 || w <= 0 ||
      h > (1 << 24) || w > (1 << 24))
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const Win win = make_window(h, w);
  const Geo g = geometry(b, h, w, win.k);
  if (g.nblocks > 0x7fffffff) return MDE_ERR_INVALID_ARG;
  const int masked = (beta == 0.f && gamma == 0.f) ? 1 : 0;
  const float c1 = (0.01f * max_depth) * (0.01f * max_depth);
  const float c2 = (0.03f * max_depth) * (0.03f * max_depth);
  float* part = (float*)workspace;
  const double numel = (double)b * h * w;
  int nparts = (int)g.nblocks;
  if (masked) {
    nparts = masked_blocks(b * h * w);
    MDE_LAUNCH(mde::K_DLOSS_FWD, 8.0 * numel, s, dloss_masked_kernel, dim3(nparts), dim3(256),
               0, (const float*)pred, (const float*)gt, b * h * w, part);
  } else if (win.k == KMAX && h * w < ((int64_t)1 << 30)) {
    const StreamGeo sg = stream_geometry(b, h, w);
    nparts = (int)sg.nwaves;
    float* coef = (float*)((char*)workspace + coef_offset(b, h, w));
    const unsigned blocks = (unsigned)mde::cdiv(sg.nwaves, 4);
    // bytes: pred + target read, 3 coefficient planes written (when beta != 0)
    if (beta != 0.f)
      MDE_LAUNCH(mde::K_DLOSS_FWD, 20.0 * numel, s, dloss_fwd_stream_kernel<true>, dim3(blocks),
                 dim3(256), 0, (const float*)pred, (const float*)gt, (int)h, (int)w, sg.strips,
                 sg.chunks, sg.chunk_rows, sg.nwaves, sym11(win), c1, c2, part, coef,
                 b * h * w);
    else
      MDE_LAUNCH(mde::K_DLOSS_FWD, 8.0 * numel, s, dloss_fwd_stream_kernel<false>, dim3(blocks),
                 dim3(256), 0, (const float*)pred, (const float*)gt, (int)h, (int)w, sg.strips,
                 sg.chunks, sg.chunk_rows, sg.nwaves, sym11(win), c1, c2, part, (float*)nullptr,
                 b * h * w);
  } else {
    MDE_LAUNCH(mde::K_DLOSS_FWD, 8.0 * numel, s, dloss_map_kernel<0>,
               dim3((unsigned)g.nblocks), dim3(256), 0, (const float*)pred,
               (const float*)gt, (int)h, (int)w, g.ho, g.wo, g.tiles_w,
               g.tiles_per_img, win, c1, c2, masked, part, (float*)nullptr,
               (const float*)nullptr, (const float*)nullptr, beta);
  }
  MDE_LAUNCH(mde::K_LOSS_FINAL, 16.0 * nparts, s, dloss_final_kernel,
             dim3(1), dim3(256), 0, part, nparts,
             (float)(1.0 / numel), (float)(1.0 / ((double)b * g.ho * g.wo)),
             alpha, beta, gamma, masked, out);
  return MDE_OK;
}

int mde_depth_loss_bwd(const void* pred, const void* gt, float alpha,
                       float beta, float gamma, float max_depth,
                       const float* fwd_out, const float* gout,
                       void* grad_pred, int64_t b, int64_t h, int64_t w,
                       void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!pred || !gt || !fwd_out || !gout || !grad_pred || !workspace ||
      b <= 0 || h <= 0 || w <= 0 || h > (1 << 24) || w > (1 << 24))
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const Win win = make_window(h, w);
  const Geo g = geometry(b, h, w, win.k);
  if (g.nblocks > 0x7fffffff) return MDE_ERR_INVALID_ARG;
  const int masked = (beta == 0.f && gamma == 0.f) ? 1 : 0;
  const int use_ssim = (!masked && beta != 0.f) ? 1 : 0;
  const float c1 = (0.01f * max_depth) * (0.01f * max_depth);
  const float c2 = (0.03f * max_depth) * (0.03f * max_depth);
  float* coef = (float*)((char*)workspace + coef_offset(b, h, w));
  const int64_t plane = b * (int64_t)g.ho * g.wo;
  const double numel = (double)b * h * w;
  if (masked) {
    MDE_LAUNCH(mde::K_DLOSS_BWD, 12.0 * numel, s, dloss_masked_bwd_kernel,
               dim3(masked_blocks(b * h * w)), dim3(256), 0, (const float*)pred,
               (const float*)gt, b * h * w, fwd_out, gout, (float*)grad_pred);
    return MDE_OK;
  }
  if (win.k == KMAX && h * w < ((int64_t)1 << 30)) {  // coefficients left by the forward
    const StreamGeo sg = stream_geometry(b, h, w);
    const unsigned blocks = (unsigned)mde::cdiv(sg.nwaves, 4);
    const float inv_n = (float)(1.0 / numel);
    // bytes: pred + target read, gradient written, 3 coefficient planes read
    const double by = 12.0 * numel + (use_ssim ? 12.0 * numel : 0.0);
    auto kern = dloss_bwd_stream_kernel<false, false>;
    if (use_ssim && gamma != 0.f)
      kern = dloss_bwd_stream_kernel<true, true>;
    else if (use_ssim)
      kern = dloss_bwd_stream_kernel<true, false>;
    else if (gamma != 0.f)
      kern = dloss_bwd_stream_kernel<false, true>;
    MDE_LAUNCH(mde::K_DLOSS_BWD, by, s, kern, dim3(blocks), dim3(256), 0, (const float*)pred,
               (const float*)gt, (int)h, (int)w, sg.strips, sg.chunks, sg.chunk_rows, sg.nwaves,
               sym11(win), (const float*)coef, b * h * w, fwd_out, gout, alpha, beta, gamma,
               inv_n, (float*)grad_pred);
    return MDE_OK;
  }
  if (use_ssim) {
    MDE_LAUNCH(mde::K_DLOSS_BWD_COEF, 8.0 * numel + 12.0 * plane, s,
               dloss_map_kernel<1>, dim3((unsigned)g.nblocks), dim3(256), 0,
               (const float*)pred, (const float*)gt, (int)h, (int)w, g.ho,
               g.wo, g.tiles_w, g.tiles_per_img, win, c1, c2, masked,
               (float*)nullptr, coef, fwd_out, gout, beta);
  }
  MDE_LAUNCH(mde::K_DLOSS_BWD, 12.0 * numel + (use_ssim ? 12.0 * plane : 0.0),
             s, dloss_grad_kernel, dim3((unsigned)g.nblocks), dim3(256), 0,
             (const float*)pred, (const float*)gt, (int)h, (int)w, g.ho, g.wo,
             g.tiles_w, g.tiles_per_img, win, masked, use_ssim, alpha, gamma,
             coef, plane, fwd_out, gout, (float*)grad_pred);
  return MDE_OK;
}

}  // extern "C"
