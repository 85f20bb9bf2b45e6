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
// The 11x11 window is applied separably in LDS.  Because the SSIM clamp acts
// on the MEAN, the gradient scale needs the forward's global result: the
// backward recomputes per-pixel SSIM coefficients (kernel 1, written to the
// workspace) and then correlates them with the window (kernel 2), reading the
// forward scalars and the upstream gradient from device memory (no host sync).
#include <cmath>

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

size_t mde_depth_loss_workspace(int64_t b, int64_t h, int64_t w) {
  const Win win = make_window(h, w);
  const Geo g = geometry(b, h, w, win.k);
  return round16(sizeof(float) * 4 * (size_t)g.nblocks) +
         sizeof(float) * 3 * (size_t)b * g.ho * g.wo;
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
  MDE_LAUNCH(mde::K_DLOSS_FWD, 8.0 * numel, s, dloss_map_kernel<0>,
             dim3((unsigned)g.nblocks), dim3(256), 0, (const float*)pred,
             (const float*)gt, (int)h, (int)w, g.ho, g.wo, g.tiles_w,
             g.tiles_per_img, win, c1, c2, masked, part, (float*)nullptr,
             (const float*)nullptr, (const float*)nullptr, beta);
  MDE_LAUNCH(mde::K_LOSS_FINAL, 16.0 * g.nblocks, s, dloss_final_kernel,
             dim3(1), dim3(256), 0, part, (int)g.nblocks,
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
  float* coef = (float*)((char*)workspace +
                         round16(sizeof(float) * 4 * (size_t)g.nblocks));
  const int64_t plane = b * (int64_t)g.ho * g.wo;
  const double numel = (double)b * h * w;
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
