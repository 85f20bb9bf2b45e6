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
// so one tiled pass produces the loss partial sums AND d loss/d pred:
//   tile 16x64 outputs, inputs staged with a 2-pixel reflected halo, per-pixel
//   SSIM statistics on the tile + 1 ring (separable 3x3 box in LDS), then the
//   transposed box of the per-pixel coefficients (with reflection
//   multiplicities) gives the gradient.  Loss partials go to a per-block slab
//   summed in block order by loss_final_kernel (deterministic).
#include "common.h"

namespace {

constexpr float kC1 = 0.01f * 0.01f;
constexpr float kC2 = 0.03f * 0.03f;
constexpr int TH = 16, TW = 64;          // output tile
constexpr int RH = TH + 4, RW = TW + 4;  // input region (2-pixel halo)
constexpr int CH = TH + 2, CW = TW + 2;  // coefficient region (1-pixel ring)

__device__ __forceinline__ int reflect1(int q, int n) {
  if (q < 0) q = -q;
  if (q > n - 1) q = 2 * (n - 1) - q;
  return q < 0 ? 0 : (q > n - 1 ? n - 1 : q);
}

// Times output index i receives the padded sample taken at window centre p.
__device__ __forceinline__ int mult(int p, int i, int n) {
  int m = 0;
#pragma unroll
  for (int dq = -1; dq <= 1; ++dq) m += reflect1(p + dq, n) == i;
  return m;
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
template <bool GT>
__global__ void __launch_bounds__(256)
    ssim3_l1_kernel(const float* __restrict__ xp, const float* __restrict__ yp,
                    const float* __restrict__ mm, int h, int w, int tiles_w,
                    int tiles_per_img, float gs_ssim, float gs_l1,
                    float* __restrict__ part, float* __restrict__ gx,
                    float* __restrict__ gy) {
  __shared__ float sx[RH][RW], sy[RH][RW];
  __shared__ float hs[5][RH][CW];
  __shared__ float ca[CH][CW], cb[CH][CW], cc[CH][CW];
  __shared__ float cay[GT ? CH : 1][GT ? CW : 1], cby[GT ? CH : 1][GT ? CW : 1];
  __shared__ float red[4];

  const int tid = threadIdx.x;
  const int img = blockIdx.x / tiles_per_img;
  const int tix = blockIdx.x % tiles_per_img;
  const int r0 = (tix / tiles_w) * TH, c0 = (tix % tiles_w) * TW;
  const int64_t base = (int64_t)img * h * w;
  const float* X = xp + base;
  const float* Y = yp + base;
  float tmn = 0.f, tden = 1.f;
  const bool norm = mm != nullptr;
  if (norm) {
    tmn = mm[0];
    tden = mm[1] - mm[0];
  }

  // 1. inputs with a reflected 2-pixel halo
  for (int e = tid; e < RH * RW; e += 256) {
    const int a = e / RW, b = e % RW;
    const int gr = reflect1(r0 - 2 + a, h), gc = reflect1(c0 - 2 + b, w);
    const int64_t off = (int64_t)gr * w + gc;
    sx[a][b] = X[off];
    const float t = Y[off];
    sy[a][b] = norm ? (t - tmn) / tden : t;
  }
  __syncthreads();

  // 2. horizontal 3-sums of x, y, x^2, y^2, xy for the coefficient columns
  for (int e = tid; e < RH * CW; e += 256) {
    const int a = e / CW, v = e % CW;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float xv = sx[a][v + k], yv = sy[a][v + k];
      s0 += xv;
      s1 += yv;
      s2 += xv * xv;
      s3 += yv * yv;
      s4 += xv * yv;
    }
    hs[0][a][v] = s0;
    hs[1][a][v] = s1;
    hs[2][a][v] = s2;
    hs[3][a][v] = s3;
    hs[4][a][v] = s4;
  }
  __syncthreads();

  // 3. per-pixel statistics, loss and gradient coefficients on tile + ring
  float lsum = 0.f;
  const float inv9 = 1.f / 9.f;
  for (int e = tid; e < CH * CW; e += 256) {
    const int u = e / CW, v = e % CW;
    const int pr = r0 - 1 + u, pc = c0 - 1 + v;
    float A = 0.f, B = 0.f, C = 0.f, Ay = 0.f, By = 0.f;
    if (pr >= 0 && pr < h && pc >= 0 && pc < w) {
      float q[5];
#pragma unroll
      for (int k = 0; k < 5; ++k)
        q[k] = (hs[k][u][v] + hs[k][u + 1][v] + hs[k][u + 2][v]) * inv9;
      const float mx = q[0], my = q[1];
      const float sxx = q[2] - mx * mx, syy = q[3] - my * my;
      const float sxy = q[4] - mx * my;
      const float n1 = 2.f * mx * my + kC1, n2 = 2.f * sxy + kC2;
      const float d1 = mx * mx + my * my + kC1, d2 = sxx + syy + kC2;
      const float D = d1 * d2;
      const float S = (n1 * n2) / D;
      const float f = (1.f - S) * 0.5f;
      const bool inside = u >= 1 && u <= TH && v >= 1 && v <= TW;
      if (inside) lsum += fminf(fmaxf(f, 0.f), 1.f);
      if (f >= 0.f && f <= 1.f) {
        const float k = gs_ssim * -0.5f;
        const float dS_dsx = -S / d2;          // = dS/dsyy
        const float dS_dsxy = 2.f * n1 / D;
        const float dS_dmx = 2.f * my * n2 / D - S * 2.f * mx / d1;
        const float dS_dmy = 2.f * mx * n2 / D - S * 2.f * my / d1;
        A = k * (dS_dmx - 2.f * mx * dS_dsx - my * dS_dsxy);
        B = k * dS_dsx;
        C = k * dS_dsxy;
        Ay = k * (dS_dmy - 2.f * my * dS_dsx - mx * dS_dsxy);
        By = B;
      }
    }
    ca[u][v] = A;
    cb[u][v] = B;
    cc[u][v] = C;
    if (GT) {
      cay[u][v] = Ay;
      cby[u][v] = By;
    }
  }
  __syncthreads();

  // 4. gradient + L1 on the tile.  Two pixels away from the image border
  // every window centre reaches each pixel exactly once (the reflected
  // windows of centres 0 and n-1 hit pixels 1 and n-2 twice), so such tiles
  // take a plain 3x3 sum.
  float l1sum = 0.f;
  const bool interior = r0 >= 2 && r0 + TH <= h - 2 && c0 >= 2 && c0 + TW <= w - 2;
  for (int e = tid; e < TH * TW; e += 256) {
    const int i0 = e / TW, j0 = e % TW;
    const int gi = r0 + i0, gj = c0 + j0;
    if (gi >= h || gj >= w) continue;
    const float xv = sx[i0 + 2][j0 + 2], yv = sy[i0 + 2][j0 + 2];
    float SA = 0.f, SB = 0.f, SC = 0.f, SAy = 0.f, SBy = 0.f;
    if (interior) {
#pragma unroll
      for (int u = i0; u < i0 + 3; ++u)
#pragma unroll
        for (int v = j0; v < j0 + 3; ++v) {
          SA += ca[u][v];
          SB += cb[u][v];
          SC += cc[u][v];
          if (GT) {
            SAy += cay[u][v];
            SBy += cby[u][v];
          }
        }
    } else {
#pragma unroll
    for (int du = -1; du <= 1; ++du) {
      const int pr = gi + du;
      if (pr < 0 || pr >= h) continue;
      const int mr = mult(pr, gi, h);
      if (!mr) continue;
#pragma unroll
      for (int dv = -1; dv <= 1; ++dv) {
        const int pc = gj + dv;
        if (pc < 0 || pc >= w) continue;
        const int m = mr * mult(pc, gj, w);
        if (!m) continue;
        const float fm = (float)m;
        const int u = i0 + 1 + du, v = j0 + 1 + dv;
        SA += fm * ca[u][v];
        SB += fm * cb[u][v];
        SC += fm * cc[u][v];
        if (GT) {
          SAy += fm * cay[u][v];
          SBy += fm * cby[u][v];
        }
      }
    }
    }
    const float diff = xv - yv;
    l1sum += fabsf(diff);
    const float sgn = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
    const int64_t off = base + (int64_t)gi * w + gj;
    if (gx) gx[off] = (SA + 2.f * xv * SB + yv * SC) * inv9 + gs_l1 * sgn;
    if (GT && gy) gy[off] = (SAy + 2.f * yv * SBy + xv * SC) * inv9 - gs_l1 * sgn;
  }

  const float ts = mde::block_sum256(lsum, red);
  const float tl = mde::block_sum256(l1sum, red);
  if (tid == 0) {
    part[2 * blockIdx.x] = ts;
    part[2 * blockIdx.x + 1] = tl;
  }
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

inline int64_t ssim_blocks(int64_t b, int64_t h, int64_t w) {
  return b * mde::cdiv(h, TH) * mde::cdiv(w, TW);
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
  return sizeof(float) * 2 * (size_t)ssim_blocks(b, h, w);
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
  const int64_t nblocks = ssim_blocks(b, h, w);
  if (nblocks > 0x7fffffff) return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t numel = b * h * w;
  const float inv = 1.f / (float)numel;
  const int tiles_w = (int)mde::cdiv(w, TW);
  const int tiles_per_img = (int)(mde::cdiv(h, TH) * tiles_w);
  float* part = (float*)workspace;
  const double bytes =
      4.0 * numel * (2.0 + (grad_pred ? 1.0 : 0.0) + (grad_target ? 1.0 : 0.0));
  if (grad_target) {
    MDE_LAUNCH(mde::K_SSIM3_L1, bytes, s, ssim3_l1_kernel<true>,
               dim3((unsigned)nblocks), dim3(256), 0, (const float*)pred,
               (const float*)target, target_minmax, (int)h, (int)w, tiles_w,
               tiles_per_img, w_ssim * inv, w_l1 * inv, part,
               (float*)grad_pred, (float*)grad_target);
  } else {
    MDE_LAUNCH(mde::K_SSIM3_L1, bytes, s, ssim3_l1_kernel<false>,
               dim3((unsigned)nblocks), dim3(256), 0, (const float*)pred,
               (const float*)target, target_minmax, (int)h, (int)w, tiles_w,
               tiles_per_img, w_ssim * inv, w_l1 * inv, part,
               (float*)grad_pred, (float*)nullptr);
  }
  MDE_LAUNCH(mde::K_LOSS_FINAL, 8.0 * nblocks, s, loss_final_kernel, dim3(1),
             dim3(256), 0, part, (int)nblocks, inv, w_ssim, w_l1, loss);
  return MDE_OK;
}

}  // extern "C"
