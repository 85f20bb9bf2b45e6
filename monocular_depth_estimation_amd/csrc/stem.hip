// DDRNet-23-slim's stem convolution under bf16 autocast: 3 -> 32 channels,
// 3x3, stride 2, padding 1, on the fp32 image (src/GuideDepth/model/
// DDRNet_23_slim.py:230-233, conv1[0]).  Autocast's semantics: the image and
// the weight rounded to bf16 (RNE), fp32 accumulation, a bf16 output, an fp32
// weight gradient; the image needs no gradient.
//
// Forward: direct convolution on the vector ALUs (27 multiply-adds per output
// value -- 4 GFLOP at cfg3, far below the HBM time of reading the image and
// writing the output), the image tile staged in LDS once per block tile.
// Weight gradient: gw [32][27] = gy [32][P] . X [P][27] over all output
// pixels P, an implicit GEMM with the pixels as the reduction dimension on
// v_mfma_f32_32x32x16_bf16: A = gy rows (16-byte reads), B = the image
// gathered per tap; the stride-2 column gather is made contiguous by staging
// the image rows as three column planes (odd-shifted, even, odd), so every B
// fragment is one 16-byte LDS read.  Per-block partials + a fixed-order
// reduction: deterministic.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"

namespace {

using mde::bf16;
using u4v = uint32_t __attribute__((ext_vector_type(4)));
using bf8v = __bf16 __attribute__((ext_vector_type(8)));
using f16v = float __attribute__((ext_vector_type(16)));
using f4v = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float rbf(float v) { return mde::bf2f(mde::f2bf(v)); }

constexpr int kCI = 3, kK = 27;  // input channels, taps x channels

// ------------------------------------------------------------------ forward
// Block tile: kFR output rows x kFC output columns; thread: 2 adjacent output
// columns of one row, all CO channels (2 CO fp32 accumulators).
constexpr int kFR = 4, kFC = 128, kFXC = 2 * kFC + 4;  // staged image columns (pitch)

template <int CO>
__global__ void __launch_bounds__(256)
    stem_bf16_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                         bf16* __restrict__ y, int h, int wi, int ho, int wo, int tiles_c,
                         int tiles_per_img, int ntiles) {
  __shared__ __attribute__((aligned(16))) float sx[kCI][2 * kFR + 1][kFXC];
  __shared__ __attribute__((aligned(16))) float swt[kK][CO];  // [ci * 9 + ky * 3 + kx][co]
  const int tid = threadIdx.x;
  for (int i = tid; i < kK * CO; i += 256) {
    const int co = i % CO, k = i / CO;
    swt[k][co] = rbf(w[co * kK + k]);
  }
  const int tr = tid >> 6, cp = tid & 63;  // output row in the tile, column pair
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int img = t / tiles_per_img, rem = t - img * tiles_per_img;
    const int r0 = (rem / tiles_c) * kFR, c0 = (rem - (rem / tiles_c) * tiles_c) * kFC;
    const float* xi = x + (int64_t)img * kCI * h * wi;
    __syncthreads();  // the previous tile's readers are done (1st: the weights)
    // image rows 2 r0 - 1 .., columns 2 c0 - 1 .. 2 c0 + 2 kFC - 1 (zero
    // padding): wave wv stages rows wv, wv + 4, .. of the 27 (channel, row)
    // rows, lanes along the columns; every load of the thread is issued before
    // the first is used (a rolled load -> store loop waits out one memory
    // latency per element)
    {
      constexpr int NC = 2 * kFC + 1, NR = kCI * (2 * kFR + 1), RPW = (NR + 3) / 4;
      constexpr int CI = (NC + 63) / 64;
      const int wv = tid >> 6, lane = tid & 63;
      float v[RPW][CI];
#pragma unroll
      for (int a = 0; a < RPW; ++a) {
        const int rowi = wv + 4 * a, ci = rowi / (2 * kFR + 1), rr = rowi - ci * (2 * kFR + 1);
        const int gr = 2 * r0 - 1 + rr;
        const bool rok = rowi < NR && gr >= 0 && gr < h;
#pragma unroll
        for (int b = 0; b < CI; ++b) {
          const int gc = 2 * c0 - 1 + lane + 64 * b;
          v[a][b] = rok && gc >= 0 && gc < wi ? xi[((int64_t)ci * h + gr) * wi + gc] : 0.f;
        }
      }
#pragma unroll
      for (int a = 0; a < RPW; ++a) {
        const int rowi = wv + 4 * a, ci = rowi / (2 * kFR + 1), rr = rowi - ci * (2 * kFR + 1);
#pragma unroll
        for (int b = 0; b < CI; ++b)
          if (rowi < NR && lane + 64 * b < NC) sx[ci][rr][lane + 64 * b] = rbf(v[a][b]);
      }
    }
    __syncthreads();
    float acc[2][CO];
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int co = 0; co < CO; ++co) acc[e][co] = 0.f;
    // (ci, ky) rolled: unrolled, the compiler hoists all 216 weight reads
#pragma unroll 1
    for (int cy = 0; cy < 3 * kCI; ++cy) {
      const int ci = cy / 3, ky = cy - 3 * ci;
      // output column c0 + 2 cp + e, tap kx reads staged column 4 cp + 2 e + kx
        const float* row = &sx[ci][2 * tr + ky][4 * cp];
        const f4v a = *reinterpret_cast<const f4v*>(row);
        const float v[5] = {a[0], a[1], a[2], a[3], row[4]};
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float* wk = swt[cy * 3 + kx];
#pragma unroll
          for (int co = 0; co < CO; co += 4) {
            const f4v wv = *reinterpret_cast<const f4v*>(wk + co);  // broadcast read
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              acc[0][co + q] = fmaf(v[kx], wv[q], acc[0][co + q]);
              acc[1][co + q] = fmaf(v[kx + 2], wv[q], acc[1][co + q]);
            }
          }
        }
    }
    const int r = r0 + tr, c = c0 + 2 * cp;
    if (r < ho && c < wo) {
      bf16* yp = y + (int64_t)img * CO * ho * wo + (int64_t)r * wo + c;
      const int64_t plane = (int64_t)ho * wo;
#pragma unroll
      for (int co = 0; co < CO; ++co) {
        if (c + 1 < wo)  // wo even: the pair is whole
          *reinterpret_cast<uint32_t*>(yp + co * plane) =
              (uint32_t)mde::f2bf(acc[0][co]) | ((uint32_t)mde::f2bf(acc[1][co]) << 16);
        else
          yp[co * plane] = mde::f2bf(acc[0][co]);
      }
    }
  }
}

// ---------------------------------------------------------- weight gradient
// gw [CO][27] = gy [CO][P] . X [P][27] for the 3-input-channel 3x3 convs
// with stride S: the stem (S = 2) and the guided-upsampling blocks' guide
// convs (S = 1, 3 -> 16 / 32 / 64 on the image, modules.py:52-54; their gy
// arrives bf16 and is read as such).  Block tile: kWR output rows x kWC
// output columns; wave w: row w, 4 K-steps of 16 pixels.  Staged image: three
// column planes per (channel, image row), plane kx holding input column
// S (c0 + jj) - 1 + kx at index jj, so a B fragment -- 8 consecutive output
// columns at one tap -- is 16 contiguous bytes.  CO = 16: the A rows 16..31
// are zero.
constexpr int kWR = 4, kWC = 64, kWP = kWC + 8;  // plane / gy row pitch (bf16)

template <int CO, int S>
__global__ void __launch_bounds__(256)
    c3in3_bf16_wgrad_kernel(const bf16* __restrict__ gy, const float* __restrict__ x,
                            float* __restrict__ part, int h, int wi, int ho, int wo, int tiles_c,
                            int tiles_per_img, int ntiles) {
  constexpr int MT = (CO + 31) / 32;
  constexpr int SR = S * (kWR - 1) + 3, NC = S * (kWC - 1) + 3;  // staged rows / columns
  __shared__ __attribute__((aligned(16))) bf16 sxp[3][kCI][SR][kWP];
  __shared__ __attribute__((aligned(16))) bf16 sg[CO][kWR][kWP];
  static_assert(sizeof(sg) >= sizeof(float) * CO * 32, "reduction buffer");
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  const int wv = tid >> 6;
  // B column (tap index k = ci * 9 + ky * 3 + kx); k >= 27 are zero columns
  const int k = l32, kci = k / 9, kky = (k / 3) % 3, kkx = k % 3;
  const bool kon = k < kK;
  f16v acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
  const int64_t plane = (int64_t)ho * wo;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int img = t / tiles_per_img, rem = t - img * tiles_per_img;
    const int r0 = (rem / tiles_c) * kWR, c0 = (rem - (rem / tiles_c) * tiles_c) * kWC;
    const float* xi = x + (int64_t)img * kCI * h * wi;
    const bf16* gi = gy + (int64_t)img * CO * plane;
    __syncthreads();
    // Every load of the thread issued before the first use (a rolled load ->
    // store loop waits out one memory latency per element).  Image columns
    // S c0 - 1 + j, j < NC, of the 3 SR (channel, row) rows (wave wv: rows
    // wv, wv + 4, ..); column j is plane kx's index (j - kx) / S.
    {
      constexpr int NR = kCI * SR, RPW = (NR + 3) / 4, CI = (NC + 63) / 64;
      float v[RPW][CI];
#pragma unroll
      for (int a = 0; a < RPW; ++a) {
        const int rowi = wv + 4 * a, ci = rowi / SR, rr = rowi - ci * SR;
        const int gr = S * r0 - 1 + rr;
        const bool rok = rowi < NR && gr >= 0 && gr < h;
#pragma unroll
        for (int b = 0; b < CI; ++b) {
          const int gc = S * c0 - 1 + lane + 64 * b;
          v[a][b] = rok && gc >= 0 && gc < wi ? xi[((int64_t)ci * h + gr) * wi + gc] : 0.f;
        }
      }
      // gy rows [co][rr][64]: 16-byte loads (8 lanes a row) when wo % 8 == 0,
      // else 4-byte ones; zero outside the plane
      constexpr int GQ = CO * kWR * 8 / 256;  // 16-byte pieces a thread
      u4v gq[GQ];
      const bool v16 = (wo & 7) == 0;
#pragma unroll
      for (int a = 0; a < GQ; ++a) {
        const int pi = tid + 256 * a, cc = 8 * (pi & 7), rr = (pi >> 3) % kWR, co = pi / (8 * kWR);
        const int r = r0 + rr, c = c0 + cc;
        const bf16* src = gi + co * plane + (int64_t)r * wo + c;
        u4v q = {0u, 0u, 0u, 0u};
        if (r < ho) {
          if (v16 && c + 8 <= wo) {
            q = *reinterpret_cast<const u4v*>(src);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (c + 2 * e < wo) q[e] = *reinterpret_cast<const uint32_t*>(src + 2 * e);
          }
        }
        gq[a] = q;
      }
#pragma unroll
      for (int a = 0; a < RPW; ++a) {
        const int rowi = wv + 4 * a, ci = rowi / SR, rr = rowi - ci * SR;
        if (rowi >= NR) continue;
#pragma unroll
        for (int b = 0; b < CI; ++b) {
          const int j = lane + 64 * b;
          if (j >= NC) continue;
          const bf16 bv = mde::f2bf(v[a][b]);
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int d = j - kx;
            if (d >= 0 && d % S == 0 && d / S < kWC) sxp[kx][ci][rr][d / S] = bv;
          }
        }
      }
#pragma unroll
      for (int a = 0; a < GQ; ++a) {
        const int pi = tid + 256 * a, cc = 8 * (pi & 7), rr = (pi >> 3) % kWR, co = pi / (8 * kWR);
        *reinterpret_cast<u4v*>(&sg[co][rr][cc]) = gq[a];
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kWC / 16; ++s) {
      const int j0 = 16 * s + 8 * hh;
      u4v b = {0u, 0u, 0u, 0u};
      if (kon) b = *reinterpret_cast<const u4v*>(&sxp[kkx][kci][S * wv + kky][j0]);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        u4v a = {0u, 0u, 0u, 0u};
        if (32 * m + l32 < CO) a = *reinterpret_cast<const u4v*>(&sg[32 * m + l32][wv][j0]);
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8v, a),
                                                          __builtin_bit_cast(bf8v, b), acc[m], 0,
                                                          0, 0);
      }
    }
  }
  // the 4 waves' accumulators in a fixed order -> part[block][co][k]
  __syncthreads();
  float* red = reinterpret_cast<float*>(&sg[0][0][0]);  // [CO][32] floats
  for (int wsel = 0; wsel < 4; ++wsel) {
    if (wv == wsel) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (co < CO) {
            float* p = red + co * 32 + l32;
            *p = wsel ? *p + acc[m][r] : acc[m][r];
          }
        }
    }
    __syncthreads();
  }
  float* o = part + (int64_t)blockIdx.x * CO * kK;
  for (int i = tid; i < CO * kK; i += 256) o[i] = red[(i / kK) * 32 + i % kK];
}

// gw[e] = sum over blocks of part[block][e]: one block an element, a fixed
// per-thread order and a fixed tree (deterministic).  TAG only tells the
// callers apart in profiles (0: the stem, 1: the guide convs).
template <int TAG>
__global__ void __launch_bounds__(256)
    stem_wreduce_kernel(const float* __restrict__ part, float* __restrict__ gw, int nblocks, int ne) {
  __shared__ float red[4];
  const int e = blockIdx.x;
  float a = 0.f;
  for (int b = threadIdx.x; b < nblocks; b += 256) a += part[(int64_t)b * ne + e];
  a = mde::block_sum256(a, red);
  if (threadIdx.x == 0) gw[e] = a;
}

int cus() {
  static const int c = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  return c;
}

bool shape_ok(int64_t n, int64_t cout, int64_t h, int64_t w) {
  return n > 0 && (cout == 32 || cout == 64) && h >= 2 && w >= 2 && w % 4 == 0 && h < (1 << 15) &&
         w < (1 << 15) && n * h * w * 3 < ((int64_t)1 << 31);
}

int wgrad_blocks(int64_t ntiles) {
  const int64_t g = 4 * (int64_t)cus();
  return (int)(ntiles < g ? ntiles : g);
}

bool guide_ok(int64_t n, int64_t cout, int64_t h, int64_t w) {
  return n > 0 && (cout == 16 || cout == 32 || cout == 64) && h >= 1 && w >= 4 && w % 4 == 0 &&
         h < (1 << 15) && w < (1 << 15) && n * h * w * 3 < ((int64_t)1 << 31);
}

template <int CO, int S>
int launch_c3in3_wgrad(const bf16* gy, const float* x, float* gw, int64_t n, int64_t h, int64_t w,
                       int ho, int wo, float* part, int kid, hipStream_t s) {
  const int tiles_c = (int)mde::cdiv(wo, kWC), tiles_r = (int)mde::cdiv(ho, kWR);
  const int64_t ntiles = n * tiles_c * tiles_r;
  if (ntiles >= ((int64_t)1 << 31)) return MDE_ERR_UNSUPPORTED;
  const int nb = wgrad_blocks(ntiles);
  const double bytes = 4.0 * n * 3 * h * w + 2.0 * n * CO * ho * wo;
  const double flops = 2.0 * kK * CO * (double)n * ho * wo;
  MDE_LAUNCH_MFMA(kid, bytes, flops, s, (c3in3_bf16_wgrad_kernel<CO, S>), dim3(nb), dim3(256), 0,
                  gy, x, part, (int)h, (int)w, ho, wo, tiles_c, tiles_c * tiles_r, (int)ntiles);
  const int ne = CO * kK;
  MDE_LAUNCH(kid, 4.0 * nb * ne, s, stem_wreduce_kernel<S == 2 ? 0 : 1>, dim3((unsigned)ne), dim3(256), 0, part,
             gw, nb, ne);
  return MDE_OK;
}

}  // namespace

extern "C" {

int mde_stem_bf16_supported(int64_t cin, int64_t cout, int64_t h, int64_t w) {
  return cin == 3 && shape_ok(1, cout, h, w) ? 1 : 0;
}

int mde_stem_bf16_fwd(const float* x, const float* weight, void* y, int64_t n, int64_t cout,
                      int64_t h, int64_t w, void* stream) {
  if (!x || !weight || !y) return MDE_ERR_INVALID_ARG;
  if (!shape_ok(n, cout, h, w)) return MDE_ERR_UNSUPPORTED;
  const int ho = (int)((h - 1) / 2 + 1), wo = (int)((w - 1) / 2 + 1);
  const int tiles_c = (int)mde::cdiv(wo, kFC), tiles_r = (int)mde::cdiv(ho, kFR);
  const int64_t ntiles = n * tiles_c * tiles_r;
  if (ntiles >= ((int64_t)1 << 31)) return MDE_ERR_UNSUPPORTED;
  const int64_t g = 8 * (int64_t)cus();
  const dim3 grid((unsigned)(ntiles < g ? ntiles : g));
  const double bytes = 4.0 * n * 3 * h * w + 2.0 * n * cout * ho * wo;
  const double flops = 2.0 * kK * cout * (double)n * ho * wo;
  hipStream_t s = (hipStream_t)stream;
  if (cout == 32)
    MDE_LAUNCH_MFMA(mde::K_STEM_FWD, bytes, flops, s, stem_bf16_fwd_kernel<32>, grid, dim3(256), 0,
                    x, weight, (bf16*)y, (int)h, (int)w, ho, wo, tiles_c, tiles_c * tiles_r,
                    (int)ntiles);
  else
    MDE_LAUNCH_MFMA(mde::K_STEM_FWD, bytes, flops, s, stem_bf16_fwd_kernel<64>, grid, dim3(256), 0,
                    x, weight, (bf16*)y, (int)h, (int)w, ho, wo, tiles_c, tiles_c * tiles_r,
                    (int)ntiles);
  return MDE_OK;
}

size_t mde_stem_bf16_wgrad_workspace(int64_t n, int64_t cout, int64_t h, int64_t w) {
  if (!shape_ok(n, cout, h, w)) return 0;
  const int64_t ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const int64_t ntiles = n * mde::cdiv(wo, kWC) * mde::cdiv(ho, kWR);
  return sizeof(float) * (size_t)wgrad_blocks(ntiles) * (size_t)(cout * kK);
}

int mde_stem_bf16_wgrad(const void* gy, const float* x, float* gweight, int64_t n, int64_t cout,
                        int64_t h, int64_t w, void* workspace, void* stream) {
  if (!gy || !x || !gweight || !workspace) return MDE_ERR_INVALID_ARG;
  if (!shape_ok(n, cout, h, w)) return MDE_ERR_UNSUPPORTED;
  const int ho = (int)((h - 1) / 2 + 1), wo = (int)((w - 1) / 2 + 1);
  if (cout == 32)
    return launch_c3in3_wgrad<32, 2>((const bf16*)gy, x, gweight, n, h, w, ho, wo,
                                     (float*)workspace, mde::K_STEM_WGRAD, (hipStream_t)stream);
  return launch_c3in3_wgrad<64, 2>((const bf16*)gy, x, gweight, n, h, w, ho, wo,
                                   (float*)workspace, mde::K_STEM_WGRAD, (hipStream_t)stream);
}

size_t mde_conv3x3_guide_bf16_wgrad_workspace(int64_t n, int64_t cout, int64_t h, int64_t w) {
  if (!guide_ok(n, cout, h, w)) return 0;
  const int64_t ntiles = n * mde::cdiv(w, kWC) * mde::cdiv(h, kWR);
  return sizeof(float) * (size_t)wgrad_blocks(ntiles) * (size_t)(cout * kK);
}

int mde_conv3x3_guide_bf16_wgrad(const void* gy, const float* x, float* gweight, int64_t n,
                                 int64_t cout, int64_t h, int64_t w, void* workspace,
                                 void* stream) {
  if (!gy || !x || !gweight || !workspace) return MDE_ERR_INVALID_ARG;
  if (!guide_ok(n, cout, h, w)) return MDE_ERR_UNSUPPORTED;
  const bf16* g = (const bf16*)gy;
  float* ws = (float*)workspace;
  hipStream_t s = (hipStream_t)stream;
  const int k = mde::K_C3_WGRAD_GUIDE;
  if (cout == 16) return launch_c3in3_wgrad<16, 1>(g, x, gweight, n, h, w, h, w, ws, k, s);
  if (cout == 32) return launch_c3in3_wgrad<32, 1>(g, x, gweight, n, h, w, h, w, ws, k, s);
  return launch_c3in3_wgrad<64, 1>(g, x, gweight, n, h, w, h, w, ws, k, s);
}

}  // extern "C"
