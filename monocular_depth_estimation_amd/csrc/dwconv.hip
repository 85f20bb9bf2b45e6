// Depthwise convolution (groups == channels, square k3/k5, stride 1/2, zero
// padding, no bias), NCHW fp32: MobileNetV3-Large's 15 depthwise stages
// (torchvision mobilenet_v3_large().features[1..15].block[*][0], used at
// src/model_mobileV3_large_newCRFs.py:165,178-182).
//
// Blocks are LDS-tiled over one (image, channel) plane: a block stages the
// input window its tile needs (tile + halo, zero-filled outside the plane)
// with coalesced reads and keeps the plane's k*k taps in registers.
//   fwd       y[oy,ox]  = sum_t w[t] x[oy*s-p+ky, ox*s-p+kx]
//             (strip-blocked: a thread computes 4 rows of one column)
//   bwd, p == k/2 (every torchvision stage): ONE fused kernel per channel
//             group -- gy window + x window staged once per tile, gx written
//             and the weight-gradient sums kept in registers across the
//             group's (image, tile) items; per-group partials are then summed
//             in a fixed order (deterministic, no atomics).
//   bwd, other p: separate data-gradient (input-space tiles) and
//             weight-gradient (per-tile partials) kernels.
//   bwd data  gx[iy,ix] = sum over taps with (iy+p-ky) % s == 0 of
//                         w[t] gy[(iy+p-ky)/s, (ix+p-kx)/s]
//   bwd wgt   gw[c,t]   = sum_{n,oy,ox} gy[oy,ox] x[oy*s-p+ky, ox*s-p+kx]
// Algorithmic HBM bytes: fwd 4(|x| + |y|), fused bwd 4(|gy| + |x| + |gx|),
// split bwd 4(|gy| + |gx|) + 4(|gy| + |x|).

#include "common.h"

namespace mde {
namespace {

// Tiles: an output (fwd, weight grad) or input (data grad) region of
// th x tw elements per block, ~1024 elements (4 per thread), with tw and th
// balanced against the plane so small late-stage planes (15x20, 30x40) are
// one or two tiles with no idle columns.  Threads walk the tile's elements in
// row-major order (coalesced global reads / writes); the input window sits in
// LDS (dynamic size), staged with all of a thread's loads in flight at once.
struct DwShape {
  int64_t c, h, w, ho, wo;
  int pad;
};

struct DwTile {
  int tw, th;   // tile extent (elements of the space the kernel writes)
  int iw, ih;   // staged LDS window
  int tx, ty;   // tiles per plane along x / y
};

constexpr int kElems = 1024;  // tile elements per block
constexpr int kChunk = 8;     // loads in flight per thread while staging

DwTile tile_for(int64_t hh, int64_t ww) {
  DwTile t;
  t.tx = (int)cdiv(ww, 64);
  t.tw = (int)cdiv(ww, t.tx);
  t.ty = (int)cdiv(hh * t.tw, kElems);
  t.th = (int)cdiv(hh, t.ty);
  t.ty = (int)cdiv(hh, t.th);
  t.iw = t.ih = 0;
  return t;
}

// tile[r * iw + col] = src[(r0 + r) * w + c0 + col], zero outside the plane.
__device__ __forceinline__ void stage_window(const float* __restrict__ src, float* tile, int ih,
                                             int iw, int64_t r0, int64_t c0, int64_t h,
                                             int64_t w) {
  const int total = ih * iw;
  for (int base = 0; base < total; base += 256 * kChunk) {
    float v[kChunk];
#pragma unroll
    for (int j = 0; j < kChunk; ++j) {
      const int e = base + threadIdx.x + 256 * j;
      const int r = e / iw, col = e - r * iw;
      const int64_t gr = r0 + r, gc = c0 + col;
      const bool ok = e < total && gr >= 0 && gr < h && gc >= 0 && gc < w;
      const float t = src[ok ? gr * w + gc : 0];
      v[j] = ok ? t : 0.f;
    }
#pragma unroll
    for (int j = 0; j < kChunk; ++j) {
      const int e = base + threadIdx.x + 256 * j;
      if (e < total) tile[e] = v[j];
    }
  }
}

__host__ __device__ constexpr int64_t floor_div(int64_t a, int64_t b) {
  return a >= 0 ? a / b : -((-a + b - 1) / b);
}

// gx[iy,ix] = sum over taps with (iy+p-ky) % S == 0 of w[t] gy[(iy+p-ky)/S, (ix+p-kx)/S]
template <int K, int S>
__global__ void __launch_bounds__(256)
    dw_bwd_data_kernel(const float* __restrict__ gy, const float* __restrict__ wt,
                       float* __restrict__ gx, DwShape d, DwTile t) {
  extern __shared__ float tile[];
  const int64_t plane = blockIdx.z;
  const int64_t ch = plane % d.c;
  const int64_t iy0 = (int64_t)blockIdx.y * t.th, ix0 = (int64_t)blockIdx.x * t.tw;
  const int64_t oy_lo = floor_div(iy0 + d.pad - (K - 1), S);
  const int64_t ox_lo = floor_div(ix0 + d.pad - (K - 1), S);
  float wk[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) wk[i] = wt[ch * K * K + i];
  stage_window(gy + plane * d.ho * d.wo, tile, t.ih, t.iw, oy_lo, ox_lo, d.ho, d.wo);
  __syncthreads();
  float* xp = gx + plane * d.h * d.w;
  for (int o = threadIdx.x; o < t.th * t.tw; o += 256) {
    const int ly = o / t.tw, lx = o - ly * t.tw;
    const int64_t iy = iy0 + ly, ix = ix0 + lx;
    if (iy >= d.h || ix >= d.w) continue;
    const int ry0 = (int)(iy + d.pad - oy_lo * S), rx0 = (int)(ix + d.pad - ox_lo * S);
    float acc = 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int ry = ry0 - ky;
      if (S > 1 && (ry % S) != 0) continue;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int rx = rx0 - kx;
        if (S > 1 && (rx % S) != 0) continue;
        acc = fmaf(tile[(ry / S) * t.iw + rx / S], wk[ky * K + kx], acc);
      }
    }
    xp[iy * d.w + ix] = acc;
  }
}

// Per-tile partial sums of the weight gradient: part[(ch * P + p) * K*K + t],
// p = (image, tile_y, tile_x) in row-major order.
template <int K, int S>
__global__ void __launch_bounds__(256)
    dw_bwd_weight_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                         float* __restrict__ part, DwShape d, DwTile t, int64_t n) {
  extern __shared__ float tile[];
  __shared__ float red[4][K * K];
  const int64_t plane = blockIdx.z;
  const int64_t ch = plane % d.c, img = plane / d.c;
  const int64_t oy0 = (int64_t)blockIdx.y * t.th, ox0 = (int64_t)blockIdx.x * t.tw;
  stage_window(x + plane * d.h * d.w, tile, t.ih, t.iw, oy0 * S - d.pad, ox0 * S - d.pad, d.h,
               d.w);
  __syncthreads();
  const float* gp = gy + plane * d.ho * d.wo;
  float acc[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
  for (int o = threadIdx.x; o < t.th * t.tw; o += 256) {
    const int ly = o / t.tw, lx = o - ly * t.tw;
    const int64_t oy = oy0 + ly, ox = ox0 + lx;
    const bool ok = oy < d.ho && ox < d.wo;
    const float gv = gp[ok ? oy * d.wo + ox : 0];
    const float g = ok ? gv : 0.f;
    const float* tp = tile + ly * S * t.iw + lx * S;
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
      for (int kx = 0; kx < K; ++kx) acc[ky * K + kx] = fmaf(g, tp[ky * t.iw + kx], acc[ky * K + kx]);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < K * K; ++i) {
    const float v = wave_sum(acc[i]);
    if (lane == 0) red[wid][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < K * K) {
    const int i = threadIdx.x;
    const int64_t tiles = (int64_t)t.tx * t.ty;
    const int64_t p = img * tiles + (int64_t)blockIdx.y * t.tx + blockIdx.x;
    part[(ch * n * tiles + p) * K * K + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// One block per channel: gw[ch, t] = sum_p part[ch, p, t] (fixed order).
template <int K>
__global__ void __launch_bounds__(256)
    dw_wreduce_kernel(const float* __restrict__ part, float* __restrict__ gw, int64_t P) {
  __shared__ float red[4][K * K];
  const int64_t ch = blockIdx.x;
  const float* pp = part + ch * P * K * K;
  float acc[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
  for (int64_t p = threadIdx.x; p < P; p += 256)
#pragma unroll
    for (int i = 0; i < K * K; ++i) acc[i] += pp[p * K * K + i];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < K * K; ++i) {
    const float v = wave_sum(acc[i]);
    if (lane == 0) red[wid][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < K * K) {
    const int i = threadIdx.x;
    gw[ch * K * K + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// ---------------------------------------------------------------------------
// Strip-blocked kernels (the fast path).  A tile is th x tw OUTPUT cells; a
// thread owns one tile column and R consecutive rows of it (a "strip"), so a
// staged LDS value feeds every output of the strip it touches from registers:
// LDS reads per output drop from K*K to (S(R-1)+K)K/R (k5 s1: 25 -> 10), which
// keeps the k5 kernels off the LDS-bandwidth ceiling.  Tiles are up to 64
// cells wide (one wave of columns) and 256/tw row groups tall.
constexpr int kStripR = 4;

struct DwStrip {
  int tw, th;  // output cells per tile (th = rg * kStripR)
  int rg;      // row groups (strips per column)
  int tx, ty;  // tiles per plane
  int gh, gw;  // staged gy window (backward)
  int xh, xw;  // staged x window
};

// Offsets (in gy rows) of the taps feeding a data-gradient cell with padding
// P = K/2: gx[S*o + a] takes gy[o + (a+P-ky)/S] for (a+P-ky) % S == 0.
__host__ __device__ constexpr int strip_lo(int K, int S) {
  int m = 1 << 20;
  for (int a = 0; a < S; ++a)
    for (int ky = 0; ky < K; ++ky) {
      const int v = a + K / 2 - ky;
      if (v % S == 0 && v / S < m) m = v / S;
    }
  return m;
}
__host__ __device__ constexpr int strip_hi(int K, int S) {
  int m = -(1 << 20);
  for (int a = 0; a < S; ++a)
    for (int ky = 0; ky < K; ++ky) {
      const int v = a + K / 2 - ky;
      if (v % S == 0 && v / S > m) m = v / S;
    }
  return m;
}

DwStrip strip_tile(const DwShape& d, int k, int s) {
  DwStrip t;
  t.tx = (int)cdiv(d.wo, 64);
  t.tw = (int)cdiv(d.wo, t.tx);
  t.rg = 256 / t.tw;
  const int need = (int)cdiv(d.ho, kStripR);
  if (t.rg > need) t.rg = need;
  t.th = t.rg * kStripR;
  t.ty = (int)cdiv(d.ho, t.th);
  t.xh = (t.th - 1) * s + k;
  t.xw = (t.tw - 1) * s + k;
  const int span = strip_hi(k, s) - strip_lo(k, s);
  t.gh = t.th + span;
  t.gw = t.tw + span;
  return t;
}

// y[oy,ox] = sum_t w[t] x[oy*S-p+ky, ox*S-p+kx]; any padding p.
template <int K, int S>
__global__ void __launch_bounds__(256)
    dw_fwd_strip_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                        float* __restrict__ y, DwShape d, DwStrip t) {
  constexpr int R = kStripR;
  extern __shared__ float tile[];
  const int64_t plane = blockIdx.z;
  const int64_t ch = plane % d.c;
  const int64_t oy0 = (int64_t)blockIdx.y * t.th, ox0 = (int64_t)blockIdx.x * t.tw;
  float wk[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) wk[i] = wt[ch * K * K + i];
  stage_window(x + plane * d.h * d.w, tile, t.xh, t.xw, oy0 * S - d.pad, ox0 * S - d.pad, d.h,
               d.w);
  __syncthreads();
  const int col = threadIdx.x % t.tw, g = threadIdx.x / t.tw;
  const int64_t ox = ox0 + col;
  if (g >= t.rg || ox >= d.wo) return;
  const float* tp = tile + g * R * S * t.xw + col * S;
  float acc[R];
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.f;
#pragma unroll
  for (int r = 0; r < S * (R - 1) + K; ++r) {
    float v[K];
#pragma unroll
    for (int kx = 0; kx < K; ++kx) v[kx] = tp[r * t.xw + kx];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int ky = r - S * j;
      if (ky < 0 || ky >= K) continue;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) acc[j] = fmaf(v[kx], wk[ky * K + kx], acc[j]);
    }
  }
  float* yp = y + plane * d.ho * d.wo;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int64_t oy = oy0 + g * R + j;
    if (oy < d.ho) yp[oy * d.wo + ox] = acc[j];
  }
}

// Fused backward for padding K/2: data gradient and weight gradient from ONE
// staging of the gy window (+ the x window), so gy is read from HBM once.
// Persistent over images: block (ch, g) walks items g, g+G, ... of the
// channel's n * tiles (image, tile) items, keeps the K*K weight-gradient sums
// in registers across items, and writes one partial per block (fixed order;
// G == 1 writes gw directly).
//   gx[S*oy+a, S*ox+b] = sum over (ky,kx) with (a+P-ky)%S == (b+P-kx)%S == 0 of
//                        w[ky,kx] gy[oy + (a+P-ky)/S, ox + (b+P-kx)/S]
//   gw[ky,kx]         += gy[oy,ox] x[S*oy-P+ky, S*ox-P+kx]
template <int K, int S>
__global__ void __launch_bounds__(256)
    dw_bwd_strip_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                        const float* __restrict__ wt, float* __restrict__ gx,
                        float* __restrict__ part, DwShape d, DwStrip t, int64_t n, int G) {
  constexpr int R = kStripR, P = K / 2;
  constexpr int LO = strip_lo(K, S), HI = strip_hi(K, S);
  constexpr int GR = R + HI - LO, GC = HI - LO + 1;
  constexpr int XR = S * (R - 1) + K;
  extern __shared__ float lds[];
  __shared__ float red[4][K * K];
  float* gyt = lds;
  float* xt = lds + t.gh * t.gw;
  const int64_t ch = blockIdx.x;
  const int g = blockIdx.y;
  const bool want_gx = gx != nullptr, want_gw = part != nullptr;
  float wk[K * K], acc[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) {
    wk[i] = want_gx ? wt[ch * K * K + i] : 0.f;
    acc[i] = 0.f;
  }
  const int col = threadIdx.x % t.tw, rgi = threadIdx.x / t.tw;
  const bool active = rgi < t.rg;
  const int ly = rgi * R;  // first tile-local output row of this strip
  const int64_t T = (int64_t)t.tx * t.ty, items = n * T;
  for (int64_t it = g; it < items; it += G) {
    const int64_t img = it / T, tl = it - img * T;
    const int64_t tyi = tl / t.tx, txi = tl - tyi * t.tx;
    const int64_t oy0 = tyi * t.th, ox0 = txi * t.tw;
    const int64_t plane = img * d.c + ch;
    __syncthreads();  // previous item's readers are done with the windows
    stage_window(gy + plane * d.ho * d.wo, gyt, t.gh, t.gw, oy0 + LO, ox0 + LO, d.ho, d.wo);
    if (want_gw)
      stage_window(x + plane * d.h * d.w, xt, t.xh, t.xw, oy0 * S - P, ox0 * S - P, d.h, d.w);
    __syncthreads();
    if (!active) continue;
    if (want_gx) {
      float gv[GR][GC];
      const float* gp = gyt + ly * t.gw + col;
#pragma unroll
      for (int a = 0; a < GR; ++a)
#pragma unroll
        for (int b = 0; b < GC; ++b) gv[a][b] = gp[a * t.gw + b];
      float* gxp = gx + plane * d.h * d.w;
#pragma unroll
      for (int j = 0; j < R; ++j)
#pragma unroll
        for (int a = 0; a < S; ++a) {
          const int64_t iy = (oy0 + ly + j) * S + a;
#pragma unroll
          for (int b = 0; b < S; ++b) {
            const int64_t ix = (ox0 + col) * S + b;
            float sacc = 0.f;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
              if ((a + P - ky) % S != 0) continue;
              const int ro = j + (a + P - ky) / S - LO;
#pragma unroll
              for (int kx = 0; kx < K; ++kx) {
                if ((b + P - kx) % S != 0) continue;
                sacc = fmaf(wk[ky * K + kx], gv[ro][(b + P - kx) / S - LO], sacc);
              }
            }
            if (iy < d.h && ix < d.w) gxp[iy * d.w + ix] = sacc;
          }
        }
    }
    if (want_gw) {
      float go[R];
#pragma unroll
      for (int j = 0; j < R; ++j) go[j] = gyt[(ly + j - LO) * t.gw + col - LO];
      const float* xp = xt + ly * S * t.xw + col * S;
#pragma unroll
      for (int r = 0; r < XR; ++r) {
        float v[K];
#pragma unroll
        for (int kx = 0; kx < K; ++kx) v[kx] = xp[r * t.xw + kx];
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const int ky = r - S * j;
          if (ky < 0 || ky >= K) continue;
#pragma unroll
          for (int kx = 0; kx < K; ++kx)
            acc[ky * K + kx] = fmaf(go[j], v[kx], acc[ky * K + kx]);
        }
      }
    }
  }
  if (!want_gw) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < K * K; ++i) {
    const float v = wave_sum(acc[i]);
    if (lane == 0) red[wid][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < K * K) {
    const int i = threadIdx.x;
    part[(ch * G + g) * K * K + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

bool dw_ok(int64_t n, int64_t c, int64_t h, int64_t w, int64_t k, int64_t stride,
           int64_t pad) {
  return n > 0 && c > 0 && h > 0 && w > 0 && (k == 3 || k == 5) &&
         (stride == 1 || stride == 2) && pad >= 0 && pad < k && n * c <= 65535 &&
         (h + 2 * pad - k) >= 0 && (w + 2 * pad - k) >= 0;
}

DwShape make_shape(int64_t c, int64_t h, int64_t w, int64_t k, int64_t s, int64_t pad) {
  DwShape d;
  d.c = c;
  d.h = h;
  d.w = w;
  d.ho = (h + 2 * pad - k) / s + 1;
  d.wo = (w + 2 * pad - k) / s + 1;
  d.pad = (int)pad;
  return d;
}

// output-space tile (fwd, weight grad): input window (th-1)*S+K x (tw-1)*S+K
DwTile out_tile(const DwShape& d, int k, int s) {
  DwTile t = tile_for(d.ho, d.wo);
  t.ih = (t.th - 1) * s + k;
  t.iw = (t.tw - 1) * s + k;
  return t;
}

// input-space tile (data grad): the gy rows / cols it can reach
DwTile in_tile(const DwShape& d, int k, int s) {
  DwTile t = tile_for(d.h, d.w);
  t.ih = (t.th + k - 2) / s + 2;
  t.iw = (t.tw + k - 2) / s + 2;
  return t;
}

template <int K, int S>
int launch_fwd(const float* x, const float* wt, float* y, int64_t n, const DwShape& d,
               hipStream_t st) {
  const DwStrip t = strip_tile(d, K, S);
  const dim3 grid((unsigned)t.tx, (unsigned)t.ty, (unsigned)(n * d.c));
  const double bytes = 4.0 * n * d.c * (d.h * d.w + d.ho * d.wo);
  MDE_LAUNCH(K_DW_FWD, bytes, st, (dw_fwd_strip_kernel<K, S>), grid, dim3(256),
             sizeof(float) * t.xh * t.xw, x, wt, y, d, t);
  return 0;
}

// Blocks per channel of the fused backward: ~2048 blocks in all (8 per CU).
int strip_groups(int64_t n, int64_t c, const DwStrip& t) {
  const int64_t items = n * (int64_t)t.tx * t.ty;
  int64_t g = cdiv(2048, c);
  if (g > items) g = items;
  return (int)(g < 1 ? 1 : g);
}

template <int K, int S>
int launch_bwd_strip(const float* gy, const float* x, const float* wt, float* gx, float* gw,
                     float* part, int64_t n, const DwShape& d, hipStream_t st) {
  const DwStrip t = strip_tile(d, K, S);
  const int G = strip_groups(n, d.c, t);
  float* dst = gw ? (G == 1 ? gw : part) : nullptr;
  const size_t lds = sizeof(float) * (t.gh * t.gw + (gw ? t.xh * t.xw : 0));
  const double bytes =
      4.0 * n * d.c * (d.ho * d.wo + (gx ? d.h * d.w : 0) + (gw ? d.h * d.w : 0));
  MDE_LAUNCH(K_DW_BWD, bytes, st, (dw_bwd_strip_kernel<K, S>), dim3((unsigned)d.c, (unsigned)G),
             dim3(256), lds, gy, x, wt, gx, dst, d, t, n, G);
  if (gw && G > 1)
    MDE_LAUNCH(K_DW_WREDUCE, 4.0 * d.c * G * K * K, st, dw_wreduce_kernel<K>,
               dim3((unsigned)d.c), dim3(256), 0, part, gw, (int64_t)G);
  return 0;
}

template <int K, int S>
int launch_bwd(const float* gy, const float* x, const float* wt, float* gx, float* gw,
               float* part, int64_t n, const DwShape& d, hipStream_t st) {
  if (d.pad == K / 2) return launch_bwd_strip<K, S>(gy, x, wt, gx, gw, part, n, d, st);
  // other paddings: separate data / weight-gradient kernels
  const double bytes = 4.0 * n * d.c * (d.h * d.w + d.ho * d.wo);
  if (gx) {
    const DwTile t = in_tile(d, K, S);
    const dim3 grid((unsigned)t.tx, (unsigned)t.ty, (unsigned)(n * d.c));
    MDE_LAUNCH(K_DW_BWD_DATA, bytes, st, (dw_bwd_data_kernel<K, S>), grid, dim3(256),
               sizeof(float) * t.ih * t.iw, gy, wt, gx, d, t);
  }
  if (gw) {
    const DwTile t = out_tile(d, K, S);
    const dim3 grid((unsigned)t.tx, (unsigned)t.ty, (unsigned)(n * d.c));
    MDE_LAUNCH(K_DW_BWD_WEIGHT, bytes, st, (dw_bwd_weight_kernel<K, S>), grid, dim3(256),
               sizeof(float) * t.ih * t.iw, gy, x, part, d, t, n);
    const int64_t P = n * (int64_t)t.tx * t.ty;
    MDE_LAUNCH(K_DW_WREDUCE, 4.0 * d.c * P * K * K, st, dw_wreduce_kernel<K>,
               dim3((unsigned)d.c), dim3(256), 0, part, gw, P);
  }
  return 0;
}

}  // namespace
}  // namespace mde

using namespace mde;

extern "C" {

size_t mde_dwconv_workspace(int64_t n, int64_t c, int64_t h, int64_t w, int64_t k,
                            int64_t stride, int64_t pad) {
  if (!dw_ok(n, c, h, w, k, stride, pad)) return 0;
  const DwShape d = make_shape(c, h, w, k, stride, pad);
  if (pad == k / 2) {
    const int G = strip_groups(n, c, strip_tile(d, (int)k, (int)stride));
    return G > 1 ? (size_t)(4 * c * G * k * k) : 0;
  }
  const DwTile t = out_tile(d, (int)k, (int)stride);
  return (size_t)(4 * c * n * (int64_t)t.tx * t.ty * k * k);
}

int mde_dwconv_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t c,
                   int64_t h, int64_t w, int64_t k, int64_t stride, int64_t pad, int dtype,
                   void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!x || !weight || !y || !dw_ok(n, c, h, w, k, stride, pad)) return MDE_ERR_INVALID_ARG;
  const DwShape d = make_shape(c, h, w, k, stride, pad);
  hipStream_t st = (hipStream_t)stream;
  const float* xp = (const float*)x;
  float* yp = (float*)y;
  if (k == 3 && stride == 1) return launch_fwd<3, 1>(xp, weight, yp, n, d, st);
  if (k == 3 && stride == 2) return launch_fwd<3, 2>(xp, weight, yp, n, d, st);
  if (k == 5 && stride == 1) return launch_fwd<5, 1>(xp, weight, yp, n, d, st);
  return launch_fwd<5, 2>(xp, weight, yp, n, d, st);
}

int mde_dwconv_bwd(const void* gy, const void* x, const float* weight, void* gx, float* gweight,
                   int64_t n, int64_t c, int64_t h, int64_t w, int64_t k, int64_t stride,
                   int64_t pad, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  if (!gy || !dw_ok(n, c, h, w, k, stride, pad) || (gx && !weight) ||
      (gweight && (!x || (!workspace && mde_dwconv_workspace(n, c, h, w, k, stride, pad) > 0))))
    return MDE_ERR_INVALID_ARG;
  const DwShape d = make_shape(c, h, w, k, stride, pad);
  hipStream_t st = (hipStream_t)stream;
  const float* g = (const float*)gy;
  const float* xp = (const float*)x;
  float* gxp = (float*)gx;
  float* part = (float*)workspace;
  if (k == 3 && stride == 1) return launch_bwd<3, 1>(g, xp, weight, gxp, gweight, part, n, d, st);
  if (k == 3 && stride == 2) return launch_bwd<3, 2>(g, xp, weight, gxp, gweight, part, n, d, st);
  if (k == 5 && stride == 1) return launch_bwd<5, 1>(g, xp, weight, gxp, gweight, part, n, d, st);
  return launch_bwd<5, 2>(g, xp, weight, gxp, gweight, part, n, d, st);
}

}  // extern "C"
