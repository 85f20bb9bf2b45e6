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

// gw[ch, t] = sum_g part[(ch * G + g), t]: one wave per channel, lane l sums
// partials l, l + 64, ... of every tap (all loads in flight), then a
// fixed-order wave reduction per tap.
template <int K>
__device__ __forceinline__ void wsum_channel(const float* __restrict__ part, float* __restrict__ gw,
                                             int G, int64_t ch, int lane) {
  const float* p = part + ch * G * (K * K);
  float acc[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
  for (int g = lane; g < G; g += 64)
#pragma unroll
    for (int i = 0; i < K * K; ++i) acc[i] += p[(int64_t)g * (K * K) + i];
#pragma unroll
  for (int i = 0; i < K * K; ++i) {
    const float v = wave_sum(acc[i]);
    if (lane == i) gw[ch * (K * K) + i] = v;
  }
}

template <int K>
__global__ void __launch_bounds__(64)
    dw_wsum_kernel(const float* __restrict__ part, float* __restrict__ gw, int G) {
  wsum_channel<K>(part, gw, G, blockIdx.x, threadIdx.x);
}

// ---------------------------------------------------------------------------
// Strip-blocked kernels (the fast path).  A tile is th x tw OUTPUT cells of
// `pb` planes; a thread owns one tile column and R consecutive rows of one of
// them (a "strip"), so a staged LDS value feeds every output of the strip it
// touches from registers: LDS reads per output drop from K*K to
// (S(R-1)+K)K/R (k5 s1: 25 -> 10), which keeps the k5 kernels off the
// LDS-bandwidth ceiling.  Tiles are up to 64 cells wide (one wave of columns)
// and 256/tw row groups tall; planes smaller than half a block (the 15x20
// late stages) are stacked pb to a block so every block keeps ~1000 loads in
// flight instead of ~300.
constexpr int kStripR = 4;

struct DwStrip {
  int tw, th;  // output cells per tile and plane (th = rg * kStripR)
  int rg;      // row groups (strips per column)
  int pb;      // planes stacked per block
  int tx, ty;  // tiles per plane
  int gh, gw;  // staged gy window per plane (backward)
  int xh, xw;  // staged x window per plane
  unsigned mgh, mgw, mxh, mxw;  // fdiv magics of the window extents
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

// e / d for 0 <= e < 2^17, d <= 4096 with m = 2^32/d + 1 (exact in that range,
// checked exhaustively); replaces a ~20-instruction integer division.
__device__ __forceinline__ int fdiv(int e, unsigned m) { return (int)__umulhi((unsigned)e, m); }
inline unsigned fdiv_magic(int d) { return (unsigned)((1ull << 32) / (unsigned)d + 1); }

// max_planes: how many planes a block may stack (fwd: n*c, bwd: n images).
DwStrip strip_tile(const DwShape& d, int k, int s, int64_t max_planes) {
  DwStrip t;
  t.tx = (int)cdiv(d.wo, 64);
  t.tw = (int)cdiv(d.wo, t.tx);
  t.rg = 256 / t.tw;
  const int need = (int)cdiv(d.ho, kStripR);
  if (t.rg > need) t.rg = need;
  t.th = t.rg * kStripR;
  t.ty = (int)cdiv(d.ho, t.th);
  t.pb = 256 / (t.tw * t.rg);
  if (t.pb > 256 / (k * k)) t.pb = 256 / (k * k);  // forward stages pb*k*k taps in LDS
  if (t.pb > max_planes) t.pb = (int)max_planes;
  if (t.pb < 1) t.pb = 1;
  t.xh = (t.th - 1) * s + k;
  t.xw = (t.tw - 1) * s + k;
  const int span = strip_hi(k, s) - strip_lo(k, s);
  t.gh = t.th + span;
  t.gw = t.tw + span;
  t.mgh = fdiv_magic(t.gh);
  t.mgw = fdiv_magic(t.gw);
  t.mxh = fdiv_magic(t.xh);
  t.mxw = fdiv_magic(t.xw);
  return t;
}

template <bool STACKED>
__device__ __forceinline__ void stage_planes_t(const float* __restrict__ src, int pstride, int np,
                                               float* tile, int ih, int iw, unsigned mih,
                                               unsigned miw, int r0, int c0, int h, int w) {
  const int total = np * ih * iw;
  for (int base = 0; base < total; base += 256 * kChunk) {
    float v[kChunk];
#pragma unroll
    for (int j = 0; j < kChunk; ++j) {
      const int e = base + threadIdx.x + 256 * j;
      const int sr = fdiv(e, miw), col = e - __mul24(sr, iw);
      int p = 0, r = sr;
      if (STACKED) {
        p = fdiv(sr, mih);
        r = sr - __mul24(p, ih);
      }
      const int gr = r0 + r, gc = c0 + col;
      const bool ok = e < total && (unsigned)gr < (unsigned)h && (unsigned)gc < (unsigned)w;
      const unsigned off = (STACKED ? (unsigned)(p * pstride) : 0u) + __mul24(gr, w) + gc;
      const float t = src[ok ? off : 0u];
      v[j] = ok ? t : 0.f;
    }
#pragma unroll
    for (int j = 0; j < kChunk; ++j) {
      const int e = base + threadIdx.x + 256 * j;
      if (e < total) tile[e] = v[j];
    }
  }
}

// tile[(p*ih + r)*iw + col] = src[p*pstride + (r0+r)*w + c0+col] for the np
// planes p < np, zero outside the plane; all 256 threads walk the flattened
// window with kChunk loads in flight (mih / miw: fdiv magics of ih / iw).
// 32-bit offsets: dw_ok bounds every tensor to < 2^31 elements and planes to
// < 2^24.
__device__ __forceinline__ void stage_planes(const float* __restrict__ src, int64_t pstride,
                                             int np, float* tile, int ih, int iw, unsigned mih,
                                             unsigned miw, int r0, int c0, int h, int w) {
  if (np == 1)
    stage_planes_t<false>(src, 0, 1, tile, ih, iw, mih, miw, r0, c0, h, w);
  else
    stage_planes_t<true>(src, (int)pstride, np, tile, ih, iw, mih, miw, r0, c0, h, w);
}

// y[oy,ox] = sum_t w[t] x[oy*S-p+ky, ox*S-p+kx]; any padding p.
// Block z covers planes z*pb .. z*pb+pb-1 (flattened n*c < 65536).
template <int K, int S>
__global__ void __launch_bounds__(256)
    dw_fwd_strip_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                        float* __restrict__ y, DwShape d, DwStrip t, int planes) {
  constexpr int R = kStripR;
  extern __shared__ float tile[];
  __shared__ float wl[256];  // the pb planes' taps (pb * K * K <= 256, see strip_tile)
  const int H = (int)d.h, W = (int)d.w, HO = (int)d.ho, WO = (int)d.wo, C = (int)d.c;
  const int plane0 = blockIdx.z * t.pb;
  const int np = planes - plane0 < t.pb ? planes - plane0 : t.pb;
  const int oy0 = blockIdx.y * t.th, ox0 = blockIdx.x * t.tw;
  for (int i = threadIdx.x; i < np * K * K; i += 256) {
    const int pl = plane0 + i / (K * K);
    wl[i] = wt[(pl % C) * K * K + i % (K * K)];
  }
  stage_planes(x + (int64_t)plane0 * H * W, (int64_t)H * W, np, tile, t.xh, t.xw, t.mxh, t.mxw,
               oy0 * S - d.pad, ox0 * S - d.pad, H, W);
  __syncthreads();
  const int per = t.tw * t.rg;
  const int p = threadIdx.x / per, q = threadIdx.x - p * per;
  const int col = q % t.tw, g = q / t.tw;
  const int ox = ox0 + col;
  if (p >= np || ox >= WO) return;
  float wk[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) wk[i] = wl[p * K * K + i];
  const float* tp = tile + (p * t.xh + g * R * S) * t.xw + col * S;
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
  float* yp = y + (int64_t)(plane0 + p) * HO * WO;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int oy = oy0 + g * R + j;
    if (oy < HO) yp[oy * WO + ox] = acc[j];
  }
}

// Fused backward for padding K/2: data gradient and weight gradient from ONE
// staging of the gy window (+ the x window), so gy is read from HBM once.
// Persistent over images: block (ch, g) walks items g, g+G, ... of the
// channel's (image group, tile) items -- an image group is pb consecutive
// images stacked in LDS.  Waves 0-1 compute the data gradient, waves 2-3 the
// weight gradient (each thread covers strips s and s+128 of the tile), so no
// thread holds both the k*k tap sums and the gy strip: ~60 VGPRs, 8 waves per
// SIMD to hide the staging latency.  The weight-gradient sums stay in
// registers across items; one partial per block (fixed order; G == 1 writes
// gw directly).
//   gx[S*oy+a, S*ox+b] = sum over (ky,kx) with (a+P-ky)%S == (b+P-kx)%S == 0 of
//                        w[ky,kx] gy[oy + (a+P-ky)/S, ox + (b+P-kx)/S]
//   gw[ky,kx]         += gy[oy,ox] x[S*oy-P+ky, S*ox-P+kx]
struct StripPos {
  int p, col, ly;  // stacked plane, tile column, first tile-local row
  bool ok;         // strip exists (s < tw * rg * pb)
};

__device__ __forceinline__ StripPos strip_pos(int s, const DwStrip& t) {
  const int per = t.tw * t.rg;
  StripPos r;
  r.p = s / per;
  const int q = s - r.p * per;
  r.col = q % t.tw;
  r.ly = q / t.tw * kStripR;
  r.ok = r.p < t.pb;
  return r;
}

struct DwItem {
  int oy0, ox0, img0, np;
};

template <int K, int S>
__device__ __forceinline__ DwItem stage_item(int it, const DwStrip& t, int nn, int C, int H,
                                             int W, int HO, int WO, int ch, const float* gy,
                                             const float* x, float* gyt, float* xt,
                                             bool want_gw) {
  constexpr int P = K / 2, LO = strip_lo(K, S);
  const int T = t.tx * t.ty;
  const int grp = it / T, tl = it - grp * T;
  const int tyi = tl / t.tx, txi = tl - tyi * t.tx;
  DwItem m;
  m.oy0 = tyi * t.th;
  m.ox0 = txi * t.tw;
  m.img0 = grp * t.pb;
  m.np = nn - m.img0 < t.pb ? nn - m.img0 : t.pb;
  __syncthreads();  // previous item's readers are done with the windows
  stage_planes(gy + ((int64_t)m.img0 * C + ch) * HO * WO, (int64_t)C * HO * WO, m.np, gyt, t.gh,
               t.gw, t.mgh, t.mgw, m.oy0 + LO, m.ox0 + LO, HO, WO);
  if (want_gw)
    stage_planes(x + ((int64_t)m.img0 * C + ch) * H * W, (int64_t)C * H * W, m.np, xt, t.xh,
                 t.xw, t.mxh, t.mxw, m.oy0 * S - P, m.ox0 * S - P, H, W);
  __syncthreads();
  return m;
}

template <int K, int S>
__device__ __forceinline__ void gx_strip(const StripPos& sp, const DwItem& m, const DwStrip& t,
                                         const float* gyt, const float* wk, float* gx, int C,
                                         int H, int W, int ch) {
  constexpr int R = kStripR, P = K / 2;
  constexpr int LO = strip_lo(K, S), HI = strip_hi(K, S);
  constexpr int GR = R + HI - LO, GC = HI - LO + 1;
  float gv[GR][GC];
  const float* gp = gyt + (sp.p * t.gh + sp.ly) * t.gw + sp.col;
#pragma unroll
  for (int a = 0; a < GR; ++a)
#pragma unroll
    for (int b = 0; b < GC; ++b) gv[a][b] = gp[a * t.gw + b];
  float* gxp = gx + ((int64_t)(m.img0 + sp.p) * C + ch) * H * W;
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int a = 0; a < S; ++a) {
      const int iy = (m.oy0 + sp.ly + j) * S + a;
#pragma unroll
      for (int b = 0; b < S; ++b) {
        const int ix = (m.ox0 + sp.col) * S + b;
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
        if (iy < H && ix < W) gxp[iy * W + ix] = sacc;
      }
    }
}

template <int K, int S>
__device__ __forceinline__ void gw_strip(const StripPos& sp, const DwStrip& t, const float* gyt,
                                         const float* xt, float* acc) {
  constexpr int R = kStripR, LO = strip_lo(K, S), XR = S * (R - 1) + K;
  float go[R];
#pragma unroll
  for (int j = 0; j < R; ++j) go[j] = gyt[(sp.p * t.gh + sp.ly + j - LO) * t.gw + sp.col - LO];
  const float* xp = xt + (sp.p * t.xh + sp.ly * S) * t.xw + sp.col * S;
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
      for (int kx = 0; kx < K; ++kx) acc[ky * K + kx] = fmaf(go[j], v[kx], acc[ky * K + kx]);
    }
  }
}

template <int K, int S>
__global__ void __launch_bounds__(256)
    dw_bwd_strip_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                        const float* __restrict__ wt, float* __restrict__ gx,
                        float* __restrict__ part, DwShape d, DwStrip t, int64_t n, int G) {
  extern __shared__ float lds[];
  __shared__ float red[2][K * K];
  float* gyt = lds;
  float* xt = lds + t.pb * t.gh * t.gw;
  const int H = (int)d.h, W = (int)d.w, HO = (int)d.ho, WO = (int)d.wo, C = (int)d.c;
  const int ch = blockIdx.x, g = blockIdx.y, nn = (int)n;
  const bool want_gx = gx != nullptr, want_gw = part != nullptr;
  const int items = (nn + t.pb - 1) / t.pb * (t.tx * t.ty);
  const StripPos sa = strip_pos(threadIdx.x & 127, t), sb = strip_pos((threadIdx.x & 127) + 128, t);
  if (threadIdx.x < 128) {  // data-gradient waves
    float wk[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) wk[i] = want_gx ? wt[ch * K * K + i] : 0.f;
    for (int it = g; it < items; it += G) {
      const DwItem m =
          stage_item<K, S>(it, t, nn, C, H, W, HO, WO, ch, gy, x, gyt, xt, want_gw);
      if (!want_gx) continue;
#pragma unroll 1
      for (int k = 0; k < 2; ++k) {
        const StripPos sp = k ? sb : sa;
        if (sp.ok && sp.p < m.np) gx_strip<K, S>(sp, m, t, gyt, wk, gx, C, H, W, ch);
      }
    }
  } else {  // weight-gradient waves
    float acc[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
    for (int it = g; it < items; it += G) {
      const DwItem m =
          stage_item<K, S>(it, t, nn, C, H, W, HO, WO, ch, gy, x, gyt, xt, want_gw);
      if (!want_gw) continue;
#pragma unroll 1
      for (int k = 0; k < 2; ++k) {
        const StripPos sp = k ? sb : sa;
        if (sp.ok && sp.p < m.np) gw_strip<K, S>(sp, t, gyt, xt, acc);
      }
    }
    const int lane = threadIdx.x & 63, wid = (threadIdx.x >> 6) - 2;
#pragma unroll
    for (int i = 0; i < K * K; ++i) {
      const float v = wave_sum(acc[i]);
      if (lane == 0) red[wid][i] = v;
    }
  }
  __syncthreads();
  if (want_gw && threadIdx.x < K * K) {
    const int i = threadIdx.x;
    part[((int64_t)ch * G + g) * K * K + i] = red[0][i] + red[1][i];
  }
}

// ---------------------------------------------------------------------------
// Column-streaming kernels (padding K/2, W == S*Wo, Wo % V == 0): the fast
// path for every MobileNetV3 stage.  No LDS staging and no barriers in the
// main loop, so HBM latency is hidden by the loads a wave keeps in flight,
// not by block-level turnover.
//
// A lane owns V consecutive OUTPUT columns (and the S*V input columns under
// them) of a band of RB output rows of one plane: a "unit".  L lanes side by
// side cover a run of L*V columns of the row (a segment); a wave holds
// spw = 64/L segments, so narrow late-stage planes (20, 40 columns) still
// fill the wave.  A lane reads its own columns with vector loads and the
// stencil's column halo with scalar loads of the neighbouring columns
// (clamped addresses + select: no divergent branches around loads); the
// K-1 halo rows at band edges are re-read (L2 hits: neighbouring bands run in
// the same wave or block).  Every row of the band is unrolled, so all of a
// band's loads are issued together and every accumulator index is a
// compile-time constant.
//   forward         y rows accumulate row by row, stored as they complete.
//   fused backward  gx (input rows S*o0 .. S*(o0+RB)) from the gy rows
//                   o0-A .. o0+RB-1+B; gw from the unit's gy rows and the x
//                   rows under them, summed over the wave (shuffles), the
//                   block's waves (LDS, fixed order) and, when a channel
//                   spans several blocks, a fixed-order partial reduce.
// Backward units are ordered (channel, image, band, segment) and a wave never
// mixes channels, so a wave-wide sum is one channel's weight gradient.
struct DwStream {
  int L, spw, nseg, nb;  // lanes per segment, segments per wave, per row, bands per plane
  int wpb, it, G;        // backward: waves per block, unit groups per wave, blocks per channel
  int fold;              // backward, gx launch: wave 0 of block ch first sums channel ch's
                         // weight-gradient partials (written by the preceding gw launch)
  int64_t upc;           // backward: units per channel
};

template <int N>
__device__ __forceinline__ void ldv(const float* p, float* v) {
  if constexpr (N == 1) {
    v[0] = p[0];
  } else if constexpr (N == 2) {
    const float2 a = *reinterpret_cast<const float2*>(p);
    v[0] = a.x;
    v[1] = a.y;
  } else {
#pragma unroll
    for (int k = 0; k < N; k += 4) {
      const float4 a = *reinterpret_cast<const float4*>(p + k);
      v[k] = a.x;
      v[k + 1] = a.y;
      v[k + 2] = a.z;
      v[k + 3] = a.w;
    }
  }
}

template <int N>
__device__ __forceinline__ void stv(float* p, const float* v) {
  if constexpr (N == 1) {
    p[0] = v[0];
  } else if constexpr (N == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else {
#pragma unroll
    for (int k = 0; k < N; k += 4)
      *reinterpret_cast<float4*>(p + k) = make_float4(v[k], v[k + 1], v[k + 2], v[k + 3]);
  }
}

// v[c - LO] = row[c0 + c] for c in [LO, HI] (row of width w; zeros outside the
// row or when !rok).  The lane's own columns [0, N) come from vector loads;
// the halo columns from the neighbouring lanes by wave shuffles (lane +-1
// owns the adjacent N columns of the same row of the same unit); a segment
// is a whole row, so its edges are the plane's zero padding.  EDGE (rows
// split into several segments): every halo column is a scalar load, issued
// by every lane at a clamped address and selected, so no branch splits the
// unrolled load stream.
template <int LO, int N, int HI, bool EDGE>
__device__ __forceinline__ void load_cols(const float* row, int c0, int w, bool rok, bool segl,
                                          bool segr, float* v) {
  static_assert(-LO <= N && HI - N + 1 <= N, "halo wider than a lane's columns");
  float own[N];
  ldv<N>(row + c0, own);
#pragma unroll
  for (int c = 0; c < N; ++c) {
    own[c] = rok ? own[c] : 0.f;
    v[c - LO] = own[c];
  }
  if constexpr (EDGE) {
    // rows split into segments: every halo column by a scalar load (faster
    // here than shuffles + edge loads: no wait on the own loads to form it)
#pragma unroll
    for (int c = LO; c <= HI; ++c) {
      if (c >= 0 && c < N) continue;
      const int col = c0 + c;
      const bool ok = col >= 0 && col < w && rok;
      const float g = row[col >= 0 && col < w ? col : 0];
      v[c - LO] = ok ? g : 0.f;
    }
  } else {
#pragma unroll
    for (int c = LO; c < 0; ++c) {
      const float t = __shfl_up(own[N + c], 1, 64);
      v[c - LO] = segl ? 0.f : t;
    }
#pragma unroll
    for (int c = N; c <= HI; ++c) {
      const float t = __shfl_down(own[c - N], 1, 64);
      v[c - LO] = segr ? 0.f : t;
    }
  }
}

template <int K, int S, int V, int RB, bool EDGE>
__global__ void __launch_bounds__(256)
    dw_fwd_stream_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                         float* __restrict__ y, DwShape d, DwStream t, int64_t units) {
  constexpr int P = K / 2, XV = S * V;
  constexpr int XL = -P, XH = S * (V - 1) - P + K - 1;  // input columns rel. to the lane's first
  constexpr int NR = S * (RB - 1) + K;                   // input rows of a band
  const int H = (int)d.h, W = (int)d.w, HO = (int)d.ho, WO = (int)d.wo, C = (int)d.c;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int sl = lane / t.L, cl = lane - sl * t.L;
  const int64_t unit = wave * t.spw + sl;
  const bool active = sl < t.spw && unit < units;
  const int64_t u = active ? unit : 0;
  const int per = t.nb * t.nseg;
  const int64_t plane = u / per;
  const int rem = (int)(u - plane * per);
  const int band = rem / t.nseg;
  const int oc0 = ((rem - band * t.nseg) * t.L + cl) * V, ic0 = oc0 * S, o0 = band * RB;
  const bool segl = cl == 0, segr = cl == t.L - 1;
  float w[K * K];
  const float* wp = wt + (plane % C) * (K * K);
#pragma unroll
  for (int i = 0; i < K * K; ++i) w[i] = wp[i];
  const float* xp = x + plane * (int64_t)H * W;
  float* yp = y + plane * (int64_t)HO * WO + oc0;
  float acc[RB][V];
#pragma unroll
  for (int j = 0; j < RB; ++j)
#pragma unroll
    for (int q = 0; q < V; ++q) acc[j][q] = 0.f;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = S * o0 - P + i;
    const bool rok = active && r >= 0 && r < H;
    float xv[XH - XL + 1];
    load_cols<XL, XV, XH, EDGE>(xp + (int64_t)(rok ? r : 0) * W, ic0, W, rok, segl, segr, xv);
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      if (i - ky < 0 || (i - ky) % S != 0 || (i - ky) / S >= RB) continue;
      const int jo = (i - ky) / S;
#pragma unroll
      for (int q = 0; q < V; ++q)
#pragma unroll
        for (int kx = 0; kx < K; ++kx) acc[jo][q] = fmaf(w[ky * K + kx], xv[S * q + kx], acc[jo][q]);
    }
  }
  // stores last: a predicated store splits the basic block, and the scheduler
  // cannot hoist the next rows' loads across it
  if (!active) return;
#pragma unroll
  for (int jo = 0; jo < RB; ++jo)
    if (o0 + jo < HO) stv<V>(yp + (int64_t)(o0 + jo) * WO, acc[jo]);
}

template <int K, int S, int V, int RB, bool EDGE, bool DATA, bool WGT>
__device__ __forceinline__ void dw_bwd_stream_body(const float* __restrict__ gy,
                                                   const float* __restrict__ x,
                                                   const float* __restrict__ wt,
                                                   float* __restrict__ gx, float* __restrict__ gw,
                                                   float* __restrict__ gwf,
                                                   const DwShape& d,
                                                   const DwStream& t, int wv) {
  constexpr int P = K / 2, XV = S * V;
  constexpr int XL = -P, XH = S * (V - 1) - P + K - 1;  // x columns for the weight gradient
  constexpr int GL = (K - 1 - P + S - 1) / S;            // gy column / row halo (data gradient)
  constexpr int GR = (S - 1 + P) / S;
  constexpr int NGY = RB + GL + GR;                      // gy rows of a band
  constexpr int NX = S * (RB - 1) + K;                   // x rows of a band
  __shared__ float red[8][K * K];
  const int H = (int)d.h, W = (int)d.w, HO = (int)d.ho, WO = (int)d.wo, C = (int)d.c;
  const int lane = threadIdx.x & 63;
  const int ch = blockIdx.x / t.G, gb = blockIdx.x - ch * t.G;
  const int sl = lane / t.L, cl = lane - sl * t.L;
  const int per = t.nb * t.nseg;
  float w[K * K], accw[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) {
    w[i] = DATA ? wt[ch * (K * K) + i] : 0.f;
    accw[i] = 0.f;
  }
  for (int itr = 0; itr < t.it; ++itr) {
    const int64_t wave = ((int64_t)gb * t.it + itr) * t.wpb + wv;  // wave within the channel
    const int64_t unit = wave * t.spw + sl;
    const bool active = sl < t.spw && unit < t.upc;
    const int64_t u = active ? unit : 0;
    const int img = (int)(u / per);
    const int rem = (int)(u - (int64_t)img * per);
    const int band = rem / t.nseg;
    const int oc0 = ((rem - band * t.nseg) * t.L + cl) * V, ic0 = oc0 * S, o0 = band * RB;
    const bool segl = cl == 0, segr = cl == t.L - 1;
    const int64_t plane = (int64_t)img * C + ch;
    const float* gp = gy + plane * HO * WO;
    float gyo[WGT ? RB : 1][V];                // the unit's own gy rows (weight gradient)
    float accx[DATA ? S * RB : 1][S * V];      // gx rows of the band (data gradient)
    if constexpr (DATA) {
#pragma unroll
      for (int a = 0; a < S * RB; ++a)
#pragma unroll
        for (int c = 0; c < S * V; ++c) accx[a][c] = 0.f;
#pragma unroll
      for (int jj = 0; jj < NGY; ++jj) {
        const int jo = jj - GL, o = o0 + jo;
        const bool rok = active && o >= 0 && o < HO;
        float gv[GL + V + GR];
        load_cols<-GL, V, V - 1 + GR, EDGE>(gp + (int64_t)(rok ? o : 0) * WO, oc0, WO, rok, segl,
                                            segr, gv);
        if constexpr (WGT) {
          if (jo >= 0 && jo < RB) {
#pragma unroll
            for (int q = 0; q < V; ++q) gyo[jo][q] = gv[GL + q];
          }
        }
        // gy row o feeds input rows S*o - P + ky
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
          const int ti = S * jo - P + ky;
          if (ti < 0 || ti >= S * RB) continue;
#pragma unroll
          for (int c = 0; c < S * V; ++c)
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
              const int e = c + P - kx + S * GL;  // S * (gy column rel. + GL), >= 0
              if (e % S != 0) continue;
              accx[ti][c] = fmaf(w[ky * K + kx], gv[e / S], accx[ti][c]);
            }
        }
      }
    } else {
#pragma unroll
      for (int jo = 0; jo < RB; ++jo) {
        const int o = o0 + jo;
        const bool rok = active && o < HO;
        float gv[V];
        load_cols<0, V, V - 1, false>(gp + (int64_t)(rok ? o : 0) * WO, oc0, WO, rok, segl, segr,
                                      gv);
#pragma unroll
        for (int q = 0; q < V; ++q) gyo[jo][q] = gv[q];
      }
    }
    if constexpr (WGT) {
      const float* xp = x + plane * (int64_t)H * W;
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        const int r = S * o0 - P + i;
        const bool rok = active && r >= 0 && r < H;
        float xv[XH - XL + 1];
        load_cols<XL, XV, XH, EDGE>(xp + (int64_t)(rok ? r : 0) * W, ic0, W, rok, segl, segr, xv);
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
          if (i - ky < 0 || (i - ky) % S != 0 || (i - ky) / S >= RB) continue;
          const int jo = (i - ky) / S;
#pragma unroll
          for (int kx = 0; kx < K; ++kx)
#pragma unroll
            for (int q = 0; q < V; ++q)
              accw[ky * K + kx] = fmaf(gyo[jo][q], xv[S * q + kx], accw[ky * K + kx]);
        }
      }
    }
    // gx stores last (a predicated store splits the basic block: loads after
    // it could not be hoisted)
    if constexpr (DATA) {
      if (active) {
        float* xo = gx + plane * (int64_t)H * W + ic0;
#pragma unroll
        for (int ti = 0; ti < S * RB; ++ti)
          if (S * o0 + ti < H) stv<S * V>(xo + (int64_t)(S * o0 + ti) * W, accx[ti]);
      }
    }
  }
  if constexpr (WGT) {
#pragma unroll
    for (int i = 0; i < K * K; ++i) {
      const float v = wave_sum(accw[i]);
      if (lane == 0) red[wv][i] = v;
    }
    __syncthreads();  // every wave of the block passes exactly one barrier (both roles)
    if (wv == 0) {
      float s = 0.f;
      if (lane < K * K)
        for (int k = 0; k < t.wpb; ++k) s += red[k][lane];
      // G == 1: the channel's gradient; else this block's partial, summed in
      // fixed order by the launch that follows on the stream (kernel
      // boundary: no cross-block hand-off inside this launch)
      if (lane < K * K) gw[(int64_t)blockIdx.x * (K * K) + lane] = s;
    }
  } else {
    __syncthreads();  // matches the gw waves' barrier
  }
}

// Backward.  MODE 1: gx only; 2: gw only; 0: both, with the block's waves
// split in two roles over the same units -- waves [0, wpb) compute gx, waves
// [wpb, 2 wpb) gw -- so a wave holds only one role's registers (the
// allocation is the larger role's, not their sum) while the second read of
// each gy row, by the other role's wave on the same CU, hits L1/L2.
// gw: written directly (G == 1) or as per-block partials.
template <int K, int S, int V, int RB, bool EDGE, int MODE>
__global__ void __launch_bounds__(512)
    dw_bwd_stream_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                         const float* __restrict__ wt, float* __restrict__ gx,
                         float* __restrict__ gw, float* __restrict__ gwf,
                         DwShape d, DwStream t, int n) {
  const int role_wave = threadIdx.x >> 6;
  if (MODE == 1 && t.fold && role_wave == 0 && blockIdx.x < d.c)
    wsum_channel<K>(gw, gwf, t.G, blockIdx.x, threadIdx.x);
  if (MODE == 0 && role_wave < t.wpb)
    dw_bwd_stream_body<K, S, V, RB, EDGE, true, false>(gy, x, wt, gx, gw, gwf, d, t,
                                                       role_wave);
  else if (MODE == 0)
    dw_bwd_stream_body<K, S, V, RB, EDGE, false, true>(gy, x, wt, gx, gw, gwf, d, t,
                                                       role_wave - t.wpb);
  else
    dw_bwd_stream_body<K, S, V, RB, EDGE, MODE == 1, MODE == 2>(gy, x, wt, gx, gw, gwf, d,
                                                                t, role_wave);
}

// Stream configuration: columns per lane V, segment lanes L (EDGE when a row
// is split into several segments), rows per band RB.
struct DwCfg {
  int v, rb;
  bool edge;
};

DwCfg stream_cfg(int s, const DwShape& d) {
  // whole rows in one segment when that keeps >= 90 % of a wave's lanes busy
  // (no halo loads at all), else segments of <= 20 lanes with edge loads
  auto util = [](int64_t l) { return (double)((64 / l) * l) / 64.0; };
  DwCfg c{};
  const int vs[2] = {s == 1 ? 4 : 2, s == 1 ? 8 : 4};
  c.v = 0;  // 0: no stream configuration (the strip kernels run)
  c.edge = true;
  for (int v : vs) {
    if (d.wo % v) continue;
    const int64_t cg = d.wo / v;
    if (cg <= 64 && util(cg) >= 0.9) {
      c.v = v;
      c.edge = false;
      break;
    }
  }
  if (!c.v && d.wo % vs[0] == 0) c.v = vs[0];
  if (!c.v) return c;
  c.rb = (s == 1 ? 8 : 4) / (c.v == vs[1] ? 2 : 1);

  return c;
}

DwStream stream_layout(const DwShape& d, const DwCfg& c) {
  DwStream t{};
  const int cg = (int)(d.wo / c.v);  // column groups per row
  t.L = 1;
  if (!c.edge) {
    t.L = cg;
  } else {
    for (int l = cg < 20 ? cg : 20; l >= 1; --l)
      if (cg % l == 0) {
        t.L = l;
        break;
      }
  }
  t.spw = 64 / t.L;
  t.nseg = cg / t.L;
  t.nb = (int)cdiv(d.ho, c.rb);
  return t;
}

bool stream_ok(const DwShape& d, int k, int s) {
  return d.pad == k / 2 && d.w == s * d.wo && d.h >= 1 && stream_cfg(s, d).v != 0;
}

bool dw_ok(int64_t n, int64_t c, int64_t h, int64_t w, int64_t k, int64_t stride,
           int64_t pad) {
  return n > 0 && c > 0 && h > 0 && w > 0 && (k == 3 || k == 5) &&
         (stride == 1 || stride == 2) && pad >= 0 && pad < k && n * c <= 65535 &&
         n * c * h * w < (int64_t(1) << 31) && h * w < (int64_t(1) << 24) &&
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

template <int K, int S, int V, int RB, bool EDGE>
int launch_fwd_stream(const float* x, const float* wt, float* y, int64_t n, const DwShape& d,
                      const DwStream& t, hipStream_t st) {
  const int64_t units = n * d.c * t.nb * t.nseg;
  const int64_t waves = cdiv(units, t.spw);
  const double bytes = 4.0 * n * d.c * (d.h * d.w + d.ho * d.wo);
  MDE_LAUNCH(K_DW_FWD, bytes, st, (dw_fwd_stream_kernel<K, S, V, RB, EDGE>),
             dim3((unsigned)cdiv(waves, 4)), dim3(256), 0, x, wt, y, d, t, units);
  return 0;
}

// Calls F.template operator()<V, RB, EDGE>() for the instantiated stream
// configurations (V0 columns x R0 rows, or 2 V0 columns x R0 / 2 rows).
template <int S, typename F>
int with_cfg(const DwCfg& c, F&& f) {
  constexpr int V0 = S == 1 ? 4 : 2, R0 = S == 1 ? 8 : 4;
  if (c.v == V0) return c.edge ? f.template operator()<V0, R0, true>()
                               : f.template operator()<V0, R0, false>();
  return c.edge ? f.template operator()<2 * V0, R0 / 2, true>()
                : f.template operator()<2 * V0, R0 / 2, false>();
}

template <int K, int S>
int launch_fwd(const float* x, const float* wt, float* y, int64_t n, const DwShape& d,
               hipStream_t st) {
  if (stream_ok(d, K, S)) {
    const DwCfg c = stream_cfg(S, d);
    const DwStream t = stream_layout(d, c);
    return with_cfg<S>(c, [&]<int V, int RB, bool EDGE>() {
      return launch_fwd_stream<K, S, V, RB, EDGE>(x, wt, y, n, d, t, st);
    });
  }
  const int64_t planes = n * d.c;
  const DwStrip t = strip_tile(d, K, S, planes);
  const dim3 grid((unsigned)t.tx, (unsigned)t.ty, (unsigned)cdiv(planes, t.pb));
  const double bytes = 4.0 * n * d.c * (d.h * d.w + d.ho * d.wo);
  MDE_LAUNCH(K_DW_FWD, bytes, st, (dw_fwd_strip_kernel<K, S>), grid, dim3(256),
             sizeof(float) * t.pb * t.xh * t.xw, x, wt, y, d, t, (int)planes);
  return 0;
}

// Blocks per channel of the fused backward: ~2048 blocks in all (8 per CU).
int strip_groups(int64_t n, int64_t c, const DwStrip& t) {
  const int64_t items = cdiv(n, t.pb) * (int64_t)t.tx * t.ty;
  int64_t g = cdiv(2048, c);
  if (g > items) g = items;
  return (int)(g < 1 ? 1 : g);
}

template <int K, int S>
int launch_bwd_strip(const float* gy, const float* x, const float* wt, float* gx, float* gw,
                     float* part, int64_t n, const DwShape& d, hipStream_t st) {
  const DwStrip t = strip_tile(d, K, S, n);
  const int G = strip_groups(n, d.c, t);
  float* dst = gw ? (G == 1 ? gw : part) : nullptr;
  const size_t lds = sizeof(float) * t.pb * (t.gh * t.gw + (gw ? t.xh * t.xw : 0));
  const double bytes =
      4.0 * n * d.c * (d.ho * d.wo + (gx ? d.h * d.w : 0) + (gw ? d.h * d.w : 0));
  MDE_LAUNCH(K_DW_BWD, bytes, st, (dw_bwd_strip_kernel<K, S>), dim3((unsigned)d.c, (unsigned)G),
             dim3(256), lds, gy, x, wt, gx, dst, d, t, n, G);
  if (gw && G > 1)
    MDE_LAUNCH(K_DW_WREDUCE, 4.0 * d.c * G * K * K, st, dw_wreduce_kernel<K>,
               dim3((unsigned)d.c), dim3(256), 0, part, gw, (int64_t)G);
  return 0;
}

// Backward stream layout: units per channel, waves per block, groups per
// wave and blocks per channel (G > 1: per-block partials + dw_wreduce).
DwStream stream_bwd_layout(int64_t n, const DwShape& d, const DwCfg& c) {
  DwStream t = stream_layout(d, c);
  t.upc = n * t.nb * t.nseg;
  const int64_t wpc = cdiv(t.upc, t.spw);  // waves per channel
  // gx and gw are separate launches (one role per block); a block of up to 8
  // waves when that holds a whole channel (no partials), else 4-wave blocks
  // (finer-grained block turnover)
  t.wpb = (int)(wpc <= 8 ? wpc : 4);
  const int64_t slots = cdiv(wpc, t.wpb);  // wave groups per channel
  // enough blocks to fill the chip (>= ~4 per CU) before looping inside a block
  int64_t g = slots, it = 1;
  while (g > 1 && d.c * g > 4096) {
    ++it;
    g = cdiv(slots, it);
  }
  t.G = (int)g;
  t.it = (int)cdiv(slots, g);
  return t;
}

template <int K, int S, int V, int RB, bool EDGE>
int launch_bwd_stream(const float* gy, const float* x, const float* wt, float* gx, float* gw,
                      float* part, int64_t n, const DwShape& d, const DwStream& t,
                      hipStream_t st) {
  float* dst = gw ? (t.G == 1 ? gw : part) : nullptr;
  const double bytes =
      4.0 * n * d.c * (d.ho * d.wo + (gx ? d.h * d.w : 0) + (gw ? d.h * d.w : 0));
  const dim3 grid((unsigned)(d.c * t.G)), block((unsigned)(64 * t.wpb));
  // gx and gw as two launches (each wave holds one role's registers; the
  // second gy read is an L2 / MALL hit for the small planes).  A channel
  // split over G > 1 blocks leaves G partials that the gx launch following
  // it sums (its block ch, wave 0, before its own units), else
  // dw_wsum_kernel: the kernel boundary orders the partials' stores before
  // their loads, so no cross-block hand-off (and no L2 flush) is needed.
  const bool sum = gw && t.G > 1;
  if (gw)
    MDE_LAUNCH(K_DW_BWD, gx ? 0.0 : bytes, st, (dw_bwd_stream_kernel<K, S, V, RB, EDGE, 2>), grid,
               block, 0, gy, x, wt, gx, dst, gw, d, t, (int)n);
  if (gx) {
    DwStream tf = t;
    tf.fold = sum ? 1 : 0;
    MDE_LAUNCH(K_DW_BWD, bytes, st, (dw_bwd_stream_kernel<K, S, V, RB, EDGE, 1>), grid, block, 0,
               gy, x, wt, gx, dst, gw, d, tf, (int)n);
  } else if (sum) {
    MDE_LAUNCH(K_DW_WREDUCE, 4.0 * d.c * t.G * K * K, st, dw_wsum_kernel<K>,
               dim3((unsigned)d.c), dim3(64), 0, part, gw, t.G);
  }
  return 0;
}

template <int K, int S>
int launch_bwd(const float* gy, const float* x, const float* wt, float* gx, float* gw,
               float* part, int64_t n, const DwShape& d, hipStream_t st) {
  if (stream_ok(d, K, S)) {
    const DwCfg c = stream_cfg(S, d);
    const DwStream t = stream_bwd_layout(n, d, c);
    return with_cfg<S>(c, [&]<int V, int RB, bool EDGE>() {
      return launch_bwd_stream<K, S, V, RB, EDGE>(gy, x, wt, gx, gw, part, n, d, t, st);
    });
  }
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
  if (stream_ok(d, (int)k, (int)stride)) {
    const DwStream t = stream_bwd_layout(n, d, stream_cfg((int)stride, d));
    return t.G > 1 ? (size_t)(4 * c * t.G * k * k) : 0;
  }
  if (pad == k / 2) {
    const int G = strip_groups(n, c, strip_tile(d, (int)k, (int)stride, n));
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
