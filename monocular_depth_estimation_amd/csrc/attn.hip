// NewCRF shifted-window attention on MFMA (gfx950, fp32, head dim 32).
//
// Reference: WindowAttention.forward (src/newcrf_layers.py:110-149) inside
// CRFBlock.forward (:195-257): LayerNorm'd tokens are zero-padded to multiples
// of the window, cyclically shifted by -shift, partitioned into ws x ws
// windows; per window and head
//     S = (q * d^-1/2) k^T + T[relative_index] (+ -100 across shifted regions)
//     O = softmax(S) v_head            (v is NOT projected: split into heads)
// and the windows are reversed, un-shifted and cropped.
//
// Here the pad / roll / partition / reverse / crop are pure index math: a
// window's token (r, c) lives at padded coordinate
//     ((wy*ws + r + shift) mod Hp, (wx*ws + c + shift) mod Wp)
// and is a real token if that is inside H x W.  The qk Linear is applied to
// the real tokens only (a GEMM outside); a padded token's q and k are the qk
// BIAS (the reference pads after the LayerNorm, before the Linear) and its v
// is 0, so padded keys take part in the softmax exactly as in the reference.
// Outputs are written straight to token order [B, H*W, C].
//
// Per (window, head) the 49x49 (padded to 64x64) score tile and the 64x32
// output tile are v_mfma_f32_16x16x4_f32 products (exact fp32, one rounding
// per product): 4 waves, wave w owns rows 16w..16w+15.
//
// Backward recomputes S and P (no saved probabilities), then
//   dP = dO V^T, dS = P (dP - rowsum(P dP)), dQ = dS K / sqrt(d),
//   dK = dS^T Q / sqrt(d), dV = P^T dO, dT[idx] = sum dS,
// with dK of padded keys summed into d(qk bias).  Table and bias gradients
// are reduced per block in a fixed order into a slab and summed by a second
// kernel: deterministic, no atomics.
#include "common.h"

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int D = 32;       // head dim (all four NewCRF stages)
constexpr int NP = 64;      // padded tokens per window (ws*ws <= 64)
constexpr int LD = 33;      // LDS row stride of the [64][32] tiles
constexpr int LP = 65;      // LDS row stride of the [64][64] tiles
constexpr int kGroup = 8;   // windows per backward block

struct Geo {
  int b, h, w, c, heads, ws, shift, hp, wp, nwh, nww, n;
  float scale;
};

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int region(int y, int hp, int ws, int shift) {
  return y < hp - ws ? 0 : (y < hp - shift ? 1 : 2);
}

// Token bookkeeping for window `win` of the shifted, padded grid.
__device__ __forceinline__ void window_tokens(const Geo& g, int win, int* tok,
                                              int* lab) {
  const int wloc = win % (g.nwh * g.nww);
  const int wy = wloc / g.nww, wx = wloc % g.nww;
  for (int i = threadIdx.x; i < NP; i += blockDim.x) {
    int t = -2, l = 0;
    if (i < g.n) {
      const int r = i / g.ws, cc = i % g.ws;
      const int ys = wy * g.ws + r, xs = wx * g.ws + cc;
      const int yp = (ys + g.shift) % g.hp, xp = (xs + g.shift) % g.wp;
      t = (yp < g.h && xp < g.w) ? yp * g.w + xp : -1;
      l = region(ys, g.hp, g.ws, g.shift) * 3 + region(xs, g.wp, g.ws, g.shift);
    }
    tok[i] = t;
    lab[i] = l;
  }
}

// Q (pre-scaled), K, V tiles of one (window, head); padded -> bias / 0.
__device__ __forceinline__ void load_qkv(const Geo& g, int bidx, int head,
                                         const float* __restrict__ qk,
                                         const float* __restrict__ qkb,
                                         const float* __restrict__ v,
                                         const int* tok, float (*Q)[LD],
                                         float (*K)[LD], float (*V)[LD]) {
  const int64_t c2 = 2 * (int64_t)g.c;
  const float* qkbase = qk + (int64_t)bidx * g.h * g.w * c2;
  const float* vbase = v + (int64_t)bidx * g.h * g.w * g.c;
  for (int e = threadIdx.x; e < NP * D; e += blockDim.x) {
    const int i = e / D, k = e % D;
    const int t = tok[i];
    float q = 0.f, kk = 0.f, vv = 0.f;
    if (t >= 0) {
      q = qkbase[t * c2 + head * D + k];
      kk = qkbase[t * c2 + g.c + head * D + k];
      vv = vbase[(int64_t)t * g.c + head * D + k];
    } else if (t == -1) {
      q = qkb[head * D + k];
      kk = qkb[g.c + head * D + k];
    }
    Q[i][k] = q * g.scale;
    K[i][k] = kk;
    V[i][k] = vv;
  }
}

// S rows of this wave (16 x 64) = Q K^T + bias (+ mask); -inf past the window.
__device__ __forceinline__ void scores(const Geo& g, float (*Q)[LD], float (*K)[LD],
                                       const float* tab, const int* lab, f4 s[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) s[ct] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < D / 4; ++kc) {
    const float a = Q[16 * w + (lane & 15)][4 * kc + (lane >> 4)];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
      s[ct] = mfma4(a, K[16 * ct + (lane & 15)][4 * kc + (lane >> 4)], s[ct]);
  }
  const int ws = g.ws, span = 2 * ws - 1;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int j = 16 * ct + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * w + (lane >> 4) * 4 + r;
      if (j >= g.n || i >= g.n) {
        s[ct][r] = j >= g.n ? -INFINITY : 0.f;
      } else {
        const int idx = (i / ws - j / ws + ws - 1) * span + (i % ws - j % ws + ws - 1);
        float v = s[ct][r] + tab[idx];
        if (g.shift && lab[i] != lab[j]) v += -100.f;
        s[ct][r] = v;
      }
    }
  }
}

// Row-wise softmax over the 64 columns held by 16 lanes x 4 column tiles.
__device__ __forceinline__ void softmax_rows(f4 s[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float m = fmaxf(fmaxf(s[0][r], s[1][r]), fmaxf(s[2][r], s[3][r]));
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float sum = 0.f;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const float e = __expf(s[ct][r] - m);
      s[ct][r] = e;
      sum += e;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
    const float inv = 1.f / sum;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) s[ct][r] *= inv;
  }
}

// Store a wave's 16 x 64 accumulator rows into a [64][LP] LDS tile.
__device__ __forceinline__ void store_rows(float (*T)[LP], const f4 s[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) T[16 * w + (lane >> 4) * 4 + r][16 * ct + (lane & 15)] = s[ct][r];
}

// out rows (16w..16w+15) x 32 = A[rows][0..63] @ B[0..63][0..31]
// TRANS_A: read A transposed from the [64][LP] tile (A[i][k] = T[k][i]).
template <bool TRANS_A>
__device__ __forceinline__ void mm_64x32(float (*A)[LP], float (*B)[LD], f4 o[2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  o[0] = f4{0.f, 0.f, 0.f, 0.f};
  o[1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < NP / 4; ++kc) {
    const int row = 16 * w + (lane & 15), k = 4 * kc + (lane >> 4);
    const float a = TRANS_A ? A[k][row] : A[row][k];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) o[dt] = mfma4(a, B[k][16 * dt + (lane & 15)], o[dt]);
  }
}

__global__ void __launch_bounds__(256)
    wattn_fwd_kernel(const float* __restrict__ qk, const float* __restrict__ qkb,
                     const float* __restrict__ v, const float* __restrict__ table,
                     float* __restrict__ out, Geo g) {
  __shared__ float Q[NP][LD], K[NP][LD], V[NP][LD];
  __shared__ float P[NP][LP];
  __shared__ float tab[256];
  __shared__ int tok[NP], lab[NP];
  const int win = blockIdx.x, head = blockIdx.y;
  const int bidx = win / (g.nwh * g.nww);
  const int ntab = (2 * g.ws - 1) * (2 * g.ws - 1);
  for (int i = threadIdx.x; i < ntab; i += blockDim.x) tab[i] = table[i * g.heads + head];
  window_tokens(g, win, tok, lab);
  __syncthreads();
  load_qkv(g, bidx, head, qk, qkb, v, tok, Q, K, V);
  __syncthreads();
  f4 s[4];
  scores(g, Q, K, tab, lab, s);
  softmax_rows(s);
  store_rows(P, s);
  __syncthreads();
  f4 o[2];
  mm_64x32<false>(P, V, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* obase = out + (int64_t)bidx * g.h * g.w * g.c;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 16 * w + (lane >> 4) * 4 + r;
    const int t = i < NP ? tok[i] : -2;
    if (t >= 0) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
        obase[(int64_t)t * g.c + head * D + 16 * dt + (lane & 15)] = o[dt][r];
    }
  }
}

// slab[(blockIdx.x * heads + head) * (ntab + D)] = {dT[0..ntab), dkbias[0..D)}
__global__ void __launch_bounds__(256)
    wattn_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ qk,
                     const float* __restrict__ qkb, const float* __restrict__ v,
                     const float* __restrict__ table, float* __restrict__ gqk,
                     float* __restrict__ gv, float* __restrict__ slab, int nwin, Geo g) {
  __shared__ float Q[NP][LD], K[NP][LD], V[NP][LD], G[NP][LD];
  __shared__ float P[NP][LP], DS[NP][LP];
  __shared__ float tab[256], dtab[256], dkb[D];
  __shared__ int tok[NP], lab[NP];
  const int head = blockIdx.y;
  const int ntab = (2 * g.ws - 1) * (2 * g.ws - 1);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c2 = 2 * (int64_t)g.c;
  for (int i = threadIdx.x; i < ntab; i += blockDim.x) {
    tab[i] = table[i * g.heads + head];
    dtab[i] = 0.f;
  }
  if (threadIdx.x < D) dkb[threadIdx.x] = 0.f;
  for (int wi = 0; wi < kGroup; ++wi) {
    const int win = blockIdx.x * kGroup + wi;
    if (win >= nwin) break;  // uniform across the block
    const int bidx = win / (g.nwh * g.nww);
    __syncthreads();
    window_tokens(g, win, tok, lab);
    __syncthreads();
    load_qkv(g, bidx, head, qk, qkb, v, tok, Q, K, V);
    const float* gbase = gout + (int64_t)bidx * g.h * g.w * g.c;
    for (int e = threadIdx.x; e < NP * D; e += blockDim.x) {
      const int i = e / D, k = e % D;
      const int t = tok[i];
      G[i][k] = t >= 0 ? gbase[(int64_t)t * g.c + head * D + k] : 0.f;
    }
    __syncthreads();
    f4 s[4];
    scores(g, Q, K, tab, lab, s);
    softmax_rows(s);
    // dP = dO V^T for this wave's rows
    f4 dp[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) dp[ct] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < D / 4; ++kc) {
      const float a = G[16 * w + (lane & 15)][4 * kc + (lane >> 4)];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        dp[ct] = mfma4(a, V[16 * ct + (lane & 15)][4 * kc + (lane >> 4)], dp[ct]);
    }
    // dS = P (dP - rowsum(P dP))
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float dl = 0.f;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) dl += s[ct][r] * dp[ct][r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) dl += __shfl_xor(dl, o, 64);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) dp[ct][r] = s[ct][r] * (dp[ct][r] - dl);
    }
    store_rows(P, s);
    store_rows(DS, dp);
    __syncthreads();
    // table gradient: entry e <- sum over the (i, j) pairs with that offset,
    // in a fixed order (deterministic)
    for (int e = threadIdx.x; e < ntab; e += blockDim.x) {
      const int span = 2 * g.ws - 1;
      const int dy = e / span - (g.ws - 1), dx = e % span - (g.ws - 1);
      float acc = 0.f;
      for (int ri = 0; ri < g.ws; ++ri) {
        const int rj = ri - dy;
        if (rj < 0 || rj >= g.ws) continue;
        for (int ci = 0; ci < g.ws; ++ci) {
          const int cj = ci - dx;
          if (cj < 0 || cj >= g.ws) continue;
          acc += DS[ri * g.ws + ci][rj * g.ws + cj];
        }
      }
      dtab[e] += acc;
    }
    f4 o[2];
    float* gqkb = gqk + (int64_t)bidx * g.h * g.w * c2;
    // dQ = dS K * scale   (rows i of this wave)
    {
      const int row = 16 * w;
      o[0] = f4{0.f, 0.f, 0.f, 0.f};
      o[1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < NP / 4; ++kc) {
        const float a = DS[row + (lane & 15)][4 * kc + (lane >> 4)];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          o[dt] = mfma4(a, K[4 * kc + (lane >> 4)][16 * dt + (lane & 15)], o[dt]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = row + (lane >> 4) * 4 + r;
        const int t = tok[i];
        if (t >= 0) {
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
            gqkb[t * c2 + head * D + 16 * dt + (lane & 15)] = o[dt][r] * g.scale;
        }
      }
    }
    // dV = P^T dO   (rows j of this wave)
    mm_64x32<true>(P, G, o);
    float* gvb = gv + (int64_t)bidx * g.h * g.w * g.c;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * w + (lane >> 4) * 4 + r;
      const int t = tok[j];
      if (t >= 0) {
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          gvb[(int64_t)t * g.c + head * D + 16 * dt + (lane & 15)] = o[dt][r];
      }
    }
    // dK = dS^T Q_scaled   (rows j of this wave); padded keys -> d(k bias)
    mm_64x32<true>(DS, Q, o);
    __syncthreads();  // every wave is done reading G (dO) before it is reused
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * w + (lane >> 4) * 4 + r;
      const int t = tok[j];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int d = 16 * dt + (lane & 15);
        if (t >= 0) gqkb[t * c2 + g.c + head * D + d] = o[dt][r];
        G[j][d] = t == -1 ? o[dt][r] : 0.f;  // stage padded-key rows
      }
    }
    __syncthreads();
    if (threadIdx.x < D) {
      float acc = 0.f;
      for (int j = 0; j < g.n; ++j) acc += G[j][threadIdx.x];
      dkb[threadIdx.x] += acc;
    }
  }
  __syncthreads();
  float* sl = slab + ((int64_t)blockIdx.x * g.heads + head) * (ntab + D);
  for (int i = threadIdx.x; i < ntab; i += blockDim.x) sl[i] = dtab[i];
  if (threadIdx.x < D) sl[ntab + threadIdx.x] = dkb[threadIdx.x];
}

// gtable[e, head] / gqkb[C + head*D + d] = sum over blocks (fixed order).
__global__ void __launch_bounds__(256)
    wattn_slab_reduce_kernel(const float* __restrict__ slab, int nblocks, int heads,
                             int ntab, int c, float* __restrict__ gtable,
                             float* __restrict__ gqkb) {
  const int head = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int per = ntab + D;
  if (e >= per) return;
  float acc = 0.f;
  for (int k = 0; k < nblocks; ++k) acc += slab[((int64_t)k * heads + head) * per + e];
  if (e < ntab)
    gtable[e * heads + head] = acc;
  else
    gqkb[c + head * D + (e - ntab)] = acc;
}

__global__ void zero_kernel(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

bool make_geo(int64_t b, int64_t h, int64_t w, int64_t c, int64_t heads, int64_t ws,
              int64_t shift, Geo* g) {
  if (b <= 0 || h <= 0 || w <= 0 || heads <= 0 || c != heads * D || ws <= 0 ||
      ws * ws > NP || shift < 0 || shift >= ws || (2 * ws - 1) * (2 * ws - 1) > 256)
    return false;
  g->b = (int)b; g->h = (int)h; g->w = (int)w; g->c = (int)c;
  g->heads = (int)heads; g->ws = (int)ws; g->shift = (int)shift;
  g->hp = (int)(mde::cdiv(h, ws) * ws);
  g->wp = (int)(mde::cdiv(w, ws) * ws);
  g->nwh = g->hp / g->ws;
  g->nww = g->wp / g->ws;
  g->n = g->ws * g->ws;
  g->scale = 1.f / sqrtf((float)D);
  return (int64_t)b * g->nwh * g->nww < (1LL << 31) && heads <= 65535;
}

}  // namespace

extern "C" {

size_t mde_window_attn_workspace(int64_t b, int64_t h, int64_t w, int64_t c,
                                 int64_t heads, int64_t window) {
  Geo g;
  if (!make_geo(b, h, w, c, heads, window, 0, &g)) return 0;
  const int64_t nwin = (int64_t)b * g.nwh * g.nww;
  const int64_t ntab = (2 * window - 1) * (2 * window - 1);
  return sizeof(float) * (size_t)(mde::cdiv(nwin, kGroup) * heads * (ntab + D));
}

int mde_window_attn_fwd(const void* qk, const float* qk_bias, const void* v,
                        const float* table, void* out, int64_t b, int64_t h,
                        int64_t w, int64_t c, int64_t heads, int64_t window,
                        int64_t shift, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  Geo g;
  if (!qk || !qk_bias || !v || !table || !out || !make_geo(b, h, w, c, heads, window, shift, &g))
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nwin = (int64_t)b * g.nwh * g.nww;
  const double bytes = 4.0 * (double)b * h * w * c * 4.0;  // q, k, v read + o written
  MDE_LAUNCH(mde::K_WATTN_FWD, bytes, s, wattn_fwd_kernel,
             dim3((unsigned)nwin, (unsigned)heads), dim3(256), 0, (const float*)qk,
             qk_bias, (const float*)v, table, (float*)out, g);
  return MDE_OK;
}

int mde_window_attn_bwd(const void* gout, const void* qk, const float* qk_bias,
                        const void* v, const float* table, void* gqk, void* gv,
                        float* gtable, float* gqk_bias, int64_t b, int64_t h,
                        int64_t w, int64_t c, int64_t heads, int64_t window,
                        int64_t shift, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  Geo g;
  if (!gout || !qk || !qk_bias || !v || !table || !gqk || !gv || !gtable ||
      !gqk_bias || !workspace || !make_geo(b, h, w, c, heads, window, shift, &g))
    return MDE_ERR_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nwin = (int64_t)b * g.nwh * g.nww;
  const int nblk = (int)mde::cdiv(nwin, kGroup);
  const int ntab = (2 * g.ws - 1) * (2 * g.ws - 1);
  const double bytes = 4.0 * (double)b * h * w * c * 7.0;  // q k v dO (x2) read, dq dk dv written
  MDE_LAUNCH(mde::K_WATTN_BWD, bytes, s, wattn_bwd_kernel,
             dim3((unsigned)nblk, (unsigned)heads), dim3(256), 0, (const float*)gout,
             (const float*)qk, qk_bias, (const float*)v, table, (float*)gqk,
             (float*)gv, (float*)workspace, (int)nwin, g);
  // q half of d(qk bias) gets nothing from padded tokens (their dO is 0)
  MDE_LAUNCH(mde::K_WATTN_BWD, 0.0, s, zero_kernel, dim3((unsigned)mde::cdiv(c, 256)),
             dim3(256), 0, gqk_bias, (int)c);
  MDE_LAUNCH(mde::K_WATTN_BWD, 4.0 * nblk * heads * (ntab + D), s,
             wattn_slab_reduce_kernel, dim3((unsigned)mde::cdiv(ntab + D, 256), (unsigned)heads),
             dim3(256), 0, (const float*)workspace, nblk, (int)heads, ntab, (int)c,
             gtable, gqk_bias);
  return MDE_OK;
}

}  // extern "C"
