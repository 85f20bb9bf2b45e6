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
// Work split: one wave per (window, head), four heads per block.  A window's
// <= 64 tokens are padded to 64 = 4 MFMA tiles.  The scores live in
// registers TRANSPOSED, S^T[j][i] (key rows, query columns), as 4x4
// v_mfma_f32_16x16x4_f32 accumulators: with the query in the C-column slot a
// lane's four accumulator values of a tile are four keys of ONE query, which
// is exactly the A-operand of the next product that contracts over keys
// (O = P V, dQ = dS K) — no LDS round trip.  The head-dim contraction of
// S^T = K Q^T uses a permuted k order (lane group g supplies dims 8g..8g+7
// over the 8 MFMA steps), so each lane's operands are 32 contiguous bytes of
// a token row: two float4 loads straight from HBM/L2, no LDS staging.
// Products contracting over queries (dV = P^T dO, dK = dS^T Q) read P / dS
// back from a per-wave LDS tile.  All f32 MFMA: exact f32 products.
//
// Backward recomputes S and P (no saved probabilities), then
//   dP = dO V^T, dS = P (dP - rowsum(P dP)), dQ = dS K / sqrt(d),
//   dK = dS^T Q / sqrt(d), dV = P^T dO, dT[idx] = sum dS,
// with dK of padded keys summed into d(qk bias).  Table and bias gradients
// are reduced per block in a fixed order into a slab and summed by a second
// kernel: deterministic, no atomics.
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.h"

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int D = 32;        // head dim (all four NewCRF stages)
constexpr int NP = 64;       // padded tokens per window (ws*ws <= 64)
constexpr int LT = 67;       // LDS row pitch of the per-wave [64][64] P / dS tile (at most
                             // 2-way bank conflicts for both the own and the transposed
                             // access pattern; 65 has 4-way)
constexpr int TABP = 256;    // table slots ((2ws-1)^2 <= 225)

// The backward's per-wave P / dS tile.  Generic windows: [64][LT].  7x7
// windows (every NewCRF / SAM stage): only keys / queries 0..48 are real, so
// the tile keeps rows and columns 0..48 plus a zero row / column 49 that the
// reads of padded keys / queries are redirected to (their P and dS are 0 by
// construction, so they are never written): 50 x 51 floats = 10.2 KB instead
// of 17.2 KB, which with <= 168 VGPRs lets three 4-wave blocks share a CU
// (three waves per SIMD instead of two).
template <int WS>
struct Tile {
  static constexpr bool kCompact = WS == 7;
  static constexpr int kValid = kCompact ? 49 : NP;  // real keys / queries
  static constexpr int kRows = kCompact ? 50 : NP;
  static constexpr int kPitch = kCompact ? 51 : LT;   // <= 2-way conflicts both ways
  static constexpr int kWords = kRows * kPitch;
  // tile row / column of key / query index v of 16-tile `t` (static t): only
  // the last tile (48..63) can hold padded indices
  template <int t>
  __device__ static __forceinline__ int clamp(int v) {
    if constexpr (kCompact && t == 3) return v < kValid ? v : kValid;
    return v;
  }
  template <int t>
  __device__ static __forceinline__ bool valid(int v) {
    if constexpr (kCompact && t == 3) return v < kValid;
    return true;
  }
  // k-steps r of a product contracting over 16-tile `t` (index 16t + 4g + r):
  // in the compact last tile only r = 0 holds a real index (48); the other
  // steps would multiply zeros
  template <int t>
  __device__ static constexpr int ksteps() {
    return kCompact && t == 3 ? 1 : 4;
  }
};
constexpr int kOccBwd7 = 3;  // blocks per CU the 7x7 backward is built for
constexpr int kHeads = 4;    // heads (= waves) per block


struct Geo {
  int b, h, w, c, heads, ws, shift, hp, wp, nwh, nww, n;
  float scale;
  const float* vb;  // v of a padded token (SAM: the kv Linear's v bias); NULL = 0 (NewCRF)
};

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int region(int y, int hp, int ws, int shift) {
  return y < hp - ws ? 0 : (y < hp - shift ? 1 : 2);
}

template <int WS>
__device__ __forceinline__ int wsize(const Geo& g) {
  return WS ? WS : g.ws;
}

// tok[i]: the token's row offset in a C-wide image tensor (token index * c,
// >= 0; a qk row is at 2 tok[i]), -1 padded (q = k = bias, v = 0),
// -2 beyond the window (i >= ws*ws); lab[i]: shifted-region label.
template <int WS>
__device__ __forceinline__ void window_tokens(const Geo& g, int win, int* tok, int* lab) {
  const int ws = wsize<WS>(g), n = ws * ws;
  const int i = threadIdx.x;
  if (i >= NP) return;
  const int wloc = win % (g.nwh * g.nww);
  const int wy = wloc / g.nww, wx = wloc - wy * g.nww;
  int t = -2, l = 0;
  if (i < n) {
    const int r = i / ws, cc = i - r * ws;
    const int ys = wy * ws + r, xs = wx * ws + cc;
    int yp = ys + g.shift, xp = xs + g.shift;
    if (yp >= g.hp) yp -= g.hp;
    if (xp >= g.wp) xp -= g.wp;
    t = (yp < g.h && xp < g.w) ? (yp * g.w + xp) * g.c : -1;
    l = region(ys, g.hp, ws, g.shift) * 3 + region(xs, g.wp, ws, g.shift);
  }
  tok[i] = t;
  lab[i] = l;
}

// Wave-uniform base pointers live in SGPRs (readfirstlane), and every access
// is base + a 32-bit BYTE offset (element index < 2^30, checked on the host):
// one global_load / global_store with an SGPR base and a VGPR offset, no
// 64-bit address arithmetic per access (it was ~2 VALU per memory op, and the
// backward is VALU-bound).
template <typename T>
__device__ __forceinline__ T* sgpr(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  // Through an explicit global-address-space pointer so the accesses stay
  // global_* (an integer->pointer round trip would otherwise make them flat_*).
  using G = __attribute__((address_space(1))) T*;
  return (T*)(G)(((uint64_t)hi << 32) | lo);
}
template <typename T>
__device__ __forceinline__ T* at(T* base, unsigned i) {
  using C = std::conditional_t<std::is_const_v<T>, const char, char>;
  return reinterpret_cast<T*>(reinterpret_cast<C*>(base) + (i << 2));
}

// 8 contiguous floats at p (32-byte aligned)
__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// Row operand: columns [off, off+8) of the row at m * t (t: a tok[] entry,
// m = 1 for C-wide tensors, 2 for qk; a compile-time constant), the bias
// for a padded token (when given), else zeros.
__device__ __forceinline__ void row8(const float* base, int m, int off, int t,
                                     const float* bias, float* v) {
  if (t >= 0) {
    load8(at(base, (unsigned)(m * t + off)), v);
  } else if (t == -1 && bias) {
    load8(at(bias, (unsigned)off), v);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = 0.f;
  }
}

// Scalar operand: element `col` of the row at m * t, bias for padded, else 0.
__device__ __forceinline__ float elem(const float* base, int m, int col, int t,
                                      const float* bias) {
  if (t >= 0) return *at(base, (unsigned)(m * t + col));
  if (t == -1 && bias) return *at(bias, (unsigned)col);
  return 0.f;
}

// One 16-key tile of sum_i T[j][i] B[i][c]: o[ct] (C layout: key 16jt + 4g + rr,
// c = 16ct + l16), B given per lane as b[it][r][ct] = B[16it + 4g + r][16ct + l16].
template <int WS, int jt>
__device__ __forceinline__ void mm_tb_tile(const float* T, const float b[4][4][2], f4 o[2],
                                           int lane) {
  using TL = Tile<WS>;
  const int l16 = lane & 15, g4 = lane >> 4;
  o[0] = f4{0.f, 0.f, 0.f, 0.f};
  o[1] = f4{0.f, 0.f, 0.f, 0.f};
  const int rowoff = TL::template clamp<jt>(16 * jt + l16) * TL::kPitch;
  auto step = [&](auto it_c) {
    constexpr int it = decltype(it_c)::value;
#pragma unroll
    for (int r = 0; r < TL::template ksteps<it>(); ++r) {
      const float a = T[rowoff + TL::template clamp<it>(16 * it + 4 * g4 + r)];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) o[ct] = mfma4(a, b[it][r][ct], o[ct]);
    }
  };
  step(std::integral_constant<int, 0>{});
  step(std::integral_constant<int, 1>{});
  step(std::integral_constant<int, 2>{});
  step(std::integral_constant<int, 3>{});
}

// T[j][i] of this lane's own entries (key 16jt + 4g + r, query 16it + l16):
// 0 for padded keys / queries (never read from LDS, never written).
template <int WS, int jt, int it>
__device__ __forceinline__ float own_get(const float* T, int r, int lane) {
  using TL = Tile<WS>;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int j = 16 * jt + 4 * g4 + r, i = 16 * it + l16;
  return T[TL::template clamp<jt>(j) * TL::kPitch + TL::template clamp<it>(i)];
}
template <int WS, int jt, int it>
__device__ __forceinline__ void own_put(float* T, int r, float v, int lane) {
  using TL = Tile<WS>;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int j = 16 * jt + 4 * g4 + r, i = 16 * it + l16;
  if (TL::template valid<jt>(j) && TL::template valid<it>(i)) T[j * TL::kPitch + i] = v;
}

// threadIdx-derived lane, opaque to the optimiser: each phase of the 7x7
// backward recomputes its lane index math instead of the compiler hoisting
// it out of the window loop and keeping ~60 registers of it live across all
// phases (which spilled at the three-waves-per-SIMD budget).
__device__ __forceinline__ int opaque_lane() {
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}

template <int N, typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

template <typename F>
__device__ __forceinline__ void static_for4(F&& f) {
  f(std::integral_constant<int, 0>{});
  f(std::integral_constant<int, 1>{});
  f(std::integral_constant<int, 2>{});
  f(std::integral_constant<int, 3>{});
}

// Per-lane operands of one window-head's scores: K rows (ka) and the
// key table offsets / region labels (kj), loaded once for all query tiles.
template <int WS>
__device__ __forceinline__ void key_operands(const Geo& g, const float* __restrict__ qkrow,
                                             const float* __restrict__ qkb, int head,
                                             const int* tok, const int* lab, int lane,
                                             float ka[4][8], int kj[16]) {
  const int l16 = lane & 15, g4 = lane >> 4;
  const int ws = wsize<WS>(g), span = 2 * ws - 1;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
    row8(qkrow, 2, g.c + head * D + 8 * g4, tok[16 * jt + l16], qkb, ka[jt]);
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jt + 4 * g4 + r;
      const int y = j / ws, x = j - y * ws;
      kj[4 * jt + r] = ((y * span + x) << 4) | lab[j];
    }
}

// P^T of query tile `it` (keys 16jt + 4g + r of query 16it + l16 in s[jt][r]):
// S^T column tile by 8 MFMA steps over the head dim, table bias + shift mask,
// softmax over the keys; padded query columns 0.  16 live score registers
// (probs_t's whole 4x4 tile holds 64).
// `qraw`: this lane's 8 head dims of query 16it + l16 (q_row(), loaded one
// tile ahead by the caller so the load latency overlaps the previous tile).
template <int WS>
__device__ __forceinline__ void q_row(const Geo& g, const float* __restrict__ qkrow,
                                      const float* __restrict__ qkb, int head, const int* tok,
                                      int it, int lane, float q[8]) {
  row8(qkrow, 2, head * D + 8 * (lane >> 4), tok[16 * it + (lane & 15)], qkb, q);
}

// One 64-key x 16-query column tile of a head-dim contraction (S^T = K Q^T,
// dP^T = V dO^T): out[jt][r] = sum_d R[16jt + 4g + r][d] C[16it + l16][d],
// rows[jt][k] = R[16jt + l16][8g + k], cols[k] = C[16it + l16][8g + k].
// Compact 7x7 windows: tile 3 holds one real key (48) and query tile 3 one
// real query (48), so 56 of the 128 MFMAs would multiply padding.  Here key
// 48's row and query 48's column come from VALU dot products instead (its
// dims broadcast from lane l16 == 0 of each lane group, the 32-dim sum over
// the four groups by two butterflies, query 48's column redistributed to the
// C layout by four shuffles per key tile): 72 MFMAs per column sweep.
template <int WS, int it>
__device__ __forceinline__ void kq_tile(const float rows[4][8], const float cols[8], f4 out[4],
                                        int lane) {
  if constexpr (!Tile<WS>::kCompact) {
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) out[jt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) out[jt] = mfma4(rows[jt][k], cols[k], out[jt]);
    return;
  }
  const int gbase = lane & 48, g4 = lane >> 4;
  {  // key 48 (tile 3, r = 0 of lane group 0): R[48] . C[16it + l16]
    float d = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) d = fmaf(__shfl(rows[3][k], gbase), cols[k], d);
    d += __shfl_xor(d, 16, 64);
    d += __shfl_xor(d, 32, 64);
    out[3] = f4{d, 0.f, 0.f, 0.f};  // keys 49.. of tile 3 are padding
  }
  if constexpr (it < 3) {
#pragma unroll
    for (int jt = 0; jt < 3; ++jt) out[jt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int jt = 0; jt < 3; ++jt) out[jt] = mfma4(rows[jt][k], cols[k], out[jt]);
  } else {
    // query 48 only (lanes l16 > 0 hold padded queries; their values are unused)
    float cq[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cq[k] = __shfl(cols[k], gbase);
#pragma unroll
    for (int jt = 0; jt < 3; ++jt) {
      float d = 0.f;  // R[16jt + l16] . C[48], summed over the four groups
#pragma unroll
      for (int k = 0; k < 8; ++k) d = fmaf(rows[jt][k], cq[k], d);
      d += __shfl_xor(d, 16, 64);
      d += __shfl_xor(d, 32, 64);
      const int src = gbase + 4 * g4;  // key 16jt + 4g + r sits in lane l16 = 4g + r
      out[jt] = f4{__shfl(d, src), __shfl(d, src + 1), __shfl(d, src + 2), __shfl(d, src + 3)};
    }
  }
}

template <int WS, int it>
__device__ __forceinline__ void probs_tile(const Geo& g, const float qraw[8], const int* lab,
                                           const float* tab, const float ka[4][8],
                                           const int kj[16], int lane, f4 s[4]) {
  const int l16 = lane & 15, g4 = lane >> 4;
  const int ws = wsize<WS>(g), n = ws * ws, span = 2 * ws - 1;
  {
    float qb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) qb[k] = qraw[k] * g.scale;
    kq_tile<WS, it>(ka, qb, s, lane);
  }
  const int i = 16 * it + l16;
  const bool iv = i < n;
  const int yi = i / ws, xi = i - yi * ws, li = lab[i];
  const int base = (yi + ws - 1) * span + xi + ws - 1;
  float m = -INFINITY;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jt + 4 * g4 + r;
      float v;
      if (j >= n) {
        v = -INFINITY;
      } else if (!iv) {
        v = 0.f;
      } else {
        const int q = kj[4 * jt + r];
        v = s[jt][r] + tab[base - (q >> 4)];
        if (g.shift && (q & 15) != li) v += -100.f;
      }
      s[jt][r] = v;
      m = fmaxf(m, v);
    }
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = __expf(s[jt][r] - m);
      s[jt][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = iv ? 1.f / sum : 0.f;  // padded query columns -> 0
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) s[jt] *= inv;
}

// The backward's P, staged query tile by query tile straight into the LDS
// tile (the register budget of three waves per SIMD).
template <int WS, typename Pre>
__device__ __forceinline__ void probs_stage(const Geo& g, const float* __restrict__ qkrow,
                                            const float* __restrict__ qkb, int head,
                                            const int* tok, const int* lab, const float* tab,
                                            float* T, Pre&& pre) {
  const int lane = opaque_lane();
  float ka[4][8];
  int kj[16];
  key_operands<WS>(g, qkrow, qkb, head, tok, lab, lane, ka, kj);
  float qn[8];
  q_row<WS>(g, qkrow, qkb, head, tok, 0, lane, qn);
  static_for4([&](auto it_c) {
    constexpr int it = decltype(it_c)::value;
    float qr[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) qr[k] = qn[k];
    if constexpr (it < 3) q_row<WS>(g, qkrow, qkb, head, tok, it + 1, lane, qn);
    else pre();  // the next phase's operands, in flight during the last tile
    f4 s[4];
    probs_tile<WS, it>(g, qr, lab, tab, ka, kj, lane, s);
    static_for4([&](auto jt_c) {
      constexpr int jt = decltype(jt_c)::value;
#pragma unroll
      for (int r = 0; r < 4; ++r) own_put<WS, jt, it>(T, r, s[jt][r], lane);
    });
  });
}

// Forward: one wave per (window, head), query tile by query tile: P^T
// columns (probs_tile), then O = P V with A = P[i][j] straight from the S^T
// accumulators (k <-> key 16jt + 4g + r) and B = V[j][d] per lane.
template <int WS>
__global__ void __launch_bounds__(256, 4)
    wattn_fwd_kernel(const float* __restrict__ qk, const float* __restrict__ qkb,
                     const float* __restrict__ v, const float* __restrict__ table,
                     float* __restrict__ out, Geo g) {
  __shared__ int tok[NP], lab[NP], kjs[NP];
  __shared__ float tab[kHeads][TABP];
  const int win = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, g4 = lane >> 4;
  const int head = blockIdx.y * kHeads + w;
  const int ws = wsize<WS>(g), ntab = (2 * ws - 1) * (2 * ws - 1);
  window_tokens<WS>(g, win, tok, lab);
  if (head < g.heads)
    for (int e = lane; e < ntab; e += 64) tab[w][e] = table[e * g.heads + head];
  __syncthreads();
  if (threadIdx.x < NP) {  // key j's table offset and region label, shared by the heads
    const int j = threadIdx.x, y = j / ws, x = j - y * ws;
    kjs[j] = ((y * (2 * ws - 1) + x) << 4) | lab[j];
  }
  __syncthreads();
  if (head >= g.heads) return;
  const int bidx = win / (g.nwh * g.nww);
  const int64_t img = (int64_t)bidx * g.h * g.w;
  const float* qkrow = sgpr(qk + img * 2 * g.c);
  float ka[4][8];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
    row8(qkrow, 2, g.c + head * D + 8 * g4, tok[16 * jt + l16], qkb, ka[jt]);
  const float* vrow = sgpr(v + img * g.c);
  float vb[4][4][2];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = tok[16 * jt + 4 * g4 + r];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
        vb[jt][r][dt] = elem(vrow, 1, head * D + 16 * dt + l16, t, g.vb);
    }
  float* orow = sgpr(out + img * g.c);
  float qn[8];
  q_row<WS>(g, qkrow, qkb, head, tok, 0, lane, qn);
  static_for4([&](auto it_c) {
    constexpr int it = decltype(it_c)::value;
    const int lane = opaque_lane(), l16 = lane & 15, g4 = lane >> 4;  // per-tile index math
    float qr[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) qr[k] = qn[k];
    if constexpr (it < 3) q_row<WS>(g, qkrow, qkb, head, tok, it + 1, lane, qn);
    int kj[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) kj[k] = kjs[16 * (k >> 2) + 4 * g4 + (k & 3)];
    f4 s[4];
    probs_tile<WS, it>(g, qr, lab, tab[w], ka, kj, lane, s);
    f4 o[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    // keys 16jt + 4g + r; in the compact last tile only r = 0 (key 48) is real
    static_for4([&](auto jt_c) {
      constexpr int jt = decltype(jt_c)::value;
#pragma unroll
      for (int r = 0; r < Tile<WS>::template ksteps<jt>(); ++r)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) o[dt] = mfma4(s[jt][r], vb[jt][r][dt], o[dt]);
    });
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int t = tok[16 * it + 4 * g4 + rr];
      if (t >= 0) {
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          *at(orow, (unsigned)(t + head * D + 16 * dt + l16)) = o[dt][rr];
      }
    }
  });
}

// slab[(blockIdx.x * heads + head) * (ntab + 2D)] = {dT[0..ntab), dkbias[0..D), dvbias[0..D)}
template <int WS>
__global__ void __launch_bounds__(256, WS == 7 ? kOccBwd7 : 2)
    wattn_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ qk,
                     const float* __restrict__ qkb, const float* __restrict__ v,
                     const float* __restrict__ table, float* __restrict__ gqk,
                     float* __restrict__ gv, float* __restrict__ slab, int nwin, int wpb,
                     Geo g) {
  using TL = Tile<WS>;
  __shared__ int tok[NP], lab[NP];
  __shared__ float tab[kHeads][TABP], dtab[kHeads][TABP];
  __shared__ float Tall[kHeads][TL::kWords];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, g4 = lane >> 4;
  const int head = blockIdx.y * kHeads + w;
  const bool active = head < g.heads;
  const int ws = wsize<WS>(g), span = 2 * ws - 1, ntab = span * span;
  const int c = g.c, c2 = 2 * g.c, hd = head * D;
  float* T = Tall[w];
  if (active)
    for (int e = lane; e < ntab; e += 64) {
      tab[w][e] = table[e * g.heads + head];
      dtab[w][e] = 0.f;
    }
  if constexpr (TL::kCompact) {  // the zero row / column padded indices read
    if (lane < TL::kRows) {
      T[TL::kValid * TL::kPitch + lane] = 0.f;
      T[lane * TL::kPitch + TL::kValid] = 0.f;
    }
  }
  float dkb[2] = {0.f, 0.f};  // d(k bias)[16ct + l16] partial of this lane
  float dvb[2] = {0.f, 0.f};  // d(v bias): dV of the padded keys (g.vb only)
  for (int wi = 0; wi < wpb; ++wi) {
    const int win = blockIdx.x * wpb + wi;
    if (win >= nwin) break;  // uniform across the block
    __syncthreads();         // previous window's tok / T readers are done
    window_tokens<WS>(g, win, tok, lab);
    __syncthreads();
    const int64_t img = (int64_t)(win / (g.nwh * g.nww)) * g.h * g.w;
    const float* qkrow = sgpr(qk + img * c2);
    const float* vrow = sgpr(v + img * c);
    const float* grow = sgpr(gout + img * c);
    float* gqkrow = sgpr(gqk + img * c2);
    float* gvrow = sgpr(gv + img * c);
    // T[w] is private to this wave: its LDS accesses are processed in program
    // order, so the P / dS round trips need no block barrier.  P and then dS
    // live in T only (not in registers across phases): the register peak is
    // one phase's operands, so the kernel runs two waves per SIMD unspilled.
    if (active) {
      // Each phase's global operands are loaded one phase ahead (after the
      // loads the current phase waits on, so its waits do not cover them).
      // B operands of a product over 16-tiles (t, r): element col of token
      // tok[16 t + 4 g + r] (padded: the bias when given), scaled.
      auto tile_elems = [&](float (&b)[4][4][2], const float* base, int m, int col0,
                            const float* bias, float scale) {
        const int lane = opaque_lane(), l16 = lane & 15, g4 = lane >> 4;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int tk = tok[16 * t + 4 * g4 + r];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
              b[t][r][ct] = scale * elem(base, m, col0 + 16 * ct + l16, tk, bias);
          }
      };
      float bdv[4][4][2];  // dV's B = dO[i][c]
      probs_stage<WS>(g, qkrow, qkb, head, tok, lab, tab[w], T,
                      [&] { tile_elems(bdv, grow, 1, hd, nullptr, 1.f); });  // P
      __builtin_amdgcn_sched_barrier(0);  // keep the phases' live ranges apart
      float va[4][8];  // dP's V rows, in flight during dV
      {
        const int lane = opaque_lane(), l16 = lane & 15, g4 = lane >> 4;
#pragma unroll
        for (int jt = 0; jt < 4; ++jt)
          row8(vrow, 1, hd + 8 * g4, tok[16 * jt + l16], g.vb, va[jt]);
      }
      // dV = P^T dO
      {
        const int lane = opaque_lane(), l16 = lane & 15, g4 = lane >> 4;
        static_for4([&](auto jt_c) {
          constexpr int jt = decltype(jt_c)::value;
          f4 o[2];
          mm_tb_tile<WS, jt>(T, bdv, o, lane);
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int t = tok[16 * jt + 4 * g4 + rr];
            if (t >= 0) {
#pragma unroll
              for (int ct = 0; ct < 2; ++ct)
                *at(gvrow, (unsigned)(t + hd + 16 * ct + l16)) = o[ct][rr];
            } else if (t == -1 && g.vb) {
#pragma unroll
              for (int ct = 0; ct < 2; ++ct) dvb[ct] += o[ct][rr];
            }
          }
        });
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the phases' live ranges apart
      // dP^T = V dO^T column by column; dS = P (dP - rowsum(P dP)), P read
      // back from T (this lane's own entries) and dS written over it
      float bq[4][4][2];  // dQ's B = K[j][c], loaded during dS's last tile
      {
        const int lane = opaque_lane(), l16 = lane & 15, g4 = lane >> 4;
        float dn[8];  // dO row of the next query tile
        row8(grow, 1, hd + 8 * g4, tok[l16], nullptr, dn);
        static_for4([&](auto it_c) {
          constexpr int it = decltype(it_c)::value;
          float db[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) db[k] = dn[k];
          if constexpr (it < 3) row8(grow, 1, hd + 8 * g4, tok[16 * (it + 1) + l16], nullptr, dn);
          else tile_elems(bq, qkrow, 2, c + hd, qkb, 1.f);
          f4 dp[4];
          kq_tile<WS, it>(va, db, dp, lane);
          float pv[4][4];
          float dl = 0.f;
          static_for4([&](auto jt_c) {
            constexpr int jt = decltype(jt_c)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              pv[jt][r] = own_get<WS, jt, it>(T, r, lane);
              dl += pv[jt][r] * dp[jt][r];
            }
          });
          dl += __shfl_xor(dl, 16, 64);
          dl += __shfl_xor(dl, 32, 64);
          static_for4([&](auto jt_c) {
            constexpr int jt = decltype(jt_c)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) own_put<WS, jt, it>(T, r, pv[jt][r] * (dp[jt][r] - dl), lane);
          });
        });
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the phases' live ranges apart
      // dQ = dS K * scale: A = dS[i][j] (this lane's own T entries), B = K[j][c] per lane
      float bk[4][4][2];  // dK's B = Q[i][c] * scale, in flight during dQ
      tile_elems(bk, qkrow, 2, hd, qkb, g.scale);
      {
        const int lane = opaque_lane(), l16 = lane & 15, g4 = lane >> 4;
        const float (&b)[4][4][2] = bq;
        static_for4([&](auto it_c) {
          constexpr int it = decltype(it_c)::value;
          f4 q[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
          static_for4([&](auto jt_c) {
            constexpr int jt = decltype(jt_c)::value;
#pragma unroll
            for (int r = 0; r < TL::template ksteps<jt>(); ++r) {
              const float a = own_get<WS, jt, it>(T, r, lane);  // dS[i][j]
#pragma unroll
              for (int ct = 0; ct < 2; ++ct) q[ct] = mfma4(a, b[jt][r][ct], q[ct]);
            }
          });
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int t = tok[16 * it + 4 * g4 + rr];
            if (t >= 0) {
#pragma unroll
              for (int ct = 0; ct < 2; ++ct)
                *at(gqkrow, (unsigned)(2 * t + hd + 16 * ct + l16)) = q[ct][rr] * g.scale;
            }
          }
        });
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the phases' live ranges apart
      // dK = dS^T Q * scale (dS from the LDS tile)
      {
        const int lane = opaque_lane(), l16 = lane & 15, g4 = lane >> 4;
        static_for4([&](auto jt_c) {
          constexpr int jt = decltype(jt_c)::value;
          f4 o[2];
          mm_tb_tile<WS, jt>(T, bk, o, lane);
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int t = tok[16 * jt + 4 * g4 + rr];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
              if (t >= 0)
                *at(gqkrow, (unsigned)(2 * t + c + hd + 16 * ct + l16)) = o[ct][rr];
              else if (t == -1)
                dkb[ct] += o[ct][rr];
            }
          }
        });
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the phases' live ranges apart
      // table gradient: entry (dy, dx) <- sum of dS over the (query, key)
      // pairs at that offset, in a fixed order (query row-major).
      if constexpr (WS > 0) {
        // Two stages over this wave's tile.  (1) lane p = ri WS + rj (one
        // query-row / key-row block pair; 49 of 64 lanes) sums each diagonal
        // dx of its WS x WS block: D[p][dx] = sum_ci dS[rj WS + ci - dx][ri WS + ci]
        // with compile-time column ranges (each of the 2401 pairs read once,
        // no masks).  (2) entry (dy, dx) sums D[ri WS + ri - dy][dx] over ri.
        // D overwrites the tile's first words once every lane's block reads
        // are issued: one wave's LDS accesses are processed in program order.
        constexpr int P = TL::kPitch, NT = 2 * WS - 1, DB = 2 * WS + 4;
        static_assert(DB + (WS * WS + WS) * NT < TL::kWords, "D fits in the tile");
        const int ri = lane / WS, rj = lane - ri * WS;
        float dsum[NT];
        if (lane < WS * WS) {
          const int base = rj * WS * P + ri * WS;
          static_for<NT>([&](auto d_c) {
            constexpr int dx = decltype(d_c)::value - (WS - 1);
            float acc = 0.f;
            static_for<WS - (dx < 0 ? -dx : dx)>([&](auto k_c) {
              constexpr int ci = decltype(k_c)::value + (dx > 0 ? dx : 0);
              acc += T[base + (ci - dx) * P + ci];
            });
            dsum[decltype(d_c)::value] = acc;
          });
        }
        __builtin_amdgcn_wave_barrier();
        if (lane < WS * WS) {
#pragma unroll
          for (int d = 0; d < NT; ++d) T[DB + lane * NT + d] = dsum[d];
        }
        __builtin_amdgcn_wave_barrier();
        for (int e = lane; e < ntab; e += 64) {
          const int dy = e / NT - (WS - 1), dx = e - (e / NT) * NT - (WS - 1);
          // D[ri WS + ri - dy][dx] = T[DB + ri (WS + 1) NT + (dx + WS - 1) - dy NT]
          const int b0 = DB + (dx + WS - 1) - dy * NT;
          float acc = 0.f;
#pragma unroll
          for (int r = 0; r < WS; ++r) {
            const bool ok = r - dy >= 0 && r - dy < WS;
            const float v = T[b0 + r * (WS + 1) * NT];
            acc += ok ? v : 0.f;
          }
          dtab[w][e] += acc;
        }
      }
      for (int e = lane; WS == 0 && e < ntab; e += 64) {
        const int dy = e / span - (ws - 1), dx = e % span - (ws - 1);
        float acc = 0.f;
        if constexpr (WS == 0) {
          for (int ri = 0; ri < ws; ++ri)
            for (int ci = 0; ci < ws; ++ci) {
              const int rj = ri - dy, cj = ci - dx;
              const bool ok = rj >= 0 && rj < ws && cj >= 0 && cj < ws;
              const float v = T[(ok ? rj * ws + cj : 0) * TL::kPitch + ri * ws + ci];
              acc += ok ? v : 0.f;
            }
        }
        dtab[w][e] += acc;
      }
    }
  }
  if (!active) return;
  float* sl = slab + ((int64_t)blockIdx.x * g.heads + head) * (ntab + 2 * D);
  for (int e = lane; e < ntab; e += 64) sl[e] = dtab[w][e];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    float t = dkb[ct], u = dvb[ct];
    t += __shfl_xor(t, 16, 64);
    t += __shfl_xor(t, 32, 64);
    u += __shfl_xor(u, 16, 64);
    u += __shfl_xor(u, 32, 64);
    if (g4 == 0) {
      sl[ntab + 16 * ct + l16] = t;
      sl[ntab + D + 16 * ct + l16] = u;
    }
  }
}

// gtable[e, head] / gqkb[C + head*D + d] / gvb[head*D + d] = sum over blocks:
// 64 entries per block of 16 waves, wave w sums blocks w, w+16, ... (8 loads
// in flight), the 16 wave sums combine in a fixed order.  Blocks (0, head)
// also zero the q half of d(qk bias), gqkb[head*D + d]: padded tokens' dO is
// 0, so it gets nothing (was a separate launch).
__global__ void __launch_bounds__(1024)
    wattn_slab_reduce_kernel(const float* __restrict__ slab, int nblocks, int heads,
                             int ntab, int c, float* __restrict__ gtable,
                             float* __restrict__ gqkb, float* __restrict__ gvb) {
  __shared__ float red[16][64];
  const int head = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (blockIdx.x == 0 && wid == 1 && lane < D) gqkb[head * D + lane] = 0.f;
  const int e = blockIdx.x * 64 + lane;
  const int per = ntab + 2 * D;
  float acc = 0.f;
  if (e < per) {
#pragma unroll 8
    for (int k = wid; k < nblocks; k += 16) acc += slab[((int64_t)k * heads + head) * per + e];
  }
  red[wid][lane] = acc;
  __syncthreads();
  if (wid != 0 || e >= per) return;
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < 16; ++w) t += red[w][lane];
  if (e < ntab)
    gtable[e * heads + head] = t;
  else if (e < ntab + D)
    gqkb[c + head * D + (e - ntab)] = t;
  else if (gvb)
    gvb[head * D + (e - ntab - D)] = t;
}

bool make_geo(int64_t b, int64_t h, int64_t w, int64_t c, int64_t heads, int64_t ws,
              int64_t shift, Geo* g) {
  if (b <= 0 || h <= 0 || w <= 0 || heads <= 0 || c != heads * D || ws <= 0 ||
      ws * ws > NP || shift < 0 || shift >= ws || (2 * ws - 1) * (2 * ws - 1) > TABP)
    return false;
  g->b = (int)b; g->h = (int)h; g->w = (int)w; g->c = (int)c;
  g->heads = (int)heads; g->ws = (int)ws; g->shift = (int)shift;
  g->hp = (int)(mde::cdiv(h, ws) * ws);
  g->wp = (int)(mde::cdiv(w, ws) * ws);
  g->nwh = g->hp / g->ws;
  g->nww = g->wp / g->ws;
  g->n = g->ws * g->ws;
  g->scale = 1.f / sqrtf((float)D);
  g->vb = nullptr;
  return (int64_t)b * g->nwh * g->nww < (1LL << 31) && mde::cdiv(heads, kHeads) <= 65535 &&
         (int64_t)h * w * 2 * c < (1LL << 30);  // 32-bit byte offsets within an image
}

}  // namespace

template <typename Kernel>
int resident_blocks(Kernel k) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 256, 0);
  return (cus > 0 ? cus : 256) * (per > 0 ? per : 1);
}

// Windows per backward block (measured, bs16 NewCRF stages; MDE_ATTN_BWD_WPB
// overrides): one, so the dispatcher balances many small blocks, unless the
// per-block slab (ntab + 2D floats per head) would get large: at 8+ rounds of
// resident blocks, the fewest windows that fit one round (C128 120x160:
// 6624 windows as 736 blocks of 9, 448 us; 1 per block 468 us, 4 per block
// 483 us).  C256 60x80 at 1: 237 us (4: 288, 5: 241); C512 30x40 at 1:
// 136 us (3: 143, 4: 154); C1024 15x20 at 1: 89 us (2: 99).
inline int windows_per_block(int64_t nwin, int64_t heads, int64_t res) {
  static const int forced = [] { const char* e = getenv("MDE_ATTN_BWD_WPB"); return e ? atoi(e) : 0; }();
  if (forced > 0) return forced;
  const int64_t blocks = nwin * ((heads + kHeads - 1) / kHeads);
  const int64_t k = blocks < 8 * res ? 1 : (blocks + res - 1) / res;
  return (int)(k > (1 << 20) ? (1 << 20) : k);
}
inline int bwd_wpb(int64_t nwin, int64_t heads, int64_t window) {
  static const int res7 = resident_blocks(wattn_bwd_kernel<7>);
  static const int res0 = resident_blocks(wattn_bwd_kernel<0>);
  return windows_per_block(nwin, heads, window == 7 ? res7 : res0);
}

extern "C" {

size_t mde_window_attn_workspace(int64_t b, int64_t h, int64_t w, int64_t c,
                                 int64_t heads, int64_t window) {
  Geo g;
  if (!make_geo(b, h, w, c, heads, window, 0, &g)) return 0;
  const int64_t nwin = (int64_t)b * g.nwh * g.nww;
  const int64_t ntab = (2 * window - 1) * (2 * window - 1);
  return sizeof(float) * (size_t)(mde::cdiv(nwin, bwd_wpb(nwin, heads, window)) * heads * (ntab + 2 * D));
}

int mde_window_attn_fwd(const void* qk, const float* qk_bias, const void* v,
                        const float* v_bias, const float* table, void* out, int64_t b,
                        int64_t h, int64_t w, int64_t c, int64_t heads, int64_t window,
                        int64_t shift, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  Geo g;
  if (!qk || !qk_bias || !v || !table || !out || !make_geo(b, h, w, c, heads, window, shift, &g))
    return MDE_ERR_INVALID_ARG;
  g.vb = v_bias;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nwin = (int64_t)b * g.nwh * g.nww;
  const double bytes = 4.0 * (double)b * h * w * c * 4.0;  // q, k, v read + o written
  const dim3 grid((unsigned)nwin, (unsigned)mde::cdiv(heads, kHeads));
  if (window == 7)
    MDE_LAUNCH(mde::K_WATTN_FWD, bytes, s, wattn_fwd_kernel<7>, grid, dim3(256), 0,
               (const float*)qk, qk_bias, (const float*)v, table, (float*)out, g);
  else
    MDE_LAUNCH(mde::K_WATTN_FWD, bytes, s, wattn_fwd_kernel<0>, grid, dim3(256), 0,
               (const float*)qk, qk_bias, (const float*)v, table, (float*)out, g);
  return MDE_OK;
}

int mde_window_attn_bwd(const void* gout, const void* qk, const float* qk_bias,
                        const void* v, const float* v_bias, const float* table, void* gqk,
                        void* gv, float* gtable, float* gqk_bias, float* gv_bias, int64_t b,
                        int64_t h, int64_t w, int64_t c, int64_t heads, int64_t window,
                        int64_t shift, void* workspace, int dtype, void* stream) {
  if (dtype != MDE_F32) return MDE_ERR_UNSUPPORTED;
  Geo g;
  if (!gout || !qk || !qk_bias || !v || !table || !gqk || !gv || !gtable ||
      !gqk_bias || !workspace || (gv_bias && !v_bias) ||
      !make_geo(b, h, w, c, heads, window, shift, &g))
    return MDE_ERR_INVALID_ARG;
  g.vb = v_bias;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nwin = (int64_t)b * g.nwh * g.nww;
  const int wpb = bwd_wpb(nwin, heads, window);
  const int nblk = (int)mde::cdiv(nwin, wpb);
  const int ntab = (2 * g.ws - 1) * (2 * g.ws - 1);
  const double bytes = 4.0 * (double)b * h * w * c * 7.0;  // q k v dO read, dq dk dv written
  const dim3 grid((unsigned)nblk, (unsigned)mde::cdiv(heads, kHeads));
  if (window == 7)
    MDE_LAUNCH(mde::K_WATTN_BWD, bytes, s, wattn_bwd_kernel<7>, grid, dim3(256), 0,
               (const float*)gout, (const float*)qk, qk_bias, (const float*)v, table,
               (float*)gqk, (float*)gv, (float*)workspace, (int)nwin, wpb, g);
  else
    MDE_LAUNCH(mde::K_WATTN_BWD, bytes, s, wattn_bwd_kernel<0>, grid, dim3(256), 0,
               (const float*)gout, (const float*)qk, qk_bias, (const float*)v, table,
               (float*)gqk, (float*)gv, (float*)workspace, (int)nwin, wpb, g);
  MDE_LAUNCH(mde::K_WATTN_BWD_REDUCE, 4.0 * nblk * heads * (ntab + 2 * D), s,
             wattn_slab_reduce_kernel,
             dim3((unsigned)mde::cdiv(ntab + 2 * D, 64), (unsigned)heads), dim3(1024), 0,
             (const float*)workspace, nblk, (int)heads, ntab, (int)c, gtable, gqk_bias, gv_bias);
  return MDE_OK;
}

}  // extern "C"
