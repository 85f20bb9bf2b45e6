// bf16 implicit-GEMM convolutions, NCHW, on v_mfma_f32_32x32x16_bf16: the
// DDRNet-23-slim convolutions of GuideDepth's encoder under bf16 autocast
// (BASELINE cfg3; src/GuideDepth/model/DDRNet_23_slim.py:41-113 BasicBlock /
// Bottleneck, :121-171 DAPPM, :230-263 stem / down / compression convs),
// which MIOpen runs as NHWC implicit GEMM behind NCHW <-> NHWC transposes and
// cast / zero-fill kernels.  Autocast's conv semantics: bf16 operands (the fp32
// weight rounded to bf16, round-to-nearest-even, as autocast's cast), fp32
// accumulation, bf16 output; the weight gradient is accumulated and returned
// in fp32 (the master weight's dtype).
//
// One forward kernel serves every pass that is a convolution of a bf16 NCHW
// source with a packed bf16 filter:
//   * 3x3 / 1x1 forward, stride 1 or 2 (MODE S1 / S2);
//   * their data gradients: stride 1 = the forward on the flipped, transposed
//     filter; stride 2 (MODE U2) = a stride-1 convolution of the flipped,
//     transposed filter over gy with zeros inserted between its rows and
//     columns (staged that way into LDS; the zero taps are multiplied, 4x the
//     MACs of the true transposed convolution -- the stride-2 convs are the
//     encoder's smallest);
// GEMM: M = output pixels (a patch of up to 128 / 256 of them: consecutive
// pixels of one image plane, or a 2D tile), N = output channels (32 / 64 a
// block), K = (tap, input channel) in chunks of 32 channels.  Per chunk the
// block stages the input patch with its halo in LDS as [pixel][32 channels]
// (80-byte pixel pitch: the 16-byte A-operand reads of 16 consecutive pixels
// hit 16 disjoint bank quads) -- transposed from NCHW on the way in (a lane
// loads 8 channels x 2 pixels as dwords and writes two 16-byte pixels), so a
// tap or a stride is a pixel offset, never a misaligned read -- and the
// chunk's filter as [tap][channel out][32 channels in] (64-byte rows, 16-byte
// pieces XOR-swizzled by the row).  Stride 2 stages each row split by column
// parity (even columns, then odd), so the three column taps of 32 consecutive
// output pixels read 32 consecutive staged pixels.  Wave = 64 pixels x 32
// channels (two 32x32 tiles sharing the B operand).  The epilogue writes bf16
// and optionally the following BatchNorm's per-block statistics (the format of
// the other conv kernels' epilogues, common.h Sh).
//
// Weight gradient: M = output channels (64 a block), N = (tap, 32 input
// channels), K = pixels.  gy is staged as [channel][pixel] rows (A operand:
// 16-byte row reads); x as the forward's [pixel][32 channels] image at a
// 64-byte pitch, read TRANSPOSED by ds_read_b64_tr_b16 (B operand: 8 pixels of
// one channel per lane, each 4-pixel row group addressed through a per-patch
// pixel -> staged-pixel table, so taps and strides are again offsets).  Waves
// = 2 channel tiles x 3 filter rows (3x3) or x 2 K halves (1x1).  Blocks split
// the pixel patches (split-K); their fp32 partials are summed in a fixed order
// (bitwise reproducible, no atomics).
#include <cstdlib>
#include <cstring>
#include <utility>

#include "common.h"

namespace {

using mde::bf16;
using bf8v = __bf16 __attribute__((ext_vector_type(8)));
using f16v = float __attribute__((ext_vector_type(16)));
using u4v = uint32_t __attribute__((ext_vector_type(4)));
using u2v = uint32_t __attribute__((ext_vector_type(2)));
using f4v = float __attribute__((ext_vector_type(4)));
using s4v = short __attribute__((ext_vector_type(4)));
using lds_s4 = __attribute__((address_space(3))) s4v;

__device__ __forceinline__ f16v mfma32(u4v a, u4v b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8v, a),
                                                 __builtin_bit_cast(bf8v, b), c, 0, 0, 0);
}

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

enum Mode : int { S1 = 0, S2 = 1, U2 = 2 };

constexpr int kPitchF = 40;  // forward image: bf16 elements per staged pixel (32 + 8 pad)
constexpr int kPitchW = 32;  // weight-gradient image (transposed reads): no pad
// weight-gradient patch pixels: 256 at stride-1 3x3 (twice the MFMAs per
// patch's fixed staging / barrier cost: 64 -> 64 @60x80 49 -> 40 us), 128
// otherwise (stride 2 at 256 spilled and took 2D tiles: 1.1-1.4x slower);
// gy rows are MBW + 8 bf16 a channel
template <int KS, int MODE>
constexpr int wgrad_mbw() { return KS == 3 && MODE == S1 ? 256 : 128; }

// Patch geometry of a pass (host-chosen, see pick_geo).
struct Geo {
  int cin, cout;   // channels of THIS pass (dgrad: cin = the forward's cout)
  int hi, wi;      // staged source plane (x; gy for U2)
  int ho, wo;      // output plane
  int pc, pr;      // 2D tiles of pr rows x pc columns; pc == 0: flat patches of mb pixels
  int mb;          // flat patch pixels
  int tiles_w;     // 2D: column tiles per band of pr rows
  int ppi;         // patches per image
  int cap;         // staged-pixel capacity (LDS image)
  int nrmax;       // output rows a patch can span: the staged row count is fixed by it
  float inv_wo, inv_pc, inv_ppi, inv_tw;  // reciprocals for fdiv
};

// a / d for 0 <= a < 2^22 from a float reciprocal, corrected to the exact quotient
__device__ __forceinline__ int fdiv(int a, int d, float inv) {
  int q = (int)((float)a * inv);
  q -= q * d > a ? 1 : 0;
  q += (q + 1) * d <= a ? 1 : 0;
  return q;
}

struct Patch {
  int img, r0, r1, c0, nc, p0, npx;
};

__device__ __forceinline__ Patch patch_of(const Geo& g, int q) {
  Patch P;
  P.img = fdiv(q, g.ppi, g.inv_ppi);
  const int k = q - P.img * g.ppi;
  if (g.pc == 0) {
    const int hw = g.ho * g.wo;
    P.p0 = k * g.mb;
    P.npx = hw - P.p0 < g.mb ? hw - P.p0 : g.mb;
    P.r0 = fdiv(P.p0, g.wo, g.inv_wo);
    P.r1 = fdiv(P.p0 + P.npx - 1, g.wo, g.inv_wo);
    P.c0 = 0;
    P.nc = g.wo;
  } else {
    const int band = fdiv(k, g.tiles_w, g.inv_tw), t = k - band * g.tiles_w;
    P.r0 = band * g.pr;
    P.r1 = (P.r0 + g.pr < g.ho ? P.r0 + g.pr : g.ho) - 1;
    P.c0 = t * g.pc;
    P.nc = g.pc;
    P.p0 = 0;
    P.npx = g.pr * g.pc;
  }
  return P;
}

// patch pixel m -> output (r, c); false if outside the plane / patch
__device__ __forceinline__ bool pix_of(const Geo& g, const Patch& P, int m, int& r, int& c) {
  if (g.pc == 0) {
    const int p = P.p0 + (m < P.npx ? m : 0);
    r = fdiv(p, g.wo, g.inv_wo);
    c = p - r * g.wo;
    return m < P.npx;
  }
  const int mr = fdiv(m, g.pc, g.inv_pc);
  r = P.r0 + mr;
  c = P.c0 + (m - mr * g.pc);
  return m < P.npx && r < g.ho && c < g.wo;
}

struct Img {
  int gr0, rs, gc0, cs, csh;
};

// The staged image of a patch: rows gr0 .. gr0 + rs - 1 and cols gc0 .. of the
// source (Z = zero-inserted gy coordinates for U2; (2 i, 2 j) for 1x1 stride 2).
// The row count is the launch's maximum (nrmax output rows), so a thread's
// staging units are the same for every patch (SrcStage::plan once per block).
template <int KS, int MODE>
__device__ __forceinline__ Img img_of(const Geo& g, const Patch& P) {
  Img I;
  const int nr = g.nrmax;
  if constexpr (KS == 3 && MODE == S2) {
    I.gr0 = 2 * P.r0 - 1;
    I.rs = 2 * nr + 1;
    I.gc0 = 2 * P.c0 - 2;
    I.csh = P.nc + 1;
    I.cs = 2 * I.csh;
  } else if constexpr (KS == 3) {  // S1, U2
    I.gr0 = P.r0 - 1;
    I.rs = nr + 2;
    I.gc0 = P.c0 - 2;
    I.cs = P.nc + 4;
    I.csh = 0;
  } else {
    I.gr0 = P.r0;
    I.rs = nr;
    I.gc0 = P.c0;
    I.cs = P.nc;
    I.csh = 0;
  }
  return I;
}

// staged-pixel index of output pixel (r, c) at tap (0, 0)
template <int KS, int MODE>
__device__ __forceinline__ int img_base(const Patch& P, const Img& I, int r, int c) {
  if constexpr (KS == 3 && MODE == S2) return 2 * (r - P.r0) * I.cs + (c - P.c0);
  if constexpr (KS == 3) return (r - P.r0) * I.cs + (c - P.c0) + 1;
  return (r - P.r0) * I.cs + (c - P.c0);
}

// offset of tap (dy, dx) from the tap-(0, 0) staged pixel
template <int KS, int MODE>
__device__ __forceinline__ int tap_off(const Img& I, int dy, int dx) {
  if constexpr (KS == 1) return 0;
  if constexpr (MODE == S2) return dy * I.cs + (dx == 0 ? I.csh : (dx == 1 ? 1 : I.csh + 1));
  return dy * I.cs + dx;
}

// two fp32 -> packed bf16 (round-to-nearest-even): one v_cvt_pk_bf16_f32
using bf2v = __bf16 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  const bf2v v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ uint32_t lo16x2(uint32_t a, uint32_t b) {  // (a.lo, b.lo)
  return __builtin_amdgcn_perm(b, a, 0x05040100u);
}
__device__ __forceinline__ uint32_t hi16x2(uint32_t a, uint32_t b) {  // (a.hi, b.hi)
  return __builtin_amdgcn_perm(b, a, 0x07060302u);
}

// Staging of 32 channels (ci0 ..) of a patch's source image into LDS as
// [pixel][channel] at pixel pitch PITCH (bf16).  Unit = (channel octet,
// staged row, staged column pair): 8 loads (8 channels x 2 source pixels as
// dwords; U2: 8 channels x 1 gy element), packed into two 16-byte pixels.
// load() issues EVERY unit's loads of the thread (clamped addresses, selects:
// no branches around loads, nothing waited on), store() packs and writes them:
// the kernels call load() for the next chunk / patch before the current one's
// MFMAs, so the load latency hides behind the matrix work.  MAXU >= the units
// a thread can own (host: pick_geo caps the staged pixels at the LDS image).
// Units are numbered octet-fastest (four lanes stage one pixel's 64 bytes)
// and, in each 8-lane group of a 16-byte LDS store (banks = dword address mod
// 32 for stores), the two quads write pixels whose offsets differ by 16 banks:
// at the forward image's 80-byte pitch by taking column units 2 or 4 apart
// (a permutation inside aligned groups), at the weight-gradient image's
// 64-byte pitch by swapping the two stores of every odd quad.  Loads are
// buffer loads: a per-unit 32-bit offset (VGPR) and a per-channel offset
// (SGPR); out-of-range units get an offset past the buffer (loads return 0),
// so no address arithmetic or select per load.
template <int KS, int MODE, int PITCH, int NT, int MAXU>
struct SrcStage {
  static constexpr bool ONE = KS == 1 && MODE == S2;     // one staged pixel a unit
  static constexpr bool EO = KS == 3 && MODE == S2;      // even / odd column halves
  static constexpr bool PAIR_PX = !ONE && !EO;           // unit jc -> pixels 2 jc, 2 jc + 1
  static constexpr int G = PITCH == kPitchF ? (PAIR_PX ? 4 : 8) : 1;  // permutation group
  static constexpr bool SWAP = PITCH != kPitchF && PAIR_PX;
  uint32_t v[MAXU][8];
  int code[MAXU];  // (swap << 30) | (octet << 28) | (staged row << 16) | column unit, -1: none
  int dA[MAXU];    // element offset of the unit's first store (< 0: none)

  __device__ static __forceinline__ int ncol(const Img& I) {
    return ONE ? I.cs : (EO ? I.csh : I.cs >> 1);
  }

  __device__ __forceinline__ void plan(const Img& I, int tid) {
    const int nc = ncol(I), total = 4 * I.rs * nc;
    // static_for, not a counted loop: a loop the compiler keeps rolled (the
    // division makes the body large) indexes code / dA dynamically and puts
    // them in scratch, reloaded at every store
    static_for<MAXU>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      const int u = tid + NT * k;
      if (u < total) {
        const int o = u & 3, rest = u >> 2;
        const int i = rest / nc;
        int jc = rest - i * nc;
        if constexpr (G > 1) {
          const int base = jc & ~(G - 1), jl = jc & (G - 1);
          if (base + G <= nc) jc = base + (jl & 1) * (G / 2) + (jl >> 1);
        }
        const bool sw = SWAP && (rest & 1);
        code[k] = ((int)sw << 30) | (o << 28) | (i << 16) | jc;
        int p0;
        if constexpr (ONE || EO)
          p0 = i * I.cs + jc;
        else
          p0 = i * I.cs + 2 * jc;
        // the second store sits dB() elements after the first (before it when swapped)
        dA[k] = (sw ? p0 + 1 : p0) * PITCH + 8 * o;
      } else {
        code[k] = -1;
        dA[k] = -1;
      }
    });
  }

  // offset of a unit's second store from its first
  __device__ static __forceinline__ int dB(const Img& I, bool sw) {
    const int d = EO ? I.csh * PITCH : PITCH;
    return sw ? -d : d;
  }

  // per patch: the buffer resource of the image and each unit's 32-bit offset
  // (channel 0 of its octet; past the buffer when outside the source plane)
  __amdgpu_buffer_rsrc_t R;
  uint32_t voff[MAXU];
  int plane;

  __device__ __forceinline__ void locate(const bf16* __restrict__ src, const Geo& g, const Img& I) {
    plane = g.hi * g.wi;
    const uint64_t a = (uint64_t)src;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    R = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                          2 * g.cin * plane, 0x00020000);
    static_for<MAXU>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      const int cd = code[k] < 0 ? 0 : code[k];
      const int o = (cd >> 28) & 3, i = (cd >> 16) & 0xfff, jc = cd & 0xffff;
      int sr, sc;
      bool ok;
      if constexpr (MODE == U2) {
        // Z[zr][zc] = gy[zr / 2][zc / 2] for even zr, zc, else 0
        const int zr = I.gr0 + i, zc = I.gc0 + 2 * jc;
        sr = zr >> 1;
        sc = zc >> 1;
        ok = (zr & 1) == 0 && zr >= 0 && sr < g.hi && zc >= 0 && sc < g.wi;
      } else if constexpr (ONE) {
        sr = 2 * (I.gr0 + i);
        sc = 2 * (I.gc0 + jc);
        ok = sr < g.hi && sc < g.wi;
      } else {
        sr = I.gr0 + i;
        sc = I.gc0 + 2 * jc;
        ok = sr >= 0 && sr < g.hi && sc >= 0 && sc < g.wi;
      }
      ok = ok && code[k] >= 0;
      voff[k] = ok ? (uint32_t)(2 * (8 * o * plane + sr * g.wi + sc)) : 0x7ffffff0u;
    });
  }

  // the loads of channels ci0 + 8 o + (0..7) of every unit (located patch)
  __device__ __forceinline__ void issue(int ci0) {
    static_for<MAXU>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int soff = 2 * (ci0 + j) * plane;
        if constexpr (MODE == U2)
          v[k][j] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(R, voff[k], soff, 0);
        else
          v[k][j] = __builtin_amdgcn_raw_buffer_load_b32(R, voff[k], soff, 0);
      }
    });
  }

  __device__ __forceinline__ void load(const bf16* __restrict__ src, const Geo& g, const Img& I,
                                       int ci0) {
    locate(src, g, I);
    issue(ci0);
  }

  __device__ __forceinline__ void store(bf16* img, const Img& I) const {
    static_for<MAXU>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      if (dA[k] >= 0) {
        u4v e, od;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (MODE == U2) {
            e[j] = v[k][2 * j] | (v[k][2 * j + 1] << 16);
            od[j] = 0u;
          } else {
            e[j] = lo16x2(v[k][2 * j], v[k][2 * j + 1]);
            od[j] = hi16x2(v[k][2 * j], v[k][2 * j + 1]);
          }
        }
        if constexpr (ONE) {
          *reinterpret_cast<u4v*>(img + dA[k]) = e;
        } else {
          const bool sw = SWAP && ((code[k] >> 30) & 1);
          *reinterpret_cast<u4v*>(img + dA[k]) = sw ? od : e;
          *reinterpret_cast<u4v*>(img + dA[k] + dB(I, sw)) = sw ? e : od;
        }
      }
    });
  }
};

// units a thread can own for a staged image of CAP pixels
template <int KS, int MODE, int CAP, int NT>
constexpr int src_units() {
  // U2 / S1: CAP / 2 column pairs; 3x3 S2: CAP / 2 source pairs; 1x1 S2: CAP pixels
  return (4 * ((KS == 1 && MODE == S2) ? CAP : CAP / 2) + NT - 1) / NT;
}

// The filter chunk [tap][NB][32] (16-byte pieces swizzled by (row >> 2) & 3,
// already so in the packed filter), register-staged like SrcStage.
template <int KK, int NB, int NT>
struct WStage {
  static constexpr int U = (KK * NB * 4 + NT - 1) / NT;
  u4v v[U];
  __device__ __forceinline__ void load(const bf16* __restrict__ src, int cout, int co0, int tid) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int u = tid + NT * k;
      const int uc = u < KK * NB * 4 ? u : 0;
      const int o = uc & 3, rest = uc >> 2, cl = rest % NB, t = rest / NB;
      v[k] = *reinterpret_cast<const u4v*>(src + ((int64_t)t * cout + co0 + cl) * 32 + 8 * o);
    }
  }
  __device__ __forceinline__ void store(bf16* sw, int tid) const {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int u = tid + NT * k;
      if (u < KK * NB * 4) {
        const int o = u & 3, rest = u >> 2, cl = rest % NB, t = rest / NB;
        *reinterpret_cast<u4v*>(sw + (t * NB + cl) * 32 + 8 * o) = v[k];  // pre-swizzled rows
      }
    }
  }
};

// The MFMAs of one staged chunk: (tap, k-half) steps over the filter rows in
// DYM (a compile-time mask: U2 tiles skip the all-zero rows), each step's B
// (filter) and A (image) fragments read PD steps ahead,
// straight-line code -- no branch around an MFMA (a branch made the compiler
// copy the accumulators between AGPRs and VGPRs at every one).
template <int KS, int DYM, int MTW, int PITCH_A>
__device__ __forceinline__ void chunk_mfmas(const bf16* __restrict__ swc, int nbrow,
                                            const bf16* __restrict__ simg, const int (&abase)[MTW],
                                            const int (&toff)[KS * KS], int boff0, int boff1, int h,
                                            f16v (&acc)[MTW]) {
  constexpr int NR = (DYM & 1) + ((DYM >> 1) & 1) + ((DYM >> 2) & 1);
  constexpr int NS = (KS == 3 ? NR * 3 : 1) * 2;
  // step s -> (tap, ks)
  auto tap_of = [](int s) constexpr {
    const int j = s >> 1;  // j-th (dy, dx) pair among the kept rows
    if constexpr (KS == 1) return 0;
    int row = 0, n = 0;
    for (int dy = 0; dy < 3; ++dy)
      if ((DYM >> dy) & 1) {
        if (j >= n * 3 && j < n * 3 + 3) row = dy * 3 + (j - n * 3);
        ++n;
      }
    return row;
  };
  // reads run PD steps ahead of the MFMAs (PD + 1 register slots): at one
  // wave per SIMD nothing else hides an LDS read's latency, and one step
  // (MTW MFMAs) is shorter than it
  constexpr int PD = 2, NSL = PD + 1;
  u4v bq[NSL], aq[NSL][MTW];
  auto ld = [&](auto s_c) {
    constexpr int s = decltype(s_c)::value, slot = s % NSL;
    constexpr int t = tap_of(s), ks = s & 1;
    bq[slot] = *reinterpret_cast<const u4v*>(swc + t * nbrow + (ks ? boff1 : boff0));
#pragma unroll
    for (int i = 0; i < MTW; ++i)
      aq[slot][i] = *reinterpret_cast<const u4v*>(simg + abase[i] + toff[t] + 16 * ks + 8 * h);
  };
  static_for<PD < NS ? PD : NS>([&](auto s_c) { ld(s_c); });
  static_for<NS>([&](auto s_c) {
    constexpr int s = decltype(s_c)::value;
    if constexpr (s + PD < NS) ld(std::integral_constant<int, s + PD>{});
    // keep the next steps' reads here: the scheduler otherwise sinks each read
    // next to its MFMA and every MFMA waits out an LDS latency
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MTW; ++i) acc[i] = mfma32(aq[s % NSL][i], bq[s % NSL], acc[i]);
    __builtin_amdgcn_sched_barrier(0);
  });
}

// chunk_mfmas for a wave tile of MTW x NTW 32x32 tiles: per (tap, k-half)
// step MTW A + NTW B reads feed MTW NTW MFMAs (2 x 2: one read per MFMA).
template <int KS, int DYM, int MTW, int NTW, int PITCH_A>
__device__ __forceinline__ void tile_mfmas(const bf16* __restrict__ swc, int nbrow,
                                           const bf16* __restrict__ simg, const int (&abase)[MTW],
                                           const int (&toff)[KS * KS], const int (&boff0)[NTW],
                                           const int (&boff1)[NTW], int h,
                                           f16v (&acc)[MTW][NTW]) {
  constexpr int NR = (DYM & 1) + ((DYM >> 1) & 1) + ((DYM >> 2) & 1);
  constexpr int NS = (KS == 3 ? NR * 3 : 1) * 2;
  auto tap_of = [](int s) constexpr {
    const int j = s >> 1;
    if constexpr (KS == 1) return 0;
    int row = 0, n = 0;
    for (int dy = 0; dy < 3; ++dy)
      if ((DYM >> dy) & 1) {
        if (j >= n * 3 && j < n * 3 + 3) row = dy * 3 + (j - n * 3);
        ++n;
      }
    return row;
  };
  constexpr int PD = 2, NSL = PD + 1;
  u4v bq[NSL][NTW], aq[NSL][MTW];
  auto ld = [&](auto s_c) {
    constexpr int s = decltype(s_c)::value, slot = s % NSL;
    constexpr int t = tap_of(s), ks = s & 1;
#pragma unroll
    for (int j = 0; j < NTW; ++j)
      bq[slot][j] = *reinterpret_cast<const u4v*>(swc + t * nbrow + (ks ? boff1[j] : boff0[j]));
#pragma unroll
    for (int i = 0; i < MTW; ++i)
      aq[slot][i] = *reinterpret_cast<const u4v*>(simg + abase[i] + toff[t] + 16 * ks + 8 * h);
  };
  static_for<PD < NS ? PD : NS>([&](auto s_c) { ld(s_c); });
  static_for<NS>([&](auto s_c) {
    constexpr int s = decltype(s_c)::value;
    if constexpr (s + PD < NS) ld(std::integral_constant<int, s + PD>{});
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[i][j] = mfma32(aq[s % NSL][i], bq[s % NSL][j], acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
  });
}

// ------------------------------------------------------------------ forward
// Block: NW waves; wave (wm, wn): output channels 32 wn .. of the block's
// 32 WN, M tiles MTW wm .. MTW wm + MTW - 1 (32 pixels each) of the patch
// (32 MTW NW / WN pixels).  8-wave blocks stage the filter chunk once per 256
// pixels (the 4-wave ones per 128: the filter is most of what a 64-channel
// block loads).
template <int KS, int MODE, int WN, int MTW, int NW, bool STATS, int CAP>
__global__ void __launch_bounds__(64 * NW, 1)
    convbf_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wp,
                      bf16* __restrict__ y, float* __restrict__ stats, Geo g) {
  constexpr int KK = KS * KS, NB = 32 * WN, WMW = NW / WN, NT = 64 * NW;
  __shared__ __attribute__((aligned(16))) bf16 simg[CAP * kPitchF];
  __shared__ __attribute__((aligned(16))) bf16 sw[KK * NB * 32];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv % WMW, wn = wv / WMW;
  const Patch P = patch_of(g, blockIdx.x);
  const Img I = img_of<KS, MODE>(g, P);
  const int co0 = blockIdx.y * NB;
  const int nmt = (P.npx + 31) >> 5;  // M tiles holding pixels

  int abase[MTW];
  bool mt_on[MTW];
  int wdymask = MODE == U2 && KS == 3 ? 0 : 7;  // filter rows some tile of the wave needs
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int mt = MTW * wm + i;
    mt_on[i] = mt < nmt;
    int r, c;
    const bool ok = pix_of(g, P, mt * 32 + l32, r, c);
    abase[i] = ok ? img_base<KS, MODE>(P, I, r, c) * kPitchF : 0;
    if constexpr (MODE == U2 && KS == 3) {
      // a tile inside one output row r reads Z rows r - 1 + dy, zero unless
      // r + dy is odd: dy = 1 for even r, dy = 0, 2 for odd r
      int r0, c0, r1, c1;
      const bool a = pix_of(g, P, mt * 32, r0, c0);
      const bool b = pix_of(g, P, mt * 32 + 31, r1, c1);
      wdymask |= !mt_on[i] ? 0 : ((a && b && r0 == r1) ? ((r0 & 1) ? 5 : 2) : 7);
    }
  }
  wdymask = __builtin_amdgcn_readfirstlane(wdymask);
  int toff[KK];
#pragma unroll
  for (int t = 0; t < KK; ++t) toff[t] = tap_off<KS, MODE>(I, t / KS, t % KS) * kPitchF;
  const int col = wn * 32 + l32;  // B column (output channel within the block)
  // the B read of k-half h takes piece (2 ks + h) ^ ((col >> 2) & 3) of the
  // row: the packed rows are swizzled, so logical piece q sits at q ^ sw
  const int sw_x = (col >> 2) & 3;
  const int boff0 = col * 32 + 8 * ((0 + h) ^ sw_x), boff1 = col * 32 + 8 * ((2 + h) ^ sw_x);

  f16v acc[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

  const bf16* xs = x + (int64_t)P.img * g.cin * g.hi * g.wi;
  const int nchunk = (g.cin + 31) >> 5;
  SrcStage<KS, MODE, kPitchF, NT, src_units<KS, MODE, CAP, NT>()> S;
  WStage<KK, NB, NT> Wt;
  S.plan(I, tid);
  S.load(xs, g, I, 0);
  Wt.load(wp, g.cout, co0, tid);
  for (int cc = 0; cc < nchunk; ++cc) {
    __syncthreads();
    S.store(simg, I);
    Wt.store(sw, tid);
    __syncthreads();
    if (cc + 1 < nchunk) {  // the next chunk's loads, in flight during this chunk's MFMAs
      S.load(xs, g, I, 32 * (cc + 1));
      Wt.load(wp + (int64_t)(cc + 1) * KK * g.cout * 32, g.cout, co0, tid);
    }
    if (MODE == U2 && KS == 3 && wdymask == 2)
      chunk_mfmas<KS, 2, MTW, kPitchF>(sw, NB * 32, simg, abase, toff, boff0, boff1, h, acc);
    else if (MODE == U2 && KS == 3 && wdymask == 5)
      chunk_mfmas<KS, 5, MTW, kPitchF>(sw, NB * 32, simg, abase, toff, boff0, boff1, h, acc);
    else
      chunk_mfmas<KS, 7, MTW, kPitchF>(sw, NB * 32, simg, abase, toff, boff0, boff1, h, acc);
  }

  // epilogue: lane (co = co0 + col, h) holds pixels 32 mt + 8 q + 4 h + (0..3), q = reg >> 2
  const int co = co0 + col;
  const int64_t hwo = (int64_t)g.ho * g.wo;
  bf16* yc = y + ((int64_t)P.img * g.cout + co) * hwo;
  mde::Sh run{0.f, 0.f, 0.f, 0.f};
  bool have_ref = false;
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    if (!mt_on[i]) continue;
    const int mt = MTW * wm + i;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = mt * 32 + 8 * q + 4 * h;
      int r, c;
      const bool ok = pix_of(g, P, m, r, c);
      const uint32_t p01 = pack2bf(acc[i][4 * q], acc[i][4 * q + 1]);
      const uint32_t p23 = pack2bf(acc[i][4 * q + 2], acc[i][4 * q + 3]);
      if constexpr (STATS) {
        const float v0 = __uint_as_float(p01 << 16), v1 = __uint_as_float(p01 & 0xffff0000u);
        const float v2 = __uint_as_float(p23 << 16), v3 = __uint_as_float(p23 & 0xffff0000u);
        if (!have_ref) {  // one shift per channel and wave: lane (co, h = 0)'s first value
          run.ref = __shfl(v0, l32, 64);
          have_ref = true;
        }
        mde::sh_add(run, v0, ok);
        mde::sh_add(run, v1, ok);
        mde::sh_add(run, v2, ok);
        mde::sh_add(run, v3, ok);
      }
      if (ok) *reinterpret_cast<u2v*>(yc + (int64_t)r * g.wo + c) = u2v{p01, p23};
    }
  }
  if constexpr (STATS) {
    run = mde::sh_xor_sum(run, 32);
    __syncthreads();
    float* part = reinterpret_cast<float*>(simg);  // [WMW][NB][4]
    if (h == 0) {
      float* p4 = part + (wm * NB + col) * 4;
      p4[0] = run.ref;
      p4[1] = run.n;
      p4[2] = run.s1;
      p4[3] = run.s2;
    }
    __syncthreads();
    if (tid < NB) {
      mde::Sh a{part[tid * 4], part[tid * 4 + 1], part[tid * 4 + 2], part[tid * 4 + 3]};
#pragma unroll
      for (int k = 1; k < WMW; ++k) {
        const float* p4 = part + (k * NB + tid) * 4;
        a = mde::sh_merge(a, {p4[0], p4[1], p4[2], p4[3]});
      }
      float* o4 = stats + ((int64_t)(co0 + tid) * gridDim.x + blockIdx.x) * 4;
      o4[0] = a.ref;
      o4[1] = a.n;
      o4[2] = a.s1;
      o4[3] = a.s2;
    }
  }
}

// Resident-filter forward: persistent blocks, each owning NB output channels
// and a contiguous range of patches, with the block's WHOLE filter slice
// ([cin / 32][tap][NB][32], <= kWRes) copied into LDS once by LDS-DMA
// (global_load_lds, 1 KiB per wave instruction, the rows pre-swizzled by the
// pack).  The pipeline runs over (patch, channel chunk) steps: the next
// step's input chunk is register-staged during this step's MFMAs, so only
// the input is staged per step (the filter -- most of what the chunked
// kernel stages -- never again).
constexpr int kWRes = 36864;  // resident filter capacity, bf16 elements (73.7 KB)

template <int KS, int MODE, int WN, bool STATS, int CAP, int NTW = 1>
__global__ void __launch_bounds__(256, 1)
    convbf_fwd_res_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wp,
                          bf16* __restrict__ y, float* __restrict__ stats, Geo g, int per,
                          int npatch) {
  // wave (wm, wn): NTW of the block's WN 32-channel tiles x MTW 32-pixel tiles
  constexpr int KK = KS * KS, NB = 32 * WN, WMW = 4 / (WN / NTW), MTW = 2, NT = 256;
  __shared__ __attribute__((aligned(16))) bf16 simg[CAP * kPitchF];
  __shared__ __attribute__((aligned(16))) bf16 sw[kWRes];
  constexpr int MB = 32 * MTW * WMW, kOP = MB + 8;  // patch pixels, output-tile row pitch
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv % WMW, wn = wv / WMW;
  const int co0 = blockIdx.y * NB;
  const int nch = (g.cin + 31) >> 5;
  const int q0 = blockIdx.x * per, q1 = q0 + per < npatch ? q0 + per : npatch;
  if (q0 >= q1) return;  // block-uniform, before any barrier
  {  // the filter slice: nch * KK segments of NB rows (NB * 64 bytes: 2 or 4 KiB)
    constexpr int SEG = NB * 64 / 1024;
    const int pieces = nch * KK * SEG;
    for (int j = wv; j < pieces; j += 4) {
      const int sg = j / SEG, within = j - sg * SEG;
      const bf16* src = wp + ((int64_t)sg * g.cout + co0) * 32 + within * 512 + lane * 8;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sw + j * 512),
                                       16, 0, 0);
    }
  }
  Patch P = patch_of(g, q0);
  Img I = img_of<KS, MODE>(g, P);
  int toff[KK];
#pragma unroll
  for (int t = 0; t < KK; ++t) toff[t] = tap_off<KS, MODE>(I, t / KS, t % KS) * kPitchF;
  // B column of tile j (output channel within the block); logical 16-byte
  // piece q of a packed filter row sits at q ^ ((col >> 2) & 3)
  int col[NTW], boff0[NTW], boff1[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    col[j] = (wn * NTW + j) * 32 + l32;
    const int sw_x = (col[j] >> 2) & 3;
    boff0[j] = col[j] * 32 + 8 * ((0 + h) ^ sw_x);
    boff1[j] = col[j] * 32 + 8 * ((2 + h) ^ sw_x);
  }
  const int64_t hwo = (int64_t)g.ho * g.wo, xplane = (int64_t)g.cin * g.hi * g.wi;

  SrcStage<KS, MODE, kPitchF, NT, src_units<KS, MODE, CAP, NT>()> S;
  S.plan(I, tid);
  S.load(x + (int64_t)P.img * xplane, g, I, 0);
  int abase[MTW];
  bool mt_on[MTW];
  int wdymask = 7;  // U2: filter rows some tile of this wave needs (wave-uniform)
  auto setup = [&](const Patch& Q, const Img& J) {
    const int nmt = (Q.npx + 31) >> 5;
    wdymask = MODE == U2 && KS == 3 ? 0 : 7;
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      const int mt = MTW * wm + i;
      mt_on[i] = mt < nmt;
      int r, c;
      const bool ok = pix_of(g, Q, mt * 32 + l32, r, c);
      abase[i] = ok ? img_base<KS, MODE>(Q, J, r, c) * kPitchF : 0;
      if constexpr (MODE == U2 && KS == 3) {
        // a tile inside one output row r reads Z rows r - 1 + dy, zero unless
        // r + dy is odd: dy = 1 for even r, dy = 0, 2 for odd r
        int r0, c0, r1, c1;
        const bool a = pix_of(g, Q, mt * 32, r0, c0);
        const bool b = pix_of(g, Q, mt * 32 + 31, r1, c1);
        wdymask |= !mt_on[i] ? 0 : ((a && b && r0 == r1) ? ((r0 & 1) ? 5 : 2) : 7);
      }
    }
    wdymask = __builtin_amdgcn_readfirstlane(wdymask);
  };
  setup(P, I);
  f16v acc[MTW][NTW];
  mde::Sh run[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) run[j] = mde::Sh{0.f, 0.f, 0.f, 0.f};
  bool have_ref[NTW] = {};  // one shift per channel and wave: its first value

  const bool flat = g.pc == 0;

  // patch-outer, chunk-inner: the accumulators are zeroed and drained once per
  // patch outside the chunk loop, so its back edge carries them in AGPRs (a
  // single flat (patch, chunk) loop made the compiler copy all of them to
  // VGPRs and back at every step)
  for (int q = q0; q < q1; ++q) {
    Patch Pn = P;
    Img In = I;
    if (q + 1 < q1) {
      Pn = patch_of(g, q + 1);
      In = img_of<KS, MODE>(g, Pn);
    }
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int cc = 0; cc < nch; ++cc) {
      __syncthreads();  // previous step's image readers are done (1st: the filter DMA drained)
      S.store(simg, I);
      __syncthreads();
      // the next step's input chunk, in flight during this step's MFMAs (the
      // unit offsets are located once a patch)
      if (cc + 1 < nch)
        S.issue(32 * (cc + 1));
      else if (q + 1 < q1)
        S.load(x + (int64_t)Pn.img * xplane, g, In, 0);
      const bf16* swc = sw + cc * KK * NB * 32;
      // U2 skips a filter row only when all of the wave's tiles do
      if (MODE == U2 && KS == 3 && wdymask == 2)
        tile_mfmas<KS, 2, MTW, NTW, kPitchF>(swc, NB * 32, simg, abase, toff, boff0, boff1, h, acc);
      else if (MODE == U2 && KS == 3 && wdymask == 5)
        tile_mfmas<KS, 5, MTW, NTW, kPitchF>(swc, NB * 32, simg, abase, toff, boff0, boff1, h, acc);
      else
        tile_mfmas<KS, 7, MTW, NTW, kPitchF>(swc, NB * 32, simg, abase, toff, boff0, boff1, h, acc);
    }
    // the patch is complete: bf16 output (+ statistics).  Flat patches (a
    // contiguous run of the output plane) go through LDS as [channel][pixel]
    // rows and leave as 16-byte stores, 256 contiguous bytes per 16 lanes (a
    // lane's own fragment -- 4 pixels of one channel -- would make every store
    // instruction touch 64 planes: store-issue-bound).  (Deferring those stores
    // into the next patch's first step, past its input loads' vmcnt wait, from
    // a separate LDS tile measured 3 % slower.)
    __syncthreads();  // every wave is done reading the image
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        if (!mt_on[i]) continue;
        const int mt = MTW * wm + i;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int m = mt * 32 + 8 * qq + 4 * h;
          const uint32_t p01 = pack2bf(acc[i][j][4 * qq], acc[i][j][4 * qq + 1]);
          const uint32_t p23 = pack2bf(acc[i][j][4 * qq + 2], acc[i][j][4 * qq + 3]);
          if constexpr (STATS) {
            int r = 0, c = 0;
            const bool ok = flat ? m < P.npx : pix_of(g, P, m, r, c);
            const float v0 = __uint_as_float(p01 << 16), v1 = __uint_as_float(p01 & 0xffff0000u);
            const float v2 = __uint_as_float(p23 << 16), v3 = __uint_as_float(p23 & 0xffff0000u);
            if (!have_ref[j]) {
              run[j].ref = __shfl(v0, l32, 64);
              have_ref[j] = true;
            }
            mde::sh_add(run[j], v0, ok);
            mde::sh_add(run[j], v1, ok);
            mde::sh_add(run[j], v2, ok);
            mde::sh_add(run[j], v3, ok);
          }
          *reinterpret_cast<u2v*>(simg + col[j] * kOP + m) = u2v{p01, p23};
        }
      }
    }
    __syncthreads();
    if (flat) {
      bf16* yb = y + ((int64_t)P.img * g.cout + co0) * hwo + P.p0;
#pragma unroll
      for (int k = 0; k < NB * MB / 8 / 256; ++k) {
        const int j = tid + 256 * k, co = j / (MB / 8), px = 8 * (j % (MB / 8));
        const u4v v = *reinterpret_cast<const u4v*>(simg + co * kOP + px);
        bf16* dst = yb + (int64_t)co * hwo + px;
        if (px + 8 <= P.npx)
          *reinterpret_cast<u4v*>(dst) = v;
        else if (px < P.npx)  // npx % 4 == 0: half a chunk
          *reinterpret_cast<u2v*>(dst) = u2v{v[0], v[1]};
      }
    } else {
      // 2D patches (pr rows x pc columns) through the same LDS rows: row
      // segments of 8 (pc % 8 == 0) or 4 pixels per lane (the fragments' own
      // 4-pixel pieces wrote 8 bytes of 64 planes per instruction)
      bf16* yb = y + ((int64_t)P.img * g.cout + co0) * hwo;
      if (g.pc % 8 == 0) {
#pragma unroll
        for (int k = 0; k < NB * MB / 8 / 256; ++k) {
          const int j = tid + 256 * k, co = j / (MB / 8), m0 = 8 * (j % (MB / 8));
          const int mr = fdiv(m0, g.pc, g.inv_pc), r = P.r0 + mr, c = P.c0 + (m0 - mr * g.pc);
          if (m0 < P.npx && r < g.ho && c < g.wo) {
            const u4v v = *reinterpret_cast<const u4v*>(simg + co * kOP + m0);
            bf16* dst = yb + (int64_t)co * hwo + (int64_t)r * g.wo + c;
            if (c + 8 <= g.wo)
              *reinterpret_cast<u4v*>(dst) = v;
            else  // wo % 4 == 0: half a chunk
              *reinterpret_cast<u2v*>(dst) = u2v{v[0], v[1]};
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < NB * MB / 4 / 256; ++k) {
          const int j = tid + 256 * k, co = j / (MB / 4), m0 = 4 * (j % (MB / 4));
          const int mr = fdiv(m0, g.pc, g.inv_pc), r = P.r0 + mr, c = P.c0 + (m0 - mr * g.pc);
          if (m0 < P.npx && r < g.ho && c < g.wo)
            *reinterpret_cast<u2v*>(yb + (int64_t)co * hwo + (int64_t)r * g.wo + c) =
                *reinterpret_cast<const u2v*>(simg + co * kOP + m0);
        }
      }
    }
    if (q + 1 < q1) {
      P = Pn;
      I = In;
      setup(P, I);
    }
  }
  if constexpr (STATS) {  // one record per channel and block
    __syncthreads();
    float* part = reinterpret_cast<float*>(simg);  // [WMW][NB][4]
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const mde::Sh a = mde::sh_xor_sum(run[j], 32);
      if (h == 0) {
        float* p4 = part + (wm * NB + col[j]) * 4;
        p4[0] = a.ref;
        p4[1] = a.n;
        p4[2] = a.s1;
        p4[3] = a.s2;
      }
    }
    __syncthreads();
    if (tid < NB) {
      mde::Sh a{part[tid * 4], part[tid * 4 + 1], part[tid * 4 + 2], part[tid * 4 + 3]};
#pragma unroll
      for (int k = 1; k < WMW; ++k) {
        const float* p4 = part + (k * NB + tid) * 4;
        a = mde::sh_merge(a, {p4[0], p4[1], p4[2], p4[3]});
      }
      float* o4 = stats + ((int64_t)(co0 + tid) * gridDim.x + blockIdx.x) * 4;
      o4[0] = a.ref;
      o4[1] = a.n;
      o4[2] = a.s1;
      o4[3] = a.s2;
    }
  }
}

// ---------------------------------------------------------- weight gradient
// Block: 64 output x 32 input channels, all taps, the patches
// [blockIdx.x * per, ...); 6 waves (3x3: wave = channel tile wc x filter row
// dy, three 32x32 accumulators, one per dx) or 4 (1x1: wc x K half).
template <int KS, int MODE, int CAP>
__global__ void __launch_bounds__(KS == 3 ? 384 : 256, 2)
    convbf_wgrad_kernel(const bf16* __restrict__ x, const bf16* __restrict__ gy,
                        float* __restrict__ part, Geo g, int per, int npatch) {
  constexpr int KK = KS * KS, NT = KS == 3 ? 384 : 256, ND = KS == 3 ? 3 : 1;
  constexpr int kMBW = wgrad_mbw<KS, MODE>(), kGP = kMBW + 8;
  constexpr int ME = 64 * KK * 32;  // partial elements: [co 64][tap][ci 32]
  __shared__ __attribute__((aligned(16))) bf16 simg[CAP * kPitchW];
  __shared__ __attribute__((aligned(16))) bf16 sg[64 * kGP];
  __shared__ int tab[kMBW];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wv & 1, wy = wv >> 1;  // 3x3: filter row wy; 1x1: K half wy
  const int ngo = (g.cout + 63) >> 6;
  const int cob = blockIdx.y % ngo, cc = blockIdx.y / ngo;
  const int co_live = g.cout - cob * 64 < 64 ? g.cout - cob * 64 : 64;  // 32 or 64
  const int q0 = blockIdx.x * per, q1 = q0 + per < npatch ? q0 + per : npatch;

  f16v acc[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[d][r] = 0.f;

  // transposed-read lane roles: 16-lane group gq, row q, column quad p
  const int gq = lane >> 4, qr = (lane >> 2) & 3, pq = lane & 3;
  const int bcol = 16 * (gq & 1) + 4 * pq;  // channel (element) offset in a staged pixel
  const int arow = (wc * 32 + l32) * kGP + 8 * h;
  const int64_t hwo = (int64_t)g.ho * g.wo;

  // gy rows: [64 channels][128 pixels], 4 pixels a unit (8-byte loads)
  constexpr int GU = (64 * (kMBW / 4) + NT - 1) / NT;
  u2v gv[GU];
  const bool flat = g.pc == 0;
  // buffer loads: a per-patch resource over the block's 64 gy planes of the
  // image, 32-bit offsets, out-of-range units past the buffer (zeros) -- no
  // 64-bit address math or selects per load
  auto gy_load = [&](const Patch& P) {
    const uint64_t a = (uint64_t)(gy + ((int64_t)P.img * g.cout + cob * 64) * hwo);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, (int)(2 * co_live * hwo), 0x00020000);
#pragma unroll
    for (int k = 0; k < GU; ++k) {
      const int u = tid + NT * k;
      const int cl = u / (kMBW / 4), m4 = 4 * (u - cl * (kMBW / 4));
      int off;
      bool ok = u < 64 * (kMBW / 4) && cl < co_live;
      if (flat) {  // a contiguous run of the plane: no (row, column) division
        ok = ok && m4 < P.npx;
        off = cl * (int)hwo + P.p0 + m4;
      } else {
        int r, c;
        ok = ok && pix_of(g, P, m4, r, c);
        off = cl * (int)hwo + r * g.wo + c;
      }
      const uint32_t voff = ok ? (uint32_t)(2 * off) : 0x7ffffff0u;
      gv[k] = __builtin_bit_cast(u2v, __builtin_amdgcn_raw_buffer_load_b64(R, voff, 0, 0));
    }
  };
  SrcStage<KS, MODE, kPitchW, NT, src_units<KS, MODE, CAP, NT>()> S;
  if (q0 < q1) {
    const Patch P = patch_of(g, q0);
    const Img I = img_of<KS, MODE>(g, P);
    S.plan(I, tid);
    S.load(x + (int64_t)P.img * g.cin * g.hi * g.wi, g, I, 32 * cc);
    gy_load(P);
  }
  for (int q = q0; q < q1; ++q) {
    const Patch P = patch_of(g, q);
    const Img I = img_of<KS, MODE>(g, P);
    __syncthreads();
    S.store(simg, I);
#pragma unroll
    for (int k = 0; k < GU; ++k) {
      const int u = tid + NT * k;
      if (u < 64 * (kMBW / 4)) {
        const int cl = u / (kMBW / 4), m4 = 4 * (u - cl * (kMBW / 4));
        *reinterpret_cast<u2v*>(sg + cl * kGP + m4) = gv[k];
      }
    }
    for (int m = tid; m < kMBW; m += NT) {
      int r, c;
      const bool ok = pix_of(g, P, m, r, c);
      tab[m] = ok ? img_base<KS, MODE>(P, I, r, c) : 0;
    }
    __syncthreads();
    if (q + 1 < q1) {  // the next patch's loads, in flight during this patch's MFMAs
      const Patch Pn = patch_of(g, q + 1);
      S.load(x + (int64_t)Pn.img * g.cin * g.hi * g.wi, g, img_of<KS, MODE>(g, Pn), 32 * cc);
      gy_load(Pn);
    }
    int toff[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) toff[d] = KS == 3 ? tap_off<KS, MODE>(I, wy, d) : 0;
    // every k-step of the patch, straight-line (a partial patch's extra steps
    // multiply zero gy rows: no branch around an MFMA), the next step's
    // operands read one step ahead; the staged-pixel offsets of all steps
    // first (tab), so no read waits on another
    constexpr int NKS = kMBW / 16 / (KS == 3 ? 1 : 2);
    u4v aq[2];
    s4v lq[2][ND], hq[2][ND];
    auto ld = [&](auto j_c, auto slot_c) {
      constexpr int j = decltype(j_c)::value, slot = decltype(slot_c)::value;
      constexpr int ks = KS == 3 ? j : -1;
      const int kk = KS == 3 ? ks : 2 * j + wy;
      // the step's staged-pixel offsets read from tab here, one step ahead like
      // the fragments (all steps' offsets held at once cost 2 NKS registers)
      const int m0 = 16 * kk + 8 * (gq >> 1) + qr;
      const int t0 = tab[m0] * kPitchW + bcol, t1 = tab[m0 + 4] * kPitchW + bcol;
      aq[slot] = *reinterpret_cast<const u4v*>(sg + arow + 16 * kk);
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        lq[slot][d] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s4*)(simg + t0 + toff[d] * kPitchW));
        hq[slot][d] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s4*)(simg + t1 + toff[d] * kPitchW));
      }
    };
    ld(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    static_for<NKS>([&](auto j_c) {
      constexpr int j = decltype(j_c)::value;
      if constexpr (j + 1 < NKS)
        ld(std::integral_constant<int, j + 1>{}, std::integral_constant<int, (j + 1) & 1>{});
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const u2v l2 = __builtin_bit_cast(u2v, lq[j & 1][d]), h2 = __builtin_bit_cast(u2v, hq[j & 1][d]);
        acc[d] = mfma32(aq[j & 1], u4v{l2.x, l2.y, h2.x, h2.y}, acc[d]);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  }

  // D[co][ci]: lane (ci = l32, h), register r -> co row (r & 3) + 8 (r >> 2) + 4 h
  float* out = part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * ME;
  if constexpr (KS == 3) {
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      const int tap = wy * 3 + d;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int col = wc * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[(col * KK + tap) * 32 + l32] = acc[d][r];
      }
    }
  } else {  // the two K halves summed through LDS, half 0 + half 1
    __syncthreads();
    float* red = reinterpret_cast<float*>(simg);  // [64 co][32 ci]
    if (wy == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(wc * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 32 + l32] = acc[0][r];
    }
    __syncthreads();
    if (wy == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int col = wc * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[col * 32 + l32] = acc[0][r] + red[col * 32 + l32];
      }
    }
  }
}

// gw[co][ci][tap] = sum over the S block partials of group (cob, cc), in order
template <int KK>
__global__ void __launch_bounds__(256)
    convbf_wreduce_kernel(const float* __restrict__ part, float* __restrict__ gw, int S, int cin,
                          int cout) {
  // block: 256 consecutive partial elements (64 float4 columns) x 4 split
  // slices; slice sl sums splits sl, sl + 4, ... in order, then slice 0 adds
  // the four in order: a fixed summation order (bitwise-repeatable), 16-byte
  // loads, and S / 4 of them in flight per thread instead of a serial chain of S
  constexpr int ME = 64 * KK * 32, SL = 4;
  const int tid = threadIdx.x, qd = tid & 63, sl = tid >> 6;
  const int e4 = blockIdx.x * 256 + 4 * qd;
  const int grp = blockIdx.y, ngo = (cout + 63) >> 6, cob = grp % ngo, cc = grp / ngo;
  const f4v* p = reinterpret_cast<const f4v*>(part + (int64_t)grp * S * ME + e4);
  f4v a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int s = sl; s < S; s += SL) a += p[(int64_t)s * (ME / 4)];
  __shared__ f4v red[SL][64];
  red[sl][qd] = a;
  __syncthreads();
  if (sl) return;
  const f4v t = ((red[0][qd] + red[1][qd]) + red[2][qd]) + red[3][qd];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = e4 + j;
    const int col = e / (KK * 32), rest = e - col * KK * 32, tap = rest / 32, ci = rest % 32;
    if (cob * 64 + col < cout) gw[((int64_t)(cob * 64 + col) * cin + cc * 32 + ci) * KK + tap] = t[j];
  }
}

// packed filter [cc][tap][co][32] (bf16, RNE) of a pass: forward (w[co][ci][tap])
// into p0, transposed + flipped (data gradient: the pass's input channels are
// the forward's outputs) into p1; either may be null (one launch packs both)
__device__ __forceinline__ bf16 pack_elem(const float* __restrict__ w, int64_t e, int cin, int cout,
                                          int kk, bool transpose) {
  const int pco = transpose ? cin : cout, pci = transpose ? cout : cin;
  const int j = (int)(e & 31);
  int64_t rest = e >> 5;
  const int co = (int)(rest % pco);
  rest /= pco;
  const int tap = (int)(rest % kk), cc = (int)(rest / kk);
  // element j of the row sits at 16-byte piece (j / 8) ^ ((co >> 2) & 3): the
  // swizzle of the LDS filter image (conflict-free B reads), so blocks copy
  // rows verbatim (register staging or LDS-DMA)
  const int jj = 8 * ((j >> 3) ^ ((co >> 2) & 3)) + (j & 7);
  const int ci = cc * 32 + jj;
  float v = 0.f;
  if (ci < pci)
    v = transpose ? w[((int64_t)ci * cin + co) * kk + (kk - 1 - tap)]
                  : w[((int64_t)co * cin + ci) * kk + tap];
  return mde::f2bf(v);
}

__global__ void __launch_bounds__(256)
    convbf_pack_kernel(const float* __restrict__ w, bf16* __restrict__ p0, bf16* __restrict__ p1,
                       int cin, int cout, int kk, int64_t total0, int64_t total1) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p0 && e < total0) p0[e] = pack_elem(w, e, cin, cout, kk, false);
  if (p1 && e < total1) p1[e] = pack_elem(w, e, cin, cout, kk, true);
}

// Every registered filter of a model in one launch (mde_convbf_pack_table):
// table row r = {weight, packed, packed_t (nullable), cin, cout, ks,
// first block, 0}; the rows' blocks are laid end to end over a 1-D grid and a
// block finds its row by binary search over the first-block column.
__global__ void __launch_bounds__(256)
    convbf_pack_table_kernel(const int64_t* __restrict__ tab, int rows) {
  const int64_t b = blockIdx.x;
  int lo = 0, hi = rows - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[(int64_t)mid * 8 + 6] <= b) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* t = tab + (int64_t)lo * 8;
  const float* w = reinterpret_cast<const float*>(t[0]);
  bf16* p0 = reinterpret_cast<bf16*>(t[1]);
  bf16* p1 = reinterpret_cast<bf16*>(t[2]);
  const int cin = (int)t[3], cout = (int)t[4], ks = (int)t[5], kk = ks * ks;
  const int64_t total0 = (int64_t)((cin + 31) / 32) * 32 * cout * kk;
  const int64_t total1 = (int64_t)((cout + 31) / 32) * 32 * cin * kk;
  const int64_t e = (b - t[6]) * 256 + threadIdx.x;
  if (p0 && e < total0) p0[e] = pack_elem(w, e, cin, cout, kk, false);
  if (p1 && e < total1) p1[e] = pack_elem(w, e, cin, cout, kk, true);
}

// ------------------------------------------------------------------- host
constexpr int kCapS1 = 420;   // staged pixels: 33.6 KB (+ 36.9 KB filter): two blocks a CU
constexpr int kCapS2 = 640;   // stride 2 / zero-inserted: 51 KB (one block a CU)
constexpr int kCapS1W = 600;  // 8-wave blocks (256 pixels): 48 KB
constexpr int kCapS2W = 1200; // 8-wave blocks, stride 2 / zero-inserted: 96 KB

struct Pass {
  int ks, mode, cin, cout, hi, wi, ho, wo;
};

inline int cap_of(const Pass& p, bool wide = false) {
  const bool s2 = p.ks == 3 && p.mode != S1;
  return wide ? (s2 ? kCapS2W : kCapS1W) : (s2 ? kCapS2 : kCapS1);
}

// staged pixels of the largest patch of a geometry
inline int img_px(const Pass& p, int pc, int pr, int mb) {
  int nr, nc;
  if (pc == 0) {
    nr = (mb + p.wo - 2) / p.wo + 1;  // rows a run of mb consecutive pixels can touch
    if (nr > p.ho) nr = p.ho;
    nc = p.wo;
  } else {
    nr = pr;
    nc = pc;
  }
  if (p.ks == 3 && p.mode == S2) return (2 * nr + 1) * 2 * (nc + 1);
  if (p.ks == 3) return (nr + 2) * (nc + 4);
  return nr * nc;
}

inline void set_inv(Geo* g) {
  g->inv_wo = 1.f / (float)g->wo;
  g->inv_pc = g->pc ? 1.f / (float)g->pc : 0.f;
  g->inv_ppi = 1.f / (float)g->ppi;
  g->inv_tw = 1.f / (float)g->tiles_w;
}

// Choose the patch geometry: flat runs of mb pixels when the image fits,
// else 2D tiles (pc columns x pr rows, pr * pc <= mb) with the fewest padded
// pixels.  False if nothing fits or the shape breaks an alignment rule.
inline bool pick_geo(const Pass& p, int mb, Geo* g, int cap = 0) {
  g->cin = p.cin;
  g->cout = p.cout;
  g->hi = p.hi;
  g->wi = p.wi;
  g->ho = p.ho;
  g->wo = p.wo;
  g->mb = mb;
  g->cap = cap ? cap : cap_of(p);
  const int64_t hw = (int64_t)p.ho * p.wo;
  if (hw >= (1 << 22)) return false;  // fdiv's exact range
  if (hw % 4 == 0 && img_px(p, 0, 0, mb) <= g->cap) {
    g->pc = g->pr = 0;
    g->tiles_w = 1;
    g->ppi = (int)mde::cdiv(hw, mb);
    int nr = (mb + p.wo - 2) / p.wo + 1;
    g->nrmax = nr > p.ho ? p.ho : nr;
    set_inv(g);
    return true;
  }
  if (p.wo % 4) return false;
  int best = -1;
  int64_t best_cost = 0;
  const int cands[] = {64, 40, 32, 20, 16, 8, 4};
  for (int pc : cands) {
    if (pc > p.wo && pc != cands[6]) continue;
    int pr = mb / pc;
    if (pr > p.ho) pr = p.ho;
    if (pr < 1 || img_px(p, pc, pr, mb) > g->cap) continue;
    const int64_t tiles = mde::cdiv(p.ho, pr) * mde::cdiv(p.wo, pc);
    const int64_t cost = tiles * ((int64_t)(pr * pc + 31) / 32 * 32);
    if (best < 0 || cost < best_cost) {
      best = pc;
      best_cost = cost;
    }
  }
  if (best < 0) return false;
  g->pc = best;
  g->pr = mb / best < p.ho ? mb / best : p.ho;
  g->tiles_w = (int)mde::cdiv(p.wo, g->pc);
  g->ppi = (int)(mde::cdiv(p.ho, g->pr) * g->tiles_w);
  g->nrmax = g->pr;
  set_inv(g);
  return true;
}

// the pass of (n, cin, cout, h, w, ks, stride) and which: 0 forward, 1 data gradient, 2 weight gradient
inline bool make_pass(int64_t cin, int64_t cout, int64_t h, int64_t w, int ks, int stride, int which,
                      Pass* p) {
  if ((ks != 1 && ks != 3) || (stride != 1 && stride != 2)) return false;
  if (cin <= 0 || cout <= 0 || h <= 0 || w <= 0 || cin % 32 || cout % 32) return false;
  if (cin > 4096 || cout > 4096 || h > 4096 || w > 4096 || w % 2) return false;
  const int pad = ks / 2;
  const int ho = (int)((h + 2 * pad - ks) / stride + 1), wo = (int)((w + 2 * pad - ks) / stride + 1);
  if (which == 1) {  // gx [cin, h, w] from gy [cout, ho, wo]
    *p = Pass{ks, stride == 1 ? S1 : U2, (int)cout, (int)cin, ho, wo, (int)h, (int)w};
  } else {
    *p = Pass{ks, stride == 1 ? S1 : S2, (int)cin, (int)cout, (int)h, (int)w, ho, wo};
  }
  if (p->wi % 2) return false;  // dword pair loads of the staged source
  return true;
}

template <int KS, int MODE, int WN, int MTW, int NW, int CAP>
int launch_fwd_t(const bf16* x, const bf16* wp, bf16* y, float* stats, const Geo& g, int64_t n,
                 int kid, double flops, double bytes, hipStream_t s) {
  const int64_t np = n * g.ppi;
  if (np >= (1 << 22)) return MDE_ERR_UNSUPPORTED;  // fdiv's exact range
  const dim3 grid((unsigned)np, (unsigned)(g.cout / (32 * WN)));
  if (stats)
    MDE_LAUNCH_MFMA(kid, bytes, flops, s, (convbf_fwd_kernel<KS, MODE, WN, MTW, NW, true, CAP>),
                    grid, dim3(64 * NW), 0, x, wp, y, stats, g);
  else
    MDE_LAUNCH_MFMA(kid, bytes, flops, s, (convbf_fwd_kernel<KS, MODE, WN, MTW, NW, false, CAP>),
                    grid, dim3(64 * NW), 0, x, wp, y, stats, g);
  return MDE_OK;
}

inline int wn_of(const Pass& p) { return p.cout % 64 == 0 ? 2 : 1; }

// forward geometry: 4-wave blocks with 2 M tiles a wave (128 pixels; 256 at
// 32 channels), or 1 when that patch's image does not fit.  MDE_CONVBF_NW8=1:
// 8-wave blocks of 256 pixels at 64 output channels (the filter staged half
// as often; measured slower at 64 -> 64 @ 60x80: 77 vs 69 us, one block a CU)
inline bool nw8_on() {
  static const bool on = [] {
    const char* e = std::getenv("MDE_CONVBF_NW8");
    return e && e[0] == '1';
  }();
  return on;
}

inline bool fwd_geo(const Pass& p, int64_t n, Geo* g, int* mtw, int* nw) {
  const int wn = wn_of(p);
  if (nw8_on() && wn == 2 && pick_geo(p, 256, g, cap_of(p, true)) &&
      n * g->ppi * (p.cout / 64) >= 512) {
    *mtw = 2;
    *nw = 8;
    return true;
  }
  const int wmw = 4 / wn;
  for (int m = 2; m >= 1; --m) {
    if (pick_geo(p, 32 * m * wmw, g)) {
      *mtw = m;
      *nw = 4;
      return true;
    }
  }
  return false;
}

// Resident-filter path (convbf_fwd_res_kernel): the block's filter slice --
// NB = 64 output channels when it fits kWRes, else 32 -- for all input
// channels.  MDE_CONVBF_RES=0: the chunked kernel always (A/B switch).
inline bool res_on() {
  static const bool on = [] {
    const char* e = std::getenv("MDE_CONVBF_RES");
    return !(e && e[0] == '0');
  }();
  return on;
}

inline int res_nb(const Pass& p) {
  const int nch = (p.cin + 31) / 32, kk = p.ks * p.ks;
  if (p.cout % 64 == 0 && nch * kk * 64 * 32 <= kWRes) return 64;
  if (nch * kk * 32 * 32 <= kWRes) return 32;
  return 0;
}

inline int device_cus() {
  static const int cus = [] {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    return c > 0 ? c : 256;
  }();
  return cus;
}

struct ResGeo {
  Geo g;
  int nb, per, blocks;  // output channels a block, patches a block, blocks per channel group
  int ntw;              // 32-channel tiles a wave: 2 = 256-pixel patches, 64 x 64 wave tiles
  int64_t np;
};

// Resident-filter variants (MDE_CONVBF_RESMODE):
//  t22  (default) 64 output channels a block, 64 x 64 wave tiles over
//       256-pixel patches where that image fits beside the filter (stride 1,
//       any 1x1); else as t21
//  t21  64 (or 32) output channels, 32 x 64 wave tiles, 128-pixel patches
// (Measured, tools/gpu_r05h.sh: two blocks a CU with a half-size filter slice
// -- 32 output channels, so one block's staging overlaps the other's MFMAs --
// ran 64 -> 64 @ 60x80 at 46.5 us against t22's 35.8: dropped.)
inline int res_mode() {
  static const int m = [] {
    const char* e = std::getenv("MDE_CONVBF_RESMODE");
    return e && !std::strcmp(e, "t21") ? 1 : 0;
  }();
  return m;
}

inline bool res_geo(const Pass& p, int64_t n, ResGeo* r) {
  r->nb = res_on() ? res_nb(p) : 0;
  if (!r->nb) return false;
  r->ntw = 1;
  const bool s1img = p.mode == S1 || p.ks == 1;
  if (res_mode() == 0 && r->nb == 64 && s1img &&
             pick_geo(p, 256, &r->g, p.ks == 3 ? kCapS1W : kCapS1)) {
    r->ntw = 2;
  } else if (!pick_geo(p, 32 * 2 * (4 / (r->nb / 32)), &r->g)) {
    return false;
  }
  r->np = n * r->g.ppi;
  if (r->np >= (1 << 22)) return false;
  const int ncob = p.cout / r->nb;
  int64_t G = device_cus() / ncob;  // one block a CU (the LDS holds one)
  if (G < 1) G = 1;
  if (G > r->np) G = r->np;
  r->per = (int)mde::cdiv(r->np, G);
  r->blocks = (int)mde::cdiv(r->np, r->per);
  return true;
}

template <int KS, int MODE, int WN, int CAP, int NTW = 1>
int launch_res_t(const bf16* x, const bf16* wp, bf16* y, float* stats, const ResGeo& r, int cout,
                 int kid, double flops, double bytes, hipStream_t s) {
  const dim3 grid((unsigned)r.blocks, (unsigned)(cout / (32 * WN)));
  if (stats)
    MDE_LAUNCH_MFMA(kid, bytes, flops, s, (convbf_fwd_res_kernel<KS, MODE, WN, true, CAP, NTW>),
                    grid, dim3(256), 0, x, wp, y, stats, r.g, r.per, (int)r.np);
  else
    MDE_LAUNCH_MFMA(kid, bytes, flops, s, (convbf_fwd_res_kernel<KS, MODE, WN, false, CAP, NTW>),
                    grid, dim3(256), 0, x, wp, y, stats, r.g, r.per, (int)r.np);
  return MDE_OK;
}

// Algorithmic MACs x 2 of a pass: the convolution's own product count,
// 2 n Ho Wo Cin Cout k^2 over the FORWARD output plane.  A forward / stride-1
// pass writes that plane; the stride-2 data gradient (U2) writes the input
// plane and reads the forward output (its staged source, hi x wi), so its
// count is over hi x wi -- not over the full-resolution gx it produces (4x
// the true work) nor over the MFMAs the zero-inserted form issues.
inline double pass_flops(const Pass& p, int64_t n) {
  const double plane = p.mode == U2 ? (double)p.hi * p.wi : (double)p.ho * p.wo;
  return 2.0 * n * plane * (double)p.cout * p.cin * p.ks * p.ks;
}

int launch_fwd(const Pass& p, const bf16* x, const bf16* wp, bf16* y, float* stats, int64_t n,
               int kid, hipStream_t s) {
  const double flops = pass_flops(p, n);
  const double bytes = 2.0 * n * ((double)p.cin * p.hi * p.wi + (double)p.cout * p.ho * p.wo);
  ResGeo rg;
  if (res_geo(p, n, &rg)) {
#define CBF_RES(KS, MODE, CAP)                                                                     \
  return rg.nb == 64 ? launch_res_t<KS, MODE, 2, CAP>(x, wp, y, stats, rg, p.cout, kid, flops, bytes, s) \
                     : launch_res_t<KS, MODE, 1, CAP>(x, wp, y, stats, rg, p.cout, kid, flops, bytes, s)
    if (rg.ntw == 2) {
      if (p.ks == 3)
        return launch_res_t<3, S1, 2, kCapS1W, 2>(x, wp, y, stats, rg, p.cout, kid, flops, bytes, s);
      if (p.mode == S1)
        return launch_res_t<1, S1, 2, kCapS1, 2>(x, wp, y, stats, rg, p.cout, kid, flops, bytes, s);
      if (p.mode == S2)
        return launch_res_t<1, S2, 2, kCapS1, 2>(x, wp, y, stats, rg, p.cout, kid, flops, bytes, s);
      return launch_res_t<1, U2, 2, kCapS1, 2>(x, wp, y, stats, rg, p.cout, kid, flops, bytes, s);
    }
    if (p.ks == 3) {
      if (p.mode == S1) { CBF_RES(3, S1, kCapS1); }
      if (p.mode == S2) { CBF_RES(3, S2, kCapS2); }
      CBF_RES(3, U2, kCapS2);
    }
    if (p.mode == S1) { CBF_RES(1, S1, kCapS1); }
    if (p.mode == S2) { CBF_RES(1, S2, kCapS1); }
    CBF_RES(1, U2, kCapS1);
#undef CBF_RES
  }
  const int wn = wn_of(p);
  Geo g;
  int mtw, nw;
  if (!fwd_geo(p, n, &g, &mtw, &nw)) return MDE_ERR_UNSUPPORTED;
#define CBF_FWD(KS, MODE, CAP, CAPW)                                                         \
  if (nw == 8)                                                                             \
    return launch_fwd_t<KS, MODE, 2, 2, 8, CAPW>(x, wp, y, stats, g, n, kid, flops, bytes, s); \
  if (wn == 2)                                                                             \
    return mtw == 2                                                                        \
               ? launch_fwd_t<KS, MODE, 2, 2, 4, CAP>(x, wp, y, stats, g, n, kid, flops, bytes, s) \
               : launch_fwd_t<KS, MODE, 2, 1, 4, CAP>(x, wp, y, stats, g, n, kid, flops, bytes, s); \
  return mtw == 2                                                                          \
             ? launch_fwd_t<KS, MODE, 1, 2, 4, CAP>(x, wp, y, stats, g, n, kid, flops, bytes, s)   \
             : launch_fwd_t<KS, MODE, 1, 1, 4, CAP>(x, wp, y, stats, g, n, kid, flops, bytes, s)
  if (p.ks == 3) {
    if (p.mode == S1) { CBF_FWD(3, S1, kCapS1, kCapS1W); }
    if (p.mode == S2) { CBF_FWD(3, S2, kCapS2, kCapS2W); }
    CBF_FWD(3, U2, kCapS2, kCapS2W);
  }
  if (p.mode == S1) { CBF_FWD(1, S1, kCapS1, kCapS1W); }
  if (p.mode == S2) { CBF_FWD(1, S2, kCapS1, kCapS1W); }
  CBF_FWD(1, U2, kCapS1, kCapS1W);
#undef CBF_FWD
}

// weight-gradient split: blocks per (output 64, input 32) channel group
// blocks a weight-gradient launch aims at (MDE_CONVBF_WBLOCKS, default 256)
inline int wgrad_blocks_target() {
  static const int v = [] {
    const char* e = std::getenv("MDE_CONVBF_WBLOCKS");
    const int b = e ? std::atoi(e) : 0;
    return b > 0 ? b : 256;
  }();
  return v;
}

// the weight-gradient kernels' staged-image capacity (its template CAP)
inline int wgrad_cap(const Pass& p) {
  return p.ks == 3 ? (p.mode == S1 ? kCapS1W : kCapS2) : kCapS1;
}

// 3x3: 256 blocks (one a CU: 191 registers x 6 waves); 1x1: 512 (two a CU,
// measured 41 -> 30 us at 64 -> 64 @60x80, 38.8 -> 27.9 at 256 -> 256 @15x20;
// the 3x3 kernel forced to two blocks a CU spills and ran 1.6x slower at stride 2)
inline int wgrad_splits(int groups, int64_t npatch, int ks) {
  int64_t s = mde::cdiv(wgrad_blocks_target() * (ks == 1 ? 2 : 1), groups);
  if (s > npatch) s = npatch;
  return (int)(s < 1 ? 1 : s);
}

inline bool wgrad_geo(const Pass& p, int64_t n, Geo* g, int* S, int* per, int64_t* npatch) {
  if (!pick_geo(p, p.ks == 3 && p.mode == S1 ? wgrad_mbw<3, S1>() : wgrad_mbw<1, S1>(), g,
                wgrad_cap(p)))
    return false;
  const int64_t np = n * g->ppi;
  if (np >= (1 << 22)) return false;  // fdiv's exact range
  *npatch = np;
  const int groups = ((p.cout + 63) / 64) * (p.cin / 32);
  const int s0 = wgrad_splits(groups, np, p.ks);
  *per = (int)mde::cdiv(np, s0);
  *S = (int)mde::cdiv(np, *per);
  return true;
}

}  // namespace

extern "C" {

int mde_convbf_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int ks, int stride,
                         int pass) {
  Pass p;
  if (pass < 0 || pass > 2 || !make_pass(cin, cout, h, w, ks, stride, pass == 1 ? 1 : 0, &p))
    return 0;
  Geo g;
  if (pass == 2) {
    int S, per;
    int64_t np;
    return wgrad_geo(p, 1, &g, &S, &per, &np) ? 1 : 0;
  }
  int mtw, nw;
  return fwd_geo(p, 1, &g, &mtw, &nw) ? 1 : 0;
}

int mde_convbf_supported_n(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, int ks,
                           int stride, int pass) {
  Pass p;
  if (n <= 0 || pass < 0 || pass > 2 ||
      !make_pass(cin, cout, h, w, ks, stride, pass == 1 ? 1 : 0, &p))
    return 0;
  Geo g;
  if (pass == 2) {
    int S, per;
    int64_t np;
    return wgrad_geo(p, n, &g, &S, &per, &np) ? 1 : 0;
  }
  // launch_fwd's own choice: the resident-filter geometry, else the chunked
  // one, whose launch refuses n * patches >= 2^22
  ResGeo rg;
  if (res_geo(p, n, &rg)) return 1;
  int mtw, nw;
  return fwd_geo(p, n, &g, &mtw, &nw) && n * g.ppi < (1 << 22) ? 1 : 0;
}

double mde_convbf_flops(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, int ks,
                        int stride, int pass) {
  Pass p;
  if (n <= 0 || pass < 0 || pass > 2 ||
      !make_pass(cin, cout, h, w, ks, stride, pass == 1 ? 1 : 0, &p))
    return 0.0;
  return pass_flops(p, n);
}

size_t mde_convbf_pack_elems(int64_t cin, int64_t cout, int ks, int transpose) {
  const int64_t pci = transpose ? cout : cin, pco = transpose ? cin : cout;
  return (size_t)(mde::cdiv(pci, 32) * 32 * pco * ks * ks);
}

int mde_convbf_pack_both(const float* weight, void* packed, void* packed_t, int64_t cin,
                         int64_t cout, int ks, void* stream) {
  if (!weight || (!packed && !packed_t) || (ks != 1 && ks != 3) || cin <= 0 || cout <= 0)
    return MDE_ERR_INVALID_ARG;
  const int64_t t0 = packed ? (int64_t)mde_convbf_pack_elems(cin, cout, ks, 0) : 0;
  const int64_t t1 = packed_t ? (int64_t)mde_convbf_pack_elems(cin, cout, ks, 1) : 0;
  const int64_t total = t0 > t1 ? t0 : t1;
  MDE_LAUNCH(mde::K_CBF_PACK, 4.0 * cin * cout * ks * ks * ((t0 > 0) + (t1 > 0)) + 2.0 * (t0 + t1),
             (hipStream_t)stream, convbf_pack_kernel, dim3((unsigned)mde::cdiv(total, 256)), dim3(256),
             0, weight, (bf16*)packed, (bf16*)packed_t, (int)cin, (int)cout, ks * ks, t0, t1);
  return MDE_OK;
}

int mde_convbf_pack_table(const int64_t* table, int rows, int64_t blocks, int64_t elems,
                          void* stream) {
  if (!table || rows <= 0 || blocks <= 0 || blocks > 0x7fffffff || elems < 0)
    return MDE_ERR_INVALID_ARG;
  MDE_LAUNCH(mde::K_CBF_PACK, 6.0 * elems, (hipStream_t)stream, convbf_pack_table_kernel,
             dim3((unsigned)blocks), dim3(256), 0, table, rows);
  return MDE_OK;
}

int mde_convbf_pack(const float* weight, void* packed, int64_t cin, int64_t cout, int ks,
                    int transpose, void* stream) {
  if (!packed) return MDE_ERR_INVALID_ARG;
  return transpose ? mde_convbf_pack_both(weight, nullptr, packed, cin, cout, ks, stream)
                   : mde_convbf_pack_both(weight, packed, nullptr, cin, cout, ks, stream);
}

int mde_convbf_stats_blocks(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, int ks,
                            int stride) {
  Pass p;
  Geo g;
  int mtw, nw;
  if (!make_pass(cin, cout, h, w, ks, stride, 0, &p)) return 0;
  ResGeo rg;
  if (res_geo(p, n, &rg)) return rg.blocks;  // one record per channel and persistent block
  if (!fwd_geo(p, n, &g, &mtw, &nw)) return 0;
  return (int)(n * g.ppi);
}

int mde_convbf_fwd(const void* x, const void* packed, void* y, float* stats, int64_t n,
                   int64_t cin, int64_t cout, int64_t h, int64_t w, int ks, int stride,
                   void* stream) {
  if (!x || !packed || !y || n <= 0) return MDE_ERR_INVALID_ARG;
  Pass p;
  if (!make_pass(cin, cout, h, w, ks, stride, 0, &p)) return MDE_ERR_UNSUPPORTED;
  return launch_fwd(p, (const bf16*)x, (const bf16*)packed, (bf16*)y, stats, n, mde::K_CBF_FWD,
                    (hipStream_t)stream);
}

int mde_convbf_bwd_data(const void* gy, const void* packed_t, void* gx, int64_t n, int64_t cin,
                        int64_t cout, int64_t h, int64_t w, int ks, int stride, void* stream) {
  if (!gy || !packed_t || !gx || n <= 0) return MDE_ERR_INVALID_ARG;
  Pass p;
  if (!make_pass(cin, cout, h, w, ks, stride, 1, &p)) return MDE_ERR_UNSUPPORTED;
  return launch_fwd(p, (const bf16*)gy, (const bf16*)packed_t, (bf16*)gx, nullptr, n,
                    mde::K_CBF_DGRAD, (hipStream_t)stream);
}

size_t mde_convbf_wgrad_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                                   int ks, int stride) {
  Pass p;
  Geo g;
  int S, per;
  int64_t np;
  if (n <= 0 || !make_pass(cin, cout, h, w, ks, stride, 0, &p) || !wgrad_geo(p, n, &g, &S, &per, &np))
    return 0;
  return sizeof(float) * (size_t)(((cout + 63) / 64) * (cin / 32) * S * 64 * ks * ks * 32);
}

int mde_convbf_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t cin,
                     int64_t cout, int64_t h, int64_t w, int ks, int stride, void* workspace,
                     void* stream) {
  if (!gy || !x || !gweight || !workspace || n <= 0) return MDE_ERR_INVALID_ARG;
  Pass p;
  Geo g;
  int S, per;
  int64_t np;
  if (!make_pass(cin, cout, h, w, ks, stride, 0, &p) || !wgrad_geo(p, n, &g, &S, &per, &np))
    return MDE_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int groups = (int)(((cout + 63) / 64) * (cin / 32));
  const double flops = 2.0 * n * p.ho * p.wo * (double)cout * cin * ks * ks;
  const double bytes = 2.0 * n * ((double)cin * h * w + (double)cout * p.ho * p.wo);
  const dim3 grid((unsigned)S, (unsigned)groups);
  float* part = (float*)workspace;
  const bf16 *gyb = (const bf16*)gy, *xb = (const bf16*)x;
  if (ks == 3) {
    if (p.mode == S1)
      MDE_LAUNCH_MFMA(mde::K_CBF_WGRAD, bytes, flops, s, (convbf_wgrad_kernel<3, S1, kCapS1W>), grid,
                      dim3(384), 0, xb, gyb, part, g, per, (int)np);
    else
      MDE_LAUNCH_MFMA(mde::K_CBF_WGRAD, bytes, flops, s, (convbf_wgrad_kernel<3, S2, kCapS2>), grid,
                      dim3(384), 0, xb, gyb, part, g, per, (int)np);
    MDE_LAUNCH(mde::K_CBF_WREDUCE, 4.0 * groups * (double)S * 64 * 9 * 32 + 4.0 * cout * cin * 9, s,
               convbf_wreduce_kernel<9>, dim3((unsigned)mde::cdiv(64 * 9 * 32, 256), groups),
               dim3(256), 0, part, gweight, S, (int)cin, (int)cout);
  } else {
    if (p.mode == S1)
      MDE_LAUNCH_MFMA(mde::K_CBF_WGRAD, bytes, flops, s, (convbf_wgrad_kernel<1, S1, kCapS1>), grid,
                      dim3(256), 0, xb, gyb, part, g, per, (int)np);
    else
      MDE_LAUNCH_MFMA(mde::K_CBF_WGRAD, bytes, flops, s, (convbf_wgrad_kernel<1, S2, kCapS1>), grid,
                      dim3(256), 0, xb, gyb, part, g, per, (int)np);
    MDE_LAUNCH(mde::K_CBF_WREDUCE, 4.0 * groups * (double)S * 64 * 32 + 4.0 * cout * cin, s,
               convbf_wreduce_kernel<1>, dim3((unsigned)mde::cdiv(64 * 32, 256), groups), dim3(256),
               0, part, gweight, S, (int)cin, (int)cout);
  }
  return MDE_OK;
}

}  // extern "C"
