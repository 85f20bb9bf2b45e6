// Shared helpers for the gfx950 kernels behind include/mde_abi.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mde_abi.h"

namespace mde {

// Kernel ids of the timing registry (mde_kernel_name gives the strings).
enum Kid : int {
  K_BILINEAR_FWD = 0,
  K_BILINEAR_BWD,
  K_NEAREST_FWD,
  K_NEAREST_BWD,
  K_SE_SQUEEZE,
  K_SE_FC,
  K_SE_SCALE,
  K_SE_BWD_DOT,
  K_SE_BWD_FC,
  K_SE_BWD_APPLY,
  K_SKIP_FWD,
  K_SKIP_BWD,
  K_SKIP_BWD_REDUCE,
  K_MINMAX,
  K_MINMAX_FINAL,
  K_DEPTHNORM,
  K_SSIM3_L1,
  K_LOSS_FINAL,
  K_DLOSS_FWD,
  K_DLOSS_BWD_COEF,
  K_DLOSS_BWD,
  K_BN_STATS,
  K_BN_FINAL,
  K_BN_APPLY,
  K_BN_BWD_REDUCE,
  K_BN_BWD_FINAL,
  K_BN_BWD_APPLY,
  K_BN_APPLY_SMALL,
  K_BN_BWD_APPLY_SMALL,
  K_WATTN_FWD,
  K_WATTN_BWD,
  K_DW_FWD,
  K_DW_BWD_DATA,
  K_DW_BWD_WEIGHT,
  K_DW_WREDUCE,
  K_LN_FWD,
  K_LN_BWD,
  K_LN_WREDUCE,
  K_TRANSPOSE,
  K_PW_FWD,
  K_PW_BWD,
  K_C3_FWD,
  K_C3_DGRAD,
  K_C3_WGRAD,
  K_C3_WREDUCE,
  K_DW_BWD,
  K_EVAL,
  K_EVAL_FINAL,
  K_NYU_AUGMENT,
  K_C3_WGRAD_GUIDE,  // the 3-channel guide convs' weight gradient (HBM-bound: ~12 flop/B)
  K_COLSUM,
  K_MLP_GELU_BWD,
  K_C3_FWD_BF16,  // the bf16 MFMA conv3x3 passes (v_mfma_f32_16x16x32_bf16: bf16 MFMA peak)
  K_C3_DGRAD_BF16,
  K_C3_WGRAD_BF16,
  K_C3_WGRAD_WIDE,  // the 64 / 128 / 256-channel NCHW weight gradients
  K_C3_WGRAD_S2,    // the stride-2 stem convolutions' weight gradients
  K_C1_FWD,         // DDRNet's wide 1x1 convolutions (conv1x1.hip)
  K_C1_DGRAD,
  K_C1_WGRAD,
  K_C1_WREDUCE,
  K_C3S2_FWD,       // DDRNet's wide stride-2 3x3 convolutions (conv3x3s2.hip)
  K_C3S2_DGRAD,
  K_C3W_FWD,        // the wide stride-1 3x3 convolutions (conv3x3s2.hip, c3s1_kernel)
  K_C3W_DGRAD,
  K_WINO_FWD,       // Winograd F(2x2, 3x3) stride-1 convolutions (wino.hip)
  K_WINO_DGRAD,
  K_WINO_WEIGHT,
  K_WATTN_BWD_REDUCE,  // the window-attention backward's table / bias slab reduction
  K_CBF_FWD,        // bf16 implicit-GEMM convolutions (convbf.hip, v_mfma_f32_32x32x16_bf16)
  K_CBF_DGRAD,
  K_CBF_WGRAD,
  K_CBF_WREDUCE,
  K_CBF_PACK,
  K_STEM_FWD,       // the bf16 stem convolution (stem.hip)
  K_STEM_WGRAD,
  K_LIN_WGRAD,      // token-major Linear weight gradients (mlp.hip, v_mfma_f32_16x16x4_f32)
  K_LIN_WREDUCE,
  K_CHANSUM,        // a biased conv's bias gradient (per-channel NCHW sums, mlp.hip)
  K_HEAD_FWD,       // the one-output-channel 3x3 conv (head.hip: the NewCRF depth head)
  K_HEAD_DGRAD,
  K_HEAD_WGRAD,
  K_COUNT
};

// Timing hooks (timing.hip).  begin() returns a token for end(); both are
// no-ops when the registry is disabled.
int timing_begin(int kid, hipStream_t s);
void timing_end(int token, hipStream_t s, double bytes, double flops = 0.0);

// Launch a kernel with optional timing and return the launch status.
#define MDE_LAUNCH(KID, BYTES, STREAM, KERNEL, GRID, BLOCK, SHMEM, ...)      \
  do {                                                                     \
    int _tok = ::mde::timing_begin((KID), (STREAM));                       \
    hipLaunchKernelGGL(KERNEL, (GRID), (BLOCK), (SHMEM), (STREAM),         \
                       __VA_ARGS__);                                       \
    hipError_t _e = hipGetLastError();                                     \
    ::mde::timing_end(_tok, (STREAM), (double)(BYTES));                    \
    if (_e != hipSuccess) return (int)_e;                                  \
  } while (0)

// Same for an MFMA kernel: FLOPS = its algorithmic floating-point operations
// (2 per multiply-accumulate), reported against the MFMA peak.
#define MDE_LAUNCH_MFMA(KID, BYTES, FLOPS, STREAM, KERNEL, GRID, BLOCK, SHMEM, ...) \
  do {                                                                     \
    int _tok = ::mde::timing_begin((KID), (STREAM));                       \
    hipLaunchKernelGGL(KERNEL, (GRID), (BLOCK), (SHMEM), (STREAM),         \
                       __VA_ARGS__);                                       \
    hipError_t _e = hipGetLastError();                                     \
    ::mde::timing_end(_tok, (STREAM), (double)(BYTES), (double)(FLOPS));   \
    if (_e != hipSuccess) return (int)_e;                                  \
  } while (0)

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Wave64 reductions.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block reduction of a float sum for blockDim.x == 256 (4 waves).  `red`
// must hold 4 floats of LDS.  Result valid in every thread.
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// Storage types of the activations / gradients: fp32, or bf16 (raw uint16,
// round-to-nearest-even like torch) under autocast.  Statistics, coefficients
// and accumulation are fp32 / fp64 either way.
using bf16 = uint16_t;
__device__ __forceinline__ float bf2f(bf16 b) { return __uint_as_float((uint32_t)b << 16); }
__device__ __forceinline__ bf16 f2bf(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16)((u >> 16) | 0x40);  // quiet NaN
  return (bf16)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16* p) { return bf2f(*p); }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16* p, float v) { *p = f2bf(v); }
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld4(const bf16* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ float2 ld2(const float* p) { return *reinterpret_cast<const float2*>(p); }
__device__ __forceinline__ float2 ld2(const bf16* p) {
  const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
  return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
}
__device__ __forceinline__ void st2(float* p, float2 v) { *reinterpret_cast<float2*>(p) = v; }
__device__ __forceinline__ void st2(bf16* p, float2 v) {
  *reinterpret_cast<uint32_t*>(p) = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
}
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void st4(bf16* p, float4 v) {
  uint2 u;
  u.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
  u.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
  *reinterpret_cast<uint2*>(p) = u;
}

// Nontemporal variants for streaming kernels (every tensor far larger than
// L2, read or written once per kernel: the BN passes measured +10 %,
// profiles/r04_bn_nt_ab.txt).
using nt4f = float __attribute__((ext_vector_type(4)));
using nt2u = uint32_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 ld4_nt(const float* p) {
  const nt4f v = __builtin_nontemporal_load(reinterpret_cast<const nt4f*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 ld4_nt(const bf16* p) {
  const nt2u u = __builtin_nontemporal_load(reinterpret_cast<const nt2u*>(p));
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ void st4_nt(float* p, float4 v) {
  __builtin_nontemporal_store(nt4f{v.x, v.y, v.z, v.w}, reinterpret_cast<nt4f*>(p));
}
__device__ __forceinline__ void st4_nt(bf16* p, float4 v) {
  const nt2u u{(uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16),
               (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16)};
  __builtin_nontemporal_store(u, reinterpret_cast<nt2u*>(p));
}

// Per-channel BatchNorm statistics emitted by a producing conv's epilogue
// (one (shift, count, s1, s2) per channel and block; mde_batchnorm_*_stats
// finalises them).  Running shifted sums of one channel's values: the shift
// `ref` (a sample of the channel, shared by the lanes that will be summed)
// keeps s2 free of cancellation; three VALU ops per value, no division.
struct Sh {
  float ref, n, s1, s2;
};

__device__ __forceinline__ void sh_add(Sh& a, float v, bool ok) {
  const float d = ok ? v - a.ref : 0.f;
  a.s1 += d;
  a.s2 = fmaf(d, d, a.s2);
  a.n += ok ? 1.f : 0.f;
}

// Sum of Sh over lanes sharing `ref` (a butterfly of plain adds over the
// given xor offsets).
__device__ __forceinline__ Sh sh_xor_sum(Sh a, int o) {
  a.n += __shfl_xor(a.n, o, 64);
  a.s1 += __shfl_xor(a.s1, o, 64);
  a.s2 += __shfl_xor(a.s2, o, 64);
  return a;
}

// a + b re-expressed on a's shift (b's shift differs from a's by O(std): both
// are samples of the channel, so the float arithmetic keeps its precision)
__device__ __forceinline__ Sh sh_merge(Sh a, Sh b) {
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float d = b.ref - a.ref;
  a.s2 += b.s2 + d * (2.f * b.s1 + b.n * d);
  a.s1 += b.s1 + b.n * d;
  a.n += b.n;
  return a;
}

// The bf16-product pointwise convolutions (pwbf.hip), called by skip.hip's
// mde_pointwise_* entry points for bf16 storage.
int pwbf_fwd(const bf16* x, const float* sc, const float* sh, const float* wt, bf16* y,
             float* stats, int64_t n, int64_t cin, int64_t cout, int64_t hw, int blocks,
             hipStream_t s);
int pwbf_bwd(const bf16* gy, const bf16* x, const float* sc, const float* sh, const float* mean,
             const float* wt, bf16* gs, float* slab, int64_t n, int64_t cin, int64_t cout,
             int64_t hw, int blocks, hipStream_t s);
bool pwbf_skip_ok(int64_t cin, int64_t cout);
int pwbf_skip_fwd(const bf16* r, const bf16* d, const float* sc, const float* sh, const float* wt,
                  const float* b, bf16* out, int64_t n, int64_t cin, int64_t cout, int64_t hw,
                  int blocks, hipStream_t s);
int pwbf_skip_bwd(const bf16* gy, const bf16* r, const bf16* d, const float* sc, const float* sh,
                  const float* mean, const float* wt, bf16* gs, float* slab, int64_t n,
                  int64_t cin, int64_t cout, int64_t hw, int blocks, hipStream_t s);

}  // namespace mde
