// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 per access width.
//
// MI355X_MICROARCH.md §HBM calibrates FETCH_SIZE (reports 1/2 of the bytes)
// and WRITE_SIZE (exact) for 16-byte-per-lane streaming accesses only and
// says other widths are uncalibrated.  Several kernels of this repo stream
// with 4- or 8-byte lanes (ssim3_l1, the depth loss, BN small-plane tables),
// so tools/pmc_traffic.py needs the factor for those widths too.  Each kernel
// here moves a known number of bytes once (1 GiB buffer: far beyond the 256
// MiB Infinity Cache) with W bytes per lane, fully coalesced, grid-stride:
//   read_w{4,8,16}   -- loads only (the sum is stored only if it equals an
//                       impossible value, so nothing is written)
//   write_w{4,8,16}  -- stores only
//   copy_w{4,16}     -- one load + one store per element
// Run:  rocprofv3 --pmc FETCH_SIZE -d DIR -o calib --output-format csv -- ./pmc_calib
// (and again with WRITE_SIZE); tools/pmc_calib.py turns the CSVs into factors.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int W>
struct Vec;
template <>
struct Vec<4> {
  using T = float;
};
template <>
struct Vec<8> {
  using T = float2;
};
template <>
struct Vec<16> {
  using T = float4;
};

__device__ inline float hsum(float v) { return v; }
__device__ inline float hsum(float2 v) { return v.x + v.y; }
__device__ inline float hsum(float4 v) { return v.x + v.y + v.z + v.w; }
__device__ inline void set(float& v, float a) { v = a; }
__device__ inline void set(float2& v, float a) { v = make_float2(a, a); }
__device__ inline void set(float4& v, float a) { v = make_float4(a, a, a, a); }

template <int W>
__global__ void __launch_bounds__(256) read_kernel(const typename Vec<W>::T* __restrict__ src,
                                                   size_t n, float* __restrict__ sink) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    acc += hsum(src[i]);
  if (acc == 1234567.0f) sink[threadIdx.x] = acc;  // never true for the fill below
}

template <int W>
__global__ void __launch_bounds__(256) write_kernel(typename Vec<W>::T* __restrict__ dst,
                                                    size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    typename Vec<W>::T t;
    set(t, v);
    dst[i] = t;
  }
}

template <int W>
__global__ void __launch_bounds__(256) copy_kernel(const typename Vec<W>::T* __restrict__ src,
                                                   typename Vec<W>::T* __restrict__ dst,
                                                   size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  char *a, *b;
  float* sink;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(a, 0, bytes));  // all zeros: the read sums stay 0
  CHECK(hipMemset(b, 0, bytes));
  const dim3 grid(256 * 8 * 4), block(256);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
#define RUN(name, launch, moved)                                                     \
  CHECK(hipEventRecord(e0));                                                         \
  launch;                                                                            \
  CHECK(hipEventRecord(e1));                                                         \
  CHECK(hipEventSynchronize(e1));                                                    \
  CHECK(hipEventElapsedTime(&ms, e0, e1));                                           \
  printf("%-9s rep %d: %.3f ms  %.1f GB/s  bytes %zu\n", name, rep, ms,              \
         (double)(moved) / (ms * 1e-3) / 1e9, (size_t)(moved));
    RUN("read_w4", (read_kernel<4><<<grid, block>>>((const float*)a, bytes / 4, sink)), bytes);
    RUN("read_w8", (read_kernel<8><<<grid, block>>>((const float2*)a, bytes / 8, sink)), bytes);
    RUN("read_w16", (read_kernel<16><<<grid, block>>>((const float4*)a, bytes / 16, sink)), bytes);
    RUN("write_w4", (write_kernel<4><<<grid, block>>>((float*)b, bytes / 4, 1.f)), bytes);
    RUN("write_w8", (write_kernel<8><<<grid, block>>>((float2*)b, bytes / 8, 1.f)), bytes);
    RUN("write_w16", (write_kernel<16><<<grid, block>>>((float4*)b, bytes / 16, 1.f)), bytes);
    RUN("copy_w4", (copy_kernel<4><<<grid, block>>>((const float*)a, (float*)b, bytes / 4)),
        2 * bytes);
    RUN("copy_w16",
        (copy_kernel<16><<<grid, block>>>((const float4*)a, (float4*)b, bytes / 16)),
        2 * bytes);
  }
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(sink));
  printf("done\n");
  return 0;
}
