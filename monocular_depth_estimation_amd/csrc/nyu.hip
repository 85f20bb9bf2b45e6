// NYU-Depth-V2 batch augmentation + tensor conversion on the GPU (SURVEY
// §8(f) rank 1, the data pipeline).
//
// Replaces the per-sample host transforms of src/data.py:157-168 --
// RandomHorizontalFlip (:16-31), RandomChannelSwap (:33-46) and ToTensor
// (:100-155) -- for a whole batch at once: the host decodes PNG/JPEG to
// uint8 (PIL, loader workers) and uploads 4 bytes per pixel instead of 16;
// one kernel applies each sample's flip / channel permutation (decided on the
// host with the reference's `random` draws) and writes the fp32 NCHW tensors
// the model and the loss take:
//   image[n, c, y, x] = img[n, y, fx(x), perm_n[c]] / 255     (HWC uint8 in)
//   depth[n, 0, y, x] = dep[n, y, fx(x)] (/ 255 for 8-bit)
// with fx(x) = W-1-x for a flipped sample, perm_n = permutations(range(3))[k]
// (k = -1: identity).  8-bit 'L' depth PNGs take ToTensor's ByteTensor path
// (.float().div(255)); 16-bit 'I;16' ones its integer path (np.int16 view,
// .float(), no scaling).  Divisions are IEEE fp32 like ATen's: bit-exact.
// Algorithmic HBM bytes: 4-5 in + 16 out per RGB-D pixel.

#include "common.h"

namespace {

// itertools.permutations(range(3), 3), in its order
__constant__ int kPerm[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};

// One block per (sample, row); threads over columns.
template <typename DT, bool DIV>
__global__ void __launch_bounds__(256)
    nyu_augment_kernel(const uint8_t* __restrict__ img, const DT* __restrict__ dep,
                       const int32_t* __restrict__ flags, float* __restrict__ img_out,
                       float* __restrict__ dep_out, int h, int w, int dh, int dw) {
  const int n = blockIdx.y, y = blockIdx.x;
  const int flip = flags[2 * n], k = flags[2 * n + 1];
  const int p0 = k >= 0 ? kPerm[k][0] : 0, p1 = k >= 0 ? kPerm[k][1] : 1,
            p2 = k >= 0 ? kPerm[k][2] : 2;
  if (y < h) {
    const uint8_t* src = img + ((int64_t)n * h + y) * w * 3;
    const int64_t plane = (int64_t)h * w;
    float* o = img_out + (int64_t)n * 3 * plane + (int64_t)y * w;
    for (int x = threadIdx.x; x < w; x += 256) {
      const uint8_t* px = src + 3 * (flip ? w - 1 - x : x);
      o[x] = (float)px[p0] / 255.f;
      o[plane + x] = (float)px[p1] / 255.f;
      o[2 * plane + x] = (float)px[p2] / 255.f;
    }
  }
  if (y < dh) {
    const DT* src = dep + ((int64_t)n * dh + y) * dw;
    float* o = dep_out + ((int64_t)n * dh + y) * dw;
    for (int x = threadIdx.x; x < dw; x += 256) {
      const float v = (float)src[flip ? dw - 1 - x : x];
      o[x] = DIV ? v / 255.f : v;
    }
  }
}

}  // namespace

extern "C" {

int mde_nyu_augment(const void* image, const void* depth, const int32_t* flags, float* image_out,
                    float* depth_out, int64_t n, int64_t h, int64_t w, int64_t dh, int64_t dw,
                    int depth_bits, void* stream) {
  if (!image || !depth || !flags || !image_out || !depth_out || n <= 0 || h <= 0 || w <= 0 ||
      dh <= 0 || dw <= 0 || n > 65535 || h > (1 << 20) || dh > (1 << 20) ||
      (depth_bits != 8 && depth_bits != 16) || n * 3 * h * w >= ((int64_t)1 << 40))
    return MDE_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(h > dh ? h : dh), (unsigned)n);
  const double bytes = (double)n * (h * w * (3.0 + 12.0) + dh * dw * (depth_bits / 8.0 + 4.0));
  if (depth_bits == 8)
    MDE_LAUNCH(mde::K_NYU_AUGMENT, bytes, st, (nyu_augment_kernel<uint8_t, true>), grid,
               dim3(256), 0, (const uint8_t*)image, (const uint8_t*)depth, flags, image_out,
               depth_out, (int)h, (int)w, (int)dh, (int)dw);
  else
    MDE_LAUNCH(mde::K_NYU_AUGMENT, bytes, st, (nyu_augment_kernel<int16_t, false>), grid,
               dim3(256), 0, (const uint8_t*)image, (const int16_t*)depth, flags, image_out,
               depth_out, (int)h, (int)w, (int)dh, (int)dw);
  return MDE_OK;
}

}  // extern "C"
