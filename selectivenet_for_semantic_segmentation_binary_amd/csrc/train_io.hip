// Training-loop I/O kernels around the UNet_B step:
//
//  * selunet_prep_batch: pre-decoded uint8 NHWC patches + uint8 label masks -> the network input
//    (NCHW fp32, `Normalization` + `ToTensor`, utils/data_utils.py:94-106,160-168, with the
//    per-image `RandomFlip` of utils/data_utils.py:108-125) and the fp32 BCE target
//    (`label/255.0` truncated to uint8, utils/data_utils.py:220-221, then `.type(FloatTensor)`,
//    train.py:189-191). Replaces the host-side PIL decode + numpy transforms of the DataLoader.
//  * selunet_seg_metrics: the per-batch host metrics of train.py:211-238 / eval.py:218-246 —
//    prediction threshold, selection threshold, rejection count and the Evaluator's 2x2
//    confusion matrix (utils/compute_metric.py:10-26) — as integer counts accumulated on the
//    device, so the loop never copies the [N,H,W] outputs to the host.
//
// Both are HBM-bound byte/int work (no MFMA): 16-B coalesced loads, one pass over the data.
#include <algorithm>

#include "common.h"

namespace selunet {

constexpr int IO_TPB = 256;

// One thread per (image, row, 4-pixel group): reads 12 B of RGB + 4 B of label (the whole
// 4-pixel group), writes 3 x 16 B of NCHW planes + 16 B of target. Flips are applied on the
// READ side (output pixel (y, x) reads source (y', x')), so the stores stay contiguous.
// CIN = 2: input_type 'GH' (utils/data_utils.py:13-27, applied before Normalization at :223-224):
// channel 0 = cv2 RGB2GRAY of the [0,1] fp32 image (0.299 R + 0.587 G + 0.114 B), channel 1 = the
// hematoxylin stain of skimage.color.separate_stains(rgb, hed_from_rgb) (stains = (log(max(rgb,
// 1e-6)) / log(1e-6)) @ hed_from_rgb, clamped at 0; column 0 of inv(rgb_from_hed)) min-max
// normalised with the reference's constants -0.66781543 / 1.87798274.
constexpr double HED_H0 = 1.8779827368521353, HED_H1 = -0.06590806222356332, HED_H2 = -0.6019073634392891;
constexpr double GH_HMIN = -0.66781543, GH_HMAX = 1.87798274;

// HRGB (CIN = 3): input_type 'H_RGB' (utils/data_utils.py:29-41): the hematoxylin stain h of
// separate_stains as above, recombined alone by skimage.color.combine_stains(stack(h, 0, 0),
// rgb_from_hed) = clip(exp(-h * (-log 1e-6) * rgb_from_hed[0]), 0, 1), rgb_from_hed[0] =
// (0.65, 0.70, 0.29).
template <int CIN, bool HRGB = false>
__global__ void prep_batch_kernel(const uint8_t* __restrict__ img, const uint8_t* __restrict__ lab,
                                  const uint8_t* __restrict__ flips, int n, int h, int w, float* __restrict__ x,
                                  float* __restrict__ target) {
  const int wq = w >> 2;
  const int64_t total = (int64_t)n * h * wq;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int xq = (int)(i % wq);
    const int64_t r = i / wq;
    const int y = (int)(r % h);
    const int b = (int)(r / h);
    const int f = flips ? flips[b] : 0;
    const int ys = (f & 2) ? h - 1 - y : y;  // np.flipud (utils/data_utils.py:118-121)
    const int64_t src_row = ((int64_t)b * h + ys) * w;
    float xv[CIN][4];
    float tv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int xo = xq * 4 + j;
      const int xs = (f & 1) ? w - 1 - xo : xo;  // np.fliplr (utils/data_utils.py:113-116)
      const uint8_t* p = img + (src_row + xs) * 3;
      // input/255.0 in float64, astype(float32) (utils/data_utils.py:220-221)
      float v[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = (float)((double)p[c] / 255.0);
      if constexpr (HRGB) {
        const float la = logf(1e-6f);
        double st = 0.0;
        st += (double)(logf(fmaxf(v[0], 1e-6f)) / la) * HED_H0;
        st += (double)(logf(fmaxf(v[1], 1e-6f)) / la) * HED_H1;
        st += (double)(logf(fmaxf(v[2], 1e-6f)) / la) * HED_H2;
        const double h = fmax(st, 0.0) * -log(1e-6);
        const double rf[3] = {0.65, 0.70, 0.29};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float o = (float)fmin(fmax(exp(-h * rf[c]), 0.0), 1.0);
          xv[c][j] = (o - 0.5f) / 0.5f;
        }
      } else if constexpr (CIN == 3) {
        // (x - 0.5) / 0.5 in float32 (Normalization, utils/data_utils.py:101)
#pragma unroll
        for (int c = 0; c < 3; ++c) xv[c][j] = (v[c] - 0.5f) / 0.5f;
      } else {
        const float gray = v[0] * 0.299f + v[1] * 0.587f + v[2] * 0.114f;
        const float la = logf(1e-6f);
        double st = 0.0;
        st += (double)(logf(fmaxf(v[0], 1e-6f)) / la) * HED_H0;
        st += (double)(logf(fmaxf(v[1], 1e-6f)) / la) * HED_H1;
        st += (double)(logf(fmaxf(v[2], 1e-6f)) / la) * HED_H2;
        const float hn = (float)((fmax(st, 0.0) - GH_HMIN) / (GH_HMAX - GH_HMIN));
        xv[0][j] = (gray - 0.5f) / 0.5f;
        xv[1][j] = (hn - 0.5f) / 0.5f;
      }
      // (label/255.0).astype(uint8): truncation, so only 255 -> 1
      tv[j] = (float)(uint8_t)((double)lab[src_row + xs] / 255.0);
    }
    const int64_t plane = (int64_t)h * w;
    const int64_t o = (int64_t)y * w + xq * 4;
#pragma unroll
    for (int c = 0; c < CIN; ++c)
      *reinterpret_cast<f32x4*>(x + ((int64_t)b * CIN + c) * plane + o) = f32x4{xv[c][0], xv[c][1], xv[c][2], xv[c][3]};
    *reinterpret_cast<f32x4*>(target + (int64_t)b * plane + o) = f32x4{tv[0], tv[1], tv[2], tv[3]};
  }
}

// counts[0..3] = confusion matrix cm[label][pred] over the counted pixels (row-major, as
// Evaluator.confusion_matrix), counts[4] = selected pixels, counts[5] = all pixels (label.size).
// A pixel is counted iff 0 <= label < 2 and (no selection head or sel >= t_sel).
// pred = out >= t_out: t_out / t_sel are the smallest fp32 logits the reference's host rule maps
// to 1 (computed once on the host from the same numpy expression, see metrics.py).
__global__ void seg_metrics_kernel(const float* __restrict__ out, const float* __restrict__ sel,
                                   const float* __restrict__ target, int64_t p, float t_out, float t_sel,
                                   unsigned long long* __restrict__ counts) {
  unsigned c[5] = {0, 0, 0, 0, 0};
  const int64_t p4 = p >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto one = [&](float o, float s, float t) {
    // label.astype('uint8') of a {0,1} float target (train.py:206; eval.py:229)
    const int lab = (int)(uint8_t)t;
    const bool selected = sel == nullptr || s >= t_sel;
    c[4] += selected;
    if (selected && lab < 2) c[lab * 2 + (o >= t_out ? 1 : 0)] += 1;
  };
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < p4; i += stride) {
    const f32x4 o = *reinterpret_cast<const f32x4*>(out + i * 4);
    const f32x4 t = *reinterpret_cast<const f32x4*>(target + i * 4);
    const f32x4 s = sel ? *reinterpret_cast<const f32x4*>(sel + i * 4) : f32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) one(o[j], s[j], t[j]);
  }
  for (int64_t i = p4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < p; i += stride)
    one(out[i], sel ? sel[i] : 0.0f, target[i]);
  __shared__ unsigned red[IO_TPB / 64][5];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    unsigned v = c[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wave][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    unsigned long long s = 0;
    for (int wv = 0; wv < IO_TPB / 64; ++wv) s += red[wv][threadIdx.x];
    atomicAdd(counts + threadIdx.x, s);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(counts + 5, (unsigned long long)p);
}

}  // namespace selunet

using namespace selunet;

extern "C" {

int selunet_prep_batch_mode(const uint8_t* img, const uint8_t* lab, const uint8_t* flips, int32_t n, int32_t h,
                            int32_t w, int32_t mode, float* x, float* target, void* stream) {
  SELUNET_REQUIRE(mode >= 0 && mode <= 2, "prep_batch_mode: mode 0 'RGB', 1 'GH', 2 'H_RGB' (got %d)", mode);
  if (mode != 2) return selunet_prep_batch(img, lab, flips, n, h, w, mode == 0 ? 3 : 2, x, target, stream);
  SELUNET_REQUIRE(img && lab && x && target && n > 0 && h > 0 && w > 0 && w % 4 == 0, "prep_batch: bad arguments");
  SELUNET_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)target & 15) == 0, "prep_batch: outputs must be 16-B aligned");
  const int64_t total = (int64_t)n * h * (w / 4);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(total, IO_TPB), 8192));
  hipLaunchKernelGGL((prep_batch_kernel<3, true>), dim3(grid), dim3(IO_TPB), 0, as_stream(stream), img, lab, flips, n, h,
                     w, x, target);
  return check_launch("prep_batch");
}

int selunet_prep_batch(const uint8_t* img, const uint8_t* lab, const uint8_t* flips, int32_t n, int32_t h, int32_t w,
                       int32_t cin, float* x, float* target, void* stream) {
  SELUNET_REQUIRE(img && lab && x && target && n > 0 && h > 0 && w > 0, "prep_batch: bad arguments");
  SELUNET_REQUIRE(cin == 3 || cin == 2, "prep_batch: cin 3 (input_type 'RGB') or 2 ('GH', utils/data_utils.py:223-224)");
  SELUNET_REQUIRE(w % 4 == 0, "prep_batch: width must be a multiple of 4");
  SELUNET_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)target & 15) == 0, "prep_batch: outputs must be 16-B aligned");
  const int64_t total = (int64_t)n * h * (w / 4);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(total, IO_TPB), 8192));
  hipLaunchKernelGGL(cin == 3 ? prep_batch_kernel<3> : prep_batch_kernel<2>, dim3(grid), dim3(IO_TPB), 0,
                     as_stream(stream), img, lab, flips, n, h, w, x, target);
  return check_launch("prep_batch");
}

int selunet_seg_metrics(const float* out, const float* sel, const float* target, int64_t p, float t_out, float t_sel,
                        unsigned long long* counts, void* stream) {
  SELUNET_REQUIRE(out && target && counts && p > 0, "seg_metrics: bad arguments");
  SELUNET_REQUIRE(((uintptr_t)out & 15) == 0 && ((uintptr_t)target & 15) == 0 && ((uintptr_t)sel & 15) == 0,
                  "seg_metrics: inputs must be 16-B aligned");
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(p / 4 + 1, IO_TPB), 2048));
  hipLaunchKernelGGL(seg_metrics_kernel, dim3(grid), dim3(IO_TPB), 0, as_stream(stream), out, sel, target, p, t_out,
                     t_sel, counts);
  return check_launch("seg_metrics");
}

}  // extern "C"
