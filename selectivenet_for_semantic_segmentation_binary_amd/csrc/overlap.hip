// One-GPU stand-in for a bucketed RCCL all-reduce kernel.
//
// RCCL's ring all-reduce runs one workgroup per channel; each workgroup reduce-copies its slice of
// the bucket (peer data + local data -> send / local buffer) and spins on peer flags while the
// other ranks catch up, so it holds its CUs for the whole collective. cu_hold_kernel reproduces
// that occupancy on one GPU: n_wg workgroups of 256 threads reduce-copy dst[i] = src[i] + dst[i]
// over their slice of a bucket-sized buffer, repeatedly, until `ticks` of the GPU wall clock have
// passed since the workgroup started. Issued on a side stream at the points GradBucketer launches
// its all-reduces, it measures how much a concurrent CU-holding kernel stretches the backward
// (tools/overlap_emulation.py). Bench / tool use only: the training path never calls it.
#include "common.h"

namespace selunet {
namespace {

constexpr int HOLD_TPB = 256;

__global__ void __launch_bounds__(HOLD_TPB) cu_hold_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                           int64_t n4, int64_t ticks) {
  const uint64_t t0 = wall_clock64();
  const int64_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = lo + per < n4 ? lo + per : n4;
  do {
    for (int64_t i = lo + threadIdx.x; i < hi; i += HOLD_TPB) {
      const float4 a = src[i];
      float4 b = dst[i];
      b.x += a.x;
      b.y += a.y;
      b.z += a.z;
      b.w += a.w;
      dst[i] = b;
    }
  } while ((int64_t)(wall_clock64() - t0) < ticks);
}

int wall_clock_khz() {
  static int khz = 0;
  if (khz == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
      khz = 100000;  // the 100 MHz constant clock of CDNA parts
  }
  return khz;
}

}  // namespace
}  // namespace selunet

using namespace selunet;

extern "C" {

int selunet_cu_hold(const float* src, float* dst, int64_t n, int32_t n_wg, float us, void* stream) {
  SELUNET_REQUIRE(src && dst && n > 0 && n % 4 == 0, "cu_hold: src, dst and n (a multiple of 4) required");
  SELUNET_REQUIRE(n_wg > 0 && n_wg <= 4096, "cu_hold: n_wg in [1, 4096] (got %d)", n_wg);
  SELUNET_REQUIRE(us >= 0.0f && us <= 1.0e5f, "cu_hold: us in [0, 1e5] (got %g)", (double)us);
  SELUNET_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "cu_hold: buffers must be 16-B aligned");
  const int64_t ticks = (int64_t)((double)us * wall_clock_khz() / 1000.0);
  hipLaunchKernelGGL(cu_hold_kernel, dim3(n_wg), dim3(HOLD_TPB), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst), n / 4, ticks);
  return check_launch("cu_hold");
}

}  // extern "C"
