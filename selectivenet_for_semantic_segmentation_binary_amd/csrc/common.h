// Shared device/host helpers for the gfx950 SelectiveUNet_B kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/selunet.h"

namespace selunet {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ error state (host)
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);

#define SELUNET_REQUIRE(cond, ...)                         \
  do {                                                     \
    if (!(cond)) return ::selunet::fail(SELUNET_EINVAL, __VA_ARGS__); \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------ options (host)
// Kernel-selection and tuning options (selunet_option in selunet.h), set only through
// selunet_set_option: the library reads no environment variables. Values < 0 mean "default".
extern int64_t g_options[SELUNET_OPT_COUNT];
inline int64_t option(int key, int64_t dflt) { return g_options[key] < 0 ? dflt : g_options[key]; }
// allocates the SELUNET_OPT_TILE_QUEUE ticket counters on the current device (conv3x3.hip); 0 on success
int x2_tile_queue_prepare();

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ------------------------------------------------------------------ element access
// 4 consecutive elements <-> float4 in registers.
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  __device__ static inline f32x4 load(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
  __device__ static inline void store(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
};
template <> struct Vec4<__bf16> {
  __device__ static inline f32x4 load(const __bf16* p) {
    bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  }
  __device__ static inline void store(__bf16* p, f32x4 v) {
    bf16x4 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    *reinterpret_cast<bf16x4*>(p) = o;
  }
};

template <typename T> __device__ inline float to_f(T v) { return (float)v; }
template <typename T> __device__ inline T from_f(float v) { return (T)v; }

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }
// numerically stable softplus(x) = log(1 + exp(x))
__device__ __forceinline__ float softplusf_(float x) { return fmaxf(x, 0.0f) + log1pf(__expf(-fabsf(x))); }

// wave64 sum
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// *amax = max(*amax, wave max of v >= 0) as one atomic per wave on the float bits (non-negative
// floats order like their bit patterns; a NaN propagates as the largest). Every lane calls it.
__device__ __forceinline__ void atomic_amax(float* amax, float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned*>(amax), __float_as_uint(v));
}

// The same as one atomic per workgroup. Same-address device atomics from all XCDs serialize at
// ~12 ns each (measured: a 4096-block BN-backward apply took 0.19 ms at any size with one atomic per
// wave), and they cluster at the end of a launch, so a wave-per-atomic tail costs 25-50 us per launch.
// Every thread of the workgroup calls it; scratch: >= blockDim.x / 64 floats of LDS the caller is
// done with (the first barrier waits for every wave's last use of it).
__device__ __forceinline__ void block_amax(float* amax, float v, float* scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (int)(blockDim.x >> 6);
    for (int w = 1; w < nw; ++w) v = fmaxf(v, scratch[w]);
    atomicMax(reinterpret_cast<unsigned*>(amax), __float_as_uint(v));
  }
}

// Power-of-two scale 2^e of a split-fp16 operand whose magnitudes are bounded by amax:
// amax * 2^e < 2^14, so the high part fp16(v * 2^e) and the low part fp16(v * 2^e - high) stay far
// below the fp16 maximum (65504) while small values keep their bits above the fp16 subnormal floor.
// amax = 0 (an all-zero operand) gives 2^14. unscale (nullable) receives 2^-e.
__device__ __forceinline__ float x2_scale(float amax, float* unscale) {
  int e = 0;
  if (amax > 0.0f) frexpf(amax, &e);  // amax < 2^e
  e = min(max(14 - e, -100), 100);
  if (unscale) *unscale = ldexpf(1.0f, -e);
  return ldexpf(1.0f, e);
}

// v -> (high, low) fp16 parts of v (already scaled): v = high + low to 22 significant bits
__device__ __forceinline__ void x2_split(float v, _Float16& h, _Float16& l) {
  h = (_Float16)v;
  l = (_Float16)(v - (float)h);
}

}  // namespace selunet
