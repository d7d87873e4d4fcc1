// Device-side operand descriptors and helpers shared by the implicit-GEMM kernels.
#pragma once

#include <type_traits>

#include "common.h"

namespace selunet {

struct SrcArg {
  const void* data;
  const float* scale;
  const float* shift;
  int C;
  int relu;
  int layout;
  int pad;
};

struct GatherArg {
  int n, h, w;       // row grid
  int taps;          // 1, 4, 9
  int nsrc;
  int Ctot;          // C0 + C1
  int hs, ws;        // source grid
  int K;             // taps * Ctot (true K)
  int small;         // element-wise gather (channels not a multiple of the staging vector)
  int64_t M;
  SrcArg src[2];
};

// Select a source by a runtime index without indexing the kernel-argument array (a dynamic
// index forces the whole argument struct onto the scratch stack: ~200 B of scratch writes per
// thread, visible as WRITE_SIZE far above the output size).
__device__ __forceinline__ SrcArg pick_src(const GatherArg& g, int s) {
  SrcArg r;
  r.data = s ? g.src[1].data : g.src[0].data;
  r.scale = s ? g.src[1].scale : g.src[0].scale;
  r.shift = s ? g.src[1].shift : g.src[0].shift;
  r.C = s ? g.src[1].C : g.src[0].C;
  r.relu = s ? g.src[1].relu : g.src[0].relu;
  r.layout = s ? g.src[1].layout : g.src[0].layout;
  r.pad = 0;
  return r;
}

constexpr int BM = SELUNET_GEMM_BM;
constexpr int ROWB = 144;  // padded LDS row bytes for a 128-B K slice

// --------------------------------------------------------------------------- gather helpers
__device__ __forceinline__ void tap_offset(int taps, int tap, int& dy, int& dx) {
  if (taps == 9) {
    dy = tap / 3 - 1;
    dx = tap - (tap / 3) * 3 - 1;
  } else if (taps == 4) {
    dy = tap >> 1;
    dx = tap & 1;
  } else {
    dy = 0;
    dx = 0;
  }
}

// source pixel of row pixel (y, x) for `tap`; returns false when it falls into the zero pad.
__device__ __forceinline__ bool src_pixel(const GatherArg& g, int tap, int y, int x, int& ys, int& xs) {
  int dy, dx;
  tap_offset(g.taps, tap, dy, dx);
  if (g.taps == 4) {
    ys = 2 * y + dy;
    xs = 2 * x + dx;
    return true;
  }
  ys = y + dy;
  xs = x + dx;
  return (unsigned)ys < (unsigned)g.hs && (unsigned)xs < (unsigned)g.ws;
}

// Linear index (in the source grid) of the pixel that row m reads for `tap`, or -1 inside the
// zero pad. Pointwise operands need no decode; otherwise 32-bit division (M < 2^31 is checked
// on the host).
__device__ __forceinline__ int64_t src_index(const GatherArg& g, int64_t m, int tap) {
  if (g.taps == 1) return m;
  const unsigned mu = (unsigned)m;
  const unsigned x = mu % (unsigned)g.w, t = mu / (unsigned)g.w;
  const unsigned y = t % (unsigned)g.h, img = t / (unsigned)g.h;
  int ys, xs;
  if (!src_pixel(g, tap, (int)y, (int)x, ys, xs)) return -1;
  return ((int64_t)img * g.hs + ys) * g.ws + xs;
}

// One gathered element (slow path, small C / non-vector channel counts). Applies the transform.
template <typename T>
__device__ __forceinline__ float gather_scalar(const GatherArg& g, int64_t m, int k) {
  if (m >= g.M || k >= g.K) return 0.0f;
  const int tap = k / g.Ctot;
  int c = k - tap * g.Ctot;
  int s = 0;
  if (g.nsrc > 1 && c >= g.src[0].C) {
    c -= g.src[0].C;
    s = 1;
  }
  const int x = (int)(m % g.w);
  const int64_t t = m / g.w;
  const int y = (int)(t % g.h);
  const int img = (int)(t / g.h);
  int ys, xs;
  if (!src_pixel(g, tap, y, x, ys, xs)) return 0.0f;
  const SrcArg sa = pick_src(g, s);
  float v;
  if (sa.layout == 1) {
    v = reinterpret_cast<const float*>(sa.data)[(((int64_t)img * sa.C + c) * g.hs + ys) * g.ws + xs];
  } else {
    v = to_f(reinterpret_cast<const T*>(sa.data)[(((int64_t)img * g.hs + ys) * g.ws + xs) * sa.C + c]);
  }
  if (sa.scale) {
    v = v * sa.scale[c] + sa.shift[c];
    if (sa.relu) v = fmaxf(v, 0.0f);
  }
  return v;
}

// --------------------------------------------------------------------------- MFMA wrappers
template <typename T> struct Mma;
template <> struct Mma<float> {
  __device__ static inline void run(f32x16& acc, uint4 a, uint4 b) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
};
template <> struct Mma<__bf16> {
  __device__ static inline void run(f32x16& acc, uint4 a, uint4 b) {
    bf16x8 av = __builtin_bit_cast(bf16x8, a);
    bf16x8 bv = __builtin_bit_cast(bf16x8, b);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
  }
};

// apply folded BN + ReLU to a 16-B vector of T (E elements), channel base c
template <typename T>
__device__ __forceinline__ uint4 transform16(uint4 raw, const float* scale, const float* shift, int c, int relu) {
  constexpr int E = 16 / sizeof(T);
  T v[E];
  __builtin_memcpy(v, &raw, 16);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float f = to_f(v[e]) * scale[c + e] + shift[c + e];
    if (relu) f = fmaxf(f, 0.0f);
    v[e] = from_f<T>(f);
  }
  uint4 out;
  __builtin_memcpy(&out, v, 16);
  return out;
}

// =========================================================================== gemm_gather
struct BnBwdArg {
  const void* y;
  const float* scale;
  const float* shift;
  const float* mean;
  const float* invstd;
  float* slab;
};

struct EpiArg {
  void* out0;
  void* out1;
  const float* bias;
  float* stats;
  int mode;
  int split;
  float* colsum;
  BnBwdArg bnb;
  float* amax;  // nullable: atomic max of |stored value| (float bits), see selunet_epilogue.amax
  const float* stats_center;  // nullable: stats are sums of (v - center), (v - center)^2
};

typedef short s16x4 __attribute__((ext_vector_type(4)));

// Bijective remap of blockIdx.x so that consecutive logical blocks (which share operand tiles)
// run on the same XCD: the dispatcher deals blocks round-robin over the 8 XCDs, each with its own
// L2. Speed only, never correctness (MI355X guide T1, bijective form for nb % 8 != 0).
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned nb) {
  const unsigned xcd = b & 7u, q = nb >> 3, r = nb & 7u;
  const unsigned base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (b >> 3);
}

// --------------------------------------------------------------------------- LDS-staged epilogue
// Accumulators of the wave's MT x NT 32x32 subtiles (tile coords (wr0 + a*32, wc0 + b*32)) ->
// fp32 LDS tile [TR][TC + 4]. C/D layout of the 32x32 MFMAs: col = lane & 31,
// row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5).
template <int MT, int NT, int TC>
__device__ __forceinline__ void acc_to_lds(float* tile, const f32x16 (&acc)[MT][NT], int wr0, int wc0, int lane) {
  const int half = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        tile[(wr0 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * half) * (TC + 4) + wc0 + b * 32 + l32] = acc[a][b][r];
}

// Per-workgroup statistics an epilogue can produce while it stores its tile (all optional):
//  stats  [2][ld]      column sum / sum of squares of the fp32 values before the bias (BN forward);
//  colsum [ld_colsum]  column sums of the stored values for global columns < colsum_cols (SPLIT:
//                      the ConvTranspose2d bias gradient of out0's half);
//  bnb                 BN-backward sums [3][ld] of the stored values as dA (PLAIN): y is read at the
//                      element the value is stored to (same [M][N] layout), da = dA*[y*sc+sh > 0],
//                      sums (da, da*xhat, xhat); the pointers are offset to the tile's first column.
struct TileStats {
  float* stats;
  int ld;
  float* colsum;
  int colsum_cols;     // global column bound for colsum
  int gcol0;           // global column of tile column 0
  BnBwdArg bnb;        // scale/shift/mean/invstd/slab offset to gcol0; y = base pointer
  const void* out0;    // base of the PLAIN output (to locate y)
  float* amax;         // nullable: running max |stored value| (atomic, float bits)
  const float* center; // nullable: stats shift per column, offset to gcol0
};

// The statistics outputs of workgroup (slab row `row`, first global column n0) of an N-column GEMM.
__device__ __forceinline__ TileStats tile_stats(const EpiArg& ep, int64_t row, int n0, int N) {
  TileStats ts;
  ts.ld = N;
  ts.stats = ep.stats ? ep.stats + row * 2 * N + n0 : nullptr;
  ts.colsum = ep.colsum ? ep.colsum + row * ep.split + n0 : nullptr;
  ts.colsum_cols = ep.split;
  ts.gcol0 = n0;
  ts.bnb = ep.bnb;
  if (ep.bnb.slab) {
    ts.bnb.scale += n0;
    ts.bnb.shift += n0;
    ts.bnb.mean += n0;
    ts.bnb.invstd += n0;
    ts.bnb.slab += row * 3 * N + n0;
  }
  ts.out0 = ep.out0;
  ts.amax = ep.amax;
  ts.center = ep.stats_center ? ep.stats_center + n0 : nullptr;
  return ts;
}

// Accumulator type of the per-thread statistics a persistent workgroup carries across its tiles:
// double for fp32 operands — a workgroup folds hundreds of values per column into each thread's
// sums, and these sums (BN batch mean / E[y^2], the BN-backward sum of dA that becomes the bias
// gradient, ConvTranspose2d bias sums) are cancellation-prone: fp32 sequential accumulation put a
// 512x512 bias gradient 2.5e-3 off the reference where the reference's own spread is 1.5e-4 —
// and float for bf16 operands, whose rounding dominates anyway.
template <typename T> struct StatAcc { using type = float; };
template <> struct StatAcc<float> { using type = double; };

// Store the LDS tile as 8-column vectors (16 B bf16 / 32 B fp32): dst(row, col) returns the
// global address of tile element (row, col) (col a multiple of 8) or nullptr for a masked row.
// bias (nullable) is indexed by bias_col(col).
// The statistics of this tile are summed per thread in fp32 (a few rows) and added into the
// thread's s1/s2/s3 (8 columns each: the thread's column chunk is tid % (TC / 8) for every tile,
// so a persistent workgroup can accumulate over its tiles, in Acc precision) and reduced across the
// workgroup by tile_stats_flush.
template <typename T, int TR, int TC, int NTHREADS, typename Dst, typename BiasCol, typename Acc>
__device__ __forceinline__ void lds_tile_store_acc(float* tile, int tid, Dst&& dst, const float* bias,
                                                   BiasCol&& bias_col, const TileStats& ts, Acc (&s1)[8],
                                                   Acc (&s2)[8], Acc (&s3)[8], float& am) {
  constexpr int CC = TC / 8;            // 8-column chunks per row
  constexpr int RS = NTHREADS / CC;     // rows per pass
  // an opaque copy of tid: in a persistent kernel the column coefficients below are invariant over
  // its tile loop, and hoisting them out of it would pin ~40 VGPRs through the MFMA main loop
  asm volatile("" : "+v"(tid));
  const int cc = tid % CC, r0 = tid / CC;
  const int col = cc * 8;
  float bv[8], cen[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = bias ? bias[bias_col(col + e)] : 0.0f;
  const bool do_st = ts.stats != nullptr;
#pragma unroll
  for (int e = 0; e < 8; ++e) cen[e] = do_st && ts.center ? ts.center[col + e] : 0.0f;
  const bool do_cs = ts.colsum != nullptr && ts.gcol0 + col < ts.colsum_cols;
  const bool do_bn = ts.bnb.slab != nullptr;
  float sc[8], sh[8], mu[8], is[8];
  if (do_bn) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = ts.bnb.scale[col + e];
      sh[e] = ts.bnb.shift[col + e];
      mu[e] = ts.bnb.mean[col + e];
      is[e] = ts.bnb.invstd[col + e];
    }
  }
  // Retire the coefficient loads above before the row loop: on gfx9 stores share vmcnt with loads, and a
  // load still pending from before the loop makes the wait-count pass put s_waitcnt vmcnt(0) ahead of
  // every row (its loop-header merge cannot count the stores in between) — one store round trip per row.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt untouched
  // per-tile fp32 partials; with fp32 accumulators they are the accumulators themselves
  constexpr bool WIDE = !std::is_same<Acc, float>::value;
  float tw1[WIDE ? 8 : 1] = {}, tw2[WIDE ? 8 : 1] = {}, tw3[WIDE ? 8 : 1] = {};
  float* t1 = WIDE ? tw1 : reinterpret_cast<float*>(s1);
  float* t2 = WIDE ? tw2 : reinterpret_cast<float*>(s2);
  float* t3 = WIDE ? tw3 : reinterpret_cast<float*>(s3);
  // rows of this thread: r0, r0 + RS, ... (TR % RS == 0). With BN-backward sums, each batch of YB
  // rows loads its y before any of its stores (the stores may alias y as far as the compiler knows,
  // so a load between them waits one memory latency per row): 2-4 % on the 128-column data
  // gradients with 4 rows; the 64-column persistent conv spills with 4 and takes 2 (1 %)
  constexpr int NR = TR / RS;
  constexpr int YB = NR < (TC >= 128 ? 4 : 2) ? NR : (TC >= 128 ? 4 : 2);
  static_assert(TR % RS == 0 && NR % YB == 0, "epilogue rows must split evenly over the threads");
#pragma unroll 1
  for (int rb = 0; rb < NR; rb += YB) {
  T yb[YB][8];
  if (do_bn) {
#pragma unroll
    for (int j = 0; j < YB; ++j) {
      const T* p = dst(r0 + (rb + j) * RS, col);
      if (p == nullptr) continue;
      const T* yp = reinterpret_cast<const T*>(ts.bnb.y) + (p - reinterpret_cast<const T*>(ts.out0));
      if constexpr (sizeof(T) == 2) {
        const uint4 u = *reinterpret_cast<const uint4*>(yp);
        __builtin_memcpy(yb[j], &u, 16);
      } else {
        const f32x4 a = *reinterpret_cast<const f32x4*>(yp), b = *reinterpret_cast<const f32x4*>(yp + 4);
        __builtin_memcpy(yb[j], &a, 16);
        __builtin_memcpy(yb[j] + 4, &b, 16);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < YB; ++j) {
    const int row = r0 + (rb + j) * RS;
    T* p = dst(row, col);
    if (p == nullptr) continue;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(tile + row * (TC + 4) + col);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(tile + row * (TC + 4) + col + 4);
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if (do_st) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[e] - cen[e];
        t1[e] += d;
        t2[e] += d * d;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += bv[e];
    T o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = from_f<T>(v[e]);
    if (ts.amax) {
#pragma unroll
      for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(to_f(o[e])));
    }
    if constexpr (sizeof(T) == 2) {
      uint4 u;
      __builtin_memcpy(&u, o, 16);
      *reinterpret_cast<uint4*>(p) = u;
    } else {
      *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
    if (do_cs) {
#pragma unroll
      for (int e = 0; e < 8; ++e) t1[e] += to_f(o[e]);
    }
    if (do_bn) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float y = to_f(yb[j][e]);
        const float da = y * sc[e] + sh[e] > 0.0f ? to_f(o[e]) : 0.0f;
        const float xh = (y - mu[e]) * is[e];
        t1[e] += da;
        t2[e] += da * xh;
        t3[e] += xh;
      }
    }
  }
  }
  if constexpr (WIDE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] += (Acc)t1[e];
      s2[e] += (Acc)t2[e];
      s3[e] += (Acc)t3[e];
    }
  }
}

// LDS bytes tile_stats_flush needs for accumulators of type Acc
template <int TC, int NTHREADS, typename Acc>
constexpr int stats_flush_bytes() { return (NTHREADS / (TC / 8)) * TC * 3 * (int)sizeof(Acc); }

// Reduce the s1/s2/s3 accumulators of lds_tile_store_acc over the workgroup (LDS scratch `red`,
// stats_flush_bytes bytes; the caller has finished with whatever `red` held) and write the slab
// row (fp32).
template <int TC, int NTHREADS, typename Acc>
__device__ __forceinline__ void tile_stats_flush(float* red_f, int tid, const TileStats& ts, const Acc (&s1)[8],
                                                 const Acc (&s2)[8], const Acc (&s3)[8], float am) {
  constexpr int CC = TC / 8;
  constexpr int RS = NTHREADS / CC;
  Acc* red = reinterpret_cast<Acc*>(red_f);
  const int cc = tid % CC, r0 = tid / CC;
  const int col = cc * 8;
  const bool do_st = ts.stats != nullptr;
  const bool do_bn = ts.bnb.slab != nullptr;
  const int nst = do_bn ? 3 : (do_st ? 2 : 1);
  if (do_st || ts.colsum != nullptr || do_bn) {
    __syncthreads();  // everyone is done reading the tile: reuse it for the column reduction
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(r0 * TC + col + e) * 3 + 0] = s1[e];
      red[(r0 * TC + col + e) * 3 + 1] = s2[e];
      red[(r0 * TC + col + e) * 3 + 2] = s3[e];
    }
    __syncthreads();
    for (int i = tid; i < TC * nst; i += NTHREADS) {
      const int c = i % TC, k = i / TC;
      Acc a = 0;
      for (int r = 0; r < RS; ++r) a += red[(r * TC + c) * 3 + k];
      if (do_bn) ts.bnb.slab[k * ts.ld + c] = a;
      else if (do_st) ts.stats[k * ts.ld + c] = a;
      else if (ts.gcol0 + c < ts.colsum_cols) ts.colsum[c] = a;
    }
  }
  // the running max |stored value| of this thread's tiles: one atomic per workgroup (an atomic per tile
  // put 0.5M same-address atomics into a full-resolution launch; one per wave, a 25-50 us tail)
  if (ts.amax) block_amax(ts.amax, am, red_f);
}

template <typename T, int TR, int TC, int NTHREADS, typename Dst, typename BiasCol>
__device__ __forceinline__ void lds_tile_store(float* tile, int tid, Dst&& dst, const float* bias, BiasCol&& bias_col,
                                               const TileStats& ts) {
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float am = 0.0f;
  lds_tile_store_acc<T, TR, TC, NTHREADS>(tile, tid, dst, bias, bias_col, ts, s1, s2, s3, am);
  tile_stats_flush<TC, NTHREADS>(tile, tid, ts, s1, s2, s3, am);
}

// host: validate a C-ABI gather descriptor and convert it (gemm.hip)
int make_gather(const selunet_gather* a, int dtype, GatherArg& g, int vec_elems);

// 3x3 conv with the input tile + halo staged once per channel chunk (conv3x3.hip). Returns
// false when the operand is not eligible (caller falls back to the generic gather GEMM).
bool conv3x3_halo_eligible(const GatherArg& g, int N, int dtype);
int64_t conv3x3_halo_tiles(const GatherArg& g);
int64_t conv3x3_halo_stats_rows(const GatherArg& g, int N, int dtype);  // slab rows of the halo epilogue
bool conv3x3_halo_one_chunk(const GatherArg& g, int dtype);             // single chunk: the ONE_CHUNK kernel
bool conv3x3_halo_persistent(const GatherArg& g, int dtype);            // multi-chunk: persistent kernel
int conv3x3_halo_launch(const GatherArg& g, const void* b, int N, int k_pad, const EpiArg& ep, int dtype,
                        hipStream_t st);
// fp32 1-D Winograd F(2,3) forward / data gradient (conv3x3.hip, selunet_conv3x3_wino)
bool conv3x3_wino_shape_ok(int h, int w, int c_in, int c_src0, int n_cols);
bool conv3x3_wgrad_wino_eligible(const GatherArg& p, const GatherArg& q, int dtype);
int64_t conv3x3_wgrad_wino_splits(const GatherArg& p, const GatherArg& q, int64_t* per_out);
int conv3x3_wgrad_wino_launch(const GatherArg& p, const GatherArg& q, float* ws, int ldw, hipStream_t st);
bool conv3x3_wino_eligible(const GatherArg& g, int N);
bool conv3x3_wino_bn128(int N, const EpiArg& ep);
bool conv3x3_x2_bn128(int N, const EpiArg& ep);
int conv3x3_wino_launch(const GatherArg& g, const float* u, int N, const EpiArg& ep, hipStream_t st);
// fp32 forward / data gradient on split-fp16 operands (conv3x3.hip, selunet_conv3x3_x2)
bool conv3x3_x2_shape_ok(int h, int w, int c_in, int c_src0, int n_cols);
bool conv3x3_x2_eligible(const GatherArg& g, int N);
int conv3x3_x2_launch(const GatherArg& g, const float* w, int N, const EpiArg& ep, const float* amax0,
                      const float* amax1, hipStream_t st);
// ConvTranspose2d forward on split-fp16 operands with resident weights (convt.hip)
bool convt_x2_eligible(const GatherArg& g, int N, const EpiArg& e);
int convt_dgrad_x2_ntb(const GatherArg& g, int N);
int64_t convt_dgrad_x2_rows(const GatherArg& g, int N);
bool convt_dgrad_x2_eligible(const GatherArg& g, int N, const EpiArg& e);
int convt_dgrad_x2_launch(const GatherArg& g, const float* w, int N, const EpiArg& e, const float* amax_src,
                          hipStream_t st);
// the LDS-DMA ring form for K >= 256 and 256-column blocks (convt_ring.hip)
bool convt_ring_dgrad_operand_ok(const GatherArg& g, int N);
int64_t convt_ring_rows(const GatherArg& g, int N);
bool convt_ring_x2_takes(const GatherArg& g, int N, const EpiArg& e);
int convt_ring_x2_launch(const GatherArg& g, const float* w, int N, const EpiArg& e, const float* amax_src,
                         hipStream_t st);
bool convt_ring_bf16_dgrad_operand_ok(const GatherArg& g, int N);
bool convt_ring_bf16_takes(const GatherArg& g, int N, const EpiArg& e);
int convt_ring_bf16_launch(const GatherArg& g, const void* w, int N, const EpiArg& e, hipStream_t st);
int convt_bf16_fwd_ntb(const GatherArg& g, int N);  // bf16 resident-weight ConvTranspose2d (convt_bf16.hip)
int convt_dgrad_bf16_ntb(const GatherArg& g, int N);
int64_t convt_dgrad_bf16_rows(const GatherArg& g, int N);
bool convt_bf16_eligible(const GatherArg& g, int N, const EpiArg& e);
bool convt_dgrad_bf16_eligible(const GatherArg& g, int N, const EpiArg& e);
int convt_bf16_launch(const GatherArg& g, const void* w, int N, const EpiArg& e, hipStream_t st);
int convt_x2_launch(const GatherArg& g, const float* w, int N, const EpiArg& e, const float* amax_src,
                    hipStream_t st);
int64_t conv3x3_persist_rows(const GatherArg& g, int N);  // workgroup rows of the persistent 3x3 kernels
int conv3x3_persist_wgs();  // their workgroup target (selunet_set_halo_workgroups; default 256 = one per CU)
// the 64-column split-fp16 kernel, two 256-thread workgroups per CU (conv3x3_x2d.hip)
bool conv3x3_x2d_eligible(const GatherArg& g, int N);
int64_t conv3x3_x2d_rows(const GatherArg& g);
int conv3x3_x2d_launch(const GatherArg& g, const float* w, const EpiArg& ep, const float* amax0, const float* amax1,
                       hipStream_t st);
bool conv3x3_wgrad_halo_eligible(const GatherArg& p, const GatherArg& q, int dtype);
int64_t conv3x3_wgrad_x2_splits(const GatherArg& p, const GatherArg& q, int64_t* per_out, bool bn = false);
int conv3x3_wgrad_x2_bi(const GatherArg& p, bool bn);
// SELUNET_OPT_TILE_QUEUE and the split-fp16 persistent kernel's statistics slab rows (conv3x3.hip)
bool x2_tile_queue();
// the 128-column split-fp16 3x3 kernel with two 256-thread workgroups per CU (conv3x3_x2p.hip)
bool conv3x3_x2p_eligible(const GatherArg& g, int N);
int64_t conv3x3_x2p_rows(const GatherArg& g, int N);
int conv3x3_x2p_launch(const GatherArg& g, const float* w, int N, const EpiArg& ep, const float* amax0,
                       const float* amax1, hipStream_t st);
int64_t conv3x3_x2_persist_rows(const GatherArg& g, int N);
// the BN-backward apply fused into the split-fp16 weight gradient's dY staging (selunet_conv3x3_wgrad_x2_bn)
struct WgradBnArg {
  const float* y;
  const float* scale;
  const float* shift;
  const float* mean;
  const float* invstd;
  const float* coef;
  float* dy;
  float* dy_amax;
  int kind;             // SELUNET_DA_*: where dA comes from (selunet_da_source)
  int nh;               // HEADS: 1 or 3
  const float* pooled;  // POOL: [n][h/2][w/2][C]
  const float* skip;    // POOL: nullable [M][C]
  const float* hw;      // HEADS: [nh][64]
  const float* g0;      // HEADS: [M] planes
  const float* g1;
  const float* g2;
};
int conv3x3_wgrad_x2_launch(const GatherArg& p, const GatherArg& q, float* ws, int ldo, const float* amax_p,
                            const float* amax_q0, const float* amax_q1, hipStream_t st,
                            const WgradBnArg* bn = nullptr);
int conv3x3_wgrad_halo_launch(const GatherArg& p, const GatherArg& q, float* out, int ldo, float* ws, int dtype,
                              hipStream_t st);
int64_t conv3x3_wgrad_halo_splits(const GatherArg& p, const GatherArg& q, int dtype, int64_t* per_out);
bool halo_enabled();

}  // namespace selunet
