// First CBR block's convolution (encoder_layer_1_1, model.py:29: C_in = 3 for RGB, 2 for GH
// input, model.py:24-27) read straight from the network's NCHW fp32 input.
//
// Forward: a 16x16-pixel tile per workgroup; the (18x18) x C_in input halo is staged in LDS and
// every thread builds its pixel's im2col row (K = 9*C_in <= 27, zero padded to 32) in LDS; one
// MFMA K-pass against the 64x32 weight tile; the LDS-staged epilogue writes y and the BatchNorm
// column statistics like every other conv. Replaces an im2col pass through HBM (a 64-column
// bf16 operand: 1 GB at bs=128) and the GEMM that re-read it.
//
// Weight gradient: dW[co][k] = sum_p dY[p][co] * im2col(x)[p][k]. Each workgroup walks a range of
// pixel tiles; per tile the threads write dY and the im2col rows TRANSPOSED into LDS ([co][pixel],
// [k][pixel]) so the MFMA's reduction dimension (pixels) is contiguous for both operands. The next
// tile's dY and input are loaded while the current one is multiplied. Per-workgroup partial sums
// go to a slab reduced deterministically in fp64 (selunet_reduce_rows).
#include "gemm_common.h"

namespace selunet {

constexpr int FK = 32;                  // padded K of the first layer (9 * C_in <= 27)
constexpr int FCO = 64;                 // output channels of encoder_layer_1_1 (model.py:29)
constexpr int FT = 16;                  // pixel tile edge
constexpr int FH = FT + 2;              // halo edge
constexpr int FPIX = FT * FT;           // 256 pixels per tile
constexpr int FTHREADS = 256;

__device__ __forceinline__ void tile_coords(unsigned t, int tiles_x, int tiles_y, int& img, int& y0, int& x0) {
  const unsigned r = t / (unsigned)tiles_x;
  x0 = (int)(t - r * (unsigned)tiles_x) * FT;
  const unsigned im = r / (unsigned)tiles_y;
  y0 = (int)(r - im * (unsigned)tiles_y) * FT;
  img = (int)im;
}

template <typename T>
__global__ void __launch_bounds__(FTHREADS, 3)
first_conv_fwd_kernel(const float* __restrict__ x, int cin, int h, int w, const T* __restrict__ wp, EpiArg ep,
                      int tiles_x, int tiles_y, int total_tiles) {
  constexpr int RB = FK * (int)sizeof(T) + 16;  // LDS row bytes (conflict-free 16-row fragment reads)
  constexpr int XR = (3 * FH * FH + FTHREADS - 1) / FTHREADS;  // halo values per thread
  // [ A rows | input halo | weights, staged once | per-wave statistics ]: 50 KB, three workgroups per
  // CU (the accumulators are stored straight from registers: no LDS epilogue tile)
  __shared__ __attribute__((aligned(16))) unsigned char smem[FPIX * RB + 3 * FH * FH * 4 + FCO * RB];
  __shared__ float red[4][2][FCO];
  unsigned char* As = smem;
  float* Xs = reinterpret_cast<float*>(smem + FPIX * RB);
  unsigned char* Bs = smem + FPIX * RB + 3 * FH * FH * 4;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  // persistent: tiles b, b + grid, ... (b XCD-remapped so neighbouring tiles share an L2)
  const unsigned b0 = xcd_remap(blockIdx.x, gridDim.x);

  // the halo of a tile, loaded unconditionally (clamped) into registers one tile ahead
  struct Halo {
    float v[XR];
  };
  auto load_halo = [&](int t) __attribute__((always_inline)) {
    Halo hv;
    int img, y0, x0;
    tile_coords((unsigned)t, tiles_x, tiles_y, img, y0, x0);
#pragma unroll
    for (int r = 0; r < XR; ++r) {
      const int i = min(r * FTHREADS + tid, cin * FH * FH - 1);
      const int c = i / (FH * FH), rr = i - c * (FH * FH);
      const int ys = min(max(y0 - 1 + rr / FH, 0), h - 1), xs = min(max(x0 - 1 + rr % FH, 0), w - 1);
      hv.v[r] = x[(((int64_t)img * cin + c) * h + ys) * w + xs];
    }
    return hv;
  };
  constexpr int WV = FK * (int)sizeof(T) / 16;  // 16-B vectors per weight row
  for (int i = tid; i < FCO * WV; i += FTHREADS) {
    const int row = i / WV, v = i - row * WV;
    *reinterpret_cast<uint4*>(Bs + row * RB + v * 16) =
        *reinterpret_cast<const uint4*>(wp + row * FK + v * (16 / sizeof(T)));
  }
  // this lane's two output columns (32x32 C layout: column lane & 31 of subtile b), their bias and
  // statistics shift
  float bias[2], cen[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    bias[b] = ep.bias ? ep.bias[b * 32 + l32] : 0.0f;
    cen[b] = ep.stats_center ? ep.stats_center[b * 32 + l32] : 0.0f;
  }

  int t = (int)b0;
  Halo cur = load_halo(t < total_tiles ? t : 0);
  for (; t < total_tiles; t += gridDim.x) {
    int img, y0, x0;
    tile_coords((unsigned)t, tiles_x, tiles_y, img, y0, x0);
#pragma unroll
    for (int r = 0; r < XR; ++r) {
      const int i = r * FTHREADS + tid;
      if (i < cin * FH * FH) {
        const int c = i / (FH * FH), rr = i - c * (FH * FH);
        const int ys = y0 - 1 + rr / FH, xs = x0 - 1 + rr % FH;
        Xs[i] = ((unsigned)ys < (unsigned)h && (unsigned)xs < (unsigned)w) ? cur.v[r] : 0.0f;
      }
    }
    const int tn = t + (int)gridDim.x;
    cur = load_halo(tn < total_tiles ? tn : t);  // next tile's input, in flight during this one
    __syncthreads();
    {
      const int py = tid / FT, px = tid % FT;
      T row[FK];
#pragma unroll
      for (int k = 0; k < FK; ++k) {
        float v = 0.0f;
        if (k < 9 * cin) {
          const int tap = k / cin, c = k - tap * cin;
          v = Xs[(c * FH + py + tap / 3) * FH + px + tap % 3];
        }
        row[k] = from_f<T>(v);
      }
#pragma unroll
      for (int v = 0; v < WV; ++v) {
        uint4 u;
        __builtin_memcpy(&u, reinterpret_cast<const unsigned char*>(row) + v * 16, 16);
        *reinterpret_cast<uint4*>(As + tid * RB + v * 16) = u;
      }
    }
    __syncthreads();

    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
#pragma unroll
    for (int q = 0; q < FK * (int)sizeof(T) / 32; ++q) {
      const int boff = q * 32 + half * 16;
      uint4 af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) af[a] = *reinterpret_cast<const uint4*>(As + (wave * 64 + a * 32 + l32) * RB + boff);
#pragma unroll
      for (int b = 0; b < 2; ++b) bfr[b] = *reinterpret_cast<const uint4*>(Bs + (b * 32 + l32) * RB + boff);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) Mma<T>::run(acc[a][b], af[a], bfr[b]);
    }

    // epilogue from registers: y (+ bias) at pixel (wave*64 + a*32 + row, column b*32 + l32) — one
    // accumulator register is two 128-B runs (fp32) — and the tile's column statistics of the values
    // before the bias (shifted by stats_center), summed over the lane's rows, its partner half-wave's
    // and the four waves
    float t1[2] = {0.f, 0.f}, t2[2] = {0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pix = wave * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        const int y = y0 + pix / FT, xx = x0 + pix % FT;
        if (y >= h || xx >= w) continue;
        T* dst = reinterpret_cast<T*>(ep.out0) + (((int64_t)img * h + y) * w + xx) * FCO;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const float v = acc[a][b][r];
          dst[b * 32 + l32] = from_f<T>(v + bias[b]);
          const float d = v - cen[b];
          t1[b] += d;
          t2[b] += d * d;
        }
      }
    if (ep.stats) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        t1[b] += __shfl_xor(t1[b], 32, 64);
        t2[b] += __shfl_xor(t2[b], 32, 64);
        if (half == 0) {
          red[wave][0][b * 32 + l32] = t1[b];
          red[wave][1][b * 32 + l32] = t2[b];
        }
      }
    }
    __syncthreads();  // statistics in LDS; A rows / halo free for the next tile
    if (ep.stats && tid < 2 * FCO) {
      const int s2 = tid / FCO, c = tid - s2 * FCO;
      ep.stats[((int64_t)t * 2 + s2) * FCO + c] = red[0][s2][c] + red[1][s2][c] + red[2][s2][c] + red[3][s2][c];
    }
  }
}

// ---------------------------------------------------------------------------------- wgrad
// BNA: the layer's BatchNorm+ReLU backward applied while staging — the kernel reads dA (`dy`) and the
// layer's conv output y and forms dy = (y sc + sh > 0 ? k0 dA : 0) - b - a y as selunet_bn_bwd_apply
// does (its coefficients from coef / invstd / mean), so encoder_layer_1_1's dy, which nothing else
// reads, is never written: one read pass of dA and y instead of apply (read both, write dy) + read dy.
struct FirstBnApply {
  const void* y;
  const float* scale;
  const float* shift;
  const float* mean;
  const float* invstd;
  const float* coef;  // [3][64] k0, k1, k2 (selunet_bn_bwd_stats_finalize)
};

template <typename T, bool BNA = false>
__global__ void __launch_bounds__(FTHREADS, 3)
first_conv_wgrad_kernel(const float* __restrict__ x, int cin, int h, int w, const T* __restrict__ dy, float* slab,
                        int tiles_x, int tiles_y, int total_tiles, int tiles_per_block, FirstBnApply bna) {
  // a tile runs as four stages of HP = 64 pixels (four tile rows each): 31 KB of LDS and 132 VGPRs
  // (fp32, BN-backward fused), three workgroups per CU. Two 128-pixel stages (54 KB, 188 VGPRs: the
  // next stage's dA and y held across the transform) ran two per CU; a whole-tile stage (104 KB) one
  constexpr int NS = 4;                          // stages per tile
  constexpr int HP = FPIX / NS;
  constexpr int PB = HP * (int)sizeof(T) + 16;  // transposed row bytes (64 pixels + pad)
  constexpr int E = 16 / (int)sizeof(T);
  constexpr int CH = FCO / NS;                   // dY channels per thread: four threads per pixel
  constexpr int DV = CH / E;                     // 16-B vectors per thread and stage
  constexpr int XR = (3 * FH * FH + FTHREADS - 1) / FTHREADS;
  __shared__ __attribute__((aligned(16))) unsigned char smem[FCO * PB + FK * PB + 3 * FH * FH * 4 + (BNA ? 5 * FCO * 4 : 0)];
  unsigned char* Ds = smem;                        // [64 co][128 px]
  unsigned char* Cs = smem + FCO * PB;             // [32 k][128 px]
  float* Xs = reinterpret_cast<float*>(Cs + FK * PB);
  float* Kc = Xs + 3 * FH * FH;                    // BNA: [5][64] sc, sh, k0, a, b

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int wa = wave & 1, wp = wave >> 1;  // co subtile, 32-pixel half of the stage
  const int sp = tid % HP, hc = tid / HP;   // staging: stage pixel, channel (dY) / k (columns) quarter
  const int tb = blockIdx.x * tiles_per_block;
  const int te = min(total_tiles, tb + tiles_per_block);

  struct Loaded {
    uint4 d[DV];
    uint4 yv[BNA ? DV : 1];
    float xh[XR];
  };
  // job j = (tile tb + j / NS, stage j % NS): this thread's dY channels of its pixel, and at stage 0
  // the tile's input halo
  auto load = [&](int j) __attribute__((always_inline)) {
    Loaded L;
    const int t = tb + j / NS, st = j % NS;
    int img, y0, x0;
    tile_coords((unsigned)t, tiles_x, tiles_y, img, y0, x0);
    const int pix = st * HP + sp;
    const int y = min(y0 + pix / FT, h - 1), xx = min(x0 + pix % FT, w - 1);
    const T* src = dy + (((int64_t)img * h + y) * w + xx) * FCO + hc * CH;
#pragma unroll
    for (int v = 0; v < DV; ++v) L.d[v] = *reinterpret_cast<const uint4*>(src + v * E);
    if constexpr (BNA) {
      const T* ysrc = reinterpret_cast<const T*>(bna.y) + (((int64_t)img * h + y) * w + xx) * FCO + hc * CH;
#pragma unroll
      for (int v = 0; v < DV; ++v) L.yv[v] = *reinterpret_cast<const uint4*>(ysrc + v * E);
    }
    if (st == 0) {
#pragma unroll
      for (int r = 0; r < XR; ++r) {
        const int i = min(r * FTHREADS + tid, cin * FH * FH - 1);
        const int c = i / (FH * FH), rr = i - c * (FH * FH);
        const int ys = min(max(y0 - 1 + rr / FH, 0), h - 1), xs = min(max(x0 - 1 + rr % FH, 0), w - 1);
        L.xh[r] = x[(((int64_t)img * cin + c) * h + ys) * w + xs];
      }
    }
    return L;
  };
  auto stage = [&](const Loaded& L, int j) __attribute__((always_inline)) {
    const int t = tb + j / NS, st = j % NS;
    int img, y0, x0;
    tile_coords((unsigned)t, tiles_x, tiles_y, img, y0, x0);
    if (st == 0) {
#pragma unroll
      for (int r = 0; r < XR; ++r) {
        const int i = r * FTHREADS + tid;
        if (i < cin * FH * FH) {
          const int c = i / (FH * FH), rr = i - c * (FH * FH);
          const int ys = y0 - 1 + rr / FH, xs = x0 - 1 + rr % FH;
          Xs[i] = ((unsigned)ys < (unsigned)h && (unsigned)xs < (unsigned)w) ? L.xh[r] : 0.0f;
        }
      }
    }
    // this thread's dY channels of stage pixel sp, transposed (a pixel outside the image contributes
    // nothing)
    const int pix = st * HP + sp;
    const bool inside = y0 + pix / FT < h && x0 + pix % FT < w;
    T* dcol = reinterpret_cast<T*>(Ds) + sp;
#pragma unroll
    for (int v = 0; v < DV; ++v) {
      T e[E];
      __builtin_memcpy(e, &L.d[v], 16);
      if constexpr (BNA) {
        T yq[E];
        __builtin_memcpy(yq, &L.yv[v], 16);
#pragma unroll
        for (int q = 0; q < E; ++q) {
          const int c = hc * CH + v * E + q;  // (one channel half per wave: the reads broadcast)
          const float yy = to_f(yq[q]);
          e[q] = from_f<T>((yy * Kc[c] + Kc[FCO + c] > 0.0f ? Kc[2 * FCO + c] * to_f(e[q]) : 0.0f) - Kc[4 * FCO + c] -
                           Kc[3 * FCO + c] * yy);
        }
      }
#pragma unroll
      for (int q = 0; q < E; ++q) dcol[(hc * CH + v * E + q) * (PB / (int)sizeof(T))] = inside ? e[q] : from_f<T>(0.0f);
    }
  };
  // im2col columns k = 8 hc .. 8 hc + 7 of stage pixel sp
  auto build_cols = [&](int st) __attribute__((always_inline)) {
    const int pix = st * HP + sp;
    const int py = pix / FT, px = pix % FT;
    T* ccol = reinterpret_cast<T*>(Cs) + sp;
#pragma unroll
    for (int kk = 0; kk < FK / NS; ++kk) {
      const int k = hc * (FK / NS) + kk;
      float v = 0.0f;
      if (k < 9 * cin) {
        const int tap = k / cin, c = k - tap * cin;
        v = Xs[(c * FH + py + tap / 3) * FH + px + tap % 3];
      }
      ccol[k * (PB / (int)sizeof(T))] = from_f<T>(v);
    }
  };

  f32x16 acc = f32x16{};
  const int jobs = NS * (te - tb);
  if constexpr (BNA) {
    for (int c = tid; c < FCO; c += FTHREADS) {
      const float k2i = bna.coef[2 * FCO + c] * bna.invstd[c];
      Kc[c] = bna.scale[c];
      Kc[FCO + c] = bna.shift[c];
      Kc[2 * FCO + c] = bna.coef[c];
      Kc[3 * FCO + c] = k2i;
      Kc[4 * FCO + c] = bna.coef[FCO + c] - k2i * bna.mean[c];
    }
    __syncthreads();
  }
  if (jobs > 0) {
    Loaded cur = load(0);
    for (int j = 0; j < jobs; ++j) {
      // the next job's loads go out before this job's staging: a whole job of cover (two register sets)
      const Loaded nxt = load(j + 1 < jobs ? j + 1 : j);
      stage(cur, j);
      __syncthreads();  // Xs, Ds written
      build_cols(j % NS);
      cur = nxt;
      __syncthreads();  // Cs written
      // out[co][k] += sum over this wave's 32 pixels of the stage
#pragma unroll
      for (int q = 0; q < 32 * (int)sizeof(T) / 32; ++q) {
        const int boff = wp * 32 * (int)sizeof(T) + q * 32 + half * 16;
        const uint4 af = *reinterpret_cast<const uint4*>(Ds + (wa * 32 + l32) * PB + boff);
        const uint4 bfr = *reinterpret_cast<const uint4*>(Cs + l32 * PB + boff);
        Mma<T>::run(acc, af, bfr);
      }
      __syncthreads();  // before the next job overwrites Ds / Cs / Xs
    }
  }
  // combine the two pixel halves, write this block's [64][32] partial sums
  float* red = reinterpret_cast<float*>(smem);  // [2][64][32]
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = wa * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
    red[(wp * FCO + co) * FK + l32] = acc[r];
  }
  __syncthreads();
  for (int i = tid; i < FCO * FK; i += FTHREADS) slab[(int64_t)blockIdx.x * FCO * FK + i] = red[i] + red[FCO * FK + i];
}

static int tiles_of(int n, int h, int w, int& tx, int& ty) {
  tx = (int)cdiv(w, FT);
  ty = (int)cdiv(h, FT);
  return n * tx * ty;
}

static int wgrad_tiles_per_block(int total) { return (int)std::max<int64_t>(1, cdiv(total, 1024)); }

}  // namespace selunet

using namespace selunet;

extern "C" int64_t selunet_first_conv_rows(int32_t n, int32_t h, int32_t w) {
  int tx, ty;
  return tiles_of(n, h, w, tx, ty);
}

extern "C" int selunet_first_conv_fwd_centered(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w,
                                               const void* wpack, void* y, float* stats, const float* center,
                                               int32_t dtype, void* stream) {
  SELUNET_REQUIRE(x && wpack && y && n > 0 && h > 0 && w > 0 && cin >= 1 && cin <= 3, "first_conv_fwd: bad arguments");
  SELUNET_REQUIRE((int64_t)n * cdiv(h, FT) * cdiv(w, FT) < (int64_t(1) << 31), "first_conv_fwd: grid too large");
  int tx, ty;
  const int tiles = tiles_of(n, h, w, tx, ty);
  SELUNET_REQUIRE(center == nullptr || stats != nullptr, "first_conv_fwd: center only with stats");
  EpiArg ep{y, nullptr, nullptr, stats, SELUNET_EP_PLAIN, 0, nullptr,
            BnBwdArg{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr}, nullptr, center};
  const unsigned blocks = (unsigned)std::min(tiles, 3072);  // (three resident workgroups per CU)
  if (dtype == SELUNET_F32)
    hipLaunchKernelGGL(first_conv_fwd_kernel<float>, dim3(blocks), dim3(FTHREADS), 0, as_stream(stream), x, cin, h, w,
                       reinterpret_cast<const float*>(wpack), ep, tx, ty, tiles);
  else if (dtype == SELUNET_BF16)
    hipLaunchKernelGGL(first_conv_fwd_kernel<__bf16>, dim3(blocks), dim3(FTHREADS), 0, as_stream(stream), x, cin, h, w,
                       reinterpret_cast<const __bf16*>(wpack), ep, tx, ty, tiles);
  else
    return fail(SELUNET_EINVAL, "first_conv_fwd: bad dtype %d", dtype);
  return check_launch("first_conv_fwd");
}

extern "C" int selunet_first_conv_fwd(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, const void* wpack,
                                      void* y, float* stats, int32_t dtype, void* stream) {
  return selunet_first_conv_fwd_centered(x, n, cin, h, w, wpack, y, stats, nullptr, dtype, stream);
}

extern "C" int64_t selunet_first_conv_wgrad_rows(int32_t n, int32_t h, int32_t w) {
  int tx, ty;
  const int total = tiles_of(n, h, w, tx, ty);
  return cdiv(total, wgrad_tiles_per_block(total));
}

static int first_wgrad_launch(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, const void* dy,
                              float* slab, int32_t dtype, const FirstBnApply* bna, void* stream) {
  SELUNET_REQUIRE(x && dy && slab && n > 0 && h > 0 && w > 0 && cin >= 1 && cin <= 3, "first_conv_wgrad: bad arguments");
  SELUNET_REQUIRE((int64_t)n * cdiv(h, FT) * cdiv(w, FT) < (int64_t(1) << 31), "first_conv_wgrad: grid too large");
  int tx, ty;
  const int total = tiles_of(n, h, w, tx, ty);
  const int per = wgrad_tiles_per_block(total);
  const unsigned blocks = (unsigned)cdiv(total, per);
  const FirstBnApply none{};
  hipStream_t st = as_stream(stream);
  if (dtype == SELUNET_F32) {
    if (bna)
      hipLaunchKernelGGL((first_conv_wgrad_kernel<float, true>), dim3(blocks), dim3(FTHREADS), 0, st, x, cin, h, w,
                         reinterpret_cast<const float*>(dy), slab, tx, ty, total, per, *bna);
    else
      hipLaunchKernelGGL((first_conv_wgrad_kernel<float, false>), dim3(blocks), dim3(FTHREADS), 0, st, x, cin, h, w,
                         reinterpret_cast<const float*>(dy), slab, tx, ty, total, per, none);
  } else if (dtype == SELUNET_BF16) {
    if (bna)
      hipLaunchKernelGGL((first_conv_wgrad_kernel<__bf16, true>), dim3(blocks), dim3(FTHREADS), 0, st, x, cin, h, w,
                         reinterpret_cast<const __bf16*>(dy), slab, tx, ty, total, per, *bna);
    else
      hipLaunchKernelGGL((first_conv_wgrad_kernel<__bf16, false>), dim3(blocks), dim3(FTHREADS), 0, st, x, cin, h, w,
                         reinterpret_cast<const __bf16*>(dy), slab, tx, ty, total, per, none);
  } else {
    return fail(SELUNET_EINVAL, "first_conv_wgrad: bad dtype %d", dtype);
  }
  return check_launch("first_conv_wgrad");
}

extern "C" int selunet_first_conv_wgrad(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, const void* dy,
                                        float* slab, int32_t dtype, void* stream) {
  return first_wgrad_launch(x, n, cin, h, w, dy, slab, dtype, nullptr, stream);
}

extern "C" int selunet_first_conv_wgrad_bn(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, const void* dz,
                                           const void* y, const float* scale, const float* shift, const float* mean,
                                           const float* invstd, const float* coef, float* slab, int32_t dtype,
                                           void* stream) {
  SELUNET_REQUIRE(y && scale && shift && mean && invstd && coef, "first_conv_wgrad_bn: BatchNorm operands missing");
  const FirstBnApply bna{y, scale, shift, mean, invstd, coef};
  return first_wgrad_launch(x, n, cin, h, w, dz, slab, dtype, &bna, stream);
}
