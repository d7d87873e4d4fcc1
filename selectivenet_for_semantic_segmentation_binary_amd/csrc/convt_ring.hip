// ConvTranspose2d forward and data gradient of fp32 training on split-fp16 operands for the two deep
// up-samplings (model.py:44-45, 51-52: unpool3 K = 512 / N = 1024 and unpool2 K = 256 / N = 512 forward;
// their data gradients K = 1024 / N = 512 and K = 512 / N = 256) — the layers where the resident-weight
// kernels of convt.hip keep only 32-128 weight columns per workgroup and re-read every A row once per
// column block, from fragment-shaped 64-B register loads with one k-step of latency cover (0.20-0.30 of
// the MFMA peak with their split VALU and stores removed, profiles/r05j_convt_ablations.txt).
//
// Here both operands stream through an LDS ring filled by LDS-DMA (global_load_lds_dwordx4):
//  * 256 x 256 output tile per 512-thread workgroup (one per CU, persistent over the row tiles of its
//    column block), 8 waves as 4 (rows) x 2 (columns), each 64 x 128 = 2 x 4 subtiles of 32 x 32: an A
//    value is transformed and split by two waves (2 x 4 waves: four, and the split VALU outgrew the
//    MFMA gaps — an MFMA leaves 24 of its 32 cycles for vector issue, MI355X guide constants table);
//  * a stage is one 16-deep k-step: A = 256 rows x 16 raw fp32 (64 B per row), B = 256 weight rows x
//    (16 high + 16 low fp16 parts) of the split-fp16 pack, 32 KiB; four stages in the ring, three in
//    flight while one is multiplied (counted s_waitcnt vmcnt + raw s_barrier: __syncthreads() would drain
//    the DMA queue at every stage);
//  * A is transformed at fragment time: each wave reads its rows' 8 fp32 values per lane from LDS,
//    applies the producer's BatchNorm+ReLU (forward), the 2^e scale and the fp16 split in registers — the
//    same arithmetic, in the same order, as convt_x2_kernel / convt_dgrad_x2_kernel, so the products and
//    their accumulation order (hl, lh, hh per 16-k step, k ascending) are those kernels';
//  * LDS images are lane-linear (an LDS-DMA writes base + lane x 16 B): the 16-B slots of a 64-B row are
//    XOR-swizzled by (row >> 2) & 3 through the per-lane SOURCE address and read back with the same XOR,
//    so the 16 rows of a ds_read_b128 lane group fall on 16 distinct slots of the 256-B bank row;
//  * epilogues straight from the accumulators as in convt.hip (forward: 2x2 scatter, bias, range word;
//    data gradient: dX, range word and the producer's BatchNorm-backward sums, one slab row per
//    workgroup, fixed reduction order).
#include "gemm_common.h"

namespace selunet {

constexpr int CR_THREADS = 512;
constexpr int CR_BM = 256, CR_BN = 256;               // workgroup tile
constexpr int CR_BK = 16;                             // k per stage (one MFMA k-step)
constexpr int CR_RING = 4;                            // LDS stages
constexpr int CR_ROWB = 64;                           // LDS bytes per row and stage
constexpr int CR_STAGE = (CR_BM + CR_BN) * CR_ROWB;   // 32 KiB
constexpr int CR_KMAX = 1024;                         // forward coefficient area (K <= 1024)

// physical 16-B slot of logical slot s in row r (an involution: the DMA lane whose physical slot is p
// loads logical slot cr_slot(r, p))
__device__ __forceinline__ int cr_slot(int r, int s) { return s ^ ((r >> 2) & 3); }

// WN: waves along the columns (2: 4 x 2 waves of 64 x 128; 1: 8 x 1 waves of 32 x 256, each A value split
// by one wave, twice the B fragment reads — the forward's default, 3-5 % faster than 4 x 2 on the same box,
// profiles/r05w_convt_ring_ab.txt; the data gradient keeps 4 x 2: its BN sums are carried per wave row in LDS)
template <bool DGRAD, int WN = 2>
__global__ void __launch_bounds__(CR_THREADS, 1)
convt_ring_x2_kernel(GatherArg g, const float* __restrict__ W, int N, int n_blocks, int P,
                     const float* __restrict__ wcs, const float* __restrict__ amax_src, float* __restrict__ out,
                     const float* __restrict__ bias, float* amax_out, const float* __restrict__ ybn, BnBwdArg bnb) {
  static_assert(WN == 2 || (WN == 1 && !DGRAD), "8 x 1 waves: forward only");
  constexpr int MT = WN, NT = 8 / WN, WR = 32 * WN, WC = 256 / WN;  // subtiles, rows / columns per wave
  // past the ring: forward: the source's BN scale / shift x 2^e per k, the columns' unscale and bias;
  // data gradient: the columns' unscale and BN coefficients, and the fp64 BN-backward sums per (wave row,
  // column) carried across tiles (registers are full: 128 accumulators + the split A and B fragments)
  constexpr int COEF = DGRAD ? 5 * CR_BN * 4 + 4 * CR_BN * 3 * 8 : 2 * CR_KMAX * 4 + 2 * CR_BN * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[CR_RING * CR_STAGE + COEF];
  float* csc = reinterpret_cast<float*>(smem + CR_RING * CR_STAGE);  // forward: source BN scale x 2^e
  float* csh = csc + CR_KMAX;                                         // ... and shift x 2^e
  float* ccol = DGRAD ? csc : csh + CR_KMAX;  // [unscale, bias | BN scale, shift, mean, invstd][256 columns]
  double* qacc = reinterpret_cast<double*>(ccol + 5 * CR_BN);        // data gradient: [4][256][3]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = lane >> 5, l32 = lane & 31;
  const int wm = wave / WN, wn = wave % WN;
  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int nb = (int)(lb % (unsigned)n_blocks);
  const int prow = (int)(lb / (unsigned)n_blocks);
  const int n0 = nb * CR_BN;
  const int K = g.K, NK = K / CR_BK;
  const int64_t m_tiles = g.M / CR_BM;  // (host: M % 256 == 0)
  const int ntl = prow < m_tiles ? (int)((m_tiles - prow + P - 1) / P) : 0;
  const int T = ntl * NK;
  const int C = g.src[0].C;  // forward: C_in (= K); data gradient: C_out (K = 4 C_out)
  const float* src = reinterpret_cast<const float*>(g.src[0].data);
  const bool do_bn = DGRAD && bnb.slab != nullptr;

  float inv;
  const float xs = x2_scale(amax_src[0], &inv);
  // ReLU as a max against 0 (or -inf: no ReLU) — one v_max per element instead of a select on a runtime flag
  const float relu_lo = !DGRAD && g.src[0].scale != nullptr && g.src[0].relu ? 0.0f : -INFINITY;
  if constexpr (!DGRAD) {
    const SrcArg& s0 = g.src[0];
    for (int c = tid; c < K; c += CR_THREADS) {
      csc[c] = (s0.scale ? s0.scale[c] : 1.0f) * xs;
      csh[c] = (s0.scale ? s0.shift[c] : 0.0f) * xs;
    }
  }
  // the block's column constants (loaded before the DMA stream starts)
  const int Cq = N / 4;  // forward: C_out
  if (tid < CR_BN) {
    const int n = n0 + tid;
    ccol[tid] = wcs[n] * inv;
    if constexpr (!DGRAD) {
      ccol[CR_BN + tid] = bias ? bias[n % Cq] : 0.0f;
    } else {
      ccol[CR_BN + tid] = do_bn ? bnb.scale[n] : 0.0f;
      ccol[2 * CR_BN + tid] = do_bn ? bnb.shift[n] : 0.0f;
      ccol[3 * CR_BN + tid] = do_bn ? bnb.mean[n] : 0.0f;
      ccol[4 * CR_BN + tid] = do_bn ? bnb.invstd[n] : 0.0f;
    }
  }
  if constexpr (DGRAD)
    for (int e = tid; e < 4 * CR_BN * 3; e += CR_THREADS) qacc[e] = 0.0;
  __syncthreads();  // coefficients visible; nothing in flight yet

  typedef const __attribute__((address_space(1))) void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  // stage t (tile t / NK, k-step t % NK) into ring slot t % 4: per thread two A rows and two weight rows
  // (rows wave*32 + r*16 + lane/4, physical slot lane & 3)
  // data gradient: dU pixel (img, 2y, 2x) of this thread's two A rows, decoded once per tile
  int64_t rbase[2] = {0, 0};
  int rb_tile = -1;
  auto issue = [&](int t) __attribute__((always_inline)) {
    const int i = t / NK, kc = t - i * NK;
    const int64_t m_base = ((int64_t)prow + (int64_t)i * P) * CR_BM;
    if constexpr (DGRAD) {
      if (i != rb_tile) {
        rb_tile = i;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const unsigned mu = (unsigned)(m_base + wave * 32 + r * 16 + (lane >> 2));
          const unsigned x = mu % (unsigned)g.w, tt = mu / (unsigned)g.w;
          const unsigned y = tt % (unsigned)g.h, img = tt / (unsigned)g.h;
          rbase[r] = ((int64_t)img * g.hs + 2 * y) * g.ws + 2 * x;
        }
      }
    }
    unsigned char* sa = smem + (t & (CR_RING - 1)) * CR_STAGE;
    unsigned char* sb = sa + CR_BM * CR_ROWB;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = wave * 32 + r * 16 + (lane >> 2);
      const int s = cr_slot(row, lane & 3);
      const int64_t m = m_base + row;
      const float* p;
      if constexpr (!DGRAD) {
        p = src + m * C + kc * CR_BK + s * 4;
      } else {
        // row m = input pixel (img, y, x); k = tap * C_out + o reads dU at (2y + tap / 2, 2x + tap % 2)
        const int k0 = kc * CR_BK, tap = k0 / C, c0 = k0 - tap * C;
        const int64_t pix = rbase[r] + (tap >> 1) * g.ws + (tap & 1);
        p = src + pix * C + c0 + s * 4;
      }
      __builtin_amdgcn_global_load_lds((gptr_t)p, (lptr_t)(sa + (wave * 32 + r * 16) * CR_ROWB), 16, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = wave * 32 + r * 16 + (lane >> 2);
      const int s = cr_slot(row, lane & 3);
      // pack row n: per 32-k slice 16 words of high parts then 16 of low parts; logical slots of a 16-k
      // step: 0 / 1 high k 0-7 / 8-15, 2 / 3 low k 0-7 / 8-15
      const float* p = W + (int64_t)(n0 + row) * K + (kc >> 1) * 32 + (kc & 1) * 8 + (s & 1) * 4 + (s >> 1) * 16;
      __builtin_amdgcn_global_load_lds((gptr_t)p, (lptr_t)(sb + (wave * 32 + r * 16) * CR_ROWB), 16, 0, 0);
    }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  auto compute = [&](int t) __attribute__((always_inline)) {
    const int kc = t % NK;
    const unsigned char* sa = smem + (t & (CR_RING - 1)) * CR_STAGE;
    const unsigned char* sb = sa + CR_BM * CR_ROWB;
    f16x8 bh[NT], bl[NT];
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int n = wn * WC + b * 32 + l32;
      bh[b] = *reinterpret_cast<const f16x8*>(sb + n * CR_ROWB + cr_slot(n, half) * 16);
      bl[b] = *reinterpret_cast<const f16x8*>(sb + n * CR_ROWB + cr_slot(n, 2 + half) * 16);
    }
    float sc[8], sh[8];
    if constexpr (!DGRAD) {
      const int k = kc * CR_BK + half * 8;
      const f32x4 s0 = *reinterpret_cast<const f32x4*>(csc + k), s1 = *reinterpret_cast<const f32x4*>(csc + k + 4);
      const f32x4 t0 = *reinterpret_cast<const f32x4*>(csh + k), t1 = *reinterpret_cast<const f32x4*>(csh + k + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc[e] = s0[e];
        sc[e + 4] = s1[e];
        sh[e] = t0[e];
        sh[e + 4] = t1[e];
      }
    }
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const int r = wm * WR + a * 32 + l32;
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(sa + r * CR_ROWB + cr_slot(r, 2 * half) * 16);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(sa + r * CR_ROWB + cr_slot(r, 2 * half + 1) * 16);
      f16x8 ah, al;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = e < 4 ? v0[e] : v1[e - 4];
        float f;
        if constexpr (DGRAD) {
          f = v * xs;
        } else {
          f = fmaxf(v * sc[e] + sh[e], relu_lo);  // (xs = 2^e > 0: relu(x) * xs == relu(x * xs), exactly)
        }
        _Float16 hh, ll;
        x2_split(f, hh, ll);
        ah[e] = hh;
        al[e] = ll;
      }
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[b], acc[a][b], 0, 0, 0);
      }
    }
  };

  // ------------------------------------------------------------ epilogues (registers -> HBM)
  float am = 0.0f;
  auto epilogue = [&](int i) __attribute__((always_inline)) {
    const int64_t m_base = ((int64_t)prow + (int64_t)i * P) * CR_BM;
    if constexpr (!DGRAD) {
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        // subtile a: pixels r0 .. r0 + 31 of one image row (w % 32 == 0), x0 = r0 % w
        const int64_t r0 = m_base + wm * WR + a * 32;
        const unsigned mu = (unsigned)r0, x0 = mu % (unsigned)g.w, tt = mu / (unsigned)g.w;
        const unsigned y = tt % (unsigned)g.h, img = tt / (unsigned)g.h;
        const int64_t row_even = ((int64_t)img * (2 * g.h) + 2 * y) * (2 * g.w);  // output row 2y
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const int cl = wn * WC + b * 32 + l32, n = n0 + cl;
          const int ab = n / Cq, o = n - ab * Cq;
          const int64_t base = row_even + (int64_t)(ab >> 1) * (2 * g.w) + (ab & 1);
          const float cf = ccol[cl], cb = ccol[CR_BN + cl];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int px = (int)x0 + (r & 3) + 8 * (r >> 2) + 4 * half;
            const float v = acc[a][b][r] * cf + cb;
            out[(base + 2 * px) * Cq + o] = v;  // (32 lanes: 128 contiguous bytes per half)
            am = fmaxf(am, fabsf(v));
          }
        }
      }
    } else {
      float s1[NT], s2[NT], s3[NT];
#pragma unroll
      for (int b = 0; b < NT; ++b) s1[b] = s2[b] = s3[b] = 0.0f;
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int64_t r0 = m_base + wm * WR + a * 32;
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const int cl = wn * WC + b * 32 + l32;
          const int64_t n = n0 + cl;
          const float cf = ccol[cl];
          const float* yp = ybn + (r0 + 4 * half) * N + n;
          float* op = out + (r0 + 4 * half) * N + n;
          float yv[16];
          if (do_bn) {
#pragma unroll
            for (int r = 0; r < 16; ++r) yv[r] = yp[(int64_t)((r & 3) + 8 * (r >> 2)) * N];
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = acc[a][b][r] * cf;
            op[(int64_t)((r & 3) + 8 * (r >> 2)) * N] = v;
            am = fmaxf(am, fabsf(v));
          }
          if (do_bn) {
            const float bsc = ccol[CR_BN + cl], bsh = ccol[2 * CR_BN + cl];
            const float bmu = ccol[3 * CR_BN + cl], bis = ccol[4 * CR_BN + cl];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float v = acc[a][b][r] * cf;
              const float da = yv[r] * bsc + bsh > 0.0f ? v : 0.0f;
              const float xh = (yv[r] - bmu) * bis;
              s1[b] += da;
              s2[b] += da * xh;
              s3[b] += xh;
            }
          }
        }
      }
      if (do_bn) {
        // the two lane halves' fp32 tile sums, then fp64 across tiles in this (wave row, column) slot
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const float t1 = s1[b] + __shfl_xor(s1[b], 32, 64), t2 = s2[b] + __shfl_xor(s2[b], 32, 64);
          const float t3 = s3[b] + __shfl_xor(s3[b], 32, 64);
          if (half == 0) {
            double* q = qacc + (wm * CR_BN + wn * WC + b * 32 + l32) * 3;
            q[0] += (double)t1;
            q[1] += (double)t2;
            q[2] += (double)t3;
          }
        }
      }
    }
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};
  };

  // ------------------------------------------------------------ main loop over the stages
  for (int t = 0; t < 3 && t < T; ++t) issue(t);
  for (int t = 0; t < T; ++t) {
    // this wave's DMAs of stage t have landed (stages t+1, t+2 may stay in flight: 4 DMAs each) ...
    const int ahead = min(T - 1 - t, 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ... and after the barrier every wave's have, and every wave is done reading stage t - 1's slot
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 3 < T) issue(t + 3);  // into slot (t - 1) % 4
    compute(t);
    if (t % NK == NK - 1) epilogue(t / NK);
  }

  __syncthreads();  // (no DMA in flight: the last stage waited for vmcnt(0)) the ring is free
  if (amax_out) block_amax(amax_out, am, reinterpret_cast<float*>(smem));
  if (do_bn) {
    // the four wave rows' sums -> one slab row per workgroup (row prow, this block's 256 columns), in order
    for (int e = tid; e < CR_BN * 3; e += CR_THREADS) {
      const int c = e % CR_BN, k = e / CR_BN;
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) v += qacc[(r * CR_BN + c) * 3 + k];
      bnb.slab[((int64_t)prow * 3 + k) * N + n0 + c] = (float)v;
    }
  }
}

// =========================================================================== bf16 form
// The same ring for the bf16 speed configuration (convt_bf16.hip's resident-weight kernels keep 64-128 weight
// columns per workgroup at unpool3 / unpool2): a stage is a 32-deep k-slice (two v_mfma_f32_32x32x16_bf16
// k-steps; A rows of 32 raw bf16 = 64 B, weight rows [N][K] of 32 bf16), nothing to split — the forward
// applies the producer's BN+ReLU at fragment time and rounds to bf16 as convt_bf16_kernel does, the data
// gradient feeds dU straight from LDS. Products, accumulation order and epilogue arithmetic are
// convt_bf16_kernel's: outputs bit-identical to it. Forward on 8 x 1 waves, data gradient 4 x 2 (BN sums).
// Taken for unpool3's forward and both data gradients (K >= 512): per launch 0.325 -> 0.263 ms (forward),
// 0.378 -> 0.196 and 0.278 -> 0.210 (data gradients), same box (profiles/r05y_convt_ring_bf16_ab.txt).
constexpr int CRB_BK = 32;

template <bool DGRAD, int WN>
__global__ void __launch_bounds__(CR_THREADS, 1)
convt_ring_bf16_kernel(GatherArg g, const __bf16* __restrict__ W, int N, int n_blocks, int P, __bf16* __restrict__ out,
                       const float* __restrict__ bias, const __bf16* __restrict__ ybn, BnBwdArg bnb) {
  static_assert(WN == 2 || (WN == 1 && !DGRAD), "8 x 1 waves: forward only");
  constexpr int MT = WN, NT = 8 / WN, WR = 32 * WN, WC = 256 / WN;
  constexpr int STAGE = (CR_BM + CR_BN) * CR_ROWB;
  constexpr int COEF = DGRAD ? 4 * CR_BN * 4 + 4 * CR_BN * 3 * 8 : 2 * CR_KMAX * 4 + CR_BN * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[CR_RING * STAGE + COEF];
  float* csc = reinterpret_cast<float*>(smem + CR_RING * STAGE);  // forward: source BN scale / shift per k
  float* csh = csc + CR_KMAX;
  float* ccol = DGRAD ? csc : csh + CR_KMAX;                    // [bias | BN scale, shift, mean, invstd][256]
  double* qacc = reinterpret_cast<double*>(ccol + 4 * CR_BN);    // data gradient: [4][256][3]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = lane >> 5, l32 = lane & 31;
  const int wm = wave / WN, wn = wave % WN;
  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int nb = (int)(lb % (unsigned)n_blocks);
  const int prow = (int)(lb / (unsigned)n_blocks);
  const int n0 = nb * CR_BN;
  const int K = g.K, NK = K / CRB_BK;
  const int64_t m_tiles = g.M / CR_BM;
  const int ntl = prow < m_tiles ? (int)((m_tiles - prow + P - 1) / P) : 0;
  const int T = ntl * NK;
  const int C = g.src[0].C;
  const __bf16* src = reinterpret_cast<const __bf16*>(g.src[0].data);
  const bool do_bn = DGRAD && bnb.slab != nullptr;
  const bool xform = !DGRAD && g.src[0].scale != nullptr;
  const bool relu = xform && g.src[0].relu;
  if constexpr (!DGRAD) {
    const SrcArg& s0 = g.src[0];
    for (int c = tid; c < K; c += CR_THREADS) {
      csc[c] = s0.scale ? s0.scale[c] : 1.0f;
      csh[c] = s0.scale ? s0.shift[c] : 0.0f;
    }
  }
  const int Cq = N / 4;
  if (tid < CR_BN) {
    const int n = n0 + tid;
    if constexpr (!DGRAD) {
      ccol[tid] = bias ? bias[n % Cq] : 0.0f;
    } else {
      ccol[tid] = do_bn ? bnb.scale[n] : 0.0f;
      ccol[CR_BN + tid] = do_bn ? bnb.shift[n] : 0.0f;
      ccol[2 * CR_BN + tid] = do_bn ? bnb.mean[n] : 0.0f;
      ccol[3 * CR_BN + tid] = do_bn ? bnb.invstd[n] : 0.0f;
    }
  }
  if constexpr (DGRAD)
    for (int e = tid; e < 4 * CR_BN * 3; e += CR_THREADS) qacc[e] = 0.0;
  __syncthreads();

  typedef const __attribute__((address_space(1))) void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  int64_t rbase[2] = {0, 0};
  int rb_tile = -1;
  auto issue = [&](int t) __attribute__((always_inline)) {
    const int i = t / NK, kc = t - i * NK;
    const int64_t m_base = ((int64_t)prow + (int64_t)i * P) * CR_BM;
    if constexpr (DGRAD) {
      if (i != rb_tile) {
        rb_tile = i;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const unsigned mu = (unsigned)(m_base + wave * 32 + r * 16 + (lane >> 2));
          const unsigned x = mu % (unsigned)g.w, tt = mu / (unsigned)g.w;
          const unsigned y = tt % (unsigned)g.h, img = tt / (unsigned)g.h;
          rbase[r] = ((int64_t)img * g.hs + 2 * y) * g.ws + 2 * x;
        }
      }
    }
    unsigned char* sa = smem + (t & (CR_RING - 1)) * STAGE;
    unsigned char* sb = sa + CR_BM * CR_ROWB;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = wave * 32 + r * 16 + (lane >> 2);
      const int s = cr_slot(row, lane & 3);
      const __bf16* p;
      if constexpr (!DGRAD) {
        p = src + (m_base + row) * C + kc * CRB_BK + s * 8;
      } else {  // k = tap * C_out + o (C_out % 32 == 0: a stage lies in one tap)
        const int k0 = kc * CRB_BK, tap = k0 / C, c0 = k0 - tap * C;
        p = src + (rbase[r] + (tap >> 1) * g.ws + (tap & 1)) * C + c0 + s * 8;
      }
      __builtin_amdgcn_global_load_lds((gptr_t)p, (lptr_t)(sa + (wave * 32 + r * 16) * CR_ROWB), 16, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = wave * 32 + r * 16 + (lane >> 2);
      const int s = cr_slot(row, lane & 3);
      const __bf16* p = W + (int64_t)(n0 + row) * K + kc * CRB_BK + s * 8;
      __builtin_amdgcn_global_load_lds((gptr_t)p, (lptr_t)(sb + (wave * 32 + r * 16) * CR_ROWB), 16, 0, 0);
    }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  auto compute = [&](int t) __attribute__((always_inline)) {
    const int kc = t % NK;
    const unsigned char* sa = smem + (t & (CR_RING - 1)) * STAGE;
    const unsigned char* sb = sa + CR_BM * CR_ROWB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int slot = 2 * ks + half;  // 8 bf16: k = ks * 16 + half * 8 .. + 7 of the stage
      bf16x8 av[MT];
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int r = wm * WR + a * 32 + l32;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(sa + r * CR_ROWB + cr_slot(r, slot) * 16);
        if constexpr (!DGRAD) {
          if (xform) {
            const int k = kc * CRB_BK + ks * 16 + half * 8;
            const f32x4 s0v = *reinterpret_cast<const f32x4*>(csc + k), s1v = *reinterpret_cast<const f32x4*>(csc + k + 4);
            const f32x4 t0v = *reinterpret_cast<const f32x4*>(csh + k), t1v = *reinterpret_cast<const f32x4*>(csh + k + 4);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              float f = (float)v[e] * (e < 4 ? s0v[e] : s1v[e - 4]) + (e < 4 ? t0v[e] : t1v[e - 4]);
              if (relu) f = fmaxf(f, 0.0f);
              v[e] = (__bf16)f;
            }
          }
        }
        av[a] = v;
      }
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const int n = wn * WC + b * 32 + l32;
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(sb + n * CR_ROWB + cr_slot(n, slot) * 16);
#pragma unroll
        for (int a = 0; a < MT; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a], bv, acc[a][b], 0, 0, 0);
      }
    }
  };

  auto epilogue = [&](int i) __attribute__((always_inline)) {
    const int64_t m_base = ((int64_t)prow + (int64_t)i * P) * CR_BM;
    if constexpr (!DGRAD) {
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int64_t r0 = m_base + wm * WR + a * 32;
        const unsigned mu = (unsigned)r0, x0 = mu % (unsigned)g.w, tt = mu / (unsigned)g.w;
        const unsigned y = tt % (unsigned)g.h, img = tt / (unsigned)g.h;
        const int64_t row_even = ((int64_t)img * (2 * g.h) + 2 * y) * (2 * g.w);
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const int cl = wn * WC + b * 32 + l32, n = n0 + cl;
          const int ab = n / Cq, o = n - ab * Cq;
          const int64_t base = row_even + (int64_t)(ab >> 1) * (2 * g.w) + (ab & 1);
          const float cb = ccol[cl];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int px = (int)x0 + (r & 3) + 8 * (r >> 2) + 4 * half;
            out[(base + 2 * px) * Cq + o] = (__bf16)(acc[a][b][r] + cb);
          }
        }
      }
    } else {
      float s1[NT], s2[NT], s3[NT];
#pragma unroll
      for (int b = 0; b < NT; ++b) s1[b] = s2[b] = s3[b] = 0.0f;
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int64_t r0 = m_base + wm * WR + a * 32;
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const int cl = wn * WC + b * 32 + l32;
          const int64_t n = n0 + cl;
          const __bf16* yp = ybn + (r0 + 4 * half) * N + n;
          __bf16* op = out + (r0 + 4 * half) * N + n;
          __bf16 yv[16];
          if (do_bn) {
#pragma unroll
            for (int r = 0; r < 16; ++r) yv[r] = yp[(int64_t)((r & 3) + 8 * (r >> 2)) * N];
          }
          __bf16 ov[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            ov[r] = (__bf16)acc[a][b][r];
            op[(int64_t)((r & 3) + 8 * (r >> 2)) * N] = ov[r];
          }
          if (do_bn) {
            const float sc = ccol[cl], sh = ccol[CR_BN + cl], mu = ccol[2 * CR_BN + cl], is = ccol[3 * CR_BN + cl];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float yf = (float)yv[r];
              const float da = yf * sc + sh > 0.0f ? (float)ov[r] : 0.0f;
              const float xh = (yf - mu) * is;
              s1[b] += da;
              s2[b] += da * xh;
              s3[b] += xh;
            }
          }
        }
      }
      if (do_bn) {
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const float t1 = s1[b] + __shfl_xor(s1[b], 32, 64), t2 = s2[b] + __shfl_xor(s2[b], 32, 64);
          const float t3 = s3[b] + __shfl_xor(s3[b], 32, 64);
          if (half == 0) {
            double* q = qacc + (wm * CR_BN + wn * WC + b * 32 + l32) * 3;
            q[0] += (double)t1;
            q[1] += (double)t2;
            q[2] += (double)t3;
          }
        }
      }
    }
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};
  };

  for (int t = 0; t < 3 && t < T; ++t) issue(t);
  for (int t = 0; t < T; ++t) {
    const int ahead = min(T - 1 - t, 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 3 < T) issue(t + 3);
    compute(t);
    if (t % NK == NK - 1) epilogue(t / NK);
  }

  __syncthreads();
  if (do_bn) {
    for (int e = tid; e < CR_BN * 3; e += CR_THREADS) {
      const int c = e % CR_BN, k = e / CR_BN;
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) v += qacc[(r * CR_BN + c) * 3 + k];
      bnb.slab[((int64_t)prow * 3 + k) * N + n0 + c] = (float)v;
    }
  }
}

// --------------------------------------------------------------------------- host side
static bool ring_on() { return option(SELUNET_OPT_CONVT_RING, 2) != 0; }

// the forward operand / epilogue this kernel takes (ConvTranspose2d forward, K = C_in of 256..1024)
static bool convt_ring_fwd_ok(const GatherArg& g, int N, const EpiArg& e) {
  if (!ring_on() || g.nsrc != 1 || g.small || g.src[0].layout != 0 || g.taps != 1) return false;
  if (g.w % 32 != 0 || g.M % CR_BM != 0 || N % CR_BN != 0 || N % 4 != 0) return false;
  if (g.K < 256 || g.K > CR_KMAX || g.K % 32 != 0 || g.src[0].C != g.K) return false;
  const bool no_sums = e.stats == nullptr && e.colsum == nullptr && e.bnb.slab == nullptr;
  return e.mode == SELUNET_EP_SCATTER2X && no_sums;
}

// The data-gradient operand (taps = 4 gather of a plain dU, K = 4 C_out >= 512): a function of the operand
// alone, so that selunet_gemm_gather_x2_stats_rows sizes the slab for the kernel that runs.
bool convt_ring_dgrad_operand_ok(const GatherArg& g, int N) {
  if (!ring_on() || g.nsrc != 1 || g.small || g.src[0].layout != 0 || g.src[0].scale != nullptr) return false;
  if (g.taps != 4 || g.w % 32 != 0 || g.M % CR_BM != 0 || N % CR_BN != 0) return false;
  return g.src[0].C % CR_BK == 0 && g.K == 4 * g.src[0].C && g.K >= 512 && g.K % 32 == 0;
}

// persistent row workgroups per column block (= statistics slab rows): one workgroup per CU overall
int64_t convt_ring_rows(const GatherArg& g, int N) {
  const int64_t m_tiles = g.M / CR_BM, blocks = std::max(1, N / CR_BN);
  return std::max<int64_t>(1, std::min<int64_t>(m_tiles, std::max<int64_t>(1, 256 / blocks)));
}

// whether selunet_gemm_gather_x2 sends this operand here (a data-gradient operand with another epilogue
// fails in convt_ring_x2_launch rather than running a kernel whose slab rows differ)
bool convt_ring_x2_takes(const GatherArg& g, int N, const EpiArg& e) {
  return convt_ring_fwd_ok(g, N, e) || convt_ring_dgrad_operand_ok(g, N);
}

int convt_ring_x2_launch(const GatherArg& g, const float* w, int N, const EpiArg& e, const float* amax_src,
                         hipStream_t st) {
  const bool fwd = convt_ring_fwd_ok(g, N, e);
  const bool dgrad = !fwd && convt_ring_dgrad_operand_ok(g, N);
  if (!fwd && !dgrad) return fail(SELUNET_EINVAL, "convt_ring_x2: operand not eligible");
  if (dgrad && !(e.mode == SELUNET_EP_PLAIN && e.out1 == nullptr && e.bias == nullptr && e.stats == nullptr &&
                 e.colsum == nullptr))
    return fail(SELUNET_EINVAL, "convt_ring_x2: a ConvTranspose2d data-gradient operand needs the PLAIN epilogue");
  if (dgrad && e.bnb.slab != nullptr && e.bnb.y == nullptr)
    return fail(SELUNET_EINVAL, "convt_ring_x2: BN-backward sums need y");
  // shapes the kernel's indexing assumes (checked here, before any launch)
  if (g.M >= (int64_t(1) << 31) || (int64_t)g.n * g.h * g.w != g.M)
    return fail(SELUNET_EINVAL, "convt_ring_x2: bad row grid");
  if (dgrad && (g.hs != 2 * g.h || g.ws != 2 * g.w)) return fail(SELUNET_EINVAL, "convt_ring_x2: dU grid is not 2x");
  const int blocks = N / CR_BN;
  const int64_t P = convt_ring_rows(g, N);
  const float* wcs = w + (int64_t)N * g.K;
  const dim3 grid((unsigned)(P * blocks)), block(CR_THREADS);
  float* out = reinterpret_cast<float*>(e.out0);
  if (fwd && option(SELUNET_OPT_CONVT_RING, 2) == 2)
    hipLaunchKernelGGL((convt_ring_x2_kernel<false, 1>), grid, block, 0, st, g, w, N, blocks, (int)P, wcs, amax_src,
                       out, e.bias, e.amax, nullptr, BnBwdArg{});
  else if (fwd)
    hipLaunchKernelGGL((convt_ring_x2_kernel<false>), grid, block, 0, st, g, w, N, blocks, (int)P, wcs, amax_src, out,
                       e.bias, e.amax, nullptr, BnBwdArg{});
  else
    hipLaunchKernelGGL((convt_ring_x2_kernel<true>), grid, block, 0, st, g, w, N, blocks, (int)P, wcs, amax_src, out,
                       nullptr, e.amax, reinterpret_cast<const float*>(e.bnb.y), e.bnb);
  return check_launch("convt_ring_x2");
}

// ---- bf16 (selunet_gemm_gather, SELUNET_BF16)
static bool convt_ring_bf16_fwd_ok(const GatherArg& g, int N, const EpiArg& e) {
  if (!ring_on() || g.nsrc != 1 || g.small || g.src[0].layout != 0 || g.taps != 1) return false;
  if (g.w % 32 != 0 || g.M % CR_BM != 0 || N % CR_BN != 0 || N % 4 != 0) return false;
  // (K = 256, unpool2: the resident kernel holds 256 weight columns and measured faster, 0.28 vs 0.31 ms)
  if (g.K < 512 || g.K > CR_KMAX || g.K % CRB_BK != 0 || g.src[0].C != g.K) return false;
  const bool no_sums = e.stats == nullptr && e.colsum == nullptr && e.bnb.slab == nullptr && e.amax == nullptr;
  return e.mode == SELUNET_EP_SCATTER2X && no_sums;
}

bool convt_ring_bf16_dgrad_operand_ok(const GatherArg& g, int N) {
  if (!ring_on() || g.nsrc != 1 || g.small || g.src[0].layout != 0 || g.src[0].scale != nullptr) return false;
  if (g.taps != 4 || g.w % 32 != 0 || g.M % CR_BM != 0 || N % CR_BN != 0) return false;
  return g.src[0].C % CRB_BK == 0 && g.K == 4 * g.src[0].C && g.K >= 512;
}

bool convt_ring_bf16_takes(const GatherArg& g, int N, const EpiArg& e) {
  return convt_ring_bf16_fwd_ok(g, N, e) || convt_ring_bf16_dgrad_operand_ok(g, N);
}

int convt_ring_bf16_launch(const GatherArg& g, const void* w, int N, const EpiArg& e, hipStream_t st) {
  const bool fwd = convt_ring_bf16_fwd_ok(g, N, e);
  const bool dgrad = !fwd && convt_ring_bf16_dgrad_operand_ok(g, N);
  if (!fwd && !dgrad) return fail(SELUNET_EINVAL, "convt_ring_bf16: operand not eligible");
  if (dgrad && !(e.mode == SELUNET_EP_PLAIN && e.out1 == nullptr && e.bias == nullptr && e.stats == nullptr &&
                 e.colsum == nullptr && e.amax == nullptr))
    return fail(SELUNET_EINVAL, "convt_ring_bf16: a ConvTranspose2d data-gradient operand needs the PLAIN epilogue");
  if (dgrad && e.bnb.slab != nullptr && e.bnb.y == nullptr)
    return fail(SELUNET_EINVAL, "convt_ring_bf16: BN-backward sums need y");
  if (g.M >= (int64_t(1) << 31) || (int64_t)g.n * g.h * g.w != g.M)
    return fail(SELUNET_EINVAL, "convt_ring_bf16: bad row grid");
  if (dgrad && (g.hs != 2 * g.h || g.ws != 2 * g.w)) return fail(SELUNET_EINVAL, "convt_ring_bf16: dU grid is not 2x");
  const int blocks = N / CR_BN;
  const int64_t P = convt_ring_rows(g, N);
  const dim3 grid((unsigned)(P * blocks)), block(CR_THREADS);
  const __bf16* W = reinterpret_cast<const __bf16*>(w);
  __bf16* out = reinterpret_cast<__bf16*>(e.out0);
  if (fwd)
    hipLaunchKernelGGL((convt_ring_bf16_kernel<false, 1>), grid, block, 0, st, g, W, N, blocks, (int)P, out, e.bias,
                       nullptr, BnBwdArg{});
  else
    hipLaunchKernelGGL((convt_ring_bf16_kernel<true, 2>), grid, block, 0, st, g, W, N, blocks, (int)P, out, nullptr,
                       reinterpret_cast<const __bf16*>(e.bnb.y), e.bnb);
  return check_launch("convt_ring_bf16");
}

}  // namespace selunet
