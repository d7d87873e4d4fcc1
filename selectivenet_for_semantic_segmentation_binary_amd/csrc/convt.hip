// ConvTranspose2d(k=2, s=2) forward of fp32 training on split-fp16 operands (model.py:44-45, 51-52,
// 57-58: unpool3/2/1), the resident-weight form of selunet_gemm_gather_x2.
//
// A short-K GEMM with a large pixel dimension: out[(2y+a, 2x+b)][o] = bias[o] +
// sum_c A[(y, x)][c] W[c][o][a][b] (M = N*h*w pixels, K = C_in, N = 4*C_out, the 2x2 scatter in the
// epilogue). The generic gather GEMM stages both operands through LDS per 32-k slice and re-stages the
// weights for every tile; its time goes to that staging. Here:
//  * a workgroup keeps one block of NTB weight columns x the whole K resident in LDS for its
//    lifetime (NTB * K = 32768 split-fp16 words = 128 KiB: all 256 columns of unpool1, 128 of
//    unpool2's 512, 64 of unpool3's 1024) — staged once, read as MFMA B fragments;
//  * the A operand never touches LDS: every lane loads its own 32-B row fragment (8 fp32 channels)
//    straight from HBM into registers, D k-steps ahead (a register ring: ~16-64 KiB in flight per
//    CU), applies the producer's BN+ReLU, the 2^e scale and the fp16 split in registers;
//  * accumulators are stored straight from registers (a 32x32 accumulator register is two 128-B
//    runs: full-rate stores), no LDS epilogue.
// Three v_mfma_f32_32x32x16_f16 per 16-k step and 32x32 subtile (hi*lo, lo*hi, hi*hi), as every
// split-fp16 kernel. One persistent 512-thread workgroup per CU walks the pixel tiles of its column
// block (tiles prow, prow + P, ...); the workgroups of one pixel tile's column blocks are neighbours
// on an XCD, so the A rows re-read per column block come from its L2.
// The data gradient (convt_dgrad_x2_kernel below) takes the same scheme for K = 4 C_out of 256 / 512
// (unpool1 / unpool2; unpool3's K = 1024 keeps the staged gather GEMM): 1.11 -> 0.83 and 0.91 -> 0.75 ms
// at bs=128. Its epilogue also reads the producer's y for the BatchNorm-backward sums; a first version
// that loaded each y between output stores the compiler had to assume alias it measured 1.66 ms.
#include "gemm_common.h"

namespace selunet {

constexpr int CT_THREADS = 512;
constexpr int CT_WORDS = 32768;  // resident weight words per workgroup (NTB * K)

// NT: 32-column subtiles per wave = NTB / 32 (K = CT_WORDS / NTB); MT = 8 / NT 32-row subtiles per
// wave (128 accumulator registers); D k-steps of A loads in flight per lane.
template <int NT>
__global__ void __launch_bounds__(CT_THREADS, 1)
convt_x2_kernel(GatherArg g, const float* __restrict__ W, int N, EpiArg ep, int n_blocks, int P,
                const float* __restrict__ wcs, const float* __restrict__ amax_src) {
  constexpr int NTB = NT * 32;
  constexpr int KC = CT_WORDS / NTB;  // K
  constexpr int NK = KC / 16;         // 16-k MFMA steps per tile
  constexpr int MT = 8 / NT;
  constexpr int D = MT >= 4 ? 1 : 2;
  constexpr int ROWS = 8 * MT * 32;   // pixel rows per tile
  constexpr int RB = 4 * KC + 16;     // LDS bytes per weight row (odd number of 16-B slots: conflict-free)
  __shared__ __attribute__((aligned(16))) unsigned char smem[NTB * RB + (2 * KC * 4)];
  float* csc = reinterpret_cast<float*>(smem + NTB * RB);  // forward: the source's BN scale / shift
  float* csh = csc + KC;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int nb = lb % n_blocks;
  const int prow = lb / n_blocks;
  const int n0 = nb * NTB;
  const int64_t M = g.M;
  const int64_t m_tiles = (M + ROWS - 1) / ROWS;
  const int ntl = prow < m_tiles ? (int)((m_tiles - prow + P - 1) / P) : 0;
  const int total = ntl * NK;

  // ------------------------------------------------------------ resident weights, coefficients
  {
    constexpr int V = KC / 4;  // uint4 per row
    for (int i = tid; i < NTB * V; i += CT_THREADS) {
      const int row = i / V, v = i - row * V;
      *reinterpret_cast<uint4*>(smem + row * RB + v * 16) =
          *reinterpret_cast<const uint4*>(W + (int64_t)(n0 + row) * KC + v * 4);
    }
    const SrcArg& s0 = g.src[0];
    for (int c = tid; c < KC; c += CT_THREADS) {
      csc[c] = s0.scale ? s0.scale[c] : 1.0f;
      csh[c] = s0.scale ? s0.shift[c] : 0.0f;
    }
  }
  float inv;
  const float xs = x2_scale(amax_src[0], &inv);
  const bool relu = g.src[0].scale != nullptr && g.src[0].relu;
  const float* src = reinterpret_cast<const float*>(g.src[0].data);
  const int C = g.src[0].C;  // C_in (= K)
  __syncthreads();

  // first pixel row of the 32-row subtile a of tile t (a 32-px run of one image row: w % 32 == 0,
  // host-checked)
  auto sub_row0 = [&](int t, int a) -> int64_t {
    return (int64_t)(prow + (int64_t)t * P) * ROWS + (wave * MT + a) * 32;
  };
  auto load = [&](f32x4 (&r)[MT][2], int j) __attribute__((always_inline)) {
    const int t = j / NK, ks = j - t * NK;
    const int k = ks * 16 + half * 8;
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      int64_t m = sub_row0(t, a) + l32;
      m = m < M ? m : M - 1;
      const float* p = src + m * C + k;
      r[a][0] = *reinterpret_cast<const f32x4*>(p);
      r[a][1] = *reinterpret_cast<const f32x4*>(p + 4);
    }
  };
  // 8 fp32 channels (k .. k+7 of this lane) -> BN+ReLU of the producer, 2^e scale, fp16 high / low parts
  auto split8 = [&](const f32x4 (&v)[2], int k, f16x8& h, f16x8& l) __attribute__((always_inline)) {
    float sc[8], sh[8];
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(csc + k), s1 = *reinterpret_cast<const f32x4*>(csc + k + 4);
    const f32x4 t0 = *reinterpret_cast<const f32x4*>(csh + k), t1 = *reinterpret_cast<const f32x4*>(csh + k + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sc[e] = s0[e] * xs;
      sc[e + 4] = s1[e] * xs;
      sh[e] = t0[e] * xs;
      sh[e + 4] = t1[e] * xs;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float f = v[e >> 2][e & 3] * sc[e] + sh[e];  // (xs = 2^e > 0: relu(x) * xs == relu(x * xs), exactly)
      if (relu) f = fmaxf(f, 0.0f);
      _Float16 hh, ll;
      x2_split(f, hh, ll);
      h[e] = hh;
      l[e] = ll;
    }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  auto mma = [&](const f32x4 (&r)[MT][2], int ks) __attribute__((always_inline)) {
    const int k = ks * 16 + half * 8;
    // B fragment of column subtile b: row b*32 + l32, 16-k step ks in its 128-B slice (high parts
    // at bytes 0-63, low parts at 64-127, ks & 1 selecting the 16-k half)
    const int boff = (ks >> 1) * 128 + (ks & 1) * 32 + half * 16;
    if constexpr (NT >= MT) {
      f16x8 ah[MT], al[MT];
#pragma unroll
      for (int a = 0; a < MT; ++a) split8(r[a], k, ah[a], al[a]);
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const unsigned char* p = smem + (b * 32 + l32) * RB + boff;
        const f16x8 bh = *reinterpret_cast<const f16x8*>(p), bl = *reinterpret_cast<const f16x8*>(p + 64);
#pragma unroll
        for (int a = 0; a < MT; ++a) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bl, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a], bh, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bh, acc[a][b], 0, 0, 0);
        }
      }
    } else {
      f16x8 bh[NT], bl[NT];
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const unsigned char* p = smem + (b * 32 + l32) * RB + boff;
        bh[b] = *reinterpret_cast<const f16x8*>(p);
        bl[b] = *reinterpret_cast<const f16x8*>(p + 64);
      }
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        f16x8 ah, al;
        split8(r[a], k, ah, al);
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[b], acc[a][b], 0, 0, 0);
        }
      }
    }
  };

  // ------------------------------------------------------------ epilogue (registers -> HBM)
  float am = 0.0f;  // running max |stored value| (the up-sampled tensor's range word)
  const int Cq = N / 4;  // C_out
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    float* out = reinterpret_cast<float*>(ep.out0);
    // the columns' bias and unscale (weight row) x 2^-e, loaded before any store: `out` may alias
    // them as far as the compiler knows, so loads between the stores would each wait a full memory
    // latency (8 per tile)
    float cbias[NT], ccf[NT];
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int n = n0 + b * 32 + l32;
      cbias[b] = ep.bias ? ep.bias[n % Cq] : 0.0f;
      ccf[b] = wcs[n] * inv;
    }
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const int64_t r0 = sub_row0(t, a);
      if (r0 >= M) continue;  // (M % 32 == 0: a subtile is entirely inside or outside)
      // subtile a: pixels r0 .. r0 + 31 of one image row (img, y), x0 = r0 % w
      const unsigned mu = (unsigned)r0, x0 = mu % (unsigned)g.w, tt = mu / (unsigned)g.w;
      const unsigned y = tt % (unsigned)g.h, img = tt / (unsigned)g.h;
      const int64_t row_even = ((int64_t)img * (2 * g.h) + 2 * y) * (2 * g.w);  // output row 2y
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const int n = n0 + b * 32 + l32;
        const int ab = n / Cq, o = n - ab * Cq;
        const float bias = cbias[b];
        const float cf = ccf[b];
        const int64_t base = row_even + (int64_t)(ab >> 1) * (2 * g.w) + (ab & 1);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int px = (int)x0 + (r & 3) + 8 * (r >> 2) + 4 * half;
          const float v = acc[a][b][r] * cf + bias;
          out[(base + 2 * px) * Cq + o] = v;  // (32 lanes: 128 contiguous bytes per half)
          am = fmaxf(am, fabsf(v));
        }
      }
    }
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};
  };

  // ------------------------------------------------------------ main loop: jobs (tile, k-step)
  f32x4 ring[D][MT][2];
#pragma unroll
  for (int u = 0; u < D; ++u) load(ring[u], u < total ? u : 0);
  for (int j0 = 0; j0 < total; j0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int j = j0 + u;
      if (j < total) {
        const int t = j / NK, ks = j - t * NK;
        mma(ring[u], ks);
        const int jn = j + D;
        load(ring[u], jn < total ? jn : j);  // (the last D jobs reload their own rows, never used)
        if (ks == NK - 1) epilogue(t);
      }
    }
  }

  if (ep.amax) block_amax(ep.amax, am, reinterpret_cast<float*>(smem));
}

// ConvTranspose2d data gradient (the backward of model.py:44-45, 51-52, 57-58): dX[(y, x)][ci] = sum over
// the 2x2 taps (a, b) and the C_out channels o of dU[(2y + a, 2x + b)][o] W[ci][o][a][b] — a gather GEMM
// with K = 4 C_out (k = tap * C_out + o, tap = 2a + b) and N = C_in. The resident-weight scheme of
// convt_x2_kernel: a block of NTB weight rows x the whole K stays in LDS for the workgroup's life, every
// lane loads its 8-channel dU fragments straight from HBM into a register ring (no source transform:
// dU only takes the 2^e scale and the split). The epilogue stores dX (PLAIN [M][N]) from the
// accumulators and folds the producer's BatchNorm-backward sums (da = dX [y sc + sh > 0], da xhat, xhat;
// the sums of lds_tile_store_acc): each 32x32 subtile's 16 y values per lane are loaded before its 16
// stores, and out / y are restrict kernel arguments, so the compiler may also issue them ahead of the
// previous subtile's stores (the staged kernel's LDS epilogue re-stages every tile). Per-lane sums are
// fp32 within a tile and fp64 across tiles, reduced in a fixed order into one slab row per workgroup.
template <int NT>
__global__ void __launch_bounds__(CT_THREADS, 1)
convt_dgrad_x2_kernel(GatherArg g, const float* __restrict__ W, int N, int n_blocks, int P,
                      const float* __restrict__ wcs, const float* __restrict__ amax_src, float* __restrict__ out,
                      const float* __restrict__ ybn, BnBwdArg bnb, float* amax_out) {
  constexpr int NTB = NT * 32;
  constexpr int KC = CT_WORDS / NTB;  // K
  constexpr int NK = KC / 16;         // 16-k MFMA steps per tile
  constexpr int MT = 8 / NT;
  constexpr int D = MT >= 4 ? 1 : 2;
  constexpr int ROWS = 8 * MT * 32;
  constexpr int RB = 4 * KC + 16;
  constexpr int RR = 16;  // partial-sum rows per column: 8 waves x 2 lane halves
  static_assert(RR * NTB * 3 * (int)sizeof(double) <= NTB * RB, "column reduction scratch exceeds the weight block");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NTB * RB + 5 * NTB * 4];
  float* cco = reinterpret_cast<float*>(smem + NTB * RB);  // [5][NTB]: unscale, BN scale, shift, mean, invstd

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int nb = lb % n_blocks;
  const int prow = lb / n_blocks;
  const int n0 = nb * NTB;
  const int64_t M = g.M;
  const int64_t m_tiles = (M + ROWS - 1) / ROWS;
  const int ntl = prow < m_tiles ? (int)((m_tiles - prow + P - 1) / P) : 0;
  const int total = ntl * NK;
  const bool do_bn = bnb.slab != nullptr;

  float inv;
  const float xs = x2_scale(amax_src[0], &inv);
  {
    constexpr int V = KC / 4;  // uint4 per row
    for (int i = tid; i < NTB * V; i += CT_THREADS) {
      const int row = i / V, v = i - row * V;
      *reinterpret_cast<uint4*>(smem + row * RB + v * 16) =
          *reinterpret_cast<const uint4*>(W + (int64_t)(n0 + row) * KC + v * 4);
    }
    for (int c = tid; c < NTB; c += CT_THREADS) {
      cco[c] = wcs[n0 + c] * inv;
      cco[NTB + c] = do_bn ? bnb.scale[n0 + c] : 0.0f;
      cco[2 * NTB + c] = do_bn ? bnb.shift[n0 + c] : 0.0f;
      cco[3 * NTB + c] = do_bn ? bnb.mean[n0 + c] : 0.0f;
      cco[4 * NTB + c] = do_bn ? bnb.invstd[n0 + c] : 0.0f;
    }
  }
  const float* src = reinterpret_cast<const float*>(g.src[0].data);
  const int C = g.src[0].C;  // C_out (K = 4 C; C % 16 == 0: a 16-k step lies in one tap)
  __syncthreads();

  auto sub_row0 = [&](int t, int a) -> int64_t {
    return (int64_t)(prow + (int64_t)t * P) * ROWS + (wave * MT + a) * 32;
  };
  auto load = [&](f32x4 (&r)[MT][2], int j) __attribute__((always_inline)) {
    const int t = j / NK, ks = j - t * NK;
    const int k = ks * 16 + half * 8;
    const int tap = k / C, c = k - tap * C;
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      int64_t r0 = sub_row0(t, a);
      r0 = r0 < M ? r0 : M - 32;
      // subtile a: pixels r0 .. r0 + 31 of one image row (img, y); this lane's pixel x0 + l32 reads
      // dU at (2y + tap / 2, 2 (x0 + l32) + tap % 2)
      const unsigned mu = (unsigned)r0, x0 = mu % (unsigned)g.w, tt = mu / (unsigned)g.w;
      const unsigned y = tt % (unsigned)g.h, img = tt / (unsigned)g.h;
      const int64_t pix = ((int64_t)img * g.hs + 2 * y + (tap >> 1)) * g.ws + 2 * (x0 + l32) + (tap & 1);
      const float* p = src + pix * C + c;
      r[a][0] = *reinterpret_cast<const f32x4*>(p);
      r[a][1] = *reinterpret_cast<const f32x4*>(p + 4);
    }
  };
  auto split8 = [&](const f32x4 (&v)[2], f16x8& h, f16x8& l) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      _Float16 hh, ll;
      x2_split(v[e >> 2][e & 3] * xs, hh, ll);
      h[e] = hh;
      l[e] = ll;
    }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  auto mma = [&](const f32x4 (&r)[MT][2], int ks) __attribute__((always_inline)) {
    const int boff = (ks >> 1) * 128 + (ks & 1) * 32 + half * 16;
    if constexpr (NT >= MT) {
      f16x8 ah[MT], al[MT];
#pragma unroll
      for (int a = 0; a < MT; ++a) split8(r[a], ah[a], al[a]);
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const unsigned char* p = smem + (b * 32 + l32) * RB + boff;
        const f16x8 bh = *reinterpret_cast<const f16x8*>(p), bl = *reinterpret_cast<const f16x8*>(p + 64);
#pragma unroll
        for (int a = 0; a < MT; ++a) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bl, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a], bh, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bh, acc[a][b], 0, 0, 0);
        }
      }
    } else {
      f16x8 bh[NT], bl[NT];
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const unsigned char* p = smem + (b * 32 + l32) * RB + boff;
        bh[b] = *reinterpret_cast<const f16x8*>(p);
        bl[b] = *reinterpret_cast<const f16x8*>(p + 64);
      }
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        f16x8 ah, al;
        split8(r[a], ah, al);
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[b], acc[a][b], 0, 0, 0);
        }
      }
    }
  };

  // ------------------------------------------------------------ epilogue (registers -> HBM)
  float am = 0.0f;
  double q1[NT], q2[NT], q3[NT];
#pragma unroll
  for (int b = 0; b < NT; ++b) q1[b] = q2[b] = q3[b] = 0.0;
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    float s1[NT], s2[NT], s3[NT];
#pragma unroll
    for (int b = 0; b < NT; ++b) s1[b] = s2[b] = s3[b] = 0.0f;
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const int64_t r0 = sub_row0(t, a);
      if (r0 >= M) continue;  // (M % 32 == 0: a subtile is entirely inside or outside)
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const int cl = b * 32 + l32;
        const int64_t n = n0 + cl;
        const float* yp = ybn + (r0 + 4 * half) * N + n;
        float* op = out + (r0 + 4 * half) * N + n;
        float yv[16];
        if (do_bn) {
#pragma unroll
          for (int r = 0; r < 16; ++r) yv[r] = yp[(int64_t)((r & 3) + 8 * (r >> 2)) * N];
        }
        const float cf = cco[cl];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = acc[a][b][r] * cf;
          op[(int64_t)((r & 3) + 8 * (r >> 2)) * N] = v;  // (32 lanes: 128 contiguous bytes per half)
          am = fmaxf(am, fabsf(v));
        }
        if (do_bn) {
          const float sc = cco[NTB + cl], sh = cco[2 * NTB + cl], mu = cco[3 * NTB + cl], is = cco[4 * NTB + cl];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = acc[a][b][r] * cf;
            const float da = yv[r] * sc + sh > 0.0f ? v : 0.0f;
            const float xh = (yv[r] - mu) * is;
            s1[b] += da;
            s2[b] += da * xh;
            s3[b] += xh;
          }
        }
      }
    }
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      q1[b] += (double)s1[b];
      q2[b] += (double)s2[b];
      q3[b] += (double)s3[b];
    }
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};
  };

  // ------------------------------------------------------------ main loop: jobs (tile, k-step)
  f32x4 ring[D][MT][2];
#pragma unroll
  for (int u = 0; u < D; ++u) load(ring[u], u < total ? u : 0);
  for (int j0 = 0; j0 < total; j0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int j = j0 + u;
      if (j < total) {
        const int t = j / NK, ks = j - t * NK;
        mma(ring[u], ks);
        const int jn = j + D;
        load(ring[u], jn < total ? jn : j);
        if (ks == NK - 1) epilogue(t);
      }
    }
  }

  if (amax_out) block_amax(amax_out, am, reinterpret_cast<float*>(smem));
  if (do_bn) {
    // per-lane sums -> one slab row per workgroup (row prow, this block's columns), fixed order
    double* red = reinterpret_cast<double*>(smem);
    __syncthreads();  // every MFMA has read its weights: the weight block is free
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      double* q = red + ((wave * 2 + half) * NTB + b * 32 + l32) * 3;
      q[0] = q1[b];
      q[1] = q2[b];
      q[2] = q3[b];
    }
    __syncthreads();
    for (int e = tid; e < NTB * 3; e += CT_THREADS) {
      const int c = e % NTB, k = e / NTB;
      double v = 0.0;
      for (int r = 0; r < RR; ++r) v += red[(r * NTB + c) * 3 + k];
      bnb.slab[((int64_t)prow * 3 + k) * N + n0 + c] = (float)v;
    }
  }
}

// --------------------------------------------------------------------------- host side
// columns of a workgroup's resident weight block for K = C_in (NTB * K = CT_WORDS), 0: not taken
static int ntb_for_k(int K) { return K == 128 ? 256 : K == 256 ? 128 : K == 512 ? 64 : 0; }

// columns per workgroup block for (K, N), or 0 when this kernel does not take the operand
static int convt_x2_ntb(const GatherArg& g, int N, const EpiArg& e) {
  if (g.nsrc != 1 || g.small || g.src[0].layout != 0) return 0;
  if (g.w % 32 != 0 || g.M % 32 != 0) return 0;
  const int ntb = ntb_for_k(g.K);
  if (ntb == 0 || N % ntb != 0) return 0;
  const bool no_sums = e.stats == nullptr && e.colsum == nullptr && e.bnb.slab == nullptr;
  if (g.taps == 1 && e.mode == SELUNET_EP_SCATTER2X && no_sums && N % 128 == 0 && g.src[0].C == g.K) return ntb;
  return 0;
}

bool convt_x2_eligible(const GatherArg& g, int N, const EpiArg& e) { return convt_x2_ntb(g, N, e) > 0; }

// persistent row workgroups per column block: one workgroup per CU overall
static int64_t convt_x2_rows(const GatherArg& g, int N, int ntb) {
  const int rows = 8 * (8 / (ntb / 32)) * 32;
  const int64_t m_tiles = cdiv(g.M, rows);
  const int64_t blocks = std::max<int64_t>(1, N / ntb);
  return std::max<int64_t>(1, std::min<int64_t>(m_tiles, std::max<int64_t>(1, 256 / blocks)));
}

int convt_x2_launch(const GatherArg& g, const float* w, int N, const EpiArg& e, const float* amax_src,
                    hipStream_t st) {
  const int ntb = convt_x2_ntb(g, N, e);
  if (ntb == 0) return fail(SELUNET_EINVAL, "convt_x2: operand not eligible");
  const int blocks = N / ntb;
  const int64_t P = convt_x2_rows(g, N, ntb);
  const float* wcs = w + (int64_t)N * g.K;
  const dim3 grid((unsigned)(P * blocks)), block(CT_THREADS);
  if (ntb == 256)
    hipLaunchKernelGGL((convt_x2_kernel<8>), grid, block, 0, st, g, w, N, e, blocks, (int)P, wcs, amax_src);
  else if (ntb == 128)
    hipLaunchKernelGGL((convt_x2_kernel<4>), grid, block, 0, st, g, w, N, e, blocks, (int)P, wcs, amax_src);
  else
    hipLaunchKernelGGL((convt_x2_kernel<2>), grid, block, 0, st, g, w, N, e, blocks, (int)P, wcs, amax_src);
  return check_launch("convt_x2");
}

// The data-gradient operand (taps = 4 gather of a plain dU, K = 4 C_out of 256 or 512): the weight-block
// columns, 0 when the resident-weight data-gradient kernel does not take it. A function of the operand
// alone, so that selunet_gemm_gather_x2_stats_rows sizes the slab for whichever kernel runs.
int convt_dgrad_x2_ntb(const GatherArg& g, int N) {
  if (g.nsrc != 1 || g.small || g.src[0].layout != 0 || g.src[0].scale != nullptr) return 0;
  if (g.taps != 4 || g.w % 32 != 0 || g.M % 32 != 0 || g.src[0].C % 16 != 0 || g.K != 4 * g.src[0].C) return 0;
  const int ntb = (g.K == 256 || g.K == 512) ? ntb_for_k(g.K) : 0;
  return ntb != 0 && N % ntb == 0 ? ntb : 0;
}

int64_t convt_dgrad_x2_rows(const GatherArg& g, int N) { return convt_x2_rows(g, N, convt_dgrad_x2_ntb(g, N)); }

bool convt_dgrad_x2_eligible(const GatherArg& g, int N, const EpiArg& e) {
  return convt_dgrad_x2_ntb(g, N) > 0 && e.mode == SELUNET_EP_PLAIN && e.out1 == nullptr && e.bias == nullptr &&
         e.stats == nullptr && e.colsum == nullptr;
}

int convt_dgrad_x2_launch(const GatherArg& g, const float* w, int N, const EpiArg& e, const float* amax_src,
                          hipStream_t st) {
  const int ntb = convt_dgrad_x2_ntb(g, N);
  if (ntb == 0 || !convt_dgrad_x2_eligible(g, N, e)) return fail(SELUNET_EINVAL, "convt_dgrad_x2: operand not eligible");
  const int blocks = N / ntb;
  const int64_t P = convt_x2_rows(g, N, ntb);
  const float* wcs = w + (int64_t)N * g.K;
  const dim3 grid((unsigned)(P * blocks)), block(CT_THREADS);
  float* out = reinterpret_cast<float*>(e.out0);
  const float* y = reinterpret_cast<const float*>(e.bnb.y);
  if (e.bnb.slab != nullptr && y == nullptr) return fail(SELUNET_EINVAL, "convt_dgrad_x2: BN-backward sums need y");
  if (ntb == 128)
    hipLaunchKernelGGL((convt_dgrad_x2_kernel<4>), grid, block, 0, st, g, w, N, blocks, (int)P, wcs, amax_src, out, y,
                       e.bnb, e.amax);
  else
    hipLaunchKernelGGL((convt_dgrad_x2_kernel<2>), grid, block, 0, st, g, w, N, blocks, (int)P, wcs, amax_src, out, y,
                       e.bnb, e.amax);
  return check_launch("convt_dgrad_x2");
}

}  // namespace selunet
