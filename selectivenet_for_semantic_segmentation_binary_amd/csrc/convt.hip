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
// The data gradient keeps the staged gather GEMM: its epilogue also reads the producer's y for the
// BatchNorm-backward sums, and with the accumulators in 128 registers those per-lane loads could not
// be batched without spilling (measured 1.66 ms against 1.05 for unpool1).
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

  if (ep.amax) atomic_amax(ep.amax, am);
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

}  // namespace selunet
