// ConvTranspose2d(k=2, s=2) forward and data gradient of the bf16 speed configuration (model.py:44-45,
// 51-52, 57-58: unpool3/2/1) — the resident-weight scheme of convt.hip with bf16 operands, behind
// selunet_gemm_gather (SELUNET_BF16).
//
// The generic gather GEMM stages both operands through LDS for every 32-k slice of every tile; on these
// short-K, large-M products it spends its time staging (gemm_gather<bf16>: 0.095 of the bf16 MFMA peak,
// 3.5 ms per bs=128 step for the six launches). Here, as for the split-fp16 kernels:
//  * a workgroup keeps NTB weight rows x the whole K resident in LDS for its lifetime (bf16: up to
//    65536 words = 128 KiB — twice the columns of the split-fp16 pack: all 256 of unpool1's forward, 256
//    of unpool2's 512, 128 of unpool3's 1024; data gradients 128 / 128 / 64 of 128 / 256 / 512);
//  * the A operand never touches LDS: every lane loads its 16-B row fragment (8 bf16 channels) straight
//    from HBM into a register ring, applies the producer's BN+ReLU there (forward; the value rounded to
//    bf16 as every bf16 stager does) and feeds v_mfma_f32_32x32x16_bf16 (one product per MAC);
//  * accumulators go straight from registers to HBM: the forward adds the bias and scatters each pixel to
//    its 2x2 output block, the data gradient stores dX and folds the producer's BatchNorm-backward sums
//    (da = dX [y sc + sh > 0], da xhat, xhat of the stored bf16 values, as lds_tile_store_acc) into one
//    slab row per workgroup, fixed order.
// One persistent 512-thread workgroup per CU walks the pixel tiles of its column block.
#include "gemm_common.h"

namespace selunet {

constexpr int CB_THREADS = 512;

// NT: 32-column subtiles per wave (NTB = 32 NT resident rows), KC: K, MT = 8 / NT row subtiles per wave,
// D: k-steps of A fragments in flight per lane. DGRAD: the taps = 4 gather of dU (K = 4 C_out, k = tap
// C_out + o) with a PLAIN store and the BN-backward sums; else the forward (taps = 1, BN+ReLU source,
// SCATTER2X store with bias).
template <int NT, int KC, bool DGRAD>
__global__ void __launch_bounds__(CB_THREADS, 1)
convt_bf16_kernel(GatherArg g, const __bf16* __restrict__ W, int N, int n_blocks, int P, __bf16* __restrict__ out,
                  const float* __restrict__ bias, const __bf16* __restrict__ ybn, BnBwdArg bnb) {
  constexpr int NTB = NT * 32;
  constexpr int NK = KC / 16;  // 16-k MFMA steps per tile
  constexpr int MT = 8 / NT;
  constexpr int D = MT >= 4 ? 2 : 4 / MT;
  constexpr int ROWS = 8 * MT * 32;  // pixel rows per tile
  constexpr int RB = 2 * KC + 16;    // LDS bytes per weight row (odd number of 16-B slots: conflict-free)
  constexpr int NCO = DGRAD ? 4 : 2;
  constexpr int RR = 16;  // partial-sum rows per column (data gradient): 8 waves x 2 lane halves
  static_assert(!DGRAD || RR * NTB * 3 * (int)sizeof(double) <= NTB * RB, "column reduction scratch exceeds the block");
  static_assert(NTB * RB + NCO * KC * 4 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NTB * RB + NCO * (DGRAD ? NTB : KC) * 4];
  float* cco = reinterpret_cast<float*>(smem + NTB * RB);  // fwd: [2][KC] scale, shift; dgrad: [4][NTB]

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
  const bool do_bn = DGRAD && bnb.slab != nullptr;
  const SrcArg& s0 = g.src[0];

  // ------------------------------------------------------------ resident weights, coefficients
  {
    constexpr int V = KC / 8;  // uint4 per row
    for (int i = tid; i < NTB * V; i += CB_THREADS) {
      const int row = i / V, v = i - row * V;
      *reinterpret_cast<uint4*>(smem + row * RB + v * 16) =
          *reinterpret_cast<const uint4*>(W + (int64_t)(n0 + row) * KC + v * 8);
    }
    if constexpr (DGRAD) {
      for (int c = tid; c < NTB; c += CB_THREADS) {
        cco[c] = do_bn ? bnb.scale[n0 + c] : 0.0f;
        cco[NTB + c] = do_bn ? bnb.shift[n0 + c] : 0.0f;
        cco[2 * NTB + c] = do_bn ? bnb.mean[n0 + c] : 0.0f;
        cco[3 * NTB + c] = do_bn ? bnb.invstd[n0 + c] : 0.0f;
      }
    } else {
      for (int c = tid; c < KC; c += CB_THREADS) {
        cco[c] = s0.scale ? s0.scale[c] : 1.0f;
        cco[KC + c] = s0.scale ? s0.shift[c] : 0.0f;
      }
    }
  }
  const bool relu = !DGRAD && s0.scale != nullptr && s0.relu;
  const bool xform = !DGRAD && s0.scale != nullptr;
  const __bf16* src = reinterpret_cast<const __bf16*>(s0.data);
  const int C = s0.C;  // fwd: C_in (= K); dgrad: C_out (K = 4 C, C % 16 == 0: a 16-k step lies in one tap)
  __syncthreads();

  auto sub_row0 = [&](int t, int a) -> int64_t {
    return (int64_t)(prow + (int64_t)t * P) * ROWS + (wave * MT + a) * 32;
  };
  auto load = [&](uint4 (&r)[MT], int j) __attribute__((always_inline)) {
    const int t = j / NK, ks = j - t * NK;
    const int k = ks * 16 + half * 8;
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      int64_t r0 = sub_row0(t, a);
      r0 = r0 < M ? r0 : M - 32;
      const __bf16* p;
      if constexpr (DGRAD) {
        // subtile a: pixels r0 .. r0 + 31 of one image row (img, y); this lane's pixel x0 + l32 reads
        // dU at (2y + tap / 2, 2 (x0 + l32) + tap % 2)
        const int tap = k / C, c = k - tap * C;
        const unsigned mu = (unsigned)r0, x0 = mu % (unsigned)g.w, tt = mu / (unsigned)g.w;
        const unsigned y = tt % (unsigned)g.h, img = tt / (unsigned)g.h;
        const int64_t pix = ((int64_t)img * g.hs + 2 * y + (tap >> 1)) * g.ws + 2 * (x0 + l32) + (tap & 1);
        p = src + pix * C + c;
      } else {
        p = src + (r0 + l32) * C + k;
      }
      r[a] = *reinterpret_cast<const uint4*>(p);
    }
  };
  // the forward's A fragment: BN+ReLU of the producer on 8 channels k .. k+7, rounded to bf16
  auto xf = [&](uint4 raw, int k) __attribute__((always_inline)) -> bf16x8 {
    bf16x8 v = __builtin_bit_cast(bf16x8, raw);
    if (!xform) return v;
    const f32x4 s0v = *reinterpret_cast<const f32x4*>(cco + k), s1v = *reinterpret_cast<const f32x4*>(cco + k + 4);
    const f32x4 t0v = *reinterpret_cast<const f32x4*>(cco + KC + k), t1v = *reinterpret_cast<const f32x4*>(cco + KC + k + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float f = (float)v[e] * (e < 4 ? s0v[e] : s1v[e - 4]) + (e < 4 ? t0v[e] : t1v[e - 4]);
      if (relu) f = fmaxf(f, 0.0f);
      v[e] = (__bf16)f;
    }
    return v;
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  auto mma = [&](const uint4 (&r)[MT], int ks) __attribute__((always_inline)) {
    const int k = ks * 16 + half * 8;
    const int boff = ks * 32 + half * 16;  // B fragment of column subtile b: row b*32 + l32, k .. k+7
    bf16x8 av[MT];
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      if constexpr (DGRAD) av[a] = __builtin_bit_cast(bf16x8, r[a]);
      else av[a] = xf(r[a], k);
    }
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(smem + (b * 32 + l32) * RB + boff);
#pragma unroll
      for (int a = 0; a < MT; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a], bv, acc[a][b], 0, 0, 0);
    }
  };

  // ------------------------------------------------------------ epilogues (registers -> HBM)
  double q1[DGRAD ? NT : 1], q2[DGRAD ? NT : 1], q3[DGRAD ? NT : 1];
#pragma unroll
  for (int b = 0; b < (DGRAD ? NT : 1); ++b) q1[b] = q2[b] = q3[b] = 0.0;
  const int Cq = N / 4;  // forward: C_out
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    if constexpr (!DGRAD) {
      float cbias[NT];
#pragma unroll
      for (int b = 0; b < NT; ++b) cbias[b] = bias ? bias[(n0 + b * 32 + l32) % Cq] : 0.0f;
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int64_t r0 = sub_row0(t, a);
        if (r0 >= M) continue;  // (M % 32 == 0: a subtile is entirely inside or outside)
        const unsigned mu = (unsigned)r0, x0 = mu % (unsigned)g.w, tt = mu / (unsigned)g.w;
        const unsigned y = tt % (unsigned)g.h, img = tt / (unsigned)g.h;
        const int64_t row_even = ((int64_t)img * (2 * g.h) + 2 * y) * (2 * g.w);  // output row 2y
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const int n = n0 + b * 32 + l32;
          const int ab = n / Cq, o = n - ab * Cq;
          const int64_t base = row_even + (int64_t)(ab >> 1) * (2 * g.w) + (ab & 1);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int px = (int)x0 + (r & 3) + 8 * (r >> 2) + 4 * half;
            out[(base + 2 * px) * Cq + o] = (__bf16)(acc[a][b][r] + cbias[b]);  // (32 lanes: 64 contiguous bytes)
          }
        }
      }
    } else {
      float s1[NT], s2[NT], s3[NT];
#pragma unroll
      for (int b = 0; b < NT; ++b) s1[b] = s2[b] = s3[b] = 0.0f;
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int64_t r0 = sub_row0(t, a);
        if (r0 >= M) continue;
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const int cl = b * 32 + l32;
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
            const float sc = cco[cl], sh = cco[NTB + cl], mu = cco[2 * NTB + cl], is = cco[3 * NTB + cl];
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
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        q1[b] += (double)s1[b];
        q2[b] += (double)s2[b];
        q3[b] += (double)s3[b];
      }
    }
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};
  };

  // ------------------------------------------------------------ main loop: jobs (tile, k-step)
  uint4 ring[D][MT];
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

  if constexpr (DGRAD) {
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
      for (int e = tid; e < NTB * 3; e += CB_THREADS) {
        const int c = e % NTB, k = e / NTB;
        double v = 0.0;
        for (int r = 0; r < RR; ++r) v += red[(r * NTB + c) * 3 + k];
        bnb.slab[((int64_t)prow * 3 + k) * N + n0 + c] = (float)v;
      }
    }
  }
}

// --------------------------------------------------------------------------- host side
// resident columns per workgroup for (K, N) of the forward / data gradient, 0: not taken
static int convt_bf16_ntb(int K, int N, bool dgrad) {
  int ntb = 0;
  if (!dgrad) ntb = K == 128 || K == 256 ? 256 : K == 512 ? 128 : 0;
  else ntb = K == 256 || K == 512 ? 128 : K == 1024 ? 64 : 0;
  return ntb != 0 && N % ntb == 0 ? ntb : 0;
}

int convt_bf16_fwd_ntb(const GatherArg& g, int N) {
  if (g.nsrc != 1 || g.small || g.src[0].layout != 0 || g.taps != 1 || g.src[0].C != g.K) return 0;
  if (g.w % 32 != 0 || g.M % 32 != 0 || N % 128 != 0) return 0;
  return convt_bf16_ntb(g.K, N, false);
}

int convt_dgrad_bf16_ntb(const GatherArg& g, int N) {
  if (g.nsrc != 1 || g.small || g.src[0].layout != 0 || g.src[0].scale != nullptr) return 0;
  if (g.taps != 4 || g.w % 32 != 0 || g.M % 32 != 0 || g.src[0].C % 16 != 0 || g.K != 4 * g.src[0].C) return 0;
  return convt_bf16_ntb(g.K, N, true);
}

bool convt_bf16_eligible(const GatherArg& g, int N, const EpiArg& e) {
  const bool no_sums = e.stats == nullptr && e.colsum == nullptr && e.bnb.slab == nullptr && e.amax == nullptr;
  return e.mode == SELUNET_EP_SCATTER2X && no_sums && convt_bf16_fwd_ntb(g, N) > 0;
}

bool convt_dgrad_bf16_eligible(const GatherArg& g, int N, const EpiArg& e) {
  return convt_dgrad_bf16_ntb(g, N) > 0 && e.mode == SELUNET_EP_PLAIN && e.out1 == nullptr && e.bias == nullptr &&
         e.stats == nullptr && e.colsum == nullptr && e.amax == nullptr;
}

// persistent row workgroups per column block: one workgroup per CU overall (= statistics slab rows)
static int64_t convt_bf16_rows(const GatherArg& g, int N, int ntb) {
  const int rows = 8 * (8 / (ntb / 32)) * 32;
  const int64_t m_tiles = cdiv(g.M, rows);
  const int64_t blocks = std::max<int64_t>(1, N / ntb);
  return std::max<int64_t>(1, std::min<int64_t>(m_tiles, std::max<int64_t>(1, 256 / blocks)));
}

int64_t convt_dgrad_bf16_rows(const GatherArg& g, int N) { return convt_bf16_rows(g, N, convt_dgrad_bf16_ntb(g, N)); }

int convt_bf16_launch(const GatherArg& g, const void* w, int N, const EpiArg& e, hipStream_t st) {
  const bool dgrad = g.taps == 4;
  const int ntb = dgrad ? convt_dgrad_bf16_ntb(g, N) : convt_bf16_fwd_ntb(g, N);
  if (ntb == 0 || !(dgrad ? convt_dgrad_bf16_eligible(g, N, e) : convt_bf16_eligible(g, N, e)))
    return fail(SELUNET_EINVAL, "convt_bf16: operand not eligible");
  if (dgrad && e.bnb.slab != nullptr && e.bnb.y == nullptr)
    return fail(SELUNET_EINVAL, "convt_bf16: BN-backward sums need y");
  const int blocks = N / ntb;
  const int64_t P = convt_bf16_rows(g, N, ntb);
  const dim3 grid((unsigned)(P * blocks)), block(CB_THREADS);
  const __bf16* W = reinterpret_cast<const __bf16*>(w);
  __bf16* out = reinterpret_cast<__bf16*>(e.out0);
  const __bf16* y = reinterpret_cast<const __bf16*>(e.bnb.y);
#define CB_LAUNCH(NT_, KC_, DG_)                                                                                  \
  hipLaunchKernelGGL((convt_bf16_kernel<NT_, KC_, DG_>), grid, block, 0, st, g, W, N, blocks, (int)P, out, e.bias, y, \
                     e.bnb)
  if (!dgrad) {
    if (g.K == 128) CB_LAUNCH(8, 128, false);
    else if (g.K == 256) CB_LAUNCH(8, 256, false);
    else CB_LAUNCH(4, 512, false);
  } else {
    if (g.K == 256) CB_LAUNCH(4, 256, true);
    else if (g.K == 512) CB_LAUNCH(4, 512, true);
    else CB_LAUNCH(2, 1024, true);
  }
#undef CB_LAUNCH
  return check_launch("convt_bf16");
}

}  // namespace selunet
