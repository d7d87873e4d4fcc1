// Implicit-GEMM MFMA kernels for the UNet_B convolutions on gfx950.
//
//  * gemm_gather: out[M][N] = G[M][K] * B[N][K]^T, where G is a gathered view of one or two
//    NHWC activations (3x3 / 1x1 / 2x2-stride-2 taps, channel concat) with the producing
//    block's BatchNorm+ReLU folded into the load. Used for conv3x3 forward (model.py:11),
//    conv3x3 data-gradient, ConvTranspose2d forward (model.py:44,51,57) and its
//    data-gradient. Epilogue: NHWC store (plain / cat-split / 2x scatter + bias) and the
//    per-workgroup BatchNorm column statistics of the fp32 accumulators.
//  * gemm_wgrad: out[I][J] += sum_m Gp[m][I] * Gq[m][J] — weight gradients, the reduction
//    over pixels split across workgroups, fp32 atomics into a packed buffer.
//
// Tiling (256 threads = 4 waves as 2x2, 64-wide wavefronts): 128 x BN output tile, one
// 128-byte K slice per stage (32 fp32 / 64 bf16), register-staged double-buffered LDS with
// the next slice's global loads in flight during the current slice's MFMAs (load early,
// write late). Rows of the LDS tiles are padded to 144 B so that the 16-B fragment reads
// (ds_read_b128) of 16 consecutive rows fall on 16 distinct bank slots.
//  fp32: v_mfma_f32_32x32x2_f32 (exact fp32); each 16-B fragment holds 4 k's of one half-wave,
//        consumed by 4 MFMAs (k = 4*half + j), B uses the same k assignment.
//  bf16: v_mfma_f32_32x32x16_bf16; a 16-B fragment is the 8 k's of one half-wave.
#include <type_traits>

#include "gemm_common.h"

namespace selunet {

// Persistent over output tiles: workgroup (prow, n_tile) owns column block n_tile and the row tiles
// prow, prow + P, prow + 2P, ...; its K stages run as one continuous pipeline across tile
// boundaries, so the first stage of the next tile is loading while this tile's last MFMAs and its
// epilogue run (short-K GEMMs — ConvTranspose2d with K = 128..512 — are otherwise one exposed load
// latency + one exposed epilogue per tile). Statistics accumulate in registers over the tiles and
// are written once per workgroup (slab row prow). P = number of row tiles gives the one-tile-per-
// workgroup launch.
//
// X2 (fp32, vector gathers only): the split-fp16 form (selunet_gemm_gather_x2; ConvTranspose2d forward
// and data gradient in fp32 training): every staged A value is scaled by 2^e (range words amax0/amax1)
// and written as fp16 high / low parts into the 128-B K slice (bytes 0-63 high, 64-127 low), B is a
// split-fp16 pack of the same layout (row unscale factors in wcs), three v_mfma_f32_32x32x16_f16 per
// 16-k step, accumulators unscaled before the epilogue — as conv3x3_halo_persist_kernel<.., X2>.
template <typename T, int BN, bool SMALL, bool X2, int BMT = BM, int NTH = 256>
__global__ void __launch_bounds__(NTH, NTH == 256 ? 2 : 1)
gemm_gather_kernel(GatherArg g, const T* __restrict__ B, int N, int k_pad, EpiArg ep, int n_tiles, int P,
                   const float* __restrict__ wcs, const float* __restrict__ amax0, const float* __restrict__ amax1) {
  static_assert(!X2 || (std::is_same<T, float>::value && !SMALL), "split-fp16 form: fp32 vector gathers");
  constexpr int E = 16 / sizeof(T);          // elements per 16-B vector
  constexpr int BKE = 128 / sizeof(T);       // K elements per stage
  constexpr int WN = BN / 2;                 // wave tile columns (waves: BMT / 64 rows x 2 columns)
  constexpr int NT = WN / 32;                // 32x32 subtiles per wave (columns)
  constexpr int MT = 2;                      // 64 rows per wave
  constexpr int RP = NTH / 8;                // rows per staging pass (8 16-B chunks per 128-B row)
  constexpr int AR = BMT / RP;               // A rows staged per thread
  constexpr int BR = BN / RP;                // B rows staged per thread
  static_assert(BMT == 64 * (NTH / 64) / 2, "two wave columns of 64-row waves");

  constexpr int SMEM_MAIN = 2 * (BMT + BN) * ROWB, SMEM_EPI = BMT * (BN + 4) * 4 + BMT * 8;  // (+ row bases)
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI];
  unsigned char* As = smem;                          // [2][BMT][ROWB]
  unsigned char* Bs = smem + 2 * BMT * ROWB;         // [2][BN][ROWB]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int half = lane >> 5, l32 = lane & 31;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int n_tile = lb % n_tiles;
  const int64_t prow = lb / n_tiles;
  const int n0 = n_tile * BN;
  const int64_t m_tiles = (g.M + BMT - 1) / BMT;
  const int nk = k_pad / BKE;
  const int64_t total = (m_tiles - prow + P - 1) / P * nk;  // stages of this workgroup (prow < P <= m_tiles)

  const int cc = tid & 7;       // 16-B chunk within the 128-B K slice
  const int rr = tid >> 3;      // base row (0..RP-1)
  float xs = 1.0f;              // X2: operand scale 2^e
  float cfac[NT] = {};          // X2: accumulator unscale per 32-column subtile (this lane's column)
  if constexpr (X2) {
    float am = amax0 ? amax0[0] : 0.0f;
    if (g.nsrc > 1 && amax1) am = fmaxf(am, amax1[0]);
    float inv;
    xs = x2_scale(am, &inv);
#pragma unroll
    for (int b = 0; b < NT; ++b) cfac[b] = wcs[n0 + wn * WN + b * 32 + l32] * inv;
  }
  // A row value quad -> LDS (X2: scaled and split into the high / low halves of the K slice)
  auto put_a = [&](unsigned char* a_dst, int row, uint4 v) __attribute__((always_inline)) {
    if constexpr (X2) {
      float f[4];
      __builtin_memcpy(f, &v, 16);
      f16x4 h, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        _Float16 x, y;
        x2_split(f[e] * xs, x, y);
        h[e] = x;
        l[e] = y;
      }
      *reinterpret_cast<f16x4*>(a_dst + row * ROWB + cc * 8) = h;
      *reinterpret_cast<f16x4*>(a_dst + row * ROWB + 64 + cc * 8) = l;
    } else {
      *reinterpret_cast<uint4*>(a_dst + row * ROWB + cc * 16) = v;
    }
  };

  // One staged K slice, held in registers between its loads and its LDS write. Loads are issued
  // unconditionally (rows / pixels clamped to valid addresses, zeroed when written to LDS) so the
  // compiler counts outstanding loads instead of waiting on each; the stage travels by value (a
  // lambda-captured register array gets demoted to scratch).
  struct Stage {
    uint4 a[AR];
    uint4 b[BR];
    float scv[E], shv[E];  // folded BN + ReLU coefficients of the staged channels (same for every row)
    unsigned ok;           // bit i: A row i is inside the image (else zero padding)
    int src;
  };

  auto load_stage = [&](int64_t m_tile, int kc) __attribute__((always_inline)) {
    Stage st;
    const int k0 = kc * BKE;
    const int64_t m0 = m_tile * BMT;
    st.ok = 0;
    st.src = 0;
    if constexpr (!SMALL) {
      const int tap = k0 / g.Ctot;
      int c0 = k0 - tap * g.Ctot;
      int s = 0;
      if (g.nsrc > 1 && c0 >= g.src[0].C) {
        c0 -= g.src[0].C;
        s = 1;
      }
      st.src = s;
      const int st_c = c0 + cc * E;
      const SrcArg sa = pick_src(g, s);
      const T* base = reinterpret_cast<const T*>(sa.data);
      // (always loaded — from the weights when there is no transform — so no branch per element)
      const bool xf = sa.scale != nullptr;
      const float* scp = xf ? sa.scale + st_c : reinterpret_cast<const float*>(B);
      const float* shp = xf ? sa.shift + st_c : reinterpret_cast<const float*>(B);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        st.scv[e] = scp[e];
        st.shv[e] = shp[e];
      }
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int64_t m = m0 + rr + RP * i;
        const bool rv = m < g.M;
        const unsigned mu = rv ? (unsigned)m : 0u;  // M < 2^31 (host check)
        const unsigned rx = mu % (unsigned)g.w, t = mu / (unsigned)g.w;
        const unsigned ry = t % (unsigned)g.h, rimg = t / (unsigned)g.h;
        int ys, xs;
        if (rv && src_pixel(g, tap, (int)ry, (int)rx, ys, xs)) st.ok |= 1u << i;
        ys = min(max(ys, 0), g.hs - 1);
        xs = min(max(xs, 0), g.ws - 1);
        const int64_t off = (((int64_t)rimg * g.hs + ys) * g.ws + xs) * sa.C + st_c;
        st.a[i] = *reinterpret_cast<const uint4*>(base + off);
      }
    } else {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        T v[E];
        const int64_t m = m0 + rr + RP * i;
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = from_f<T>(gather_scalar<T>(g, m, k0 + cc * E + e));
        __builtin_memcpy(&st.a[i], v, 16);
        st.ok |= 1u << i;
      }
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = n0 + rr + RP * i;
      st.b[i] = *reinterpret_cast<const uint4*>(B + (int64_t)n * k_pad + k0 + cc * E);
    }
    return st;
  };

  auto store_stage = [&](const Stage& st, int buf) __attribute__((always_inline)) {
    unsigned char* a_dst = As + buf * BMT * ROWB;
    unsigned char* b_dst = Bs + buf * BN * ROWB;
    const SrcArg sa = pick_src(g, st.src);
    if (!SMALL && sa.scale != nullptr) {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        T v[E];
        __builtin_memcpy(v, &st.a[i], 16);
        const bool ok = (st.ok >> i) & 1u;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          float f = to_f(v[e]) * st.scv[e] + st.shv[e];
          f = sa.relu ? fmaxf(f, 0.0f) : f;
          v[e] = from_f<T>(ok ? f : 0.0f);
        }
        uint4 o;
        __builtin_memcpy(&o, v, 16);
        put_a(a_dst, rr + RP * i, o);
      }
    } else {
#pragma unroll
      for (int i = 0; i < AR; ++i) put_a(a_dst, rr + RP * i, ((st.ok >> i) & 1u) ? st.a[i] : make_uint4(0, 0, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < BR; ++i)
      *reinterpret_cast<uint4*>(b_dst + (rr + RP * i) * ROWB + cc * 16) = st.b[i];
  };

  auto mma_stage = [&](f32x16 (&acc)[MT][NT], int buf) __attribute__((always_inline)) {
    const unsigned char* a_src = As + buf * BMT * ROWB;
    const unsigned char* b_src = Bs + buf * BN * ROWB;
    if constexpr (X2) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        f16x8 ah[MT], al[MT], bh[NT], bl[NT];
#pragma unroll
        for (int a = 0; a < MT; ++a) {
          const unsigned char* p = a_src + (wm * 64 + a * 32 + l32) * ROWB + half * 16;
          ah[a] = *reinterpret_cast<const f16x8*>(p + ks * 32);
          al[a] = *reinterpret_cast<const f16x8*>(p + (2 + ks) * 32);
        }
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const unsigned char* p = b_src + (wn * WN + b * 32 + l32) * ROWB + half * 16;
          bh[b] = *reinterpret_cast<const f16x8*>(p + ks * 32);
          bl[b] = *reinterpret_cast<const f16x8*>(p + (2 + ks) * 32);
        }
#pragma unroll
        for (int a = 0; a < MT; ++a)
#pragma unroll
          for (int b = 0; b < NT; ++b) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
          }
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int boff = q * 32 + half * 16;
      uint4 af[MT], bfr[NT];
#pragma unroll
      for (int a = 0; a < MT; ++a)
        af[a] = *reinterpret_cast<const uint4*>(a_src + (wm * 64 + a * 32 + l32) * ROWB + boff);
#pragma unroll
      for (int b = 0; b < NT; ++b)
        bfr[b] = *reinterpret_cast<const uint4*>(b_src + (wn * WN + b * 32 + l32) * ROWB + boff);
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) Mma<T>::run(acc[a][b], af[a], bfr[b]);
    }
  };

  // ------------------------------------------------------------------ epilogue (LDS-staged)
  float* tile = reinterpret_cast<float*>(smem);  // [BMT][BN + 4] over the (idle) stage buffers
  int64_t* rowbase = reinterpret_cast<int64_t*>(smem + BMT * (BN + 4) * 4);
  const int Cq = N >> 2;
  const TileStats ts = tile_stats(ep, prow, n0, N);
  using Acc = typename StatAcc<T>::type;
  static_assert(stats_flush_bytes<BN, NTH, Acc>() <= (int)sizeof(smem), "statistics scratch exceeds LDS");
  Acc s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float amx = 0.0f;  // running max |stored value| (epilogue range word)
  auto epilogue = [&](f32x16 (&acc)[MT][NT], int64_t m_tile) __attribute__((always_inline)) {
    const int64_t m0 = m_tile * BMT;
    if constexpr (X2) {
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] *= cfac[b];
    }
    acc_to_lds<MT, NT, BN>(tile, acc, wm * 64, wn * WN, lane);
    // SCATTER2X: each tile row's output base (pixel (img, 2y, 2x) of the 2x-upsampled grid) decoded
    // once into LDS past the tile, instead of three integer divisions per stored 16-B chunk
    if (ep.mode == SELUNET_EP_SCATTER2X && tid < BMT) {
      const int64_t m = m0 + tid;
      int64_t base = -1;
      if (m < g.M) {
        const unsigned mu = (unsigned)m, x = mu % (unsigned)g.w, t = mu / (unsigned)g.w;
        const unsigned y = t % (unsigned)g.h, img = t / (unsigned)g.h;
        base = (((int64_t)img * (2 * g.h) + 2 * y) * (2 * g.w) + 2 * x) * Cq;
      }
      rowbase[tid] = base;
    }
    __syncthreads();
    auto dst = [&](int row, int c) -> T* {
      const int col = n0 + c;
      if (ep.mode == SELUNET_EP_SCATTER2X) {
        const int64_t base = rowbase[row];
        if (base < 0) return nullptr;
        const int ab = col / Cq, cq = col - ab * Cq;
        return reinterpret_cast<T*>(ep.out0) + base + ((int64_t)(ab >> 1) * (2 * g.w) + (ab & 1)) * Cq + cq;
      }
      const int64_t m = m0 + row;
      if (m >= g.M) return nullptr;
      if (ep.mode == SELUNET_EP_PLAIN) return reinterpret_cast<T*>(ep.out0) + m * N + col;
      return col < ep.split ? reinterpret_cast<T*>(ep.out0) + m * ep.split + col
                            : reinterpret_cast<T*>(ep.out1) + m * (N - ep.split) + (col - ep.split);
    };
    auto bias_col = [&](int c) { return ep.mode == SELUNET_EP_SCATTER2X ? (n0 + c) % Cq : n0 + c; };
    lds_tile_store_acc<T, BMT, BN, NTH>(tile, tid, dst, ep.bias, bias_col, ts, s1, s2, s3, amx);
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  {
    const Stage st0 = load_stage(prow, 0);
    store_stage(st0, 0);
  }
  __syncthreads();

  int64_t mt = prow;
  int kc = 0;
  for (int64_t s = 0; s < total; ++s) {
    const bool last_k = kc + 1 == nk;
    const bool more = s + 1 < total;
    const int64_t nmt = last_k ? mt + P : mt;
    const int nkc = last_k ? 0 : kc + 1;
    // the next stage (of this tile or the next one) loads while this one multiplies; the last
    // stage reloads its own slice (valid addresses, never stored)
    const Stage nxt = load_stage(more ? nmt : mt, more ? nkc : kc);
    __builtin_amdgcn_sched_barrier(0);  // all of the next stage's loads ahead of this stage's MFMAs
    mma_stage(acc, (int)(s & 1));
    if (last_k) {
      __syncthreads();  // both stage buffers idle: the tile is staged over them
      epilogue(acc, mt);
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};
      __syncthreads();
    }
    if (more) store_stage(nxt, (int)((s + 1) & 1));
    __syncthreads();
    mt = nmt;
    kc = nkc;
  }
  tile_stats_flush<BN, NTH>(tile, tid, ts, s1, s2, s3, amx);
}

// =========================================================================== gemm_wgrad
// out[I][J] += sum_m P[m][i] Q[m][j]; fp32 operands via v_mfma_f32_32x32x2_f32. LDS tiles are
// [32 rows (m)][BI or BJ] fp32 so the MFMA operands (one element per lane: A[i][k], B[k][j])
// are single conflict-free ds_read_b32 along a row.
template <typename T>
__device__ __forceinline__ f32x4 gather_vec4(const GatherArg& g, int64_t m, int k, int tap, int s, int c,
                                    bool vec) {
  if (!vec) {
    return f32x4{gather_scalar<T>(g, m, k), gather_scalar<T>(g, m, k + 1), gather_scalar<T>(g, m, k + 2),
                 gather_scalar<T>(g, m, k + 3)};
  }
  if (m >= g.M) return f32x4{0, 0, 0, 0};
  const int64_t pix = src_index(g, m, tap);
  if (pix < 0) return f32x4{0, 0, 0, 0};
  const SrcArg sa = pick_src(g, s);
  f32x4 v = Vec4<T>::load(reinterpret_cast<const T*>(sa.data) + pix * sa.C + c);
  if (sa.scale) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float f = v[e] * sa.scale[c + e] + sa.shift[c + e];
      v[e] = sa.relu ? fmaxf(f, 0.0f) : f;
    }
  }
  return v;
}

template <typename T, int BI, int BJ, bool SMALL>
__global__ void __launch_bounds__(256, 2)
gemm_wgrad_kernel(GatherArg P, GatherArg Q, float* __restrict__ out, int ldo, int64_t mchunk,
                  int tiles_j, int tiles, float* __restrict__ ws, int64_t ws_stride) {
  constexpr int KM = 32;              // pixels per stage
  constexpr int WI = BI / 2, WJ = BJ / 2;
  constexpr int MT = WI / 32, NT = WJ / 32;
  constexpr int CPI = BI / 4, CPJ = BJ / 4;       // float4 chunks per row
  constexpr int RPI = 256 / CPI, RPJ = 256 / CPJ; // rows per pass
  constexpr int PI = KM / RPI, PJ = KM / RPJ;     // passes

  __shared__ __attribute__((aligned(16))) float Ps[2][KM][BI];
  __shared__ __attribute__((aligned(16))) float Qs[2][KM][BJ];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const int half = lane >> 5, l32 = lane & 31;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lb % tiles;
  const int64_t split = lb / tiles;
  const int i0 = (tile / tiles_j) * BI;
  const int j0 = (tile % tiles_j) * BJ;
  const int64_t mb = split * mchunk;
  const int64_t me = min(P.M, mb + mchunk);
  if (mb >= me) return;

  // fixed column chunk of this thread -> (tap, source, channel) for P and Q
  const int pc = tid % CPI, pr = tid / CPI;
  const int qc = tid % CPJ, qr = tid / CPJ;
  const int pk = i0 + pc * 4, qk = j0 + qc * 4;
  int ptap = 0, ps = 0, pch = 0, qtap = 0, qs = 0, qch = 0;
  const bool pvec = !SMALL || !P.small, qvec = !SMALL || !Q.small;
  if (pvec) {
    ptap = pk / P.Ctot;
    pch = pk - ptap * P.Ctot;
    if (P.nsrc > 1 && pch >= P.src[0].C) { pch -= P.src[0].C; ps = 1; }
  }
  if (qvec) {
    qtap = qk / Q.Ctot;
    qch = qk - qtap * Q.Ctot;
    if (Q.nsrc > 1 && qch >= Q.src[0].C) { qch -= Q.src[0].C; qs = 1; }
  }
  const bool pin = pk < P.K, qin = qk < Q.K;

  f32x4 rp[PI], rq[PJ];
  auto load_stage = [&](int64_t m_base) {
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const int64_t m = m_base + pr + RPI * i;
      rp[i] = (pin && m < me) ? gather_vec4<T>(P, m, pk, ptap, ps, pch, pvec) : f32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < PJ; ++i) {
      const int64_t m = m_base + qr + RPJ * i;
      rq[i] = (qin && m < me) ? gather_vec4<T>(Q, m, qk, qtap, qs, qch, qvec) : f32x4{0, 0, 0, 0};
    }
  };
  auto store_stage = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PI; ++i) *reinterpret_cast<f32x4*>(&Ps[buf][pr + RPI * i][pc * 4]) = rp[i];
#pragma unroll
    for (int i = 0; i < PJ; ++i) *reinterpret_cast<f32x4*>(&Qs[buf][qr + RPJ * i][qc * 4]) = rq[i];
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  const int64_t nst = (me - mb + KM - 1) / KM;
  load_stage(mb);
  store_stage(0);
  __syncthreads();
  for (int64_t st = 0; st < nst; ++st) {
    const int buf = (int)(st & 1);
    if (st + 1 < nst) load_stage(mb + (st + 1) * KM);
#pragma unroll
    for (int kk = 0; kk < KM / 2; ++kk) {
      const int row = 2 * kk + half;
      float av[MT], bv[NT];
#pragma unroll
      for (int a = 0; a < MT; ++a) av[a] = Ps[buf][row][wi * WI + a * 32 + l32];
#pragma unroll
      for (int b = 0; b < NT; ++b) bv[b] = Qs[buf][row][wj * WJ + b * 32 + l32];
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    if (st + 1 < nst) store_stage(buf ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int j = j0 + wj * WJ + b * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + wi * WI + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (ws) ws[split * ws_stride + (int64_t)i * ldo + j] = acc[a][b][r];
        else atomicAdd(out + (int64_t)i * ldo + j, acc[a][b][r]);
      }
    }
}

// =========================================================================== gemm_wgrad (split fp16)
// fp32 weight gradient on split-fp16 operands (selunet_gemm_wgrad_x2: the ConvTranspose2d weight
// gradient in fp32 training): the bf16 kernel's structure (natural [pixel][column] LDS tiles,
// ds_read_b64_tr_b16 operand reads) with each fp32 operand column scaled by its source's 2^e and
// stored as two fp16 planes (high, low); three v_mfma_f32_32x32x16_f16 per 16-pixel step (hl, lh,
// hh); each output (i, j) is unscaled by its two columns' 2^-e before the split partial is written.
// NTH = 512: 256-column tiles on 8 waves (2 x 4), one workgroup per CU — the ConvTranspose2d weight
// gradients re-read each operand once per tile of the other, so wider tiles halve that traffic.
template <int BI, int BJ, int NTH = 256>
__global__ void __launch_bounds__(NTH, NTH == 256 ? 2 : 1)
gemm_wgrad_x2_kernel(GatherArg P, GatherArg Q, int ldo, int64_t mchunk, int tiles_j, int tiles, float* __restrict__ ws,
                     int64_t ws_stride, const float* __restrict__ amax_p0, const float* __restrict__ amax_p1,
                     const float* __restrict__ amax_q0, const float* __restrict__ amax_q1) {
  constexpr int KM = 32;                           // pixels per stage
  constexpr int PADE = 32;                         // 64 B row pad (bank spread for tr reads)
  constexpr int LDI = BI + PADE, LDJ = BJ + PADE;  // row strides in halves
  constexpr int WGJ = NTH / 128;                   // waves along j (2 along i)
  constexpr int WI = BI / 2, WJ = BJ / WGJ;
  constexpr int MT = WI / 32, NT = WJ / 32;
  constexpr int CPI = BI / 4, CPJ = BJ / 4;        // 16-B fp32 chunks per row
  constexpr int RPI = NTH / CPI, RPJ = NTH / CPJ;
  constexpr int PI = KM / RPI, PJ = KM / RPJ;
  static_assert(PI >= 1 && PJ >= 1 && MT >= 1 && NT >= 1, "stage rows must cover the threads");

  __shared__ __attribute__((aligned(16))) _Float16 Ps[2][2][KM][LDI];
  __shared__ __attribute__((aligned(16))) _Float16 Qs[2][2][KM][LDJ];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wi = wave / WGJ, wj = wave % WGJ;
  const int half = lane >> 5, l32 = lane & 31;
  const int grp_hi = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lb % tiles;
  const int64_t split = lb / tiles;
  const int i0 = (tile / tiles_j) * BI;
  const int j0 = (tile % tiles_j) * BJ;
  const int64_t mb = split * mchunk;
  const int64_t me = min(P.M, mb + mchunk);

  const int pc = tid % CPI, pr = tid / CPI;
  const int qc = tid % CPJ, qr = tid / CPJ;
  const int pk = i0 + pc * 4, qk = j0 + qc * 4;
  int ptap = pk / P.Ctot, pch = pk - ptap * P.Ctot, ps = 0;
  if (P.nsrc > 1 && pch >= P.src[0].C) { pch -= P.src[0].C; ps = 1; }
  int qtap = qk / Q.Ctot, qch = qk - qtap * Q.Ctot, qs = 0;
  if (Q.nsrc > 1 && qch >= Q.src[0].C) { qch -= Q.src[0].C; qs = 1; }
  const bool pin = pk < P.K, qin = qk < Q.K;
  const SrcArg psa = pick_src(P, ps), qsa = pick_src(Q, qs);
  const float sp = x2_scale((ps ? amax_p1 : amax_p0)[0], nullptr);
  const float sq = x2_scale((qs ? amax_q1 : amax_q0)[0], nullptr);
  // BN scale / shift with the operand's 2^e folded in (relu(x) 2^e == relu(x 2^e), and fma(x, sc 2^e, sh 2^e)
  // == 2^e fma(x, sc, sh) exactly: the same values as scaling after the transform, one multiply fewer)
  float psc[4], psh[4], qsc[4], qsh[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    psc[e] = (psa.scale && pin ? psa.scale[pch + e] : 1.0f) * sp;
    psh[e] = (psa.scale && pin ? psa.shift[pch + e] : 0.0f) * sp;
    qsc[e] = (qsa.scale && qin ? qsa.scale[qch + e] : 1.0f) * sq;
    qsh[e] = (qsa.scale && qin ? qsa.shift[qch + e] : 0.0f) * sq;
  }
  const float plo = psa.scale && psa.relu ? 0.0f : -INFINITY;  // ReLU as one max (no per-element select)
  const float qlo = qsa.scale && qsa.relu ? 0.0f : -INFINITY;
  float4 rp[PI], rq[PJ];
  unsigned pok = 0, qok = 0;  // bit i: staged row i is a real (non-padding) pixel
  auto raw_row = [&](const GatherArg& g, const SrcArg& sa, int64_t m, int tap, int c, bool in, unsigned& ok,
                     int bit) __attribute__((always_inline)) {
    int64_t pix = (in && m < me) ? src_index(g, m, tap) : -1;
    ok |= (pix >= 0 ? 1u : 0u) << bit;
    pix = pix >= 0 ? pix : 0;
    return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(sa.data) + pix * sa.C + c);
  };
  auto put = [&](float4 raw, bool ok, const SrcArg& sa, const float* sc, const float* sh, float lo, _Float16* hp,
                 _Float16* lp) __attribute__((always_inline)) {
    float f[4] = {raw.x, raw.y, raw.z, raw.w};
    f16x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      _Float16 a, b;
      x2_split(ok ? fmaxf(f[e] * sc[e] + sh[e], lo) : 0.0f, a, b);
      h[e] = a;
      l[e] = b;
    }
    *reinterpret_cast<f16x4*>(hp) = h;
    *reinterpret_cast<f16x4*>(lp) = l;
  };
  // A stage's KM rows are KM consecutive pixels; when every stage starts a KM-pixel run inside one image row
  // (w % KM == 0, split starts on stage boundaries) the 2x2-tap gather of Q needs one pixel decode per stage
  // instead of one per staged row (the per-row divisions outweighed the MFMAs in the stage's vector issue)
  const bool q_run = Q.taps == 4 && Q.w % KM == 0 && mchunk % KM == 0 && P.taps == 1;
  auto load_stage = [&](int64_t m_base) __attribute__((always_inline)) {
    pok = qok = 0;
#pragma unroll
    for (int i = 0; i < PI; ++i) rp[i] = raw_row(P, psa, m_base + pr + RPI * i, ptap, pch, pin, pok, i);
    if (q_run) {
      const unsigned mu = (unsigned)m_base, x0 = mu % (unsigned)Q.w, t = mu / (unsigned)Q.w;
      const unsigned y = t % (unsigned)Q.h, img = t / (unsigned)Q.h;
      int dy, dx;
      tap_offset(4, qtap, dy, dx);
      const int64_t row0 = (((int64_t)img * Q.hs + 2 * y + dy) * Q.ws + 2 * x0 + dx) * qsa.C + qch;
#pragma unroll
      for (int i = 0; i < PJ; ++i) {
        const int r = qr + RPJ * i;
        const bool ok = qin && m_base + r < me;
        qok |= (ok ? 1u : 0u) << i;
        rq[i] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(qsa.data) +
                                                 (ok ? row0 + (int64_t)(2 * r) * qsa.C : 0));
      }
    } else {
#pragma unroll
      for (int i = 0; i < PJ; ++i) rq[i] = raw_row(Q, qsa, m_base + qr + RPJ * i, qtap, qch, qin, qok, i);
    }
  };
  auto store_stage = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PI; ++i)
      put(rp[i], (pok >> i) & 1u, psa, psc, psh, plo, &Ps[buf][0][pr + RPI * i][pc * 4], &Ps[buf][1][pr + RPI * i][pc * 4]);
#pragma unroll
    for (int i = 0; i < PJ; ++i)
      put(rq[i], (qok >> i) & 1u, qsa, qsc, qsh, qlo, &Qs[buf][0][qr + RPJ * i][qc * 4], &Qs[buf][1][qr + RPJ * i][qc * 4]);
  };
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  auto tr8 = [&](const _Float16* p0, const _Float16* p1) __attribute__((always_inline)) {
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  const int64_t nst = me > mb ? (me - mb + KM - 1) / KM : 0;
  if (nst > 0) {
    load_stage(mb);
    store_stage(0);
    __syncthreads();
  }
  for (int64_t st = 0; st < nst; ++st) {
    const int buf = (int)(st & 1);
    if (st + 1 < nst) load_stage(mb + (st + 1) * KM);
#pragma unroll
    for (int ks = 0; ks < KM / 16; ++ks) {
      const int row = 16 * ks + 8 * half + q4;
      f16x8 ah[MT], al[MT], bh[NT], bl[NT];
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int col = wi * WI + a * 32 + 16 * grp_hi + 4 * p4;
        ah[a] = tr8(&Ps[buf][0][row][col], &Ps[buf][0][row + 4][col]);
        al[a] = tr8(&Ps[buf][1][row][col], &Ps[buf][1][row + 4][col]);
      }
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const int col = wj * WJ + b * 32 + 16 * grp_hi + 4 * p4;
        bh[b] = tr8(&Qs[buf][0][row][col], &Qs[buf][0][row + 4][col]);
        bl[b] = tr8(&Qs[buf][1][row][col], &Qs[buf][1][row + 4][col]);
      }
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
    }
    if (st + 1 < nst) store_stage(buf ^ 1);
    __syncthreads();
  }

  // unscale: column i of P and column j of Q carry their sources' scales
  auto col_unscale = [&](const GatherArg& g, int k, const float* a0, const float* a1) -> float {
    int c = k % g.Ctot;
    const bool s1 = g.nsrc > 1 && c >= g.src[0].C;
    float u;
    x2_scale((s1 ? a1 : a0)[0], &u);
    return u;
  };
#pragma unroll
  for (int b = 0; b < NT; ++b) {
    const int j = j0 + wj * WJ + b * 32 + l32;
    const float uq = col_unscale(Q, min(j, Q.K - 1), amax_q0, amax_q1);
#pragma unroll
    for (int a = 0; a < MT; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + wi * WI + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        const float up = col_unscale(P, min(i, P.K - 1), amax_p0, amax_p1);
        ws[split * ws_stride + (int64_t)i * ldo + j] = acc[a][b][r] * (up * uq);
      }
    }
  }
}

// =========================================================================== gemm_wgrad (bf16)
// Same contraction with v_mfma_f32_32x32x16_bf16. The LDS tiles stay in their natural gathered
// layout [pixel m][column] (coalesced staging); the MFMA operands need 8 consecutive m per
// column, which ds_read_b64_tr_b16 delivers: per 16-lane group it reads a 4(m) x 16(col) block
// and hands lane j column j's 4 values, so two reads give lane (col = l & 31, half = l >> 5)
// the k-run m = 8*half .. 8*half+7 of its column. Rows are padded by 64 B so the 32 lanes of a
// read touch 64 distinct banks (row stride = 16 dwords mod 64).

__device__ __forceinline__ uint4 gather_vec8_bf16(const GatherArg& g, int64_t m, int k, int tap, int s, int c, bool vec,
                                         bool in) {
  if (!in || m >= g.M) return make_uint4(0, 0, 0, 0);
  if (!vec) {
    __bf16 v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (__bf16)gather_scalar<__bf16>(g, m, k + e);
    uint4 o;
    __builtin_memcpy(&o, v, 16);
    return o;
  }
  const int64_t pix = src_index(g, m, tap);
  if (pix < 0) return make_uint4(0, 0, 0, 0);
  const SrcArg sa = pick_src(g, s);
  uint4 raw = *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(sa.data) + pix * sa.C + c);
  if (sa.scale) raw = transform16<__bf16>(raw, sa.scale, sa.shift, c, sa.relu);
  return raw;
}

// NTH = 512 (round 4): 256-column tiles on 8 waves (2 x 4), one workgroup per CU, as gemm_wgrad_x2_kernel —
// the ConvTranspose2d weight gradients re-read each operand once per tile of the other
template <int BI, int BJ, bool SMALL, int NTH = 256>
__global__ void __launch_bounds__(NTH, NTH == 256 ? 2 : 1)
gemm_wgrad_bf16_kernel(GatherArg P, GatherArg Q, float* __restrict__ out, int ldo, int64_t mchunk, int tiles_j,
                       int tiles, float* __restrict__ ws, int64_t ws_stride) {
  constexpr int KM = 64;                           // pixels per stage
  constexpr int PADE = 32;                         // 64 B row pad (bank spread for tr reads)
  constexpr int LDI = BI + PADE, LDJ = BJ + PADE;  // row strides in elements
  constexpr int WGJ = NTH / 128;                   // waves along j (2 along i)
  constexpr int WI = BI / 2, WJ = BJ / WGJ;
  constexpr int MT = WI / 32, NT = WJ / 32;
  constexpr int CPI = BI / 8, CPJ = BJ / 8;        // 16-B chunks per row
  constexpr int RPI = NTH / CPI, RPJ = NTH / CPJ;
  constexpr int PI = KM / RPI, PJ = KM / RPJ;
  static_assert(PI >= 1 && PJ >= 1 && MT >= 1 && NT >= 1, "stage rows must cover the threads");

  __shared__ __attribute__((aligned(16))) unsigned short Ps[2][KM][LDI];
  __shared__ __attribute__((aligned(16))) unsigned short Qs[2][KM][LDJ];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wi = wave / WGJ, wj = wave % WGJ;
  const int half = lane >> 5, l32 = lane & 31;
  const int grp_hi = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lb % tiles;
  const int64_t split = lb / tiles;
  const int i0 = (tile / tiles_j) * BI;
  const int j0 = (tile % tiles_j) * BJ;
  const int64_t mb = split * mchunk;
  const int64_t me = min(P.M, mb + mchunk);
  if (mb >= me) return;

  const int pc = tid % CPI, pr = tid / CPI;
  const int qc = tid % CPJ, qr = tid / CPJ;
  const int pk = i0 + pc * 8, qk = j0 + qc * 8;
  int ptap = 0, ps = 0, pch = 0, qtap = 0, qs = 0, qch = 0;
  const bool pvec = !SMALL || !P.small, qvec = !SMALL || !Q.small;
  if (pvec) {
    ptap = pk / P.Ctot;
    pch = pk - ptap * P.Ctot;
    if (P.nsrc > 1 && pch >= P.src[0].C) { pch -= P.src[0].C; ps = 1; }
  }
  if (qvec) {
    qtap = qk / Q.Ctot;
    qch = qk - qtap * Q.Ctot;
    if (Q.nsrc > 1 && qch >= Q.src[0].C) { qch -= Q.src[0].C; qs = 1; }
  }
  const bool pin = pk < P.K, qin = qk < Q.K;

  uint4 rp[PI], rq[PJ];
  // Vector path (!SMALL): the raw 16-B loads are issued unconditionally (out-of-image / padding rows
  // clamped to pixel 0) and stay in flight across the current stage's MFMAs; the producer's
  // BN+ReLU and the zeroing are applied when the stage is written to LDS. (Transforming right after
  // the load made every stage wait out the full global latency.)
  const SrcArg psa = pick_src(P, ps), qsa = pick_src(Q, qs);
  float psc[8], psh[8], qsc[8], qsh[8];
  unsigned pok = 0, qok = 0;  // bit i: staged row i is a real (non-padding) pixel
  if constexpr (!SMALL) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      psc[e] = psa.scale && pin ? psa.scale[pch + e] : 1.0f;
      psh[e] = psa.scale && pin ? psa.shift[pch + e] : 0.0f;
      qsc[e] = qsa.scale && qin ? qsa.scale[qch + e] : 1.0f;
      qsh[e] = qsa.scale && qin ? qsa.shift[qch + e] : 0.0f;
    }
  }
  auto raw_row = [&](const GatherArg& g, const SrcArg& sa, int64_t m, int tap, int c, bool in, unsigned& ok,
                     int bit) __attribute__((always_inline)) {
    int64_t pix = (in && m < me) ? src_index(g, m, tap) : -1;
    ok |= (pix >= 0 ? 1u : 0u) << bit;
    pix = pix >= 0 ? pix : 0;
    return *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(sa.data) + pix * sa.C + c);
  };
  auto finish = [&](uint4 raw, bool ok, const SrcArg& sa, const float* sc, const float* sh)
      __attribute__((always_inline)) {
    if (!ok) return make_uint4(0, 0, 0, 0);
    if (!sa.scale) return raw;
    __bf16 v[8];
    __builtin_memcpy(v, &raw, 16);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float f = (float)v[e] * sc[e] + sh[e];
      if (sa.relu) f = fmaxf(f, 0.0f);
      v[e] = (__bf16)f;
    }
    __builtin_memcpy(&raw, v, 16);
    return raw;
  };
  // one dU pixel decode per stage where a stage's KM pixels are one run of an image row (gemm_wgrad_x2_kernel)
  const bool q_run = !SMALL && Q.taps == 4 && Q.w % KM == 0 && mchunk % KM == 0 && P.taps == 1;
  auto load_stage = [&](int64_t m_base) {
    if constexpr (!SMALL) {
      pok = qok = 0;
#pragma unroll
      for (int i = 0; i < PI; ++i) rp[i] = raw_row(P, psa, m_base + pr + RPI * i, ptap, pch, pin, pok, i);
      if (q_run) {
        const unsigned mu = (unsigned)m_base, x0 = mu % (unsigned)Q.w, t = mu / (unsigned)Q.w;
        const unsigned y = t % (unsigned)Q.h, img = t / (unsigned)Q.h;
        int dy, dx;
        tap_offset(4, qtap, dy, dx);
        const int64_t row0 = (((int64_t)img * Q.hs + 2 * y + dy) * Q.ws + 2 * x0 + dx) * qsa.C + qch;
#pragma unroll
        for (int i = 0; i < PJ; ++i) {
          const int r = qr + RPJ * i;
          const bool ok = qin && m_base + r < me;
          qok |= (ok ? 1u : 0u) << i;
          rq[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(qsa.data) +
                                                  (ok ? row0 + (int64_t)(2 * r) * qsa.C : 0));
        }
      } else {
#pragma unroll
        for (int i = 0; i < PJ; ++i) rq[i] = raw_row(Q, qsa, m_base + qr + RPJ * i, qtap, qch, qin, qok, i);
      }
    } else {
#pragma unroll
      for (int i = 0; i < PI; ++i) {
        const int64_t m = m_base + pr + RPI * i;
        rp[i] = gather_vec8_bf16(P, m < me ? m : P.M, pk, ptap, ps, pch, pvec, pin);
      }
#pragma unroll
      for (int i = 0; i < PJ; ++i) {
        const int64_t m = m_base + qr + RPJ * i;
        rq[i] = gather_vec8_bf16(Q, m < me ? m : Q.M, qk, qtap, qs, qch, qvec, qin);
      }
    }
  };
  auto store_stage = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      uint4 v = rp[i];
      if constexpr (!SMALL) v = finish(v, (pok >> i) & 1u, psa, psc, psh);
      *reinterpret_cast<uint4*>(&Ps[buf][pr + RPI * i][pc * 8]) = v;
    }
#pragma unroll
    for (int i = 0; i < PJ; ++i) {
      uint4 v = rq[i];
      if constexpr (!SMALL) v = finish(v, (qok >> i) & 1u, qsa, qsc, qsh);
      *reinterpret_cast<uint4*>(&Qs[buf][qr + RPJ * i][qc * 8]) = v;
    }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  const int64_t nst = (me - mb + KM - 1) / KM;
  load_stage(mb);
  store_stage(0);
  __syncthreads();
  for (int64_t st = 0; st < nst; ++st) {
    const int buf = (int)(st & 1);
    if (st + 1 < nst) load_stage(mb + (st + 1) * KM);
#pragma unroll
    for (int ks = 0; ks < KM / 16; ++ks) {
      const int row = 16 * ks + 8 * half + q4;
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int col = wi * WI + a * 32 + 16 * grp_hi + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(&Ps[buf][row][col]));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(&Ps[buf][row + 4][col]));
        af[a] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const int col = wj * WJ + b * 32 + 16 * grp_hi + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(&Qs[buf][row][col]));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(&Qs[buf][row + 4][col]));
        bfr[b] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
    if (st + 1 < nst) store_stage(buf ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int j = j0 + wj * WJ + b * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + wi * WI + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (ws) ws[split * ws_stride + (int64_t)i * ldo + j] = acc[a][b][r];
        else atomicAdd(out + (int64_t)i * ldo + j, acc[a][b][r]);
      }
    }
}

// =========================================================================== host side
int make_gather(const selunet_gather* a, int dtype, GatherArg& g, int vec_elems) {
  SELUNET_REQUIRE(a != nullptr, "gather descriptor is NULL");
  SELUNET_REQUIRE(a->n > 0 && a->h > 0 && a->w > 0, "gather grid must be positive (%d,%d,%d)", a->n, a->h, a->w);
  SELUNET_REQUIRE(a->taps == 1 || a->taps == 4 || a->taps == 9, "taps must be 1, 4 or 9 (got %d)", a->taps);
  SELUNET_REQUIRE(a->nsrc == 1 || a->nsrc == 2, "nsrc must be 1 or 2");
  std::memset(&g, 0, sizeof(g));
  g.n = a->n;
  g.h = a->h;
  g.w = a->w;
  g.taps = a->taps;
  g.nsrc = a->nsrc;
  g.hs = a->taps == 4 ? 2 * a->h : a->h;
  g.ws = a->taps == 4 ? 2 * a->w : a->w;
  g.M = (int64_t)a->n * a->h * a->w;
  SELUNET_REQUIRE(g.M * (a->taps == 4 ? 4 : 1) < (int64_t(1) << 31), "gather grid too large (%lld rows)",
                  (long long)g.M);
  int ctot = 0;
  bool vec = true;
  for (int s = 0; s < a->nsrc; ++s) {
    const selunet_source& src = a->src[s];
    SELUNET_REQUIRE(src.data != nullptr, "source %d data is NULL", s);
    SELUNET_REQUIRE(src.channels > 0, "source %d channels must be positive", s);
    SELUNET_REQUIRE((src.scale == nullptr) == (src.shift == nullptr), "scale/shift must both be set or both NULL");
    SELUNET_REQUIRE(src.layout == 0 || (src.layout == 1 && a->nsrc == 1 && src.scale == nullptr),
                    "NCHW (fp32) sources are only supported as a single untransformed source");
    g.src[s].data = src.data;
    g.src[s].scale = src.scale;
    g.src[s].shift = src.shift;
    g.src[s].C = src.channels;
    g.src[s].relu = src.relu;
    g.src[s].layout = src.layout;
    if (src.channels % vec_elems != 0 || src.layout != 0) vec = false;
    if ((reinterpret_cast<uintptr_t>(src.data) & 15) != 0) vec = false;
    ctot += src.channels;
  }
  g.Ctot = ctot;
  g.K = a->taps * ctot;
  g.small = vec ? 0 : 1;
  if (g.small) {
    SELUNET_REQUIRE(a->nsrc == 1 && a->src[0].scale == nullptr,
                    "element-wise gather (channels %% %d != 0) supports one untransformed source", vec_elems);
  }
  return 0;
}

template <typename T, int BN, bool SMALL>
static void launch_gather_impl(const GatherArg& g, const void* b, int N, int k_pad, const EpiArg& ep, hipStream_t st);
template <typename T, int BI, int BJ, bool SMALL>
static void launch_wgrad_impl(const GatherArg& p, const GatherArg& q, float* out, int ldo, int ni, int nj_pad,
                              float* ws, hipStream_t st);

// pixel splits of the generic weight gradient (rows per split a multiple of the 64-pixel stage)
static int64_t wgrad_splits(int64_t M, int tiles, int64_t* mchunk_out, int64_t wgs = 0) {
  // workgroup target over (tile, pixel split): 512 (two per CU) measured 6.43 vs 6.57 ms/step at
  // 16 images/GPU against 2048 (fewer split partials to reduce), equal at 128; 256 and 1024 in
  // between (SELUNET_GEMM_WGRAD_WGS overrides); wgs: a kernel's own target (one workgroup per CU)
  const int64_t target = wgs > 0 ? wgs : std::max<int64_t>(1, option(SELUNET_OPT_GEMM_WGRAD_WGS, 512));
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(cdiv(M, 256), cdiv(target, tiles)));
  const int64_t mchunk = cdiv(cdiv(M, splits), 64) * 64;
  if (mchunk_out) *mchunk_out = mchunk;
  return cdiv(M, mchunk);
}

template <typename T, int BN>
static void launch_gather(const GatherArg& g, const void* b, int N, int k_pad, const EpiArg& ep, hipStream_t st) {
  if (g.small) {
    launch_gather_impl<T, BN, true>(g, b, N, k_pad, ep, st);
    return;
  }
  launch_gather_impl<T, BN, false>(g, b, N, k_pad, ep, st);
}

// Resident gather-GEMM workgroups the persistent launch aims for (2 per CU; a constant, not the
// device's CU count, so slab rows never depend on the device); 0 = one tile per workgroup.
// SELUNET_OPT_GATHER_WGS (selunet_set_option) or selunet_set_gather_workgroups (tests) override it.
static int64_t gather_wgs() { return option(SELUNET_OPT_GATHER_WGS, 512); }

// Row-tile workgroups (= statistics slab rows) of the gather GEMM for N output columns; independent
// of the column tile width (64 or 128) so the caller can size slabs from (operand, N) alone.
static int64_t gather_rows(const GatherArg& g, int N) {
  const int64_t m_tiles = cdiv(g.M, BM);
  const int64_t wgs = gather_wgs();
  if (wgs == 0) return m_tiles;
  return std::max<int64_t>(1, std::min<int64_t>(m_tiles, wgs / cdiv(N, 128)));
}

template <typename T, int BN, bool SMALL>
static void launch_gather_impl(const GatherArg& g, const void* b, int N, int k_pad, const EpiArg& ep, hipStream_t st) {
  const int n_tiles = N / BN;
  const int64_t P = gather_rows(g, N);
  hipLaunchKernelGGL((gemm_gather_kernel<T, BN, SMALL, false>), dim3((unsigned)(P * n_tiles)), dim3(256), 0, st, g,
                     reinterpret_cast<const T*>(b), N, k_pad, ep, n_tiles, (int)P, nullptr, nullptr, nullptr);
}

template <typename T, int BI, int BJ>
static void launch_wgrad(const GatherArg& p, const GatherArg& q, float* out, int ldo, int ni, int nj_pad,
                         hipStream_t st, float* ws = nullptr) {
  if (p.small || q.small) launch_wgrad_impl<T, BI, BJ, true>(p, q, out, ldo, ni, nj_pad, ws, st);
  else launch_wgrad_impl<T, BI, BJ, false>(p, q, out, ldo, ni, nj_pad, ws, st);
}

template <typename T, int BI, int BJ, bool SMALL>
static void launch_wgrad_impl(const GatherArg& p, const GatherArg& q, float* out, int ldo, int ni, int nj_pad,
                              float* ws, hipStream_t st) {
  const int tiles_j = nj_pad / BJ;
  const int tiles = (ni / BI) * tiles_j;
  int64_t mchunk;
  const int64_t splits = wgrad_splits(p.M, tiles, &mchunk);
  if constexpr (std::is_same<T, float>::value)
    hipLaunchKernelGGL((gemm_wgrad_kernel<T, BI, BJ, SMALL>), dim3((unsigned)(tiles * splits)), dim3(256), 0, st, p, q, out,
                       ldo, mchunk, tiles_j, tiles, ws, (int64_t)ni * ldo);
  else
    hipLaunchKernelGGL((gemm_wgrad_bf16_kernel<BI, BJ, SMALL>), dim3((unsigned)(tiles * splits)), dim3(256), 0, st, p, q,
                       out, ldo, mchunk, tiles_j, tiles, ws, (int64_t)ni * ldo);
}

}  // namespace selunet

using namespace selunet;

bool selunet::halo_enabled() { return option(SELUNET_OPT_HALO, 1) != 0; }

extern "C" int32_t selunet_set_gather_workgroups(int32_t wgs) {
  const int32_t prev = (int32_t)selunet::gather_wgs();
  g_options[SELUNET_OPT_GATHER_WGS] = wgs < 0 ? -1 : wgs;
  return prev;
}

extern "C" int64_t selunet_gemm_stats_rows(const selunet_gather* a, int32_t n_cols, int32_t dtype) {
  const int esz = dtype == SELUNET_F32 ? 4 : 2;
  GatherArg g;
  if (make_gather(a, dtype, g, 16 / esz)) return -1;
  if (halo_enabled() && conv3x3_halo_eligible(g, n_cols, dtype)) return conv3x3_halo_stats_rows(g, n_cols, dtype);
  // the bf16 ConvTranspose2d data gradient (BN-backward sums): the resident-weight kernel's rows
  if (dtype == SELUNET_BF16 && convt_ring_bf16_dgrad_operand_ok(g, n_cols)) return convt_ring_rows(g, n_cols);
  if (dtype == SELUNET_BF16 && convt_dgrad_bf16_ntb(g, n_cols) > 0) return convt_dgrad_bf16_rows(g, n_cols);
  return gather_rows(g, n_cols);
}

// Name of the kernel selunet_gemm_gather / selunet_gemm_wgrad dispatch to for these operands
// (profiling and roofline attribution; matches the rocprofv3 kernel names' template arguments).
extern "C" const char* selunet_gemm_kernel_name(const selunet_gather* a, const selunet_gather* q, int32_t n_cols,
                                                int32_t mode, int32_t dtype) {
  const bool bf = dtype == SELUNET_BF16;
  const int esz = bf ? 2 : 4;
  GatherArg g;
  if (q == nullptr) {
    if (make_gather(a, dtype, g, 16 / esz)) return "invalid";
    if (mode != SELUNET_EP_SCATTER2X && halo_enabled() && conv3x3_halo_eligible(g, n_cols, dtype)) {
      // (SPLIT epilogues in this network split the columns in half: torch.cat of equal halves)
      const bool one = conv3x3_halo_one_chunk(g, dtype);  // single channel chunk: 64-column tiles, 2 WG/CU
      const bool bn128 = !one && n_cols % 128 == 0 && !(mode == SELUNET_EP_SPLIT && (n_cols / 2) % 128 != 0);
      if (one) return bf ? "conv3x3_halo1<bf16,64>" : "conv3x3_halo1<f32,64>";
      if (conv3x3_halo_persistent(g, dtype))
        return bf ? (bn128 ? "conv3x3_halo_persist<bf16,128>" : "conv3x3_halo_persist<bf16,64>")
                  : (bn128 ? "conv3x3_halo_persist<f32,128>" : "conv3x3_halo_persist<f32,64>");
      return bf ? (bn128 ? "conv3x3_halo<bf16,128>" : "conv3x3_halo<bf16,64>")
                : (bn128 ? "conv3x3_halo<f32,128>" : "conv3x3_halo<f32,64>");
    }
    if (bf && mode == SELUNET_EP_SCATTER2X && convt_bf16_fwd_ntb(g, n_cols) > 0) return "convt<bf16>";
    if (bf && mode == SELUNET_EP_PLAIN && convt_dgrad_bf16_ntb(g, n_cols) > 0) return "convt_dgrad<bf16>";
    return bf ? "gemm_gather<bf16>" : "gemm_gather<f32>";
  }
  GatherArg gq;
  const int vec = bf ? 8 : 4;
  if (make_gather(a, dtype, g, vec) || make_gather(q, dtype, gq, vec)) return "invalid";
  if (halo_enabled() && conv3x3_wgrad_wino_eligible(g, gq, dtype)) return "conv3x3_wgrad_wino_f32<64>";
  if (halo_enabled() && conv3x3_wgrad_halo_eligible(g, gq, dtype)) {
    if (bf) return g.K % 128 == 0 ? "conv3x3_wgrad_halo<128>" : "conv3x3_wgrad_halo<64>";
    return g.K % 128 == 0 ? "conv3x3_wgrad_halo_f32<128>" : "conv3x3_wgrad_halo_f32<64>";
  }
  return bf ? "gemm_wgrad_bf16" : "gemm_wgrad<f32>";
}

// Argument checks shared by selunet_gemm_gather and selunet_conv3x3_wino; fills g and e.
static int check_gather_call(const selunet_gather* a, const void* b, int32_t n_cols, int32_t k_pad,
                             const selunet_epilogue* ep, int32_t dtype, GatherArg& g, EpiArg& e) {
  SELUNET_REQUIRE(dtype == SELUNET_F32 || dtype == SELUNET_BF16, "dtype must be SELUNET_F32 or SELUNET_BF16");
  const int esz = dtype == SELUNET_F32 ? 4 : 2;
  const int bke = 128 / esz;
  if (int rc = make_gather(a, dtype, g, 16 / esz)) return rc;
  SELUNET_REQUIRE(b != nullptr && ep != nullptr && ep->out0 != nullptr, "B / epilogue / out0 must be non-NULL");
  SELUNET_REQUIRE(n_cols > 0 && n_cols % 64 == 0, "n_cols must be a positive multiple of 64 (got %d)", n_cols);
  SELUNET_REQUIRE(k_pad >= g.K && k_pad % bke == 0, "k_pad (%d) must be >= K (%d) and a multiple of %d", k_pad, g.K,
                  bke);
  SELUNET_REQUIRE(g.small || (g.Ctot % bke == 0 && (a->nsrc == 1 || a->src[0].channels % bke == 0)),
                  "vector gather needs channel counts that are multiples of %d", bke);
  SELUNET_REQUIRE(ep->mode >= 0 && ep->mode <= 2, "bad epilogue mode");
  if (ep->mode == SELUNET_EP_SPLIT)
    SELUNET_REQUIRE(ep->out1 != nullptr && ep->split > 0 && ep->split < n_cols && ep->split % 64 == 0,
                    "split epilogue needs out1 and 0 < split < n_cols, split %% 64 == 0");
  if (ep->mode == SELUNET_EP_SCATTER2X)
    SELUNET_REQUIRE(n_cols % 4 == 0 && a->taps == 1, "scatter2x epilogue needs taps == 1 and n_cols % 4 == 0");
  SELUNET_REQUIRE(ep->stats == nullptr || ep->mode == SELUNET_EP_PLAIN, "stats only with the plain epilogue");
  SELUNET_REQUIRE(ep->colsum == nullptr || ep->mode == SELUNET_EP_SPLIT, "colsum only with the split epilogue");
  const selunet_bn_bwd_stats& bb = ep->bnb;
  if (bb.slab != nullptr)
    SELUNET_REQUIRE(ep->mode == SELUNET_EP_PLAIN && ep->stats == nullptr && bb.y && bb.scale && bb.shift && bb.mean &&
                        bb.invstd && ep->bias == nullptr,
                    "bn-backward sums need the plain epilogue without stats/bias and y/scale/shift/mean/invstd");
  e = EpiArg{ep->out0, ep->out1, ep->bias, ep->stats, ep->mode, ep->split, ep->colsum,
             BnBwdArg{bb.y, bb.scale, bb.shift, bb.mean, bb.invstd, bb.slab}, ep->amax, ep->stats_center};
  SELUNET_REQUIRE(ep->stats_center == nullptr || ep->stats != nullptr, "stats_center only with stats");
  return SELUNET_OK;
}

extern "C" int selunet_gemm_gather(const selunet_gather* a, const void* b, int32_t n_cols, int32_t k_pad,
                                   const selunet_epilogue* ep, int32_t dtype, void* stream) {
  GatherArg g;
  EpiArg e;
  if (int rc = check_gather_call(a, b, n_cols, k_pad, ep, dtype, g, e)) return rc;
  hipStream_t st = as_stream(stream);
  if (ep->mode != SELUNET_EP_SCATTER2X && halo_enabled() && conv3x3_halo_eligible(g, n_cols, dtype))
    return conv3x3_halo_launch(g, b, n_cols, k_pad, e, dtype, st);
  if (dtype == SELUNET_BF16) {  // ConvTranspose2d forward / data gradient: the ring (unpool3 / 2) or resident kernels
    if (convt_ring_bf16_takes(g, n_cols, e)) return convt_ring_bf16_launch(g, b, n_cols, e, st);
    if (convt_bf16_eligible(g, n_cols, e) || convt_dgrad_bf16_eligible(g, n_cols, e))
      return convt_bf16_launch(g, b, n_cols, e, st);
    SELUNET_REQUIRE(convt_dgrad_bf16_ntb(g, n_cols) == 0 || (e.stats == nullptr && e.colsum == nullptr &&
                                                             e.bnb.slab == nullptr),
                    "gemm_gather: statistics epilogue on a ConvTranspose2d data-gradient operand that "
                    "selunet_gemm_stats_rows sizes for the resident-weight kernel (PLAIN, no amax / bias)");
  }
  const bool bn128 = n_cols % 128 == 0 && !(ep->mode == SELUNET_EP_SPLIT && ep->split % 128 != 0);
  if (dtype == SELUNET_F32) {
    if (bn128) launch_gather<float, 128>(g, b, n_cols, k_pad, e, st);
    else launch_gather<float, 64>(g, b, n_cols, k_pad, e, st);
  } else {
    if (bn128) launch_gather<__bf16, 128>(g, b, n_cols, k_pad, e, st);
    else launch_gather<__bf16, 64>(g, b, n_cols, k_pad, e, st);
  }
  return check_launch("gemm_gather");
}

extern "C" int32_t selunet_conv3x3_wino_ok(int32_t h, int32_t w, int32_t c_in, int32_t c_src0, int32_t n_cols) {
  return halo_enabled() && conv3x3_wino_shape_ok(h, w, c_in, c_src0, n_cols) ? 1 : 0;
}

extern "C" const char* selunet_conv3x3_wino_kernel_name(int32_t n_cols, int32_t mode, int32_t split) {
  EpiArg e{};
  e.mode = mode;
  e.split = split;
  return conv3x3_wino_bn128(n_cols, e) ? "conv3x3_wino<f32,128>" : "conv3x3_wino<f32,64>";
}

extern "C" int selunet_conv3x3_wino(const selunet_gather* a, const float* u, int32_t n_cols,
                                   const selunet_epilogue* ep, void* stream) {
  GatherArg g;
  EpiArg e;
  SELUNET_REQUIRE(a != nullptr && a->taps == 9, "conv3x3_wino: a 3x3 (taps = 9) gather is required");
  if (int rc = check_gather_call(a, u, n_cols, 12 * a->src[0].channels + 12 * (a->nsrc > 1 ? a->src[1].channels : 0),
                                 ep, SELUNET_F32, g, e))
    return rc;
  SELUNET_REQUIRE(ep->mode != SELUNET_EP_SCATTER2X, "conv3x3_wino: scatter epilogue not supported");
  SELUNET_REQUIRE(halo_enabled() && conv3x3_wino_eligible(g, n_cols),
                  "conv3x3_wino: operand not eligible (%dx%d, C=%d, n_cols=%d; see selunet_conv3x3_wino_ok)", g.h, g.w,
                  g.Ctot, n_cols);
  return conv3x3_wino_launch(g, u, n_cols, e, as_stream(stream));
}

// The split-fp16 gather GEMM (ConvTranspose2d forward and data gradient in fp32 training) runs 256 x 128
// tiles with 512 threads, one persistent workgroup per CU (x2_rows): 1.33x the MACs per staged byte of
// the 128 x 128 tiles (256 x 256 tiles spill: 696 B of scratch per lane). N not a multiple of 128: the
// 128 x 64 kernel.
constexpr int X2_BM = 256;

static int x2_bn(int n_cols, const EpiArg& e) {
  if (n_cols % 128 != 0 || (e.mode == SELUNET_EP_SPLIT && e.split % 128 != 0)) return 64;
  return 128;
}

// statistics slab rows (= persistent row workgroups) of the split-fp16 gather GEMM; independent of
// the column tile width (128 / 256), like gather_rows. N not a multiple of 128: the 128-row kernel.
static int64_t x2_rows(const GatherArg& g, int N) {
  if (convt_ring_dgrad_operand_ok(g, N)) return convt_ring_rows(g, N);    // (whichever kernel the epilogue picks)
  if (convt_dgrad_x2_ntb(g, N) > 0) return convt_dgrad_x2_rows(g, N);
  if (N % 128 != 0) return gather_rows(g, N);
  const int64_t m_tiles = cdiv(g.M, X2_BM);
  const int64_t wgs = gather_wgs();  // (the gather knob: half as many of these one-per-CU workgroups)
  if (wgs == 0) return m_tiles;
  return std::max<int64_t>(1, std::min<int64_t>(m_tiles, std::max<int64_t>(1, wgs / 2) / cdiv(N, 128)));
}

extern "C" int64_t selunet_gemm_gather_x2_stats_rows(const selunet_gather* a, int32_t n_cols) {
  GatherArg g;
  if (make_gather(a, SELUNET_F32, g, 4)) return -1;
  return x2_rows(g, n_cols);
}

extern "C" int selunet_gemm_gather_x2(const selunet_gather* a, const float* w, int32_t n_cols, int32_t k_pad,
                                      const selunet_epilogue* ep, const float* amax0, const float* amax1,
                                      void* stream) {
  GatherArg g;
  EpiArg e;
  if (int rc = check_gather_call(a, w, n_cols, k_pad, ep, SELUNET_F32, g, e)) return rc;
  SELUNET_REQUIRE(!g.small && k_pad == g.K && g.K % 32 == 0,
                  "gemm_gather_x2: vector gathers with K (%d) a multiple of 32 and k_pad == K", g.K);
  SELUNET_REQUIRE(amax0 != nullptr && (a->nsrc == 1 || amax1 != nullptr),
                  "gemm_gather_x2: every source needs its range word (amax0, amax1)");
  hipStream_t st = as_stream(stream);
  // unpool3 / unpool2 forward and data gradient (K >= 256, 256-column blocks): the LDS-DMA ring kernel
  if (convt_ring_x2_takes(g, n_cols, e)) return convt_ring_x2_launch(g, w, n_cols, e, amax0, st);
  // the ConvTranspose2d forward (scatter epilogue): the resident-weight kernel (convt.hip)
  if (convt_x2_eligible(g, n_cols, e)) return convt_x2_launch(g, w, n_cols, e, amax0, st);
  // its data gradient (PLAIN, BN-backward sums): the resident-weight data-gradient kernel
  if (convt_dgrad_x2_eligible(g, n_cols, e)) return convt_dgrad_x2_launch(g, w, n_cols, e, amax0, st);
  const int bn = x2_bn(n_cols, e);
  const int64_t P = x2_rows(g, n_cols);
  const float* wcs = w + (int64_t)n_cols * k_pad;
  const dim3 grid((unsigned)(P * (n_cols / bn)));
  if (bn == 128)
    hipLaunchKernelGGL((gemm_gather_kernel<float, 128, false, true, X2_BM, 512>), grid, dim3(512), 0, st, g, w,
                       n_cols, k_pad, e, n_cols / 128, (int)P, wcs, amax0, amax1);
  else
    hipLaunchKernelGGL((gemm_gather_kernel<float, 64, false, true>), grid, dim3(256), 0, st, g, w, n_cols, k_pad, e,
                       n_cols / 64, (int)P, wcs, amax0, amax1);
  return check_launch("gemm_gather_x2");
}

extern "C" int32_t selunet_conv3x3_x2_ok(int32_t h, int32_t w, int32_t c_in, int32_t c_src0, int32_t n_cols) {
  return halo_enabled() && conv3x3_x2_shape_ok(h, w, c_in, c_src0, n_cols) ? 1 : 0;
}

extern "C" const char* selunet_conv3x3_x2_kernel_name(const selunet_gather* a, int32_t n_cols, int32_t mode,
                                                      int32_t split) {
  EpiArg e{};
  e.mode = mode;
  e.split = split;
  GatherArg g;
  if (make_gather(a, SELUNET_F32, g, 4)) return "?";
  if (conv3x3_x2d_eligible(g, n_cols)) return "conv3x3_x2d<f32,64>";
  if (conv3x3_x2p_eligible(g, n_cols)) return "conv3x3_x2p<f32,128>";
  return conv3x3_x2_bn128(n_cols, e) ? "conv3x3_x2<f32,128>" : "conv3x3_x2<f32,64>";
}

extern "C" int64_t selunet_conv3x3_x2_stats_rows(const selunet_gather* a, int32_t n_cols) {
  GatherArg g;
  if (make_gather(a, SELUNET_F32, g, 4)) return -1;
  if (conv3x3_x2d_eligible(g, n_cols)) return conv3x3_x2d_rows(g);
  return conv3x3_x2_persist_rows(g, n_cols);
}

extern "C" int selunet_conv3x3_x2(const selunet_gather* a, const float* w, int32_t n_cols, const selunet_epilogue* ep,
                                  const float* amax0, const float* amax1, void* stream) {
  GatherArg g;
  EpiArg e;
  SELUNET_REQUIRE(a != nullptr && a->taps == 9, "conv3x3_x2: a 3x3 (taps = 9) gather is required");
  if (int rc = check_gather_call(a, w, n_cols, 9 * (a->src[0].channels + (a->nsrc > 1 ? a->src[1].channels : 0)), ep,
                                 SELUNET_F32, g, e))
    return rc;
  SELUNET_REQUIRE(ep->mode != SELUNET_EP_SCATTER2X, "conv3x3_x2: scatter epilogue not supported");
  SELUNET_REQUIRE(amax0 != nullptr && (a->nsrc == 1 || amax1 != nullptr),
                  "conv3x3_x2: every source needs its range word (amax0, amax1)");
  SELUNET_REQUIRE(halo_enabled() && conv3x3_x2_eligible(g, n_cols),
                  "conv3x3_x2: operand not eligible (%dx%d, C=%d, n_cols=%d; see selunet_conv3x3_x2_ok)", g.h, g.w,
                  g.Ctot, n_cols);
  return conv3x3_x2_launch(g, w, n_cols, e, amax0, amax1, as_stream(stream));
}

// Deterministic split reduction of the weight-gradient partials: out[i][j] = sum_s ws[s][i][j]
// for j < kq (fixed split order), 0 in the pad columns. LAYOUT != PACKED writes the reference
// parameter layout instead of the packed [ni][ldo] one (the unpack pass folded into the reduction):
// CONV3X3: packed column j = tap*ci + c of row o -> out[o][c][tap] (Conv2d weight [co][ci][3][3]);
// CONVT: packed column j = ab*co + o of row c -> out[c][o][ab] (ConvTranspose2d weight [ci][co][2][2]).
enum { WG_PACKED = 0, WG_CONV3X3 = 1, WG_CONVT = 2 };
template <int LAYOUT>
__global__ void __launch_bounds__(64) wgrad_reduce_kernel(const float* __restrict__ ws, int64_t splits,
                                                          int64_t stride, int ni, int ldo, int kq,
                                                          float* __restrict__ out) {
  // one wave per block, 4 floats per lane, 16 split loads in flight per lane (the splits of one
  // element are 4*stride bytes apart: latency, not bandwidth, bounds a one-load-at-a-time loop)
  constexpr int U = 16;
  const int64_t n4 = (int64_t)ni * ldo / 4;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n4; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * 4;
    const int j = (int)(e % ldo);
    f32x4 acc = {0, 0, 0, 0};
    if (j < kq) {
      int64_t sp = 0;
      for (; sp + U <= splits; sp += U) {
        f32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = *reinterpret_cast<const f32x4*>(ws + (sp + u) * stride + e);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += x[u];
      }
      for (; sp < splits; ++sp) acc += *reinterpret_cast<const f32x4*>(ws + sp * stride + e);
      if (j + 4 > kq)
        for (int u = 0; u < 4; ++u)
          if (j + u >= kq) acc[u] = 0.0f;
    }
    if constexpr (LAYOUT == WG_PACKED) {
      *reinterpret_cast<f32x4*>(out + e) = acc;
    } else {
      const int64_t row = e / ldo;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int jj = j + u;
        if (jj >= kq) continue;
        if constexpr (LAYOUT == WG_CONV3X3) {
          const int ci = kq / 9, tap = jj / ci, c = jj - tap * ci;
          out[(row * ci + c) * 9 + tap] = acc[u];
        } else {
          const int co = kq / 4, ab = jj / co, o = jj - ab * co;
          out[(row * co + o) * 4 + ab] = acc[u];
        }
      }
    }
  }
}

// Fixed-order split reduction of the fp32 Winograd weight gradient's M planes
// (conv3x3_wgrad_wino_f32_kernel: ws[split][co][(dy*4 + xi)*C + c]) with the output transform
// dW[dy][0] = M0 + (M1+M2)/2, dW[dy][1] = (M1-M2)/2, dW[dy][2] = (M1+M2)/2 + M3, written as the
// packed [co][ldo] (column tap*C + c) or the Conv2d [co][C][3][3] layout. One lane per (co, dy, 4 c).
template <int LAYOUT>
__global__ void __launch_bounds__(64) wgrad_wino_reduce_kernel(const float* __restrict__ ws, int64_t splits,
                                                               int64_t stride, int ni, int ctot, int ldo,
                                                               float* __restrict__ out) {
  const int c4n = ctot / 4;
  const int64_t n = (int64_t)ni * 3 * c4n;
  const int ldw = 12 * ctot;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(v % c4n) * 4;
    const int64_t r2 = v / c4n;
    const int dy = (int)(r2 % 3);
    const int64_t row = r2 / 3;
    const float* base = ws + row * ldw + dy * 4 * ctot + c;
    f32x4 m[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    constexpr int U = 4;
    int64_t sp = 0;
    for (; sp + U <= splits; sp += U) {
      f32x4 x[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) x[u][k] = *reinterpret_cast<const f32x4*>(base + (sp + u) * stride + k * ctot);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] += x[u][k];
    }
    for (; sp < splits; ++sp)
#pragma unroll
      for (int k = 0; k < 4; ++k) m[k] += *reinterpret_cast<const f32x4*>(base + sp * stride + k * ctot);
    const f32x4 s12 = (m[1] + m[2]) * 0.5f;
    const f32x4 t[3] = {m[0] + s12, (m[1] - m[2]) * 0.5f, s12 + m[3]};
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int tap = dy * 3 + dx;
      if constexpr (LAYOUT == WG_PACKED) {
        *reinterpret_cast<f32x4*>(out + row * ldo + tap * ctot + c) = t[dx];
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) out[(row * ctot + c + u) * 9 + tap] = t[dx][u];
      }
    }
  }
}

struct WgradPlan {
  GatherArg gp, gq;
  int ni, bj, nj_pad;
  bool halo;
  bool wino;       // fp32 Winograd planes (split-partials paths only): ws row length 12 * C
  int64_t splits;  // pixel splits whose partials the fixed-order reduction sums
  int wide_bi;     // bf16 generic path on 256-column tiles (512 threads, one workgroup per CU): 256 / 128, or 0
};

static int plan_wgrad(const selunet_gather* p, const selunet_gather* q, int32_t dtype, WgradPlan& w) {
  SELUNET_REQUIRE(dtype == SELUNET_F32 || dtype == SELUNET_BF16, "dtype must be SELUNET_F32 or SELUNET_BF16");
  const int vec = dtype == SELUNET_F32 ? 4 : 8;  // elements per staged vector
  if (int rc = make_gather(p, dtype, w.gp, vec)) return rc;
  if (int rc = make_gather(q, dtype, w.gq, vec)) return rc;
  SELUNET_REQUIRE(w.gp.M == w.gq.M && p->n == q->n && p->h == q->h && p->w == q->w, "P and Q must share the row grid");
  SELUNET_REQUIRE(w.gp.K % 64 == 0, "P columns (%d) must be a multiple of 64", w.gp.K);
  SELUNET_REQUIRE(w.gp.small == 0, "P must be vector-gatherable");
  w.ni = w.gp.K;
  w.wide_bi = 0;
  w.bj = (w.gq.K % 128 == 0 || w.gq.K > 512) ? 128 : 64;
  w.nj_pad = (int)(cdiv(w.gq.K, w.bj) * w.bj);
  w.halo = halo_enabled() && conv3x3_wgrad_halo_eligible(w.gp, w.gq, dtype);
  w.wino = w.halo && conv3x3_wgrad_wino_eligible(w.gp, w.gq, dtype);
  if (w.wino) {
    w.splits = conv3x3_wgrad_wino_splits(w.gp, w.gq, nullptr);
  } else if (w.halo) {
    w.splits = conv3x3_wgrad_halo_splits(w.gp, w.gq, dtype, nullptr);
  } else {
    // bf16, vector operands, 256-column tiles possible (the ConvTranspose2d weight gradients): 256 x 256 or
    // 128 x 256 tiles, pixel splits sized for 256 workgroups (gemm_wgrad_x2's tiling)
    if (dtype == SELUNET_BF16 && !w.gp.small && !w.gq.small && w.gq.K % 256 == 0 && (w.ni % 256 == 0 || w.ni == 128)) {
      w.wide_bi = w.ni % 256 == 0 ? 256 : 128;
      w.nj_pad = w.gq.K;
      w.splits = wgrad_splits(w.gp.M, (w.ni / w.wide_bi) * (w.nj_pad / 256), nullptr, 256);
      return 0;
    }
    const int bi = w.ni % 128 == 0 ? 128 : 64;
    w.splits = wgrad_splits(w.gp.M, (w.ni / bi) * (w.nj_pad / w.bj), nullptr);
  }
  return 0;
}

// workspace floats per split: [ni][nj_pad], or [ni][12 C] for the Winograd planes
static int64_t wgrad_ws_row(const WgradPlan& w) { return w.wino ? 12 * (int64_t)w.gq.Ctot : (int64_t)w.nj_pad; }

// Winograd planes -> the split reduction with the output transform (layout WG_PACKED: out [ni][nj_pad])
static void launch_wino_reduce(const WgradPlan& w, float* ws, int layout, float* out, hipStream_t st) {
  const int64_t n = (int64_t)w.ni * 3 * (w.gq.Ctot / 4);
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 64), 16384));
  const int64_t stride = (int64_t)w.ni * wgrad_ws_row(w);
  if (layout == WG_CONV3X3)
    hipLaunchKernelGGL(wgrad_wino_reduce_kernel<WG_CONV3X3>, dim3(blocks), dim3(64), 0, st, ws, w.splits, stride, w.ni,
                       w.gq.Ctot, w.nj_pad, out);
  else
    hipLaunchKernelGGL(wgrad_wino_reduce_kernel<WG_PACKED>, dim3(blocks), dim3(64), 0, st, ws, w.splits, stride, w.ni,
                       w.gq.Ctot, w.nj_pad, out);
}

static void launch_wgrad_any(const WgradPlan& w, float* out, float* ws, int32_t dtype, hipStream_t st) {
  const GatherArg &gp = w.gp, &gq = w.gq;
  const int ni = w.ni, nj_pad = w.nj_pad, bj = w.bj;
  if (w.halo) {
    conv3x3_wgrad_halo_launch(gp, gq, out, nj_pad, ws, dtype, st);
    return;
  }
  const bool bi128 = ni % 128 == 0;
  if (w.wide_bi && ws) {  // bf16 256-column tiles (split partials only)
    const int tiles_j = nj_pad / 256, tiles = (ni / w.wide_bi) * tiles_j;
    int64_t mchunk;
    const int64_t splits = wgrad_splits(gp.M, tiles, &mchunk, 256);
    const dim3 grid((unsigned)(tiles * splits));
    if (w.wide_bi == 256)
      hipLaunchKernelGGL((gemm_wgrad_bf16_kernel<256, 256, false, 512>), grid, dim3(512), 0, st, gp, gq, out, nj_pad,
                         mchunk, tiles_j, tiles, ws, (int64_t)ni * nj_pad);
    else
      hipLaunchKernelGGL((gemm_wgrad_bf16_kernel<128, 256, false, 512>), grid, dim3(512), 0, st, gp, gq, out, nj_pad,
                         mchunk, tiles_j, tiles, ws, (int64_t)ni * nj_pad);
    return;
  }
  // out is [ni][nj_pad] where nj_pad = roundup(Kq, 64 or 128): see selunet_wgrad_ld()
  if (dtype == SELUNET_F32) {
    if (bi128 && bj == 128) launch_wgrad<float, 128, 128>(gp, gq, out, nj_pad, ni, nj_pad, st, ws);
    else if (bj == 128) launch_wgrad<float, 64, 128>(gp, gq, out, nj_pad, ni, nj_pad, st, ws);
    else if (bi128) launch_wgrad<float, 128, 64>(gp, gq, out, nj_pad, ni, nj_pad, st, ws);
    else launch_wgrad<float, 64, 64>(gp, gq, out, nj_pad, ni, nj_pad, st, ws);
  } else {
    if (bi128 && bj == 128) launch_wgrad<__bf16, 128, 128>(gp, gq, out, nj_pad, ni, nj_pad, st, ws);
    else if (bj == 128) launch_wgrad<__bf16, 64, 128>(gp, gq, out, nj_pad, ni, nj_pad, st, ws);
    else if (bi128) launch_wgrad<__bf16, 128, 64>(gp, gq, out, nj_pad, ni, nj_pad, st, ws);
    else launch_wgrad<__bf16, 64, 64>(gp, gq, out, nj_pad, ni, nj_pad, st, ws);
  }
}

extern "C" int selunet_gemm_wgrad(const selunet_gather* p, const selunet_gather* q, float* out, int32_t dtype,
                                  void* stream) {
  WgradPlan w;
  if (int rc = plan_wgrad(p, q, dtype, w)) return rc;
  SELUNET_REQUIRE(out != nullptr, "out is NULL");
  w.wino = false;  // atomics into the packed output: the direct kernels
  launch_wgrad_any(w, out, nullptr, dtype, as_stream(stream));
  return check_launch("gemm_wgrad");
}

extern "C" int64_t selunet_gemm_wgrad_ws_bytes(const selunet_gather* p, const selunet_gather* q, int32_t dtype) {
  WgradPlan w;
  if (plan_wgrad(p, q, dtype, w)) return -1;
  return w.splits * (int64_t)w.ni * wgrad_ws_row(w) * 4;
}

extern "C" int selunet_gemm_wgrad_ws(const selunet_gather* p, const selunet_gather* q, float* out, float* ws,
                                     int64_t ws_bytes, int32_t dtype, void* stream) {
  WgradPlan w;
  if (int rc = plan_wgrad(p, q, dtype, w)) return rc;
  SELUNET_REQUIRE(out != nullptr, "out is NULL");
  const int64_t need = w.splits * (int64_t)w.ni * wgrad_ws_row(w) * 4;
  hipStream_t st = as_stream(stream);
  if (w.wino) {
    SELUNET_REQUIRE(ws != nullptr && ws_bytes >= need, "workspace of %lld bytes needed (got %lld)", (long long)need,
                    (long long)ws_bytes);
    if (int rc = conv3x3_wgrad_wino_launch(w.gp, w.gq, ws, 12 * w.gq.Ctot, st)) return rc;
    SELUNET_REQUIRE(hipMemsetAsync(out, 0, (size_t)w.ni * w.nj_pad * 4, st) == hipSuccess, "hipMemsetAsync failed");
    launch_wino_reduce(w, ws, WG_PACKED, out, st);
    return check_launch("gemm_wgrad_ws");
  }
  if (need == 0) {  // no split-partials path for these operands: zero + atomics
    SELUNET_REQUIRE(hipMemsetAsync(out, 0, (size_t)w.ni * w.nj_pad * 4, st) == hipSuccess, "hipMemsetAsync failed");
    launch_wgrad_any(w, out, nullptr, dtype, st);
    return check_launch("gemm_wgrad_ws");
  }
  SELUNET_REQUIRE(ws != nullptr && ws_bytes >= need, "workspace of %lld bytes needed (got %lld)", (long long)need,
                  (long long)ws_bytes);
  launch_wgrad_any(w, out, ws, dtype, st);
  const int64_t n4 = (int64_t)w.ni * w.nj_pad / 4;
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n4, 64), 16384));
  hipLaunchKernelGGL(wgrad_reduce_kernel<WG_PACKED>, dim3(blocks), dim3(64), 0, st, ws, w.splits, (int64_t)w.ni * w.nj_pad,
                     w.ni, w.nj_pad, w.gq.K, out);
  return check_launch("gemm_wgrad_ws");
}

// selunet_gemm_wgrad_ws with the result written straight in the reference parameter layout
// (layout 1: Conv2d [co][ci][3][3], 2: ConvTranspose2d [ci][co][2][2]); `packed` ([ni][ld] fp32)
// is scratch for the operands without a split-partials path (atomics, then the unpack kernel).
extern "C" int selunet_gemm_wgrad_ws_to(const selunet_gather* p, const selunet_gather* q, float* packed, float* ws,
                                        int64_t ws_bytes, int32_t layout, float* out, int32_t dtype, void* stream) {
  WgradPlan w;
  if (int rc = plan_wgrad(p, q, dtype, w)) return rc;
  SELUNET_REQUIRE(out != nullptr && (layout == WG_CONV3X3 || layout == WG_CONVT), "wgrad_ws_to: bad arguments");
  SELUNET_REQUIRE(w.gq.K % (layout == WG_CONV3X3 ? 9 : 4) == 0, "wgrad_ws_to: K_q = %d is not a multiple of %d",
                  w.gq.K, layout == WG_CONV3X3 ? 9 : 4);
  const int64_t need = w.splits * (int64_t)w.ni * wgrad_ws_row(w) * 4;
  if (w.wino) {
    SELUNET_REQUIRE(layout == WG_CONV3X3, "wgrad_ws_to: the Winograd planes are a 3x3 weight gradient");
    SELUNET_REQUIRE(ws != nullptr && ws_bytes >= need, "workspace of %lld bytes needed (got %lld)", (long long)need,
                    (long long)ws_bytes);
    hipStream_t st = as_stream(stream);
    if (int rc = conv3x3_wgrad_wino_launch(w.gp, w.gq, ws, 12 * w.gq.Ctot, st)) return rc;
    launch_wino_reduce(w, ws, WG_CONV3X3, out, st);
    return check_launch("gemm_wgrad_ws_to");
  }
  if (need == 0) {
    SELUNET_REQUIRE(packed != nullptr, "wgrad_ws_to: packed scratch is NULL");
    if (int rc = selunet_gemm_wgrad_ws(p, q, packed, ws, ws_bytes, dtype, stream)) return rc;
    return layout == WG_CONV3X3 ? selunet_unpack_conv3x3_grad(packed, w.ni, w.gq.K / 9, w.nj_pad, out, stream)
                                : selunet_unpack_convT_grad(packed, w.ni, w.gq.K / 4, out, stream);
  }
  SELUNET_REQUIRE(ws != nullptr && ws_bytes >= need, "workspace of %lld bytes needed (got %lld)", (long long)need,
                  (long long)ws_bytes);
  hipStream_t st = as_stream(stream);
  launch_wgrad_any(w, nullptr, ws, dtype, st);
  const int64_t n4 = (int64_t)w.ni * w.nj_pad / 4;
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n4, 64), 16384));
  if (layout == WG_CONV3X3)
    hipLaunchKernelGGL(wgrad_reduce_kernel<WG_CONV3X3>, dim3(blocks), dim3(64), 0, st, ws, w.splits,
                       (int64_t)w.ni * w.nj_pad, w.ni, w.nj_pad, w.gq.K, out);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<WG_CONVT>, dim3(blocks), dim3(64), 0, st, ws, w.splits,
                       (int64_t)w.ni * w.nj_pad, w.ni, w.nj_pad, w.gq.K, out);
  return check_launch("gemm_wgrad_ws_to");
}

// fp32 3x3 weight gradient on split-fp16 operands (conv3x3_wgrad_x2_kernel + the fixed-order split
// reduction into the Conv2d layout)
static int plan_wgrad_x2(const selunet_gather* p, const selunet_gather* q, WgradPlan& w, bool bn = false) {
  if (int rc = plan_wgrad(p, q, SELUNET_F32, w)) return rc;
  SELUNET_REQUIRE(halo_enabled() && conv3x3_wgrad_halo_eligible(w.gp, w.gq, SELUNET_F32) && w.gq.K % 9 == 0,
                  "conv3x3_wgrad_x2: operands not eligible (P: 1 tap, K %% 64 == 0; Q: 3x3, channels %% 64 == 0, "
                  "h >= 8, w >= 16)");
  w.splits = conv3x3_wgrad_x2_splits(w.gp, w.gq, nullptr, bn);
  return 0;
}

extern "C" int64_t selunet_conv3x3_wgrad_x2_ws_bytes(const selunet_gather* p, const selunet_gather* q) {
  WgradPlan w, wb;  // (the plain and the BN-fused forms' split plans)
  if (plan_wgrad_x2(p, q, w) || plan_wgrad_x2(p, q, wb, true)) return -1;
  return std::max(w.splits, wb.splits) * (int64_t)w.ni * w.nj_pad * 4;
}

extern "C" int selunet_conv3x3_wgrad_x2(const selunet_gather* p, const selunet_gather* q, float* ws, int64_t ws_bytes,
                                        float* out, const float* amax_p, const float* amax_q0, const float* amax_q1,
                                        void* stream) {
  WgradPlan w;
  if (int rc = plan_wgrad_x2(p, q, w)) return rc;
  const int64_t need = w.splits * (int64_t)w.ni * w.nj_pad * 4;
  SELUNET_REQUIRE(out != nullptr && ws != nullptr && ws_bytes >= need, "conv3x3_wgrad_x2: out / workspace of %lld bytes",
                  (long long)need);
  SELUNET_REQUIRE(amax_p != nullptr && amax_q0 != nullptr && (q->nsrc == 1 || amax_q1 != nullptr),
                  "conv3x3_wgrad_x2: every operand source needs its range word");
  hipStream_t st = as_stream(stream);
  if (int rc = conv3x3_wgrad_x2_launch(w.gp, w.gq, ws, w.nj_pad, amax_p, amax_q0, amax_q1, st)) return rc;
  const int64_t n4 = (int64_t)w.ni * w.nj_pad / 4;
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n4, 64), 16384));
  hipLaunchKernelGGL(wgrad_reduce_kernel<WG_CONV3X3>, dim3(blocks), dim3(64), 0, st, ws, w.splits,
                     (int64_t)w.ni * w.nj_pad, w.ni, w.nj_pad, w.gq.K, out);
  return check_launch("conv3x3_wgrad_x2");
}

extern "C" int selunet_conv3x3_wgrad_x2_bn_src(const selunet_gather* p, const selunet_gather* q, float* ws,
                                               int64_t ws_bytes, float* out, const float* amax_p, const float* amax_q0,
                                               const float* amax_q1, const selunet_bn_bwd_stats* bnb, const float* coef,
                                               const selunet_da_source* src, float* dy, float* dy_amax, void* stream) {
  WgradPlan w;
  if (int rc = plan_wgrad_x2(p, q, w, true)) return rc;
  const int64_t need = w.splits * (int64_t)w.ni * w.nj_pad * 4;
  SELUNET_REQUIRE(out != nullptr && ws != nullptr && ws_bytes >= need, "conv3x3_wgrad_x2_bn: out / workspace of %lld bytes",
                  (long long)need);
  SELUNET_REQUIRE(amax_p != nullptr && amax_q0 != nullptr && (q->nsrc == 1 || amax_q1 != nullptr),
                  "conv3x3_wgrad_x2_bn: every operand source needs its range word");
  SELUNET_REQUIRE(bnb && bnb->y && bnb->scale && bnb->shift && bnb->mean && bnb->invstd && coef,
                  "conv3x3_wgrad_x2_bn: y, scale, shift, mean, invstd and coef are required");
  SELUNET_REQUIRE(p->nsrc == 1 && p->src[0].scale == nullptr && p->src[0].layout == 0,
                  "conv3x3_wgrad_x2_bn: p gathers dA alone (one source, no transform)");
  SELUNET_REQUIRE((dy == nullptr) == (dy_amax == nullptr), "conv3x3_wgrad_x2_bn: dy and dy_amax go together");
  WgradBnArg bn{reinterpret_cast<const float*>(bnb->y), bnb->scale, bnb->shift, bnb->mean, bnb->invstd, coef, dy,
                dy_amax, SELUNET_DA_TENSOR, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  const int kind = src ? src->kind : SELUNET_DA_TENSOR;
  if (kind == SELUNET_DA_TENSOR) {
    SELUNET_REQUIRE(dy == nullptr || (dy != p->src[0].data && dy != bnb->y), "conv3x3_wgrad_x2_bn: dy must not alias dA or y");
  } else if (kind == SELUNET_DA_POOL) {
    SELUNET_REQUIRE(w.gp.K == 64 && w.gp.h % 2 == 0 && w.gp.w % 2 == 0 && src->pooled != nullptr,
                    "conv3x3_wgrad_x2_bn: a pool source needs C = 64, an even grid and the pooled gradient");
    SELUNET_REQUIRE(dy == nullptr || (dy != src->pooled && dy != src->skip && dy != bnb->y),
                    "conv3x3_wgrad_x2_bn: dy must not alias y, the pooled or the skip gradient");
    bn.pooled = src->pooled;
    bn.skip = src->skip;
  } else if (kind == SELUNET_DA_HEADS) {
    SELUNET_REQUIRE(w.gp.K == 64 && (src->nh == 1 || src->nh == 3) && src->head_w && src->g[0] &&
                        (src->nh == 1 || (src->g[1] && src->g[2])),
                    "conv3x3_wgrad_x2_bn: a heads source needs C = 64, nh = 1 or 3, the head weights and planes");
    SELUNET_REQUIRE(dy == nullptr || dy != bnb->y, "conv3x3_wgrad_x2_bn: dy must not alias y");
    bn.nh = src->nh;
    bn.hw = src->head_w;
    bn.g0 = src->g[0];
    bn.g1 = src->g[1];
    bn.g2 = src->g[2];
  } else {
    return fail(SELUNET_EINVAL, "conv3x3_wgrad_x2_bn: unknown dA source kind %d", kind);
  }
  bn.kind = kind;
  hipStream_t st = as_stream(stream);
  if (int rc = conv3x3_wgrad_x2_launch(w.gp, w.gq, ws, w.nj_pad, amax_p, amax_q0, amax_q1, st, &bn)) return rc;
  const int64_t n4 = (int64_t)w.ni * w.nj_pad / 4;
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n4, 64), 16384));
  hipLaunchKernelGGL(wgrad_reduce_kernel<WG_CONV3X3>, dim3(blocks), dim3(64), 0, st, ws, w.splits,
                     (int64_t)w.ni * w.nj_pad, w.ni, w.nj_pad, w.gq.K, out);
  return check_launch("conv3x3_wgrad_x2_bn");
}

extern "C" int selunet_conv3x3_wgrad_x2_bn(const selunet_gather* p, const selunet_gather* q, float* ws, int64_t ws_bytes,
                                           float* out, const float* amax_p, const float* amax_q0, const float* amax_q1,
                                           const selunet_bn_bwd_stats* bnb, const float* coef, float* dy, float* dy_amax,
                                           void* stream) {
  return selunet_conv3x3_wgrad_x2_bn_src(p, q, ws, ws_bytes, out, amax_p, amax_q0, amax_q1, bnb, coef, nullptr, dy,
                                         dy_amax, stream);
}

// generic fp32 weight gradient on split-fp16 operands (gemm_wgrad_x2_kernel + the fixed-order split
// reduction into the reference layout)
// tile of the generic split-fp16 weight gradient: 256 columns (512 threads, one workgroup per CU)
// where the operands allow, else 128 / 64 (256 threads, two per CU)
struct Gx2Tile {
  int bi, bj, nth;
};
static Gx2Tile gx2_tile(const WgradPlan& w) {
  if (w.nj_pad % 256 == 0 && (w.ni % 256 == 0 || w.ni == 128)) return {w.ni % 256 == 0 ? 256 : 128, 256, 512};
  return {w.ni % 128 == 0 ? 128 : 64, w.bj, 256};
}

static int plan_wgrad_gx2(const selunet_gather* p, const selunet_gather* q, WgradPlan& w) {
  if (int rc = plan_wgrad(p, q, SELUNET_F32, w)) return rc;
  SELUNET_REQUIRE(!w.gp.small && !w.gq.small && w.gp.K % 64 == 0 && w.gq.K % 64 == 0,
                  "gemm_wgrad_x2: vector gathers with K_p, K_q multiples of 64 (got %d, %d)", w.gp.K, w.gq.K);
  const Gx2Tile t = gx2_tile(w);
  w.splits = wgrad_splits(w.gp.M, (w.ni / t.bi) * (w.nj_pad / t.bj), nullptr, t.nth == 512 ? 256 : 0);
  return 0;
}

extern "C" int64_t selunet_gemm_wgrad_x2_ws_bytes(const selunet_gather* p, const selunet_gather* q) {
  WgradPlan w;
  if (plan_wgrad_gx2(p, q, w)) return -1;
  return w.splits * (int64_t)w.ni * w.nj_pad * 4;
}

extern "C" int selunet_gemm_wgrad_x2(const selunet_gather* p, const selunet_gather* q, float* ws, int64_t ws_bytes,
                                     int32_t layout, float* out, const float* amax_p0, const float* amax_p1,
                                     const float* amax_q0, const float* amax_q1, void* stream) {
  WgradPlan w;
  if (int rc = plan_wgrad_gx2(p, q, w)) return rc;
  SELUNET_REQUIRE(out != nullptr && (layout == WG_CONV3X3 || layout == WG_CONVT), "gemm_wgrad_x2: bad arguments");
  SELUNET_REQUIRE(w.gq.K % (layout == WG_CONV3X3 ? 9 : 4) == 0, "gemm_wgrad_x2: K_q = %d is not a multiple of %d",
                  w.gq.K, layout == WG_CONV3X3 ? 9 : 4);
  const int64_t need = w.splits * (int64_t)w.ni * w.nj_pad * 4;
  SELUNET_REQUIRE(ws != nullptr && ws_bytes >= need, "gemm_wgrad_x2: workspace of %lld bytes needed", (long long)need);
  SELUNET_REQUIRE(amax_p0 && amax_q0 && (p->nsrc == 1 || amax_p1) && (q->nsrc == 1 || amax_q1),
                  "gemm_wgrad_x2: every operand source needs its range word");
  hipStream_t st = as_stream(stream);
  const Gx2Tile t = gx2_tile(w);
  const int bi = t.bi;
  const int tiles_j = w.nj_pad / t.bj, tiles = (w.ni / bi) * tiles_j;
  int64_t mchunk;
  wgrad_splits(w.gp.M, tiles, &mchunk, t.nth == 512 ? 256 : 0);
  const unsigned blocks = (unsigned)(tiles * w.splits);
  const int64_t stride = (int64_t)w.ni * w.nj_pad;
  if (t.nth == 512 && bi == 256)
    hipLaunchKernelGGL((gemm_wgrad_x2_kernel<256, 256, 512>), dim3(blocks), dim3(512), 0, st, w.gp, w.gq, w.nj_pad,
                       mchunk, tiles_j, tiles, ws, stride, amax_p0, amax_p1, amax_q0, amax_q1);
  else if (t.nth == 512)
    hipLaunchKernelGGL((gemm_wgrad_x2_kernel<128, 256, 512>), dim3(blocks), dim3(512), 0, st, w.gp, w.gq, w.nj_pad,
                       mchunk, tiles_j, tiles, ws, stride, amax_p0, amax_p1, amax_q0, amax_q1);
  else if (bi == 128 && w.bj == 128)
    hipLaunchKernelGGL((gemm_wgrad_x2_kernel<128, 128>), dim3(blocks), dim3(256), 0, st, w.gp, w.gq, w.nj_pad, mchunk,
                       tiles_j, tiles, ws, stride, amax_p0, amax_p1, amax_q0, amax_q1);
  else if (w.bj == 128)
    hipLaunchKernelGGL((gemm_wgrad_x2_kernel<64, 128>), dim3(blocks), dim3(256), 0, st, w.gp, w.gq, w.nj_pad, mchunk,
                       tiles_j, tiles, ws, stride, amax_p0, amax_p1, amax_q0, amax_q1);
  else if (bi == 128)
    hipLaunchKernelGGL((gemm_wgrad_x2_kernel<128, 64>), dim3(blocks), dim3(256), 0, st, w.gp, w.gq, w.nj_pad, mchunk,
                       tiles_j, tiles, ws, stride, amax_p0, amax_p1, amax_q0, amax_q1);
  else
    hipLaunchKernelGGL((gemm_wgrad_x2_kernel<64, 64>), dim3(blocks), dim3(256), 0, st, w.gp, w.gq, w.nj_pad, mchunk,
                       tiles_j, tiles, ws, stride, amax_p0, amax_p1, amax_q0, amax_q1);
  if (int rc = check_launch("gemm_wgrad_x2")) return rc;
  const int64_t n4 = (int64_t)w.ni * w.nj_pad / 4;
  const unsigned rblocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n4, 64), 16384));
  if (layout == WG_CONV3X3)
    hipLaunchKernelGGL(wgrad_reduce_kernel<WG_CONV3X3>, dim3(rblocks), dim3(64), 0, st, ws, w.splits, stride, w.ni,
                       w.nj_pad, w.gq.K, out);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<WG_CONVT>, dim3(rblocks), dim3(64), 0, st, ws, w.splits, stride, w.ni,
                       w.nj_pad, w.gq.K, out);
  return check_launch("gemm_wgrad_x2");
}

// leading dimension of the packed wgrad output for a Q operand with kq columns
extern "C" int32_t selunet_wgrad_ld(int32_t kq) {
  const int bj = (kq % 128 == 0 || kq > 512) ? 128 : 64;
  return (int32_t)(cdiv(kq, bj) * bj);
}
