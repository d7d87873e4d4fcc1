// 3x3 / stride 1 / pad 1 convolution (model.py:11) as an MFMA implicit GEMM whose A operand is
// staged once per channel chunk as a (16+2) x (16+2)-pixel halo tile in LDS: the nine taps read
// shifted 16x16 windows of the same tile instead of re-gathering every input pixel nine times
// through L2. Used for the conv forward (BN+ReLU of the producer folded into the staging, torch.cat
// sources read in place) and for the data-gradient (dY with the flipped/transposed weight pack).
//
// Workgroup: 512 threads = 8 waves (2 per SIMD), output tile 16x16 pixels x BN channels
// (BN = 128: waves 4(M) x 2(N), 64 px x 64 ch each; BN = 64: 8 x 1, 32 px x 64 ch). One K-step =
// one tap x one 128-B channel chunk (32 fp32 / 64 bf16 channels). B (weights) is double-buffered
// per step; the next chunk's halo is loaded a 16-B slice per thread per tap during the current
// chunk's first six taps (load early, write late) into the second halo buffer.
// Weight rows in LDS are 144 B (128 B + 16 B pad) so ds_read_b128 fragment reads of 16 consecutive
// rows hit 16 distinct bank slots; halo rows use the swizzled 160-B layout below (AROWB).
#include <cstdlib>

#include "gemm_common.h"

namespace selunet {

constexpr int TH = 16, TW = 16;         // output tile (pixels)
constexpr int HHT = TH + 2, HWT = TW + 2;  // halo tile
constexpr int HPIX = HHT * HWT;         // 324 halo pixels
constexpr int HTHREADS = 512;
constexpr int A_ROUNDS = (HPIX * 8 + HTHREADS - 1) / HTHREADS;  // 16-B halo loads per thread per chunk
// Halo rows are 160 B (10 bank units of 16 B) with the two 16-B halves of each 32-B k slice
// swapped on odd halo lines (slot ^ (hy & 1)): the fragment reads of a wave's 32 pixels (two image
// rows, i.e. halo rows R..R+15 and R+18..R+33) then hit 16 distinct bank units in every ds_read_b128
// lane group for all nine tap offsets (144-B rows: 2-way conflicts on this pattern).
constexpr int AROWB = 160;
__device__ __forceinline__ int halo_off(int hp, int cc) { return hp * AROWB + ((cc ^ ((hp / HWT) & 1)) << 4); }

// ONE_CHUNK: the whole K of a tap fits one chunk (C == CK): a single halo buffer, no halo
// prefetch, and LDS small enough for two workgroups per CU so one's prologue/epilogue overlaps
// the other's MFMAs.
template <typename T, int BN, bool ONE_CHUNK>
__global__ void __launch_bounds__(HTHREADS, ONE_CHUNK ? 2 : 1)
conv3x3_halo_kernel(GatherArg g, const T* __restrict__ B, int N, int k_pad, EpiArg ep, int n_tiles, int tiles_x,
                    int tiles_y) {
  constexpr int E = 16 / sizeof(T);       // elements per 16-B vector
  constexpr int CK = 128 / sizeof(T);     // channels per chunk
  constexpr int WAVES_N = BN / 64;
  constexpr int WAVES_M = 8 / WAVES_N;
  constexpr int WPIX = (TH * TW) / WAVES_M;  // 64 or 32 pixels per wave
  constexpr int MT = WPIX / 32;
  constexpr int NT = 2;                   // 64 channels per wave
  constexpr int B_ROUNDS = BN * 8 / HTHREADS;
  static_assert(B_ROUNDS * HTHREADS == BN * 8, "weight tile rows must split evenly over the threads");
  constexpr int NHBUF = ONE_CHUNK ? 1 : 2;
  constexpr int AD = 3;                   // halo slice loaded at tap r is written at tap r + AD

  constexpr int SMEM_MAIN = NHBUF * HPIX * AROWB + 2 * BN * ROWB + (ONE_CHUNK ? 0 : 2 * CK * 8);
  constexpr int SMEM_EPI = TH * TW * (BN + 4) * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI];
  unsigned char* As = smem;
  unsigned char* Bs = smem + NHBUF * HPIX * AROWB;
  // folded BN coefficients of the prefetched chunk: [2 buffers][CK] scale, then [2][CK] shift
  float* Ss = reinterpret_cast<float*>(Bs + 2 * BN * ROWB);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int half = lane >> 5, l32 = lane & 31;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int n_tile = lb % n_tiles;
  const int ptile = lb / n_tiles;
  const int tx_t = ptile % tiles_x;
  const int rest = ptile / tiles_x;
  const int ty_t = rest % tiles_y;
  const int img = rest / tiles_y;
  const int y0 = ty_t * TH, x0 = tx_t * TW;
  const int n0 = n_tile * BN;

  const int nchunks = g.Ctot / CK;
  const int nsteps = nchunks * 9;

  // ---------------------------------------------------------------- staging helpers
  // halo slice `round` of this thread: halo pixel hp, 16-B column cc; false outside the slice
  // (hp clamped into the tile for the partial last round, so loads can be issued unconditionally)
  auto a_slot = [&](int round, int& hp, int& cc) -> bool {
    const int hidx = round * HTHREADS + tid;
    hp = min(hidx >> 3, HPIX - 1);
    cc = hidx & 7;
    return hidx < HPIX * 8;
  };
  auto a_inside = [&](int hp) -> bool {
    const int hy = hp / HWT, hx = hp - (hp / HWT) * HWT;
    return (unsigned)(y0 - 1 + hy) < (unsigned)g.h && (unsigned)(x0 - 1 + hx) < (unsigned)g.w;
  };
  // global address of chunk `chunk`'s 16-B slice (hp, cc), the pixel clamped into the image (the
  // zero padding is applied when the slice is written to LDS); a chunk never straddles sources
  auto a_ptr = [&](int chunk, int hp, int cc) -> const uint4* {
    int c = chunk * CK;
    const bool s1 = g.nsrc > 1 && c >= g.src[0].C;
    if (s1) c -= g.src[0].C;
    const SrcArg sa = pick_src(g, s1 ? 1 : 0);
    const int hy = hp / HWT, hx = hp - (hp / HWT) * HWT;
    const int ys = min(max(y0 - 1 + hy, 0), g.h - 1), xs = min(max(x0 - 1 + hx, 0), g.w - 1);
    return reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(sa.data) +
                                          (((int64_t)img * g.h + ys) * g.w + xs) * sa.C + c + cc * E);
  };
  struct BRegs {
    uint4 v[B_ROUNDS];
  };
  auto b_load = [&](int step) __attribute__((always_inline)) {
    const int chunk = step / 9, tap = step - chunk * 9;
    const int k0 = tap * g.Ctot + chunk * CK;
    BRegs rb;
#pragma unroll
    for (int r = 0; r < B_ROUNDS; ++r) {
      const int idx = r * HTHREADS + tid;
      const int row = idx >> 3, cc = idx & 7;
      rb.v[r] = *reinterpret_cast<const uint4*>(B + (int64_t)(n0 + row) * k_pad + k0 + cc * E);
    }
    return rb;
  };
  auto b_store = [&](const BRegs& rb, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < B_ROUNDS; ++r) {
      const int idx = r * HTHREADS + tid;
      const int row = idx >> 3, cc = idx & 7;
      *reinterpret_cast<uint4*>(Bs + (buf * BN + row) * ROWB + cc * 16) = rb.v[r];
    }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x16{};

  // per-lane halo row of pixel (subtile a, lane) for tap (0,0), and the 16-B half it reads after the
  // odd-line swap (half ^ parity of the halo line; the tap's dy flips the parity)
  int hrow0[MT], hsw0[MT];
#pragma unroll
  for (int a = 0; a < MT; ++a) {
    const int pix = wm * WPIX + a * 32 + l32;
    hrow0[a] = (pix / TW) * HWT + (pix % TW);
    hsw0[a] = half ^ ((pix / TW) & 1);
  }

  auto mma_step = [&](int hbuf, int bbuf, int t) __attribute__((always_inline)) {
    const unsigned char* a_src = As + hbuf * HPIX * AROWB;
    const unsigned char* b_src = Bs + bbuf * BN * ROWB;
    const int dy = t / 3, dx = t - (t / 3) * 3;
    const int tap_off = dy * HWT + dx;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int boff = q * 32 + half * 16;
      uint4 af[MT], bfr[NT];
#pragma unroll
      for (int a = 0; a < MT; ++a)
        af[a] = *reinterpret_cast<const uint4*>(a_src + (hrow0[a] + tap_off) * AROWB + q * 32 + ((hsw0[a] ^ dy) & 1) * 16);
#pragma unroll
      for (int b = 0; b < NT; ++b)
        bfr[b] = *reinterpret_cast<const uint4*>(b_src + (wn * 64 + b * 32 + l32) * ROWB + boff);
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) Mma<T>::run(acc[a][b], af[a], bfr[b]);
    }
  };

  // ---------------------------------------------------------------- prologue: chunk 0, B(0), B(1)
  {
    const int c0 = 0;
    const SrcArg sa = pick_src(g, 0);
    uint4 v0[A_ROUNDS];
#pragma unroll
    for (int r = 0; r < A_ROUNDS; ++r) {
      int hp, cc;
      a_slot(r, hp, cc);
      v0[r] = *a_ptr(0, hp, cc);
    }
#pragma unroll
    for (int r = 0; r < A_ROUNDS; ++r) {
      int hp, cc;
      if (!a_slot(r, hp, cc)) continue;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a_inside(hp)) {
        v = v0[r];
        if (sa.scale) v = transform16<T>(v, sa.scale, sa.shift, c0 + cc * E, sa.relu);
      }
      *reinterpret_cast<uint4*>(As + halo_off(hp, cc)) = v;
    }
  }
  BRegs rb_next = b_load(0);
  b_store(rb_next, 0);
  rb_next = b_load(nsteps > 1 ? 1 : 0);
  __syncthreads();

  if constexpr (ONE_CHUNK) {
    // ------------------------------------------------------------ 9 taps of the single chunk
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      BRegs rb_far = rb_next;
      if (t + 2 < 9) rb_far = b_load(t + 2);
      mma_step(0, t & 1, t);
      if (t + 1 < 9) b_store(rb_next, (t + 1) & 1);
      __syncthreads();
      rb_next = rb_far;
    }
  } else {
    // ------------------------------------------------------------ main loop over chunks
    uint4 ra[A_ROUNDS];
    for (int c = 0; c < nchunks; ++c) {
      const int cn = c + 1 < nchunks ? c + 1 : c;  // prefetched chunk (the last one reloads itself)
      int cs = cn * CK;
      const bool s1 = g.nsrc > 1 && cs >= g.src[0].C;
      if (s1) cs -= g.src[0].C;
      const SrcArg sn = pick_src(g, s1 ? 1 : 0);
      float* ssc = Ss + ((c + 1) & 1) * CK;
      float* ssh = Ss + 2 * CK + ((c + 1) & 1) * CK;
      float coef = 0.0f;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int s = c * 9 + t;
        const BRegs rb_far = b_load(s + 2 < nsteps ? s + 2 : nsteps - 1);
        if (t == 0 && sn.scale && tid < 2 * CK) coef = tid < CK ? sn.scale[cs + tid] : sn.shift[cs + tid - CK];
        if (t < A_ROUNDS) {
          int hp, cc;
          a_slot(t, hp, cc);
          ra[t] = *a_ptr(cn, hp, cc);
        }
        mma_step(c & 1, s & 1, t);
        b_store(rb_next, (s + 1) & 1);
        if (t == 1 && sn.scale && tid < 2 * CK) (tid < CK ? ssc[tid] : ssh[tid - CK]) = coef;
        if (t >= AD && t - AD < A_ROUNDS) {
          const int r = t - AD;
          int hp, cc;
          if (a_slot(r, hp, cc)) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (a_inside(hp)) {
              v = ra[r];
              if (sn.scale) {
                // transform with the coefficients staged in LDS at t == 1 (visible after its barrier)
                T e[E];
                __builtin_memcpy(e, &v, 16);
#pragma unroll
                for (int j = 0; j < E; ++j) {
                  float f = to_f(e[j]) * ssc[cc * E + j] + ssh[cc * E + j];
                  if (sn.relu) f = fmaxf(f, 0.0f);
                  e[j] = from_f<T>(f);
                }
                __builtin_memcpy(&v, e, 16);
              }
            }
            *reinterpret_cast<uint4*>(As + ((c + 1) & 1) * HPIX * AROWB + halo_off(hp, cc)) = v;
          }
        }
        __syncthreads();
        rb_next = rb_far;
      }
    }
  }

  // ---------------------------------------------------------------- epilogue (LDS-staged)
  float* tile = reinterpret_cast<float*>(smem);  // [256][BN + 4]; the loop ended with a barrier
  acc_to_lds<MT, NT, BN>(tile, acc, wm * WPIX, wn * 64, lane);
  __syncthreads();
  auto dst = [&](int pix, int c) -> T* {
    const int y = y0 + pix / TW, x = x0 + pix % TW;
    if (y >= g.h || x >= g.w) return nullptr;
    const int64_t m = ((int64_t)img * g.h + y) * g.w + x;
    const int col = n0 + c;
    if (ep.mode == SELUNET_EP_SPLIT)
      return col < ep.split ? reinterpret_cast<T*>(ep.out0) + m * ep.split + col
                            : reinterpret_cast<T*>(ep.out1) + m * (N - ep.split) + (col - ep.split);
    return reinterpret_cast<T*>(ep.out0) + m * N + col;
  };
  auto bias_col = [&](int c) { return n0 + c; };
  lds_tile_store<T, TH * TW, BN, HTHREADS>(tile, tid, dst, ep.bias, bias_col, tile_stats(ep, ptile, n0, N));
}

// =========================================================================== persistent variant
// Multi-chunk layers (C > one chunk) at one workgroup per CU: a non-persistent workgroup exposes
// its prologue (first halo chunk and weights from HBM, nothing else resident to overlap it) and its
// epilogue on every tile. Here each workgroup keeps one column tile (n0) and walks the output tiles
// prow, prow + gp, prow + 2 gp, ...; its (tile, chunk) jobs form one stream, so the first chunk of
// tile i+1 and its weights are loaded during the last chunk of tile i. Those loads stay in registers
// until the epilogue of tile i (which uses the whole LDS) is done, then go to LDS. The epilogue's
// column sums (BN statistics / colsum / BN-backward sums) accumulate in registers over the tiles
// and are reduced once: one slab row per workgroup (row prow, see conv3x3_halo_stats_rows).
//
// X2 (fp32 sources only): the split-fp16 form of the fp32 convolution (selunet_conv3x3_x2). The halo
// stager scales every transformed value by 2^e (from the operand range words amax0/amax1) and
// writes it as two fp16 parts into the same 128-B pixel row a 32-channel fp32 chunk occupies:
// bytes 0-63 the 32 high parts, 64-127 the 32 low parts, so 16-B units q = 0, 1 hold the high
// parts of the two 16-channel k-steps and q = 2, 3 their low parts. The weights
// (SELUNET_PACK_CONV3X3_X2) have the same 128-B layout per (tap, chunk) and are staged unchanged.
// Per tap: 2 k-steps x 3 v_mfma_f32_32x32x16_f16 (hh, hl, lh) per 32x32 subtile instead of 16 fp32
// MFMAs (32 vs 64 cycles each: 5.3x fewer MFMA cycles); the accumulators are unscaled by
// 2^-e * (row unscale of the weights) before the epilogue.
// M16 (X2 only, used at BN = 64): v_mfma_f32_16x16x32_f16 instead of 32x32x16 — the same cycles per
// FLOP, but the chip holds a higher clock on the smaller shape under a power-limited load (MI355X
// guide, DVFS item 7).
// A wave's 16x16 subtiles: one tile row (16 px) x 16 columns; one MFMA covers a tap's whole
// 32-channel chunk (lane: row/column lane & 15, channels 8 (lane >> 4) .. + 7); weight rows are 160 B
// so the 16 rows of a ds_read_b128 lane group hit distinct bank slots.
// TQ (split-fp16 only, SELUNET_OPT_TILE_QUEUE): the workgroups of a column tile take their pixel tiles from an
// atomic ticket counter instead of the static walk prow, prow + gp, ..., so a launch whose workgroups cannot
// all start at once (CUs held by a concurrent RCCL all-reduce kernel) rebalances instead of
// ending with its late workgroups' whole share. The next tile is claimed one tile ahead (tap 0 of chunk 0,
// consumed at chunk 1), so the atomic's latency hides under the MFMAs. The statistics (BN sums, BN-backward
// sums, column sums) are flushed per tile into slab row = tile index — results are independent of which
// workgroup ran a tile, so the launch stays deterministic. tq: [2][n_tiles] counters (tickets, finished
// workgroups), zero between launches: the last workgroup of a column tile to finish resets both.
template <typename T, int BN, bool X2, bool M16 = false, bool TQ = false>
__global__ void __launch_bounds__(HTHREADS, 1)
conv3x3_halo_persist_kernel(GatherArg g, const T* __restrict__ B, int N, int k_pad, EpiArg ep, int n_tiles,
                            int tiles_x, int tiles_y, int ptiles, int gp, const float* __restrict__ wcs,
                            const float* __restrict__ amax0, const float* __restrict__ amax1,
                            unsigned* __restrict__ tq = nullptr) {
  static_assert(!TQ || X2, "tile queue: split-fp16 kernel only");
  static_assert(!X2 || std::is_same<T, float>::value, "split-fp16 form of fp32 operands only");
  static_assert(!M16 || X2, "16x16x32 form: split-fp16 only (the bf16 form lost every A/B, retired in round 6)");
  constexpr int E = 16 / sizeof(T);
  constexpr int CK = 128 / sizeof(T);
  constexpr int WAVES_N = BN / 64;
  constexpr int WAVES_M = 8 / WAVES_N;
  constexpr int WPIX = (TH * TW) / WAVES_M;
  constexpr int MT = WPIX / 32;
  constexpr int NT = 2;
  constexpr int RT = WPIX / 16;  // M16: 16-px subtiles (tile rows) per wave
  // accumulators: MT x NT 32x32 subtiles, or (M16) RT x 4 16x16 subtiles — the same registers
  using AccT = std::conditional_t<M16, f32x4, f32x16>;
  constexpr int AM = M16 ? RT : MT, AN = M16 ? 4 : NT;
  constexpr int WROWB = M16 ? 160 : ROWB;  // LDS bytes per weight row
  constexpr int B_ROUNDS = BN * 8 / HTHREADS;
  static_assert(B_ROUNDS * HTHREADS == BN * 8, "weight tile rows must split evenly over the threads");
  // tap at which halo slice r of the next job is loaded / written to LDS (written at >= 2: the
  // coefficients staged at tap 1 are visible from tap 2 on)
  auto halo_load_tap = [](int r) { return r; };
  auto halo_write_tap = [](int r) { return r + 3; };
  static_assert(A_ROUNDS <= 6, "halo slice schedule covers six slices");

  constexpr int SMEM_MAIN = 2 * HPIX * AROWB + 2 * BN * WROWB + 2 * CK * 8;
  constexpr int SMEM_EPI = TH * TW * (BN + 4) * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI];
  unsigned char* As = smem;
  unsigned char* Bs = smem + 2 * HPIX * AROWB;
  float* Ss = reinterpret_cast<float*>(Bs + 2 * BN * WROWB);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int half = lane >> 5, l32 = lane & 31;
  const int l16 = lane & 15, kg = lane >> 4;  // M16 fragment coordinates

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int n_tile = lb % n_tiles;
  const int prow = lb / n_tiles;
  const int n0 = n_tile * BN;
  const int nchunks = g.Ctot / CK;
  const int ntl = TQ ? 0 : (prow < ptiles ? (ptiles - prow + gp - 1) / gp : 0);  // host: gp <= ptiles, so >= 1
  // TQ: this workgroup's tiles are claimed tickets (>= ptiles: none left); static: prow, prow + gp, ...
  __shared__ int tq_slot;
  int pt_cur = 0, pt_next = 0;
  if constexpr (TQ) {
    if (tid == 0) tq_slot = (int)min(atomicAdd(tq + n_tile, 1u), (unsigned)ptiles);
    __syncthreads();
    pt_cur = tq_slot;
  }
  const int csteps = nchunks * 9;  // steps per tile
  float xs = 1.0f;       // X2: operand scale 2^e
  float cfac[AN] = {};   // X2: accumulator unscale per column subtile (this lane's column)
  if constexpr (X2) {
    float am = amax0 ? amax0[0] : 0.0f;
    if (g.nsrc > 1 && amax1) am = fmaxf(am, amax1[0]);
    float inv;
    xs = x2_scale(am, &inv);
#pragma unroll
    for (int b = 0; b < AN; ++b)
      cfac[b] = wcs[n0 + wn * 64 + (M16 ? b * 16 + l16 : b * 32 + l32)] * inv;
  }
  // one 16-B halo slice (4 transformed fp32 values or E raw elements) to halo buffer hb
  auto halo_store = [&](int hb, int hp, int cc, uint4 v) __attribute__((always_inline)) {
    unsigned char* base = As + hb * HPIX * AROWB + hp * AROWB;
    if constexpr (X2) {
      float f[4];
      __builtin_memcpy(f, &v, 16);
      f16x4 h, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        _Float16 a, b;
        x2_split(f[e] * xs, a, b);
        h[e] = a;
        l[e] = b;
      }
      const int par = (hp / HWT) & 1;
      *reinterpret_cast<f16x4*>(base + (((cc >> 1) ^ par) << 4) + (cc & 1) * 8) = h;
      *reinterpret_cast<f16x4*>(base + (((4 + (cc >> 1)) ^ par) << 4) + (cc & 1) * 8) = l;
    } else {
      *reinterpret_cast<uint4*>(base + (((cc ^ ((hp / HWT) & 1))) << 4)) = v;
    }
  };

  // a slice already transformed (X2: and split, high parts in .x/.y, low parts in .z/.w) in the last job
  auto halo_store_prepped = [&](int hb, int hp, int cc, uint4 v) __attribute__((always_inline)) {
    unsigned char* base = As + hb * HPIX * AROWB + hp * AROWB;
    if constexpr (X2) {
      const int par = (hp / HWT) & 1;
      *reinterpret_cast<uint2*>(base + (((cc >> 1) ^ par) << 4) + (cc & 1) * 8) = make_uint2(v.x, v.y);
      *reinterpret_cast<uint2*>(base + (((4 + (cc >> 1)) ^ par) << 4) + (cc & 1) * 8) = make_uint2(v.z, v.w);
    } else {
      *reinterpret_cast<uint4*>(base + (((cc ^ ((hp / HWT) & 1))) << 4)) = v;
    }
  };
  auto tile_xy = [&](int pt_i, int& img, int& y0, int& x0) __attribute__((always_inline)) {
    const unsigned pt = (unsigned)pt_i;
    const unsigned r = pt / (unsigned)tiles_x;
    x0 = (int)(pt - r * (unsigned)tiles_x) * TW;
    const unsigned r2 = r / (unsigned)tiles_y;
    y0 = (int)(r - r2 * (unsigned)tiles_y) * TH;
    img = (int)r2;
  };
  auto a_slot = [&](int round, int& hp, int& cc) -> bool {
    const int hidx = round * HTHREADS + tid;
    hp = min(hidx >> 3, HPIX - 1);
    cc = hidx & 7;
    return hidx < HPIX * 8;
  };
  auto a_inside = [&](int y0, int x0, int hp) -> bool {
    const int hy = hp / HWT, hx = hp - (hp / HWT) * HWT;
    return (unsigned)(y0 - 1 + hy) < (unsigned)g.h && (unsigned)(x0 - 1 + hx) < (unsigned)g.w;
  };
  // source (and its channel base) of chunk `chunk`; a chunk never straddles sources
  auto chunk_src = [&](int chunk, int& c) -> SrcArg {
    c = chunk * CK;
    const bool s1 = g.nsrc > 1 && c >= g.src[0].C;
    if (s1) c -= g.src[0].C;
    return pick_src(g, s1 ? 1 : 0);
  };
  auto a_ptr = [&](const SrcArg& sa, int c, int img, int y0, int x0, int hp, int cc) -> const uint4* {
    const int hy = hp / HWT, hx = hp - (hp / HWT) * HWT;
    const int ys = min(max(y0 - 1 + hy, 0), g.h - 1), xs = min(max(x0 - 1 + hx, 0), g.w - 1);
    return reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(sa.data) +
                                          (((int64_t)img * g.h + ys) * g.w + xs) * sa.C + c + cc * E);
  };
  struct BRegs {
    uint4 v[B_ROUNDS];
  };
  auto b_load = [&](int st) __attribute__((always_inline)) {  // st: step within a tile
    const int chunk = st / 9, tap = st - chunk * 9;
    const int k0 = tap * g.Ctot + chunk * CK;
    BRegs rb;
#pragma unroll
    for (int r = 0; r < B_ROUNDS; ++r) {
      const int idx = r * HTHREADS + tid;
      const int row = idx >> 3, cc = idx & 7;
      rb.v[r] = *reinterpret_cast<const uint4*>(B + (int64_t)(n0 + row) * k_pad + k0 + cc * E);
    }
    return rb;
  };
  auto b_store = [&](const BRegs& rb, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < B_ROUNDS; ++r) {
      const int idx = r * HTHREADS + tid;
      const int row = idx >> 3, cc = idx & 7;
      *reinterpret_cast<uint4*>(Bs + (buf * BN + row) * WROWB + cc * 16) = rb.v[r];
    }
  };

  AccT acc[AM][AN];
#pragma unroll
  for (int a = 0; a < AM; ++a)
#pragma unroll
    for (int b = 0; b < AN; ++b) acc[a][b] = AccT{};
  int hrow0[MT], hsw0[MT];
#pragma unroll
  for (int a = 0; a < MT; ++a) {
    const int pix = wm * WPIX + a * 32 + l32;
    hrow0[a] = (pix / TW) * HWT + (pix % TW);
    hsw0[a] = half ^ ((pix / TW) & 1);
  }
  auto mma_step = [&](int hbuf, int bbuf, int t) __attribute__((always_inline)) {
    const unsigned char* a_src = As + hbuf * HPIX * AROWB;
    const unsigned char* b_src = Bs + bbuf * BN * WROWB;
    const int dy = t / 3, dx = t - (t / 3) * 3;
    const int tap_off = dy * HWT + dx;
    if constexpr (M16) {
      // the wave's 4 column subtiles' weight fragments (high, low), then per tile row its halo
      // fragments and 12 MFMAs; unit kg ^ (halo row parity) undoes the halo swizzle (halo_store)
      f16x8 bh[4], bl[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const unsigned char* p = b_src + (wn * 64 + b * 16 + l16) * WROWB + kg * 16;
        bh[b] = *reinterpret_cast<const f16x8*>(p);
        bl[b] = *reinterpret_cast<const f16x8*>(p + 64);
      }
#pragma unroll
      for (int a = 0; a < RT; ++a) {
        const int py = wm * RT + a;
        const unsigned char* p =
            a_src + ((py + dy) * HWT + l16 + dx) * AROWB + ((kg ^ ((py + dy) & 1)) << 4);
        const f16x8 ah = *reinterpret_cast<const f16x8*>(p);
        const f16x8 al = *reinterpret_cast<const f16x8*>(p + 64);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[b], acc[a][b], 0, 0, 0);
        }
      }
    } else if constexpr (X2) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        f16x8 ah[MT], al[MT], bh[NT], bl[NT];
#pragma unroll
        for (int a = 0; a < MT; ++a) {
          const unsigned char* p = a_src + (hrow0[a] + tap_off) * AROWB + ((hsw0[a] ^ dy) & 1) * 16;
          ah[a] = *reinterpret_cast<const f16x8*>(p + ks * 32);
          al[a] = *reinterpret_cast<const f16x8*>(p + (2 + ks) * 32);
        }
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const unsigned char* p = b_src + (wn * 64 + b * 32 + l32) * ROWB + half * 16;
          bh[b] = *reinterpret_cast<const f16x8*>(p + ks * 32);
          bl[b] = *reinterpret_cast<const f16x8*>(p + (2 + ks) * 32);
        }
        // the three products of one accumulator back to back (product-major order, consecutive
        // MFMAs sharing an operand, and hoisting both k-steps' reads were measured: DESIGN.md §3)
#pragma unroll
        for (int a = 0; a < MT; ++a)
#pragma unroll
          for (int b = 0; b < NT; ++b) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
          }
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int boff = q * 32 + half * 16;
        uint4 af[MT], bfr[NT];
#pragma unroll
        for (int a = 0; a < MT; ++a)
          af[a] = *reinterpret_cast<const uint4*>(a_src + (hrow0[a] + tap_off) * AROWB + q * 32 + ((hsw0[a] ^ dy) & 1) * 16);
#pragma unroll
        for (int b = 0; b < NT; ++b)
          bfr[b] = *reinterpret_cast<const uint4*>(b_src + (wn * 64 + b * 32 + l32) * WROWB + boff);
#pragma unroll
        for (int a = 0; a < MT; ++a)
#pragma unroll
          for (int b = 0; b < NT; ++b) Mma<T>::run(acc[a][b], af[a], bfr[b]);
      }
    }
  };
  // write halo slice `r` (raw registers v) of chunk source sa/c of the tile at (y0, x0) to buffer
  // hb, transformed with the global coefficients (used outside the steady-state loop)
  auto halo_put_global = [&](uint4 v, int r, const SrcArg& sa, int c, int y0, int x0, int hb)
      __attribute__((always_inline)) {
    int hp, cc;
    if (!a_slot(r, hp, cc)) return;
    uint4 o = make_uint4(0, 0, 0, 0);
    if (a_inside(y0, x0, hp)) o = sa.scale ? transform16<T>(v, sa.scale, sa.shift, c + cc * E, sa.relu) : v;
    halo_store(hb, hp, cc, o);
  };

  // ---------------------------------------------------------------- prologue: tile 0 chunk 0, B(0), B(1)
  if (!TQ || pt_cur < ptiles) {
    int img, y0, x0;
    tile_xy(TQ ? pt_cur : prow, img, y0, x0);
    int c0;
    const SrcArg sa = chunk_src(0, c0);
    uint4 v0[A_ROUNDS];
#pragma unroll
    for (int r = 0; r < A_ROUNDS; ++r) {
      int hp, cc;
      a_slot(r, hp, cc);
      v0[r] = *a_ptr(sa, c0, img, y0, x0, hp, cc);
    }
#pragma unroll
    for (int r = 0; r < A_ROUNDS; ++r) halo_put_global(v0[r], r, sa, c0, y0, x0, 0);
  }
  BRegs rb_next = b_load(0);
  b_store(rb_next, 0);
  rb_next = b_load(1 % csteps);
  __syncthreads();

  // (X2 at BN = 128: fp32 statistics registers, as the Winograd kernel — fp64 ones spill)
  using Acc = std::conditional_t<X2 && BN == 128, float, typename StatAcc<T>::type>;
  static_assert(stats_flush_bytes<BN, HTHREADS, Acc>() <= (int)sizeof(smem), "statistics scratch exceeds LDS");
  Acc s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float amx = 0.0f;  // running max |stored value| (epilogue range word)
  const TileStats ts = tile_stats(ep, TQ ? 0 : prow, n0, N);
  float* tile = reinterpret_cast<float*>(smem);  // epilogue: [256][BN + 4] over the whole LDS
  uint4 ra[A_ROUNDS];
  int J = 0;  // job (tile, chunk) counter: halo buffer J & 1
  int S = 0;  // step counter: weight buffer S & 1
  unsigned claimed = 0;  // TQ: the ticket tid 0 claims during a tile
  for (int i = 0; TQ ? pt_cur < ptiles : i < ntl; ++i) {
    int img, y0, x0;
    tile_xy(TQ ? pt_cur : prow + i * gp, img, y0, x0);
    BRegs rb_hold;
    for (int c = 0; c < nchunks; ++c, ++J) {
      if constexpr (TQ) {
        if (c == 1) pt_next = tq_slot;  // the ticket claimed at chunk 0 (nchunks >= 2)
      }
      const bool last_c = c + 1 == nchunks;
      const bool has_next = !last_c || (TQ ? pt_next < ptiles : i + 1 < ntl);
      const bool defer = last_c && has_next;  // next job is the next tile: LDS writes after the epilogue
      int nimg = img, ny0 = y0, nx0 = x0;
      if (defer) tile_xy(TQ ? pt_next : prow + (i + 1) * gp, nimg, ny0, nx0);
      const int nc = !has_next ? c : (last_c ? 0 : c + 1);
      int cs;
      const SrcArg sn = chunk_src(nc, cs);
      float* ssc = Ss + ((J + 1) & 1) * CK;
      float* ssh = Ss + 2 * CK + ((J + 1) & 1) * CK;
      float coef = 0.0f;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int st2 = c * 9 + t + 2;  // weights are loaded two steps ahead
        const BRegs rb_far = b_load(st2 < csteps ? st2 : st2 - csteps);  // next tile's steps wrap
        if (t == 0 && sn.scale && tid < 2 * CK) coef = tid < CK ? sn.scale[cs + tid] : sn.shift[cs + tid - CK];
#pragma unroll
        for (int r = 0; r < A_ROUNDS; ++r) {
          if (halo_load_tap(r) == t) {
            int hp, cc;
            a_slot(r, hp, cc);
            ra[r] = *a_ptr(sn, cs, nimg, ny0, nx0, hp, cc);
          }
        }
        if constexpr (TQ) {
          if (c == 0 && t == 0 && tid == 0) claimed = atomicAdd(tq + n_tile, 1u);  // the next tile's ticket
        }
        mma_step(J & 1, S & 1, t);
        if constexpr (TQ) {
          if (c == 0 && t == 8 && tid == 0) tq_slot = (int)min(claimed, (unsigned)ptiles);  // read at chunk 1
        }
        if (defer && t == 8) rb_hold = rb_next;  // B(S + 1): stored after the epilogue
        else b_store(rb_next, (S + 1) & 1);
        if (t == 1 && sn.scale && tid < 2 * CK) (tid < CK ? ssc[tid] : ssh[tid - CK]) = coef;
#pragma unroll
        for (int r = 0; r < A_ROUNDS; ++r) {
          if (halo_write_tap(r) != t) continue;
          int hp, cc;
          if (a_slot(r, hp, cc)) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (a_inside(ny0, nx0, hp)) {
              v = ra[r];
              if (sn.scale) {
                T e[E];
                __builtin_memcpy(e, &v, 16);
#pragma unroll
                for (int j = 0; j < E; ++j) {
                  float f = to_f(e[j]) * ssc[cc * E + j] + ssh[cc * E + j];
                  if (sn.relu) f = fmaxf(f, 0.0f);
                  e[j] = from_f<T>(f);
                }
                __builtin_memcpy(&v, e, 16);
              }
            }
            if (!defer) {
              halo_store((J + 1) & 1, hp, cc, v);
            } else {
              // the next tile's first job: its slice is transformed (and split) here, under this job's
              // MFMAs, and written to LDS after the epilogue (which uses the whole LDS) with no global reads
              if constexpr (X2) {
                float f[4];
                __builtin_memcpy(f, &v, 16);
                f16x4 h, l;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  _Float16 a, b;
                  x2_split(f[e] * xs, a, b);
                  h[e] = a;
                  l[e] = b;
                }
                __builtin_memcpy(&v.x, &h, 8);
                __builtin_memcpy(&v.z, &l, 8);
              }
              ra[r] = v;
            }
          }
        }
        __syncthreads();
        rb_next = rb_far;
        ++S;
      }
      if (defer) {
        // (kept for after the epilogue: ra[] = next tile's chunk 0, rb_hold = B(S), rb_next = B(S+1))
      }
    }

    // ------------------------------------------------------------ epilogue of tile i
    if constexpr (X2) {
#pragma unroll
      for (int a = 0; a < AM; ++a)
#pragma unroll
        for (int b = 0; b < AN; ++b) acc[a][b] *= cfac[b];
    }
    if constexpr (M16) {
      // 16x16 C layout: column lane & 15, rows 4 (lane >> 4) + i of the subtile (tile row py)
#pragma unroll
      for (int a = 0; a < RT; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            tile[(wm * WPIX + a * 16 + 4 * kg + i) * (BN + 4) + wn * 64 + b * 16 + l16] = acc[a][b][i];
    } else {
      acc_to_lds<MT, NT, BN>(tile, acc, wm * WPIX, wn * 64, lane);
    }
#pragma unroll
    for (int a = 0; a < AM; ++a)
#pragma unroll
      for (int b = 0; b < AN; ++b) acc[a][b] = AccT{};
    __syncthreads();
    auto dst = [&](int pix, int cl) -> T* {
      const int y = y0 + pix / TW, x = x0 + pix % TW;
      if (y >= g.h || x >= g.w) return nullptr;
      const int64_t m = ((int64_t)img * g.h + y) * g.w + x;
      const int col = n0 + cl;
      if (ep.mode == SELUNET_EP_SPLIT)
        return col < ep.split ? reinterpret_cast<T*>(ep.out0) + m * ep.split + col
                              : reinterpret_cast<T*>(ep.out1) + m * (N - ep.split) + (col - ep.split);
      return reinterpret_cast<T*>(ep.out0) + m * N + col;
    };
    auto bias_col = [&](int cl) { return n0 + cl; };
    if constexpr (TQ) {
      // this tile's statistics go to slab row pt_cur; the range word stays per workgroup (tracked by the store pass,
      // one atomic at the end — a null amax in the store pass left it 0, i.e. an operand scale of 2^14 for the
      // consumer, which overflowed the fp16 split once |values| passed 4: the divergence found in round 6)
      TileStats tt = tile_stats(ep, pt_cur, n0, N);
      lds_tile_store_acc<T, TH * TW, BN, HTHREADS>(tile, tid, dst, ep.bias, bias_col, tt, s1, s2, s3, amx);
      tt.amax = nullptr;
      tile_stats_flush<BN, HTHREADS>(tile, tid, tt, s1, s2, s3, 0.0f);
#pragma unroll
      for (int e = 0; e < 8; ++e) s1[e] = s2[e] = s3[e] = 0;
    } else {
      lds_tile_store_acc<T, TH * TW, BN, HTHREADS>(tile, tid, dst, ep.bias, bias_col, ts, s1, s2, s3, amx);
    }
    if (TQ ? pt_next < ptiles : i + 1 < ntl) {
      __syncthreads();  // the tile has been read: LDS back to halo / weights
      // (slots recomputed from an opaque copy of tid: kept from the prologue they would be spilled, and a
      // scratch reload here waits for every store of the epilogue above)
      int tid2 = tid;
      asm volatile("" : "+v"(tid2));
#pragma unroll
      for (int r = 0; r < A_ROUNDS; ++r) {
        const int hidx = r * HTHREADS + tid2;
        if (hidx < HPIX * 8) halo_store_prepped(J & 1, hidx >> 3, hidx & 7, ra[r]);  // (transformed in the last job)
      }
      b_store(rb_hold, S & 1);
      __syncthreads();
    }
    if constexpr (TQ) pt_cur = pt_next;
  }
  if constexpr (TQ) {
    if (ts.amax) block_amax(ts.amax, amx, tile);
    if (tid == 0 && atomicAdd(tq + n_tiles + n_tile, 1u) == (unsigned)gp - 1u) {
      // every workgroup of this column tile has made its last claim: reset for the next launch
      atomicExch(tq + n_tile, 0u);
      atomicExch(tq + n_tiles + n_tile, 0u);
    }
  } else {
    tile_stats_flush<BN, HTHREADS>(tile, tid, ts, s1, s2, s3, amx);
  }
}

// =========================================================================== fp32 Winograd F(2,3)
// fp32 forward / data gradient of the multi-chunk layers as a 1-D Winograd F(2,3) along x: for each
// kernel row dy, a pair of outputs (x, x+1) is
//   y(x)   = M0 + M1 + M2,   y(x+1) = M1 - M2 - M3,   M_xi = sum_c U_xi[dy][c] * V_xi[c]
// with V0 = d0 - d2, V1 = d1 + d2, V2 = d2 - d1, V3 = d1 - d3 (d_j = input at x - 1 + j, row y + dy)
// and U0 = g0, U1 = (g0 + g1 + g2) / 2, U2 = (g0 - g1 + g2) / 2, U3 = g2 (the kernel row's taps,
// transformed once per step by selunet_pack_weights). Per output pixel that is 3 x 4 / 2 = 6 fp32
// MFMA k-passes over the input channels instead of 9: the exact-fp32 MFMA work drops by 1.5x; the
// transforms are one fp32 add per operand element (rounding comparable to the direct sum: measured
// relative RMS 3.1e-7 vs 1.8e-7 direct at C = 512, fp64 reference).
// Structure as conv3x3_halo_persist_kernel (persistent column-tile walk, halo prefetch across the
// epilogue, statistics in registers) with 12 steps (dy, xi) per 32-channel chunk. The halo tile's
// columns are stored deinterleaved by parity (even x first), so the d_j reads of a wave's 32 output
// pairs (8 pairs x 4 rows) are 4 runs of 8 consecutive LDS rows, as the direct kernel's reads.
// Waves: 4 (pair rows) x 2 (column halves of BN); accumulators acc[xi][BN/64] per wave.
constexpr int WINO_STEPS = 12;
__device__ __forceinline__ int wino_row(int hp) {
  const int hy = hp / HWT, hx = hp - hy * HWT;
  return hy * HWT + (hx & 1) * (HWT / 2) + (hx >> 1);
}

// XS = transformed planes (xi) per step: 1 (BN = 128: 12 steps per chunk) or 2 (BN = 64: 6 steps,
// so a step carries as many MFMAs per barrier as the BN = 128 one; two planes of weights per buffer)
template <int BN, int XS>
__global__ void __launch_bounds__(HTHREADS, 1)
conv3x3_wino_persist_kernel(GatherArg g, const float* __restrict__ B, int N, int k_pad, EpiArg ep, int n_tiles,
                            int tiles_x, int tiles_y, int ptiles, int gp) {
  using T = float;
  constexpr int E = 4;
  constexpr int CK = 32;
  constexpr int NT = BN / 64;  // 32-column subtiles per wave
  constexpr int STEPS = WINO_STEPS / XS;
  constexpr int BROWS = XS * BN;  // weight rows per step (plane-major)
  constexpr int B_ROUNDS = BROWS * 8 / HTHREADS;
  static_assert(XS == 1 || XS == 2, "one or two planes per step");
  // halo slice r of the next job: loaded at step lt(r), written to LDS at lt(r) + 3
  auto lt = [](int r) { return XS == 1 ? r : r >> 1; };
  static_assert(B_ROUNDS * HTHREADS == BROWS * 8, "weight tile rows must split evenly over the threads");
  static_assert(A_ROUNDS <= 6, "halo slice schedule covers six slices");

  constexpr int SMEM_MAIN = 2 * HPIX * AROWB + 2 * BROWS * ROWB + 2 * CK * 8;
  constexpr int SMEM_EPI = TH * TW * (BN + 4) * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI];
  unsigned char* As = smem;
  unsigned char* Bs = smem + 2 * HPIX * AROWB;
  float* Ss = reinterpret_cast<float*>(Bs + 2 * BROWS * ROWB);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int half = lane >> 5, l32 = lane & 31;
  // this lane's output pair: tile row py, pixels 2 px2 and 2 px2 + 1
  const int pair = wm * 32 + l32, py = pair >> 3, px2 = pair & 7;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int n_tile = lb % n_tiles;
  const int prow = lb / n_tiles;
  const int n0 = n_tile * BN;
  const int ntl = prow < ptiles ? (ptiles - prow + gp - 1) / gp : 0;
  const int nchunks = g.Ctot / CK;
  const int csteps = nchunks * STEPS;

  auto tile_xy = [&](int i, int& img, int& y0, int& x0) __attribute__((always_inline)) {
    const unsigned pt = (unsigned)(prow + i * gp);
    const unsigned r = pt / (unsigned)tiles_x;
    x0 = (int)(pt - r * (unsigned)tiles_x) * TW;
    const unsigned r2 = r / (unsigned)tiles_y;
    y0 = (int)(r - r2 * (unsigned)tiles_y) * TH;
    img = (int)r2;
  };
  auto a_slot = [&](int round, int& hp, int& cc) -> bool {
    const int hidx = round * HTHREADS + tid;
    hp = min(hidx >> 3, HPIX - 1);
    cc = hidx & 7;
    return hidx < HPIX * 8;
  };
  auto a_inside = [&](int y0, int x0, int hp) -> bool {
    const int hy = hp / HWT, hx = hp - (hp / HWT) * HWT;
    return (unsigned)(y0 - 1 + hy) < (unsigned)g.h && (unsigned)(x0 - 1 + hx) < (unsigned)g.w;
  };
  auto chunk_src = [&](int chunk, int& c) -> SrcArg {
    c = chunk * CK;
    const bool s1 = g.nsrc > 1 && c >= g.src[0].C;
    if (s1) c -= g.src[0].C;
    return pick_src(g, s1 ? 1 : 0);
  };
  auto a_ptr = [&](const SrcArg& sa, int c, int img, int y0, int x0, int hp, int cc) -> const uint4* {
    const int hy = hp / HWT, hx = hp - (hp / HWT) * HWT;
    const int ys = min(max(y0 - 1 + hy, 0), g.h - 1), xs = min(max(x0 - 1 + hx, 0), g.w - 1);
    return reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(sa.data) +
                                          (((int64_t)img * g.h + ys) * g.w + xs) * sa.C + c + cc * E);
  };
  struct BRegs {
    uint4 v[B_ROUNDS];
  };
  auto b_load = [&](int st) __attribute__((always_inline)) {  // st: step within a tile
    const int chunk = st / STEPS, t = st - chunk * STEPS;
    BRegs rb;
#pragma unroll
    for (int r = 0; r < B_ROUNDS; ++r) {
      const int idx = r * HTHREADS + tid;
      const int row = idx >> 3, cc = idx & 7;
      const int pl = row / BN, co = row - pl * BN;  // plane t*XS + pl, output column co
      const int k0 = (t * XS + pl) * g.Ctot + chunk * CK;
      rb.v[r] = *reinterpret_cast<const uint4*>(B + (int64_t)(n0 + co) * k_pad + k0 + cc * E);
    }
    return rb;
  };
  auto b_store = [&](const BRegs& rb, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < B_ROUNDS; ++r) {
      const int idx = r * HTHREADS + tid;
      const int row = idx >> 3, cc = idx & 7;
      *reinterpret_cast<uint4*>(Bs + (buf * BROWS + row) * ROWB + cc * 16) = rb.v[r];
    }
  };

  f32x16 acc[4][NT];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[x][b] = f32x16{};
  const int prow0 = py * HWT + px2;  // LDS row of d_0 at dy = 0

  // step t = (dy, xi) (XS = 1) or (dy, xi pair) (XS = 2): V_xi from d_j rows of the halo, one MFMA
  // pass per plane and column subtile
  auto mma_step = [&](int hbuf, int bbuf, int t) __attribute__((always_inline)) {
    const unsigned char* a_src = As + hbuf * HPIX * AROWB;
    const unsigned char* b_src = Bs + bbuf * BROWS * ROWB;
    const int dy = (t * XS) >> 2, x0i = (t * XS) & 3;
    const int sw = ((half ^ (py + dy)) & 1) * 16;
    auto drow = [&](int j) { return a_src + (prow0 + dy * HWT + (j & 1) * (HWT / 2) + (j >> 1)) * AROWB + sw; };
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint4 bfr[XS][NT];
#pragma unroll
      for (int p = 0; p < XS; ++p)
#pragma unroll
        for (int b = 0; b < NT; ++b)
          bfr[p][b] = *reinterpret_cast<const uint4*>(b_src + (p * BN + wn * (BN / 2) + b * 32 + l32) * ROWB + q * 32 +
                                                      half * 16);
      float4 v[XS];
      if (XS == 1) {
        const int xi = x0i;
        const int ja = xi == 0 ? 0 : (xi == 2 ? 2 : 1);
        const int jb = xi == 3 ? 3 : (xi == 2 ? 1 : 2);
        const float4 da = *reinterpret_cast<const float4*>(drow(ja) + q * 32);
        const float4 db = *reinterpret_cast<const float4*>(drow(jb) + q * 32);
        v[0] = xi == 1 ? make_float4(da.x + db.x, da.y + db.y, da.z + db.z, da.w + db.w)
                       : make_float4(da.x - db.x, da.y - db.y, da.z - db.z, da.w - db.w);
      } else {
        // xi 0,1: d0 - d2, d1 + d2;  xi 2,3: d2 - d1, d1 - d3
        const int j0 = x0i == 0 ? 0 : 1;
        const float4 e0 = *reinterpret_cast<const float4*>(drow(j0) + q * 32);
        const float4 e1 = *reinterpret_cast<const float4*>(drow(j0 + 1) + q * 32);
        const float4 e2 = *reinterpret_cast<const float4*>(drow(j0 + 2) + q * 32);
        if (x0i == 0) {
          v[0] = make_float4(e0.x - e2.x, e0.y - e2.y, e0.z - e2.z, e0.w - e2.w);
          v[XS - 1] = make_float4(e1.x + e2.x, e1.y + e2.y, e1.z + e2.z, e1.w + e2.w);
        } else {
          v[0] = make_float4(e1.x - e0.x, e1.y - e0.y, e1.z - e0.z, e1.w - e0.w);
          v[XS - 1] = make_float4(e0.x - e2.x, e0.y - e2.y, e0.z - e2.z, e0.w - e2.w);
        }
      }
#pragma unroll
      for (int p = 0; p < XS; ++p) {
        const uint4 av = make_uint4(__float_as_uint(v[p].x), __float_as_uint(v[p].y), __float_as_uint(v[p].z),
                                    __float_as_uint(v[p].w));
#pragma unroll
        for (int b = 0; b < NT; ++b) Mma<float>::run(acc[x0i + p][b], av, bfr[p][b]);
      }
    }
  };
  auto halo_put_global = [&](uint4 v, int r, const SrcArg& sa, int c, int y0, int x0, int hb)
      __attribute__((always_inline)) {
    int hp, cc;
    if (!a_slot(r, hp, cc)) return;
    uint4 o = make_uint4(0, 0, 0, 0);
    if (a_inside(y0, x0, hp)) o = sa.scale ? transform16<T>(v, sa.scale, sa.shift, c + cc * E, sa.relu) : v;
    *reinterpret_cast<uint4*>(As + hb * HPIX * AROWB + halo_off(wino_row(hp), cc)) = o;
  };

  // ---------------------------------------------------------------- prologue: tile 0 chunk 0, B(0), B(1)
  {
    int img, y0, x0;
    tile_xy(0, img, y0, x0);
    int c0;
    const SrcArg sa = chunk_src(0, c0);
    uint4 v0[A_ROUNDS];
#pragma unroll
    for (int r = 0; r < A_ROUNDS; ++r) {
      int hp, cc;
      a_slot(r, hp, cc);
      v0[r] = *a_ptr(sa, c0, img, y0, x0, hp, cc);
    }
#pragma unroll
    for (int r = 0; r < A_ROUNDS; ++r) halo_put_global(v0[r], r, sa, c0, y0, x0, 0);
  }
  BRegs rb_next = b_load(0);
  b_store(rb_next, 0);
  rb_next = b_load(1 % csteps);
  __syncthreads();

  // Statistics registers: fp64 as in the direct kernel at BN = 64; at BN = 128 the 48 registers of fp64
  // sums (8 columns x 3 sets) push the kernel past 256 VGPRs (39 spills: +240 MB of scratch writes per
  // launch, PMC) — there they are fp32 (4.5% faster, tools/ab_conv.sh). The per-tile partials are
  // fp32 either way; the fp32 sum over a workgroup's ~128 tiles adds ~sqrt(128) ulp to BN-backward
  // and bias sums that the fp64 slab reduction then combines; the forward's first-pass mean only
  // centres the second, exact pass (selunet_bn_centered_partials).
  using Acc = std::conditional_t<BN == 128, float, typename StatAcc<T>::type>;
  static_assert(stats_flush_bytes<BN, HTHREADS, Acc>() <= (int)sizeof(smem), "statistics scratch exceeds LDS");
  Acc s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float amx = 0.0f;  // running max |stored value| (epilogue range word)
  const TileStats ts = tile_stats(ep, prow, n0, N);
  float* tile = reinterpret_cast<float*>(smem);
  uint4 ra[A_ROUNDS];
  int J = 0;
  int S = 0;
  for (int i = 0; i < ntl; ++i) {
    int img, y0, x0;
    tile_xy(i, img, y0, x0);
    BRegs rb_hold;
    for (int c = 0; c < nchunks; ++c, ++J) {
      const bool last_c = c + 1 == nchunks;
      const bool has_next = !last_c || i + 1 < ntl;
      const bool defer = last_c && has_next;
      int nimg = img, ny0 = y0, nx0 = x0;
      if (defer) tile_xy(i + 1, nimg, ny0, nx0);
      const int nc = !has_next ? c : (last_c ? 0 : c + 1);
      int cs;
      const SrcArg sn = chunk_src(nc, cs);
      float* ssc = Ss + ((J + 1) & 1) * CK;
      float* ssh = Ss + 2 * CK + ((J + 1) & 1) * CK;
      float coef = 0.0f;
#pragma unroll
      for (int t = 0; t < STEPS; ++t) {
        const int st2 = c * STEPS + t + 2;
        const BRegs rb_far = b_load(st2 < csteps ? st2 : st2 - csteps);
        if (t == 0 && !defer && sn.scale && tid < 2 * CK) coef = tid < CK ? sn.scale[cs + tid] : sn.shift[cs + tid - CK];
#pragma unroll
        for (int r = 0; r < A_ROUNDS; ++r) {
          if (lt(r) == t) {
            int hp, cc;
            a_slot(r, hp, cc);
            ra[r] = *a_ptr(sn, cs, nimg, ny0, nx0, hp, cc);
          }
        }
        mma_step(J & 1, S & 1, t);
        if (defer && t == STEPS - 1) rb_hold = rb_next;
        else b_store(rb_next, (S + 1) & 1);
        if (!defer) {
          if (t == 1 && sn.scale && tid < 2 * CK) (tid < CK ? ssc[tid] : ssh[tid - CK]) = coef;
#pragma unroll
          for (int r = 0; r < A_ROUNDS; ++r) {
            if (lt(r) + 3 != t) continue;
            int hp, cc;
            if (a_slot(r, hp, cc)) {
              uint4 v = make_uint4(0, 0, 0, 0);
              if (a_inside(ny0, nx0, hp)) {
                v = ra[r];
                if (sn.scale) {
                  float e[E];
                  __builtin_memcpy(e, &v, 16);
#pragma unroll
                  for (int j = 0; j < E; ++j) {
                    float f = e[j] * ssc[cc * E + j] + ssh[cc * E + j];
                    if (sn.relu) f = fmaxf(f, 0.0f);
                    e[j] = f;
                  }
                  __builtin_memcpy(&v, e, 16);
                }
              }
              *reinterpret_cast<uint4*>(As + ((J + 1) & 1) * HPIX * AROWB + halo_off(wino_row(hp), cc)) = v;
            }
          }
        }
        __syncthreads();
        rb_next = rb_far;
        ++S;
      }
    }

    // ------------------------------------------------------------ epilogue of tile i
    // output transform in registers (the lane holds all four M_xi of its pairs), pixels -> LDS
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int col = wn * (BN / 2) + b * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        const int e = (pr >> 3) * TW + 2 * (pr & 7);
        const float m0 = acc[0][b][r], m1 = acc[1][b][r], m2 = acc[2][b][r], m3 = acc[3][b][r];
        tile[e * (BN + 4) + col] = (m0 + m1) + m2;
        tile[(e + 1) * (BN + 4) + col] = (m1 - m2) - m3;
      }
    }
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[x][b] = f32x16{};
    __syncthreads();
    auto dst = [&](int pix, int cl) -> T* {
      const int y = y0 + pix / TW, x = x0 + pix % TW;
      if (y >= g.h || x >= g.w) return nullptr;
      const int64_t m = ((int64_t)img * g.h + y) * g.w + x;
      const int col = n0 + cl;
      if (ep.mode == SELUNET_EP_SPLIT)
        return col < ep.split ? reinterpret_cast<T*>(ep.out0) + m * ep.split + col
                              : reinterpret_cast<T*>(ep.out1) + m * (N - ep.split) + (col - ep.split);
      return reinterpret_cast<T*>(ep.out0) + m * N + col;
    };
    auto bias_col = [&](int cl) { return n0 + cl; };
    lds_tile_store_acc<T, TH * TW, BN, HTHREADS>(tile, tid, dst, ep.bias, bias_col, ts, s1, s2, s3, amx);
    if (i + 1 < ntl) {
      __syncthreads();
      int nimg, ny0, nx0;
      tile_xy(i + 1, nimg, ny0, nx0);
      int cs;
      const SrcArg sn = chunk_src(0, cs);
#pragma unroll
      for (int r = 0; r < A_ROUNDS; ++r) halo_put_global(ra[r], r, sn, cs, ny0, nx0, J & 1);
      b_store(rb_hold, S & 1);
      __syncthreads();
    }
  }
  tile_stats_flush<BN, HTHREADS>(tile, tid, ts, s1, s2, s3, amx);
}

// =========================================================================== weight gradient
// dW[co][tap][ci] = sum_p dY[p][co] * X[p + off(tap)][ci] for one co tile (BI) and one 64-channel
// ci chunk, reduced over the pixel tiles (8 x 16) of a split; fp32 atomics at the end.
// Each pixel tile stages dY [128 px][BI] and the input halo [10 x 18 px][64 ch] in LDS in their
// natural layouts; the MFMA k dimension is the pixel, so both operands are read with
// ds_read_b64_tr_b16 (4 pixels x 16 channels per 16-lane group). One dY fragment feeds the MFMAs
// of every tap the wave owns. 8 waves: (BI/32 co subtiles) x (2 ci subtiles) x (taps split in two
// groups when BI = 64). Rows are padded to a stride of 16 dwords mod 64 so the transposed reads
// of 4 consecutive rows hit distinct banks.
constexpr int WTH = 8, WTW = 16;                 // pixel tile
constexpr int WHH = WTH + 2, WHW = WTW + 2;      // halo
constexpr int WHP = WHH * WHW;                   // 180 halo pixels
constexpr int WPIXT = WTH * WTW;                 // 128 pixels

template <int BI>
__global__ void __launch_bounds__(512, 2)
conv3x3_wgrad_halo_kernel(GatherArg P, GatherArg Q, float* __restrict__ out, int ldo, int co_tiles, int ci_chunks,
                          int64_t tiles_per_split, int tiles_x, int tiles_y, int64_t total_tiles,
                          float* __restrict__ ws, int64_t ws_stride) {
  constexpr int LDP = BI + 32;                   // dY tile row stride (elements)
  constexpr int LDX = 64 + 32;                   // halo row stride (elements)
  constexpr int TG = BI == 64 ? 2 : 1;           // tap groups
  constexpr int NTAP = TG == 1 ? 9 : 5;          // accumulators per wave
  constexpr int P_ROUNDS = (WPIXT * BI / 8) / 512;
  constexpr int X_ROUNDS = (WHP * 8 + 511) / 512;

  __shared__ __attribute__((aligned(16))) unsigned short Ps[2][WPIXT][LDP];
  __shared__ __attribute__((aligned(16))) unsigned short Xs[2][WHP][LDX];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wj = wave & 1;                       // ci subtile
  const int wi = (wave >> 1) % (BI / 32);        // co subtile
  const int tg = (wave >> 1) / (BI / 32);        // tap group
  const int tap0 = tg * 5;
  const int ntap = TG == 1 ? 9 : (tg == 0 ? 5 : 4);
  const int half = lane >> 5, l32 = lane & 31;
  const int grp_hi = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int cot = lb % co_tiles;
  const int rest = lb / co_tiles;
  const int cik = rest % ci_chunks;
  const int64_t split = rest / ci_chunks;
  const int i0 = cot * BI;
  const int c0 = cik * 64;
  const int64_t pt_begin = split * tiles_per_split;
  const int64_t pt_end = min(total_tiles, pt_begin + tiles_per_split);
  if (pt_begin >= pt_end) return;

  // source of this ci chunk
  int xs_src = 0, xc = c0;
  if (Q.nsrc > 1 && xc >= Q.src[0].C) {
    xc -= Q.src[0].C;
    xs_src = 1;
  }
  const SrcArg xa = pick_src(Q, xs_src);
  const SrcArg& pa = P.src[0];
  const int H = P.h, W = P.w;

  // folded BN coefficients of the block's dY and X channels, staged once in LDS and applied when a
  // tile is written to LDS (the raw loads stay in flight across the previous tile's MFMAs)
  __shared__ float Ks[2 * BI + 2 * 64];
  if (tid < 2 * BI + 128) {
    float v;
    if (tid < 2 * BI) {
      const int c = i0 + (tid % BI);
      v = pa.scale ? (tid < BI ? pa.scale[c] : pa.shift[c]) : 0.0f;
    } else {
      const int c = xc + ((tid - 2 * BI) % 64);
      v = xa.scale ? (tid < 2 * BI + 64 ? xa.scale[c] : xa.shift[c]) : 0.0f;
    }
    Ks[tid] = v;
  }

  auto tile_origin = [&](int pt, int& img, int& y0, int& x0) __attribute__((always_inline)) {
    const unsigned r2 = (unsigned)pt / (unsigned)tiles_x;
    x0 = ((unsigned)pt - r2 * (unsigned)tiles_x) * WTW;
    const unsigned r3 = r2 / (unsigned)tiles_y;
    y0 = (r2 - r3 * (unsigned)tiles_y) * WTH;
    img = (int)r3;
  };
  auto apply = [&](uint4 v, const float* sc, const float* sh, int relu) __attribute__((always_inline)) {
    __bf16 e[8];
    __builtin_memcpy(e, &v, 16);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = (float)e[j] * sc[j] + sh[j];
      if (relu) f = fmaxf(f, 0.0f);
      e[j] = (__bf16)f;
    }
    __builtin_memcpy(&v, e, 16);
    return v;
  };
  // unconditional loads (pixels clamped into the image; zeroed when written), so the compiler can
  // count the outstanding loads instead of waiting for each one
  uint4 rp[P_ROUNDS], rx[X_ROUNDS];
  auto load_tile = [&](int pt) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < P_ROUNDS; ++r) {
      const int idx = r * 512 + tid;
      const int px = idx / (BI / 8), cc = idx % (BI / 8);
      const int y = min(y0 + px / WTW, H - 1), x = min(x0 + px % WTW, W - 1);
      rp[r] = *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(pa.data) +
                                             (((int64_t)img * H + y) * W + x) * pa.C + i0 + cc * 8);
    }
#pragma unroll
    for (int r = 0; r < X_ROUNDS; ++r) {
      const int idx = r * 512 + tid;
      const int hp = min(idx >> 3, WHP - 1), cc = idx & 7;
      const int y = min(max(y0 - 1 + hp / WHW, 0), H - 1), x = min(max(x0 - 1 + hp % WHW, 0), W - 1);
      rx[r] = *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(xa.data) +
                                             (((int64_t)img * H + y) * W + x) * xa.C + xc + cc * 8);
    }
  };
  auto store_tile = [&](int pt, int buf) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < P_ROUNDS; ++r) {
      const int idx = r * 512 + tid;
      const int px = idx / (BI / 8), cc = idx % (BI / 8);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (y0 + px / WTW < H && x0 + px % WTW < W)
        v = pa.scale ? apply(rp[r], Ks + cc * 8, Ks + BI + cc * 8, pa.relu) : rp[r];
      *reinterpret_cast<uint4*>(&Ps[buf][px][cc * 8]) = v;
    }
#pragma unroll
    for (int r = 0; r < X_ROUNDS; ++r) {
      const int idx = r * 512 + tid;
      if (idx < WHP * 8) {
        const int hp = idx >> 3, cc = idx & 7;
        const int y = y0 - 1 + hp / WHW, x = x0 - 1 + hp % WHW;
        uint4 v = make_uint4(0, 0, 0, 0);
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
          v = xa.scale ? apply(rx[r], Ks + 2 * BI + cc * 8, Ks + 2 * BI + 64 + cc * 8, xa.relu) : rx[r];
        *reinterpret_cast<uint4*>(&Xs[buf][hp][cc * 8]) = v;
      }
    }
  };

  f32x16 acc[NTAP];
#pragma unroll
  for (int t = 0; t < NTAP; ++t) acc[t] = f32x16{};

  load_tile((int)pt_begin);
  __syncthreads();  // coefficients visible
  store_tile((int)pt_begin, 0);
  __syncthreads();
  // the tap count is a template constant of the tile loop: a per-k-step branch on the wave's (runtime)
  // tap group would split the scheduled MFMA/read groups into blocks joined by LDS-counter drains
  auto tile_loop = [&](auto ntc) __attribute__((always_inline)) {
    constexpr int NTP = decltype(ntc)::value;
    int buf = 0;
    for (int pt = (int)pt_begin; pt < (int)pt_end; ++pt) {
      const bool more = pt + 1 < (int)pt_end;
      load_tile(more ? pt + 1 : pt);
      __builtin_amdgcn_sched_barrier(0);  // keep the next tile's loads ahead of this tile's MFMAs
  #pragma unroll
      for (int ks = 0; ks < WTH; ++ks) {   // one tile row (16 pixels) per k-step
        const int prow = ks * WTW + 8 * half + q4;
        const int pcol = wi * 32 + 16 * grp_hi + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)&Ps[buf][prow][pcol]);
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)&Ps[buf][prow + 4][pcol]);
        const bf16x8 af = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        const int xcol = wj * 32 + 16 * grp_hi + 4 * p4;
        // tap fragments are read PF taps ahead of their MFMA (a rolling window of PF+1 fragments:
        // hoisting all nine would spill), pinned in that order with sched_group_barrier so the LDS
        // latency hides behind the MFMAs already issued instead of being waited out per MFMA
        constexpr int PF = 3;
        auto read_tap = [&](int t) __attribute__((always_inline)) {
          const int tap = min(tap0 + t, 8);
          const int dy = tap / 3, dx = tap - (tap / 3) * 3;
          const int xrow = (ks + dy) * WHW + 8 * half + dx + q4;
          s16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)&Xs[buf][xrow][xcol]);
          s16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)&Xs[buf][xrow + 4][xcol]);
          return __builtin_bit_cast(bf16x8, __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7));
        };
        bf16x8 bfr[NTAP];
  #pragma unroll
        for (int t = 0; t < PF && t < NTAP; ++t) bfr[t] = read_tap(t);
        __builtin_amdgcn_sched_group_barrier(0x100, 2 + 2 * PF, 0);
  #pragma unroll
        for (int t = 0; t < NTAP; ++t) {
          if (t < NTP) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr[t], acc[t], 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (t + PF < NTAP) {
            bfr[t + PF] = read_tap(t + PF);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          }
        }
      }
      if (more) store_tile(pt + 1, buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  };
  if (TG == 1) tile_loop(std::integral_constant<int, 9>{});
  else if (tg == 0) tile_loop(std::integral_constant<int, 5>{});
  else tile_loop(std::integral_constant<int, 4>{});

  const int ctot = Q.Ctot;
#pragma unroll
  for (int t = 0; t < NTAP; ++t) {
    if (t < ntap) {
      const int tap = tap0 + t;
      const int j = tap * ctot + c0 + wj * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + wi * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (ws) ws[split * ws_stride + (int64_t)i * ldo + j] = acc[t][r];  // this split's partial
        else atomicAdd(out + (int64_t)i * ldo + j, acc[t][r]);
      }
    }
  }
}

// =========================================================================== split-fp16 weight gradient
// fp32 3x3 weight gradient on split-fp16 operands (selunet_conv3x3_wgrad_x2): the bf16 halo kernel's
// structure (MFMA k = pixel, both operands read with ds_read_b64_tr_b16 from their natural
// [pixel][channel] tiles, one dY fragment feeding every tap of the wave) with each operand staged as
// two fp16 planes, h = fp16(v * 2^e) and l = fp16(v * 2^e - h), and three v_mfma_f32_32x32x16_f16
// per tap and k-step (hl, lh, hh). 8 x 8-pixel tiles (10 x 10 halo) so that both planes of both
// operands double-buffer in LDS (BI = 128: 155 KB). The partials are unscaled by 2^-(e_dy + e_x)
// (one source per 64-channel chunk, so one scale per workgroup) and reduced like the halo kernels'.
constexpr int XTH = 8, XTW = 8, XHW = XTW + 2, XHP = (XTH + 2) * XHW, XPIX = XTH * XTW;

// The BN-backward apply fused into the weight gradient's dY staging (selunet_conv3x3_wgrad_x2_bn): P gathers
// the layer's dA; y, the forward's folded scale / shift (ReLU mask), mean / invstd and the coefficients coef
// [3][C] of selunet_bn_bwd_stats_finalize form dy = (y sc + sh > 0 ? k0 dA : 0) - k1 - k2 invstd (y - mean)
// exactly as bn_bwd_apply_kernel; dy is written once per element (pixel px of a tile by the workgroup of
// channel chunk px % ci_chunks) with its exact max |dy| (atomic max) for the layer's data gradient
// (WgradBnArg, gemm_common.h). BNA: 0 no apply; 1 dA from P; 2 dA = route(pooled) + skip of a max-pooled
// layer (bn_bwd_apply_pool_kernel's dA: the first maximum of relu(y sc + sh) in row-major window order);
// 3 dA = sum_h w_h g_h of the 1x1 heads (bn_bwd_apply_heads_kernel's). Modes 2 and 3 are BI = 64 only.
// TQ (SELUNET_OPT_TILE_QUEUE bit 1): the `splits` workgroups of a (co tile, ci chunk) group take their
// pixel tiles from the group's ticket counter instead of a fixed run, so a launch whose workgroups cannot all
// start at once (CUs held by a concurrent RCCL all-reduce) rebalances instead of ending with the late workgroups'
// whole run. Two tickets are claimed at the start (the next tile's loads are issued before a tile's MFMAs) and one
// more per tile at its first k-step. A workgroup's partial then sums the tiles it happened to take: the weight
// gradient is the same sum in another order (not bit-reproducible run to run); dy and max |dy| are unchanged.
// tq: [2][groups] counters (tickets, finished workgroups), zero between launches (the group's last workgroup
// resets both).
template <int BI, int BNA = 0, bool TQ = false>
__global__ void __launch_bounds__(512, 1)
conv3x3_wgrad_x2_kernel(GatherArg P, GatherArg Q, int ldo, int co_tiles, int ci_chunks, int64_t tiles_per_split,
                        int tiles_x, int tiles_y, int64_t total_tiles, float* __restrict__ ws, int64_t ws_stride,
                        const float* __restrict__ amax_p, const float* __restrict__ amax_q0,
                        const float* __restrict__ amax_q1, WgradBnArg bn, unsigned* __restrict__ tq = nullptr) {
  constexpr int LDP = BI + 32;                   // dY plane row stride (halves): 16 dwords mod 64
  constexpr int LDX = 64 + 32;                   // halo plane row stride (halves)
  constexpr int TG = BI == 64 ? 2 : 1;           // tap groups
  constexpr int NTAP = TG == 1 ? 9 : 5;          // accumulators per wave
  constexpr int P_ROUNDS = (XPIX * BI / 4) / 512;
  constexpr int X_ROUNDS = (XHP * 16 + 511) / 512;
  constexpr bool POOL = BNA == 2, HEADS = BNA == 3;
  // coefficient area: dY side (sc, sh[, k0, a, b[, w0, w1, w2]]), then the halo's
  constexpr int KX = BNA ? (HEADS ? 8 : 5) * BI : 2 * BI;
  constexpr int NWIN = XPIX * BI / 16;            // POOL: 2x2 windows x 4 channels of a dY tile, one per thread
  static_assert(P_ROUNDS * 512 == XPIX * BI / 4, "dY tile must split evenly over the threads");
  static_assert(!(POOL || HEADS) || (BI == 64 && NWIN <= 512), "pool / heads sources are BI = 64 forms");

  __shared__ __attribute__((aligned(16))) _Float16 Ps[2][2][XPIX][LDP];  // [buffer][h, l][pixel][co]
  __shared__ __attribute__((aligned(16))) _Float16 Xs[2][2][XHP][LDX];   // [buffer][h, l][halo pixel][ci]
  __shared__ __attribute__((aligned(16))) float Ks[KX + 2 * 64];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wj = wave & 1;                       // ci subtile
  const int wi = (wave >> 1) % (BI / 32);        // co subtile
  const int tg = (wave >> 1) / (BI / 32);        // tap group
  const int tap0 = tg * 5;
  const int ntap = TG == 1 ? 9 : (tg == 0 ? 5 : 4);
  const int half = lane >> 5, l32 = lane & 31;
  const int grp_hi = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int cot = lb % co_tiles;
  const int rest = lb / co_tiles;
  const int cik = rest % ci_chunks;
  const int64_t split = rest / ci_chunks;
  const int i0 = cot * BI;
  const int c0 = cik * 64;
  const int ngroups = co_tiles * ci_chunks, grp = (int)(lb % (unsigned)ngroups);
  // tiles pt_first, pt_second, ... below pt_stop: static, the split's run; TQ, claimed tickets (>= total: none)
  __shared__ int tq_slot[2];
  int pt_first, pt_second, pt_stop;
  if constexpr (TQ) {
    if (tid == 0) {
      const unsigned t = atomicAdd(tq + grp, 2u);
      tq_slot[0] = (int)min(t, (unsigned)total_tiles);
      tq_slot[1] = (int)min(t + 1u, (unsigned)total_tiles);
    }
    __syncthreads();
    pt_first = tq_slot[0];
    pt_second = tq_slot[1];
    pt_stop = (int)total_tiles;
  } else {
    pt_first = (int)(split * tiles_per_split);
    pt_second = pt_first + 1;
    pt_stop = (int)min(total_tiles, (int64_t)pt_first + tiles_per_split);
  }

  int xs_src = 0, xc = c0;
  if (Q.nsrc > 1 && xc >= Q.src[0].C) {
    xc -= Q.src[0].C;
    xs_src = 1;
  }
  const SrcArg xa = pick_src(Q, xs_src);
  const SrcArg& pa = P.src[0];
  const int H = P.h, W = P.w;
  float uns_p, uns_x;
  const float sp = x2_scale(amax_p[0], &uns_p);
  const float sx = x2_scale((xs_src ? amax_q1 : amax_q0)[0], &uns_x);

  if constexpr (BNA) {
    for (int k = tid; k < KX; k += 512) {
      const int c = i0 + (k % BI), C = P.Ctot;
      float v;
      switch (k / BI) {
        case 0: v = bn.scale[c]; break;
        case 1: v = bn.shift[c]; break;
        case 2: v = bn.coef[c]; break;                                       // k0
        case 3: v = bn.coef[2 * C + c] * bn.invstd[c]; break;                // a = k2 invstd
        case 4: v = bn.coef[C + c] - bn.coef[2 * C + c] * bn.invstd[c] * bn.mean[c]; break;  // b = k1 - a mean
        default: {                                                            // HEADS: w_h[c]
          const int hd = k / BI - 5;
          v = hd < bn.nh ? bn.hw[hd * 64 + c] : 0.0f;
        }
      }
      Ks[k] = v;
    }
    if (tid < 128) {
      const int c = xc + (tid % 64);
      Ks[KX + tid] = xa.scale ? (tid < 64 ? xa.scale[c] : xa.shift[c]) : 0.0f;
    }
  } else if (tid < 2 * BI + 128) {
    float v;
    if (tid < 2 * BI) {
      const int c = i0 + (tid % BI);
      v = pa.scale ? (tid < BI ? pa.scale[c] : pa.shift[c]) : 0.0f;
    } else {
      const int c = xc + ((tid - 2 * BI) % 64);
      v = xa.scale ? (tid < 2 * BI + 64 ? xa.scale[c] : xa.shift[c]) : 0.0f;
    }
    Ks[tid] = v;
  }
  float dam = 0.0f;                               // BNA: running max |dy| of this workgroup's stores
  // BNA: every channel chunk's workgroup forms the whole dY tile; the dy stores are shared out by pixel
  // (pixel px of a tile is stored by chunk px % ci_chunks), so no chunk's workgroups carry all of them
  const bool dy_out = BNA && bn.dy != nullptr;

  auto tile_origin = [&](int pt, int& img, int& y0, int& x0) __attribute__((always_inline)) {
    const unsigned r2 = (unsigned)pt / (unsigned)tiles_x;
    x0 = ((unsigned)pt - r2 * (unsigned)tiles_x) * XTW;
    const unsigned r3 = r2 / (unsigned)tiles_y;
    y0 = (r2 - r3 * (unsigned)tiles_y) * XTH;
    img = (int)r3;
  };
  // 4 fp32 channels -> (BN+ReLU) -> scale -> h / l fp16 quads at plane rows hp / lp
  auto put = [&](float4 v, const float* sc, const float* sh, int relu, float s, _Float16* hp, _Float16* lp)
      __attribute__((always_inline)) {
    float f[4] = {v.x, v.y, v.z, v.w};
    f16x4 h, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float t = f[j];
      if (sc) {
        t = t * sc[j] + sh[j];
        if (relu) t = fmaxf(t, 0.0f);
      }
      _Float16 a, b;
      x2_split(t * s, a, b);
      h[j] = a;
      l[j] = b;
    }
    *reinterpret_cast<f16x4*>(hp) = h;
    *reinterpret_cast<f16x4*>(lp) = l;
  };
  float4 rp[P_ROUNDS], rx[X_ROUNDS];
  float4 ry[BNA ? P_ROUNDS : 1];                  // BNA: y at the dA elements
  float rg[HEADS ? P_ROUNDS : 1][3];              // HEADS: the heads' gradients at the pixel
  float4 wy[POOL ? 4 : 1], wk[POOL ? 4 : 1], wg;  // POOL: y and skip at a window's 4 pixels, the pooled gradient
  // rounds [r0, r1) of the dY tile (BNA at BI = 128 stages it in two halves: dA and y of half a tile live
  // at a time, as many registers as the plain kernel's whole dY tile)
  auto load_p = [&](int pt, int r0, int r1) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
    if constexpr (POOL) {  // window wi = tid / (BI / 4) of the tile, channels (tid % (BI / 4)) * 4
      if (r0 == 0 && tid < NWIN) {
        const int wi = tid / (BI / 4), cg = tid % (BI / 4);
        const int yy = min(y0 + 2 * (wi / (XTW / 2)), H - 2), xx = min(x0 + 2 * (wi % (XTW / 2)), W - 2);
        const int64_t b0 = (((int64_t)img * H + yy) * W + xx) * pa.C + i0 + cg * 4, rs = (int64_t)W * pa.C;
        const int64_t off[4] = {b0, b0 + pa.C, b0 + rs, b0 + rs + pa.C};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          wy[k] = *reinterpret_cast<const float4*>(bn.y + off[k]);
          wk[k] = bn.skip ? *reinterpret_cast<const float4*>(bn.skip + off[k]) : make_float4(0, 0, 0, 0);
        }
        wg = *reinterpret_cast<const float4*>(
            bn.pooled + (((int64_t)img * (H / 2) + yy / 2) * (W / 2) + xx / 2) * pa.C + i0 + cg * 4);
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < P_ROUNDS; ++r) {
      if (r < r0 || r >= r1) continue;
      const int idx = r * 512 + tid;
      const int px = idx / (BI / 4), cc = idx % (BI / 4);
      const int y = min(y0 + px / XTW, H - 1), x = min(x0 + px % XTW, W - 1);
      const int64_t pix = ((int64_t)img * H + y) * W + x;
      const int64_t off = pix * pa.C + i0 + cc * 4;
      if constexpr (HEADS) {
        rg[r][0] = bn.g0[pix];
        rg[r][1] = bn.nh > 1 ? bn.g1[pix] : 0.0f;
        rg[r][2] = bn.nh > 1 ? bn.g2[pix] : 0.0f;
      } else {
        rp[r] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(pa.data) + off);
      }
      if constexpr (BNA) ry[r] = *reinterpret_cast<const float4*>(bn.y + off);
    }
  };
  auto load_x = [&](int pt) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < X_ROUNDS; ++r) {
      const int idx = r * 512 + tid;
      const int hp = min(idx >> 4, XHP - 1), cc = idx & 15;
      const int y = min(max(y0 - 1 + hp / XHW, 0), H - 1), x = min(max(x0 - 1 + hp % XHW, 0), W - 1);
      rx[r] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(xa.data) +
                                               (((int64_t)img * H + y) * W + x) * xa.C + xc + cc * 4);
    }
  };
  auto store_p = [&](int pt, int buf, int r0, int r1) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
    if constexpr (POOL) {
      if (r0 == 0 && tid < NWIN) {
        const int wi = tid / (BI / 4), cg = tid % (BI / 4);
        const int wyy = 2 * (wi / (XTW / 2)), wxx = 2 * (wi % (XTW / 2));
        const bool in = y0 + wyy < H && x0 + wxx < W;  // (H, W even: a window is wholly in or out)
        const f32x4 csc = *reinterpret_cast<const f32x4*>(Ks + cg * 4);
        const f32x4 csh = *reinterpret_cast<const f32x4*>(Ks + BI + cg * 4);
        const f32x4 ck0 = *reinterpret_cast<const f32x4*>(Ks + 2 * BI + cg * 4);
        const f32x4 ca = *reinterpret_cast<const f32x4*>(Ks + 3 * BI + cg * 4);
        const f32x4 cb = *reinterpret_cast<const f32x4*>(Ks + 4 * BI + cg * 4);
        const float yv[4][4] = {{wy[0].x, wy[0].y, wy[0].z, wy[0].w}, {wy[1].x, wy[1].y, wy[1].z, wy[1].w},
                                {wy[2].x, wy[2].y, wy[2].z, wy[2].w}, {wy[3].x, wy[3].y, wy[3].z, wy[3].w}};
        const float gv[4] = {wg.x, wg.y, wg.z, wg.w};
        int arg[4] = {0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float best = fmaxf(yv[0][e] * csc[e] + csh[e], 0.0f);
#pragma unroll
          for (int k = 1; k < 4; ++k) {
            const float v = fmaxf(yv[k][e] * csc[e] + csh[e], 0.0f);
            if (v > best) {  // first maximum in row-major window order (strict >), as bn_bwd_apply_pool_kernel
              best = v;
              arg[e] = k;
            }
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float d[4] = {wk[k].x, wk[k].y, wk[k].z, wk[k].w};
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (arg[e] == k) d[e] += gv[e];
            o[e] = (yv[k][e] * csc[e] + csh[e] > 0.0f ? ck0[e] * d[e] : 0.0f) - cb[e] - ca[e] * yv[k][e];
          }
          const int py = wyy + (k >> 1), pxx = wxx + (k & 1), px = py * XTW + pxx;
          const float4 dv = in ? make_float4(o[0], o[1], o[2], o[3]) : make_float4(0, 0, 0, 0);
          if (dy_out && in && px % ci_chunks == cik) {
            const int64_t off = (((int64_t)img * H + y0 + py) * W + x0 + pxx) * pa.C + i0 + cg * 4;
            *reinterpret_cast<float4*>(bn.dy + off) = dv;
            dam = fmaxf(dam, fmaxf(fmaxf(fabsf(dv.x), fabsf(dv.y)), fmaxf(fabsf(dv.z), fabsf(dv.w))));
          }
          put(dv, nullptr, nullptr, 0, sp, &Ps[buf][0][px][cg * 4], &Ps[buf][1][px][cg * 4]);
        }
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < P_ROUNDS; ++r) {
      if (r < r0 || r >= r1) continue;
      const int idx = r * 512 + tid;
      const int px = idx / (BI / 4), cc = idx % (BI / 4);
      const bool in = y0 + px / XTW < H && x0 + px % XTW < W;
      if constexpr (BNA) {
        // dy of 4 channels (bn_bwd_apply_kernel's arithmetic)
        float g[4] = {rp[r].x, rp[r].y, rp[r].z, rp[r].w};
        const float yv[4] = {ry[r].x, ry[r].y, ry[r].z, ry[r].w};
        if constexpr (HEADS) {  // dA = w0 g0 + w1 g1 + w2 g2 (bn_bwd_apply_heads_kernel's form)
          const f32x4 w0 = *reinterpret_cast<const f32x4*>(Ks + 5 * BI + cc * 4);
          const f32x4 w1 = *reinterpret_cast<const f32x4*>(Ks + 6 * BI + cc * 4);
          const f32x4 w2 = *reinterpret_cast<const f32x4*>(Ks + 7 * BI + cc * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) g[e] = w0[e] * rg[r][0] + w1[e] * rg[r][1] + w2[e] * rg[r][2];
        }
        // the 4 channels' coefficients: one 16-B LDS read per coefficient row
        const f32x4 csc = *reinterpret_cast<const f32x4*>(Ks + cc * 4);
        const f32x4 csh = *reinterpret_cast<const f32x4*>(Ks + BI + cc * 4);
        const f32x4 ck0 = *reinterpret_cast<const f32x4*>(Ks + 2 * BI + cc * 4);
        const f32x4 ca = *reinterpret_cast<const f32x4*>(Ks + 3 * BI + cc * 4);
        const f32x4 cb = *reinterpret_cast<const f32x4*>(Ks + 4 * BI + cc * 4);
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[e] = (yv[e] * csc[e] + csh[e] > 0.0f ? ck0[e] * g[e] : 0.0f) - cb[e] - ca[e] * yv[e];
        const float4 d = in ? make_float4(o[0], o[1], o[2], o[3]) : make_float4(0, 0, 0, 0);
        if (dy_out && in && px % ci_chunks == cik) {
          const int64_t off = (((int64_t)img * H + y0 + px / XTW) * W + x0 + px % XTW) * pa.C + i0 + cc * 4;
          *reinterpret_cast<float4*>(bn.dy + off) = d;
          dam = fmaxf(dam, fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), fabsf(d.w))));
        }
        put(d, nullptr, nullptr, 0, sp, &Ps[buf][0][px][cc * 4], &Ps[buf][1][px][cc * 4]);
      } else {
        put(in ? rp[r] : make_float4(0, 0, 0, 0), pa.scale && in ? Ks + cc * 4 : nullptr, Ks + BI + cc * 4, pa.relu,
            sp, &Ps[buf][0][px][cc * 4], &Ps[buf][1][px][cc * 4]);
      }
    }
  };
  auto store_x = [&](int pt, int buf) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < X_ROUNDS; ++r) {
      const int idx = r * 512 + tid;
      if (idx < XHP * 16) {
        const int hp = idx >> 4, cc = idx & 15;
        const int y = y0 - 1 + hp / XHW, x = x0 - 1 + hp % XHW;
        const bool in = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        put(in ? rx[r] : make_float4(0, 0, 0, 0), xa.scale && in ? Ks + KX + cc * 4 : nullptr,
            Ks + KX + 64 + cc * 4, xa.relu, sx, &Xs[buf][0][hp][cc * 4], &Xs[buf][1][hp][cc * 4]);
      }
    }
  };

  f32x16 acc[NTAP];
#pragma unroll
  for (int t = 0; t < NTAP; ++t) acc[t] = f32x16{};

  if (pt_first < pt_stop) {
    load_p(pt_first, 0, P_ROUNDS);
    load_x(pt_first);
    __syncthreads();  // coefficients visible
    store_p(pt_first, 0, 0, P_ROUNDS);
    store_x(pt_first, 0);
    __syncthreads();
  }
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  auto tr8 = [&](const _Float16* p0, const _Float16* p1) __attribute__((always_inline)) {
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto tile_loop = [&](auto ntc) __attribute__((always_inline)) {
    constexpr int NTP = decltype(ntc)::value;
    int buf = 0;
    int pt_tq = pt_second;  // TQ: the next tile's ticket
    for (int pt = pt_first; pt < pt_stop;) {
      const int ptn = TQ ? pt_tq : pt + 1;  // the next tile
      const bool more = ptn < pt_stop;
      unsigned claimed = 0;  // TQ: the ticket tid 0 claims during this tile (the tile after next)
      // the next tile goes to the free buffer in two halves (dY after k-step 1, the halo at the end),
      // so only one half's staging registers are live at a time (BNA at BI = 128: dA and y in two
      // quarters, stored after k-steps 0 and 2)
      constexpr bool QSPLIT = BNA && BI == 128;
      constexpr int PH = QSPLIT ? P_ROUNDS / 2 : P_ROUNDS;
      load_p(more ? ptn : pt, 0, PH);
      __builtin_amdgcn_sched_barrier(0);  // keep the next tile's loads ahead of this tile's MFMAs
#pragma unroll
      for (int ks = 0; ks < XPIX / 16; ++ks) {  // two tile rows (16 pixels) per k-step
        if (QSPLIT && ks == 1) {
          if (more) store_p(ptn, buf ^ 1, 0, PH);
          load_p(more ? ptn : pt, PH, P_ROUNDS);
          __builtin_amdgcn_sched_barrier(0);
        }
        // (QSPLIT: the second dY half is stored at k-step 3, two k-steps after its loads, and the halo's loads get
        // the last k-step — the halo rows are L2-hot more often: 1.5 % on the fused 128-column weight gradients,
        // profiles/r05p_wgrad_bn_schedule_ab.txt. BI = 64, whose registers allow both operands in flight at once:
        // the halo loaded at k-step 1 and the dY tile stored at k-step 3, three k-steps of cover each: 3-4 %,
        // profiles/r05q_wgrad64_schedule_ab.txt)
        if (BI == 64 && ks == 1) {
          load_x(more ? ptn : pt);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (ks == (QSPLIT || BI == 64 ? 3 : 2)) {
          if (more) store_p(ptn, buf ^ 1, QSPLIT ? PH : 0, P_ROUNDS);
          if (BI != 64) load_x(more ? ptn : pt);
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (TQ) {
          if (ks == 0 && tid == 0) claimed = atomicAdd(tq + grp, 1u);
        }
        const int prow = ks * 16 + 8 * half + q4;
        const int pcol = wi * 32 + 16 * grp_hi + 4 * p4;
        const f16x8 ah = tr8(&Ps[buf][0][prow][pcol], &Ps[buf][0][prow + 4][pcol]);
        const f16x8 al = tr8(&Ps[buf][1][prow][pcol], &Ps[buf][1][prow + 4][pcol]);
        const int xcol = wj * 32 + 16 * grp_hi + 4 * p4;
        constexpr int PF = BI == 128 ? 1 : 2;  // tap fragments read ahead (BI = 128: register-bound)
        struct Frag {
          f16x8 h, l;
        };
        auto read_tap = [&](int t) __attribute__((always_inline)) {
          const int tap = min(tap0 + t, 8);
          const int dy = tap / 3, dx = tap - (tap / 3) * 3;
          const int xrow = (2 * ks + half + dy) * XHW + dx + q4;
          Frag f;
          f.h = tr8(&Xs[buf][0][xrow][xcol], &Xs[buf][0][xrow + 4][xcol]);
          f.l = tr8(&Xs[buf][1][xrow][xcol], &Xs[buf][1][xrow + 4][xcol]);
          return f;
        };
        Frag bfr[NTAP];
#pragma unroll
        for (int t = 0; t < PF && t < NTAP; ++t) bfr[t] = read_tap(t);
        __builtin_amdgcn_sched_group_barrier(0x100, 4 + 4 * PF, 0);
#pragma unroll
        for (int t = 0; t < NTAP; ++t) {
          if (t < NTP) {
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bfr[t].l, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bfr[t].h, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bfr[t].h, acc[t], 0, 0, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
          if (t + PF < NTAP) {
            bfr[t + PF] = read_tap(t + PF);
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
          }
        }
      }
      if constexpr (TQ) {
        if (tid == 0) tq_slot[buf] = (int)min(claimed, (unsigned)pt_stop);  // read after the barrier
      }
      if (more) store_x(ptn, buf ^ 1);
      __syncthreads();
      if constexpr (TQ) pt_tq = tq_slot[buf];
      pt = ptn;
      buf ^= 1;
    }
  };
  if (TG == 1) tile_loop(std::integral_constant<int, 9>{});
  else if (tg == 0) tile_loop(std::integral_constant<int, 5>{});
  else tile_loop(std::integral_constant<int, 4>{});

  if constexpr (BNA) {
    // the exact max |dy| of the stored dy: one atomic per workgroup (uniform branch)
    if (bn.dy_amax) block_amax(bn.dy_amax, dam, Ks);
  }
  if constexpr (TQ) {
    const unsigned splits = gridDim.x / (unsigned)ngroups;
    if (tid == 0 && atomicAdd(tq + ngroups + grp, 1u) == splits - 1u) {
      // every workgroup of this group has made its last claim: reset for the next launch
      atomicExch(tq + grp, 0u);
      atomicExch(tq + ngroups + grp, 0u);
    }
  }
  const float ofac = uns_p * uns_x;
  const int ctot = Q.Ctot;
#pragma unroll
  for (int t = 0; t < NTAP; ++t) {
    if (t < ntap) {
      const int tap = tap0 + t;
      const int j = tap * ctot + c0 + wj * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + wi * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        ws[split * ws_stride + (int64_t)i * ldo + j] = acc[t][r] * ofac;
      }
    }
  }
}

// fp32 weight gradient (v_mfma_f32_32x32x2_f32: exact fp32 products, the parity configuration).
// An MFMA operand is one fp32 per lane (A[i = co][k = pixel], B[k = pixel][j = ci]), read with
// ds_read_b32 straight from the natural [pixel][channel] tiles: lanes 0-31 take pixel 2s and
// lanes 32-63 pixel 2s + 1 — the two 32-lane groups of ds_read_b32 never conflict with each other
// and 32 consecutive floats in a group hit 32 distinct banks, so the tiles need no padding.
//
// 512 threads (two waves per SIMD). A wave owns WCO co x 32 ci and one group of taps: BI = 128
// with WCO = 64 splits the 9 taps in two groups (5 / 4), BI = 64 with WCO = 32 likewise, so a
// wave keeps at most 10 accumulators and per k-step issues WCO/32 dY reads + one halo read per
// tap for (WCO/32) x taps MFMAs; the operands of the next k-step are read while the current one
// multiplies. The pixel tile is 8 x 8 (10 x 10 halo) and LDS holds two tiles: the next tile's
// loads are issued before a tile's MFMAs and written (BN+ReLU of the producer applied, padding
// zeroed) into the other buffer after them, so a tile boundary costs one barrier. Measured against
// the alternatives (tools/ab_wgrad.sh, fp32 bs=128 layers): 9 taps per wave at 2 waves/SIMD
// 118 TF/s; one wave per SIMD with 18 accumulators 85; the next tile written to LDS in the middle
// of the MFMA loop 98-107; this layout 126 (BI = 128) / 118 (BI = 64).
constexpr int FTH = 8, FTW = 8;                  // fp32 pixel tile

template <int BI, int WCO>
__global__ void __launch_bounds__(512, 1)
conv3x3_wgrad_halo_f32_kernel(GatherArg P, GatherArg Q, float* __restrict__ out, int ldo, int co_tiles,
                              int ci_chunks, int64_t tiles_per_split, int tiles_x, int tiles_y, int64_t total_tiles,
                              float* __restrict__ ws, int64_t ws_stride) {
  constexpr int CJ = 64;                         // ci channels per chunk
  constexpr int WTH = FTH, WTW = FTW, WHW = FTW + 2, WPIXT = FTH * FTW, WHP = (FTH + 2) * (FTW + 2);
  constexpr int NT = 512;
  constexpr int MA = WCO / 32;                   // co subtiles per wave
  constexpr int COH = BI / WCO;                  // co groups
  constexpr int TGN = 8 / (COH * 2);             // tap groups: 2 (taps 0-4, 5-8) or 4 (0-2, 3-4, 5-6, 7-8)
  static_assert(TGN == 2 || TGN == 4, "8 waves = co groups x 2 ci halves x tap groups");
  constexpr int NTAP = TGN == 2 ? 5 : 3;
  constexpr int P_ROUNDS = (WPIXT * BI / 4) / NT;
  constexpr int X_ROUNDS = (WHP * (CJ / 4) + NT - 1) / NT;
  constexpr int KS = WPIXT / 2;                  // k-steps per tile
  // k-steps unrolled: 4 at BI = 64 (120 vs 110 TF/s), 2 at BI = 128 (4 spills 22 registers: 126 vs 119)
  constexpr int UNR = BI == 128 ? 2 : 4;
  static_assert(P_ROUNDS * NT == WPIXT * BI / 4, "dY tile must split evenly over the threads");

  __shared__ __attribute__((aligned(16))) float Ps[2][WPIXT][BI];
  __shared__ __attribute__((aligned(16))) float Xs[2][WHP][CJ];
  __shared__ float Ks[2 * BI + 2 * CJ];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wj = wave & 1;                       // ci half (32 channels)
  const int wc = (wave >> 1) % COH;              // co group
  const int tg = (wave >> 1) / COH;              // tap group
  const int tap0 = TGN == 2 ? tg * 5 : (tg == 0 ? 0 : 1 + 2 * tg);
  const int ntap = TGN == 2 ? (tg == 0 ? 5 : 4) : (tg == 0 ? 3 : 2);
  const int half = lane >> 5, l32 = lane & 31;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int cot = lb % co_tiles;
  const int rest = lb / co_tiles;
  const int cik = rest % ci_chunks;
  const int64_t split = rest / ci_chunks;
  const int i0 = cot * BI;
  const int c0 = cik * CJ;
  const int64_t pt_begin = split * tiles_per_split;
  const int64_t pt_end = min(total_tiles, pt_begin + tiles_per_split);
  if (pt_begin >= pt_end) return;

  int xs_src = 0, xc = c0;
  if (Q.nsrc > 1 && xc >= Q.src[0].C) {
    xc -= Q.src[0].C;
    xs_src = 1;
  }
  const SrcArg xa = pick_src(Q, xs_src);
  const SrcArg& pa = P.src[0];
  const int H = P.h, W = P.w;

  if (tid < 2 * BI + 2 * CJ) {
    float v;
    if (tid < 2 * BI) {
      const int c = i0 + (tid % BI);
      v = pa.scale ? (tid < BI ? pa.scale[c] : pa.shift[c]) : 0.0f;
    } else {
      const int c = xc + ((tid - 2 * BI) % CJ);
      v = xa.scale ? (tid < 2 * BI + CJ ? xa.scale[c] : xa.shift[c]) : 0.0f;
    }
    Ks[tid] = v;
  }

  auto tile_origin = [&](int pt, int& img, int& y0, int& x0) __attribute__((always_inline)) {
    const unsigned r2 = (unsigned)pt / (unsigned)tiles_x;
    x0 = ((unsigned)pt - r2 * (unsigned)tiles_x) * WTW;
    const unsigned r3 = r2 / (unsigned)tiles_y;
    y0 = (r2 - r3 * (unsigned)tiles_y) * WTH;
    img = (int)r3;
  };
  auto apply = [&](f32x4 v, const float* sc, const float* sh, int relu) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float f = v[j] * sc[j] + sh[j];
      v[j] = relu ? fmaxf(f, 0.0f) : f;
    }
    return v;
  };
  // raw loads of a tile's dY part / halo part (pixels clamped into the image; zeroed when written)
  f32x4 rp[P_ROUNDS], rx[X_ROUNDS];
  auto load_p = [&](int pt) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < P_ROUNDS; ++r) {
      const int idx = r * NT + tid;
      const int px = idx / (BI / 4), cc = idx % (BI / 4);
      const int y = min(y0 + px / WTW, H - 1), x = min(x0 + px % WTW, W - 1);
      rp[r] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(pa.data) +
                                              (((int64_t)img * H + y) * W + x) * pa.C + i0 + cc * 4);
    }
  };
  auto load_x = [&](int pt) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < X_ROUNDS; ++r) {
      const int idx = r * NT + tid;
      const int hp = min(idx >> 4, WHP - 1), cc = idx & 15;
      const int y = min(max(y0 - 1 + hp / WHW, 0), H - 1), x = min(max(x0 - 1 + hp % WHW, 0), W - 1);
      rx[r] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(xa.data) +
                                              (((int64_t)img * H + y) * W + x) * xa.C + xc + cc * 4);
    }
  };
  auto store_p = [&](int pt, int buf) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < P_ROUNDS; ++r) {
      const int idx = r * NT + tid;
      const int px = idx / (BI / 4), cc = idx % (BI / 4);
      f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
      if (y0 + px / WTW < H && x0 + px % WTW < W)
        v = pa.scale ? apply(rp[r], Ks + cc * 4, Ks + BI + cc * 4, pa.relu) : rp[r];
      *reinterpret_cast<f32x4*>(&Ps[buf][px][cc * 4]) = v;
    }
  };
  auto store_x = [&](int pt, int buf) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < X_ROUNDS; ++r) {
      const int idx = r * NT + tid;
      if (idx < WHP * (CJ / 4)) {
        const int hp = idx >> 4, cc = idx & 15;
        const int y = y0 - 1 + hp / WHW, x = x0 - 1 + hp % WHW;
        f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
          v = xa.scale ? apply(rx[r], Ks + 2 * BI + cc * 4, Ks + 2 * BI + CJ + cc * 4, xa.relu) : rx[r];
        *reinterpret_cast<f32x4*>(&Xs[buf][hp][cc * 4]) = v;
      }
    }
  };

  f32x16 acc[MA][NTAP];
#pragma unroll
  for (int a = 0; a < MA; ++a)
#pragma unroll
    for (int t = 0; t < NTAP; ++t) acc[a][t] = f32x16{};

  int toff[NTAP];
#pragma unroll
  for (int t = 0; t < NTAP; ++t) {
    const int tap = min(tap0 + t, 8);
    toff[t] = ((tap / 3) * WHW + tap % 3) * CJ;
  }
  struct Frag {
    float a[MA], b[NTAP];
  };
  // operands of k-step ks (k = the lane half's pixel) from buffer buf
  auto frag = [&](int buf, int ks) __attribute__((always_inline)) {
    Frag f;
    const int p = 2 * ks + half;
    const float* pr = &Ps[buf][p][wc * WCO + l32];
#pragma unroll
    for (int a = 0; a < MA; ++a) f.a[a] = pr[a * 32];
    const float* xr = &Xs[buf][(p / WTW) * WHW + p % WTW][wj * 32 + l32];
#pragma unroll
    for (int t = 0; t < NTAP; ++t) f.b[t] = xr[toff[t]];
    return f;
  };

  load_p((int)pt_begin);
  load_x((int)pt_begin);
  __syncthreads();  // coefficients visible
  store_p((int)pt_begin, 0);
  store_x((int)pt_begin, 0);
  __syncthreads();
  int buf = 0;
  for (int pt = (int)pt_begin; pt < (int)pt_end; ++pt) {
    const bool more = pt + 1 < (int)pt_end;
    if (more) { load_p(pt + 1); load_x(pt + 1); }
    Frag cur = frag(buf, 0);
#pragma unroll UNR
    for (int ks = 0; ks < KS; ++ks) {
      const Frag nxt = frag(buf, ks + 1 < KS ? ks + 1 : 0);
#pragma unroll
      for (int t = 0; t < NTAP; ++t)
        if (t < ntap) {
#pragma unroll
          for (int a = 0; a < MA; ++a)
            acc[a][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.a[a], cur.b[t], acc[a][t], 0, 0, 0);
        }

      cur = nxt;
    }
    if (more) { store_p(pt + 1, buf ^ 1); store_x(pt + 1, buf ^ 1); }
    __syncthreads();  // the next tile is in buf ^ 1; everyone is done with buf
    buf ^= 1;
  }

  // (an opaque copy of the lane: the store addresses below are loop-invariant, and hoisting them
  // above the tile loop would pin ~70 registers through it)
  int ln = lane;
  asm volatile("" : "+v"(ln));
  const int ctot = Q.Ctot;
#pragma unroll
  for (int t = 0; t < NTAP; ++t) {
    if (t < ntap) {
      const int tap = tap0 + t;
      const int j = tap * ctot + c0 + wj * 32 + (ln & 31);
#pragma unroll
      for (int a = 0; a < MA; ++a)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = i0 + wc * WCO + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
          if (ws) ws[split * ws_stride + (int64_t)i * ldo + j] = acc[a][t][r];
          else atomicAdd(out + (int64_t)i * ldo + j, acc[a][t][r]);
        }
    }
  }
}

// fp32 weight gradient as the transpose of the Winograd F(2,3) forward (1-D along x). With
// δ0, δ1 = dY at an output pair (x, x+1) and d_j = X at (x - 1 + j, row + dy):
//   dW[dy][0] = M0 + (M1 + M2)/2,  dW[dy][1] = (M1 - M2)/2,  dW[dy][2] = (M1 + M2)/2 + M3,
//   M_xi = sum over pairs of A_xi * B_xi,  A = (δ0, δ0 + δ1, δ0 - δ1, -δ1),
//   B = (d0 - d2, d1 + d2, d2 - d1, d1 - d3)
// (dW_i = dL/dg_i of the forward's Winograd form: the M_xi carry the G-transposed weights). The MFMA
// k dimension is the output pair (two per k-step: one per lane half), so a 8x8 tile is 16 k-steps
// of 4 products per dy instead of 32 of 3 taps: 2/3 of the direct kernel's MFMA work. Workgroup:
// 64 co x 64 ci x the 12 (dy, xi) planes; 8 waves = 2 co halves x 2 ci halves x 2 plane groups
// (planes 0-5 = dy 0 and dy 1 xi 0-1; 6-11 = dy 1 xi 2-3 and dy 2), 6 accumulators each. Each split
// stores its M planes (plain stores, every plane has one owner) to ws[split][co][plane * C + ci]; the
// fixed-order split reduction applies the output transform (wgrad_wino_reduce_kernel, gemm.hip).
// Tiles are staged as in conv3x3_wgrad_halo_f32_kernel (double-buffered, next tile loaded during
// the MFMAs, BN+ReLU of the producer applied at the LDS write).
// NW = 8 waves (2 plane groups of 6: dy 0 + dy 1 xi 0-1 / dy 1 xi 2-3 + dy 2) or 12 waves (3 plane
// groups, one kernel row dy each: 4 accumulators, 6 LDS reads per 4 MFMAs, three waves per SIMD)
template <int TWW, int NW>
__global__ void __launch_bounds__(NW * 64, 1)
conv3x3_wgrad_wino_f32_kernel(GatherArg P, GatherArg Q, int co_tiles, int ci_chunks, int64_t tiles_per_split,
                              int tiles_x, int tiles_y, int64_t total_tiles, float* __restrict__ ws, int64_t ws_stride,
                              int ldw) {
  constexpr int BI = 64, CJ = 64;
  // pixel tile 8 x TWW (TWW = 16: 64 output pairs, 32 k-steps per tile, half the per-tile overhead of 8 x 8)
  constexpr int WTH = FTH, WTW = TWW, WHW = TWW + 2, WPIXT = FTH * TWW, WHP = (FTH + 2) * (TWW + 2);
  constexpr int NT = NW * 64;
  constexpr int P_VEC = WPIXT * BI / 4;
  constexpr int P_ROUNDS = (P_VEC + NT - 1) / NT;
  constexpr int X_ROUNDS = (WHP * (CJ / 4) + NT - 1) / NT;
  constexpr int NACC = NW == 8 ? 6 : 4;  // planes per wave
  constexpr int KS = WPIXT / 4;  // k-steps per tile: two pairs per k-step
  constexpr int PPR = TWW / 2;   // pairs per tile row
  static_assert(NW == 8 || NW == 12, "8 or 12 waves");

  __shared__ __attribute__((aligned(16))) float Ps[2][WPIXT][BI];
  __shared__ __attribute__((aligned(16))) float Xs[2][WHP][CJ];
  __shared__ float Ks[2 * BI + 2 * CJ];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wj = wave & 1;          // ci half
  const int wc = (wave >> 1) & 1;   // co half
  const int tg = wave >> 2;         // plane group (NW = 12: the kernel row dy)
  const int half = lane >> 5, l32 = lane & 31;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int cot = lb % co_tiles;
  const int rest = lb / co_tiles;
  const int cik = rest % ci_chunks;
  const int64_t split = rest / ci_chunks;
  const int i0 = cot * BI;
  const int c0 = cik * CJ;
  const int64_t pt_begin = split * tiles_per_split;
  const int64_t pt_end = min(total_tiles, pt_begin + tiles_per_split);

  int xs_src = 0, xc = c0;
  if (Q.nsrc > 1 && xc >= Q.src[0].C) {
    xc -= Q.src[0].C;
    xs_src = 1;
  }
  const SrcArg xa = pick_src(Q, xs_src);
  const SrcArg& pa = P.src[0];
  const int H = P.h, W = P.w;

  if (tid < 2 * BI + 2 * CJ) {
    float v;
    if (tid < 2 * BI) {
      const int c = i0 + (tid % BI);
      v = pa.scale ? (tid < BI ? pa.scale[c] : pa.shift[c]) : 0.0f;
    } else {
      const int c = xc + ((tid - 2 * BI) % CJ);
      v = xa.scale ? (tid < 2 * BI + CJ ? xa.scale[c] : xa.shift[c]) : 0.0f;
    }
    Ks[tid] = v;
  }

  auto tile_origin = [&](int pt, int& img, int& y0, int& x0) __attribute__((always_inline)) {
    const unsigned r2 = (unsigned)pt / (unsigned)tiles_x;
    x0 = ((unsigned)pt - r2 * (unsigned)tiles_x) * WTW;
    const unsigned r3 = r2 / (unsigned)tiles_y;
    y0 = (r2 - r3 * (unsigned)tiles_y) * WTH;
    img = (int)r3;
  };
  auto apply = [&](f32x4 v, const float* sc, const float* sh, int relu) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float f = v[j] * sc[j] + sh[j];
      v[j] = relu ? fmaxf(f, 0.0f) : f;
    }
    return v;
  };
  f32x4 rp[P_ROUNDS], rx[X_ROUNDS];
  auto load_p = [&](int pt) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < P_ROUNDS; ++r) {
      const int idx = min(r * NT + tid, P_VEC - 1);
      const int px = idx / (BI / 4), cc = idx % (BI / 4);
      const int y = min(y0 + px / WTW, H - 1), x = min(x0 + px % WTW, W - 1);
      rp[r] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(pa.data) +
                                              (((int64_t)img * H + y) * W + x) * pa.C + i0 + cc * 4);
    }
  };
  auto load_x = [&](int pt) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < X_ROUNDS; ++r) {
      const int idx = r * NT + tid;
      const int hp = min(idx >> 4, WHP - 1), cc = idx & 15;
      const int y = min(max(y0 - 1 + hp / WHW, 0), H - 1), x = min(max(x0 - 1 + hp % WHW, 0), W - 1);
      rx[r] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(xa.data) +
                                              (((int64_t)img * H + y) * W + x) * xa.C + xc + cc * 4);
    }
  };
  auto store_p = [&](int pt, int buf) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < P_ROUNDS; ++r) {
      const int idx = r * NT + tid;
      if (P_VEC % NT != 0 && idx >= P_VEC) continue;
      const int px = idx / (BI / 4), cc = idx % (BI / 4);
      f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
      if (y0 + px / WTW < H && x0 + px % WTW < W)
        v = pa.scale ? apply(rp[r], Ks + cc * 4, Ks + BI + cc * 4, pa.relu) : rp[r];
      *reinterpret_cast<f32x4*>(&Ps[buf][px][cc * 4]) = v;
    }
  };
  auto store_x = [&](int pt, int buf) __attribute__((always_inline)) {
    int img, y0, x0;
    tile_origin(pt, img, y0, x0);
#pragma unroll
    for (int r = 0; r < X_ROUNDS; ++r) {
      const int idx = r * NT + tid;
      if (idx < WHP * (CJ / 4)) {
        const int hp = idx >> 4, cc = idx & 15;
        const int y = y0 - 1 + hp / WHW, x = x0 - 1 + hp % WHW;
        f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
          v = xa.scale ? apply(rx[r], Ks + 2 * BI + cc * 4, Ks + 2 * BI + CJ + cc * 4, xa.relu) : rx[r];
        *reinterpret_cast<f32x4*>(&Xs[buf][hp][cc * 4]) = v;
      }
    }
  };

  f32x16 acc[NACC];
#pragma unroll
  for (int t = 0; t < NACC; ++t) acc[t] = f32x16{};

  // raw operands of one k-step: δ0, δ1 of the lane's pair and the seven d_j rows its planes use
  // (group 0: dy 0 d0..d3, dy 1 d0..d2; group 1: dy 1 d1..d3, dy 2 d0..d3). The plane group is a
  // template constant of the whole tile loop (tile_loop below): a per-k-step branch on it splits the
  // loop into blocks at whose joins the compiler drains the LDS counter, serialising the next
  // k-step's reads behind the current MFMAs.
  struct Frag {
    float a0, a1, d[7];
  };
  auto tile_loop = [&](auto tgc) __attribute__((always_inline)) {
    constexpr int TG = decltype(tgc)::value;
    auto frag = [&](int buf, int ks) __attribute__((always_inline)) {
      Frag f;
      const int pp = 2 * ks + half, r = pp / PPR, c2 = pp % PPR;
      const float* pr = &Ps[buf][r * WTW + 2 * c2][wc * 32 + l32];
      f.a0 = pr[0];
      f.a1 = pr[BI];
      const float* xr = &Xs[buf][r * WHW + 2 * c2][wj * 32 + l32];
      if constexpr (NW == 12) {
#pragma unroll
        for (int j = 0; j < 4; ++j) f.d[j] = xr[(TG * WHW + j) * CJ];  // dy = TG: d0..d3
      } else if constexpr (TG == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) f.d[j] = xr[j * CJ];              // dy 0
#pragma unroll
        for (int j = 0; j < 3; ++j) f.d[4 + j] = xr[(WHW + j) * CJ];  // dy 1, j = 0..2
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) f.d[j] = xr[(WHW + 1 + j) * CJ];      // dy 1, j = 1..3
#pragma unroll
        for (int j = 0; j < 4; ++j) f.d[3 + j] = xr[(2 * WHW + j) * CJ];  // dy 2
      }
      return f;
    };
    auto mma = [&](const Frag& f) __attribute__((always_inline)) {
      const float A0 = f.a0, A1 = f.a0 + f.a1, A2 = f.a0 - f.a1, A3 = -f.a1;
      const float* d = f.d;
      if constexpr (NW == 12) {  // one kernel row: xi 0..3
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, d[0] - d[2], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, d[1] + d[2], acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(A2, d[2] - d[1], acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(A3, d[1] - d[3], acc[3], 0, 0, 0);
      } else if constexpr (TG == 0) {  // dy 0: d[0..3]; dy 1: d[4..6] = d0..d2
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, d[0] - d[2], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, d[1] + d[2], acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(A2, d[2] - d[1], acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(A3, d[1] - d[3], acc[3], 0, 0, 0);
        acc[4] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, d[4] - d[6], acc[4], 0, 0, 0);
        acc[5] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, d[5] + d[6], acc[5], 0, 0, 0);
      } else {  // dy 1: d[0..2] = d1..d3; dy 2: d[3..6] = d0..d3
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A2, d[1] - d[0], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A3, d[0] - d[2], acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, d[3] - d[5], acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, d[4] + d[5], acc[3], 0, 0, 0);
        acc[4] = __builtin_amdgcn_mfma_f32_32x32x2f32(A2, d[5] - d[4], acc[4], 0, 0, 0);
        acc[5] = __builtin_amdgcn_mfma_f32_32x32x2f32(A3, d[4] - d[6], acc[5], 0, 0, 0);
      }
    };
    if (pt_begin < pt_end) {
      load_p((int)pt_begin);
      load_x((int)pt_begin);
    }
    __syncthreads();  // coefficients visible
    if (pt_begin < pt_end) {
      store_p((int)pt_begin, 0);
      store_x((int)pt_begin, 0);
    }
    __syncthreads();
    int buf = 0;
    for (int pt = (int)pt_begin; pt < (int)pt_end; ++pt) {
      const bool more = pt + 1 < (int)pt_end;
      if (more) { load_p(pt + 1); load_x(pt + 1); }
      Frag cur = frag(buf, 0);
#pragma unroll 4
      for (int ks = 0; ks < KS; ++ks) {
        const Frag nxt = frag(buf, ks + 1 < KS ? ks + 1 : 0);
        // the next k-step's LDS reads stay ahead of this one's MFMAs (left alone, the scheduler sinks
        // them next to their use across the unrolled k-steps and waits each out with lgkmcnt(0))
        __builtin_amdgcn_sched_barrier(0);
        mma(cur);
        cur = nxt;
      }
      if (more) { store_p(pt + 1, buf ^ 1); store_x(pt + 1, buf ^ 1); }
      __syncthreads();
      buf ^= 1;
    }
  };
  if (tg == 0) tile_loop(std::integral_constant<int, 0>{});
  else if (NW == 8 || tg == 1) tile_loop(std::integral_constant<int, 1>{});
  else tile_loop(std::integral_constant<int, 2>{});

  // planes of this wave: group 0 -> 0..5, group 1 -> 6..11 (plane = dy * 4 + xi)
  int ln = lane;
  asm volatile("" : "+v"(ln));
  const int ctot = Q.Ctot;
#pragma unroll
  for (int t = 0; t < NACC; ++t) {
    const int plane = tg * NACC + t;
    const int j = plane * ctot + c0 + wj * 32 + (ln & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = i0 + wc * 32 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
      ws[split * ws_stride + (int64_t)i * ldw + j] = acc[t][r];
    }
  }
}

bool conv3x3_wgrad_wino_eligible(const GatherArg& p, const GatherArg& q, int dtype) {
  return option(SELUNET_OPT_WINO_WGRAD, 1) != 0 && dtype == SELUNET_F32 && conv3x3_wgrad_halo_eligible(p, q, dtype) && q.w % 2 == 0;
}

// splits of the Winograd weight gradient (64 x 64 tiles): ~256 workgroups over (co tile, ci chunk, split)
static int wino_wgrad_tw() { return option(SELUNET_OPT_WINO_WGRAD_TW, 16) == 8 ? 8 : 16; }

int64_t conv3x3_wgrad_wino_splits(const GatherArg& p, const GatherArg& q, int64_t* per_out) {
  const int co_tiles = p.K / 64, ci_chunks = q.Ctot / 64;
  const int64_t total = (int64_t)q.n * cdiv(q.w, wino_wgrad_tw()) * cdiv(q.h, FTH);
  const int64_t target = std::max<int64_t>(1, option(SELUNET_OPT_WGRAD_WGS, 256));
  const int64_t want = std::max<int64_t>(1, cdiv(target, (int64_t)co_tiles * ci_chunks));
  const int64_t per = cdiv(total, std::min(total, want));
  if (per_out) *per_out = per;
  return cdiv(total, per);
}

int conv3x3_wgrad_wino_launch(const GatherArg& p, const GatherArg& q, float* ws, int ldw, hipStream_t st) {
  const int co_tiles = p.K / 64, ci_chunks = q.Ctot / 64;
  const int tw = wino_wgrad_tw();
  const int tiles_x = (int)cdiv(q.w, tw), tiles_y = (int)cdiv(q.h, FTH);
  const int64_t total = (int64_t)q.n * tiles_x * tiles_y;
  int64_t per;
  const int64_t splits = conv3x3_wgrad_wino_splits(p, q, &per);
  const unsigned blocks = (unsigned)(co_tiles * ci_chunks * splits);
  const int nw = option(SELUNET_OPT_WINO_WGRAD_WAVES, 12) == 8 ? 8 : 12;
  auto kern = tw == 8 ? (nw == 8 ? conv3x3_wgrad_wino_f32_kernel<8, 8> : conv3x3_wgrad_wino_f32_kernel<8, 12>)
                      : (nw == 8 ? conv3x3_wgrad_wino_f32_kernel<16, 8> : conv3x3_wgrad_wino_f32_kernel<16, 12>);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(nw * 64), 0, st, p, q, co_tiles, ci_chunks, per, tiles_x, tiles_y,
                     total, ws, (int64_t)p.K * ldw, ldw);
  return check_launch("conv3x3_wgrad_wino");
}

// column tile of the split-fp16 weight gradient (plain and BN-fused forms alike; 64-column tiles for the fused
// 128+-channel layers measured 4 % slower, profiles/r05g_wgrad_bn_bi64_ab.txt)
int conv3x3_wgrad_x2_bi(const GatherArg& p, bool /*bn*/) { return p.K % 128 == 0 ? 128 : 64; }

// pixel-tile splits of the split-fp16 weight gradient: ~256 workgroups over (co tile, ci chunk, split)
int64_t conv3x3_wgrad_x2_splits(const GatherArg& p, const GatherArg& q, int64_t* per_out, bool bn) {
  const int bi = conv3x3_wgrad_x2_bi(p, bn);
  const int co_tiles = p.K / bi, ci_chunks = q.Ctot / 64;
  const int64_t total = (int64_t)q.n * cdiv(q.w, XTW) * cdiv(q.h, XTH);
  const int64_t target = std::max<int64_t>(1, option(SELUNET_OPT_X2_WGRAD_WGS, 256));
  const int64_t want = std::max<int64_t>(1, cdiv(target, (int64_t)co_tiles * ci_chunks));
  const int64_t per = cdiv(total, std::min(total, want));
  if (per_out) *per_out = per;
  return cdiv(total, per);
}

static unsigned* tq_counters(hipStream_t st);
// SELUNET_OPT_TILE_QUEUE bit 1: the split-fp16 weight gradients take their pixel tiles from ticket counters
static bool x2_wgrad_tile_queue() { return (option(SELUNET_OPT_TILE_QUEUE, 0) & 2) != 0; }

int conv3x3_wgrad_x2_launch(const GatherArg& p, const GatherArg& q, float* ws, int ldo, const float* amax_p,
                            const float* amax_q0, const float* amax_q1, hipStream_t st, const WgradBnArg* bn) {
  const int bi = conv3x3_wgrad_x2_bi(p, bn != nullptr);
  const int co_tiles = p.K / bi, ci_chunks = q.Ctot / 64;
  const int tiles_x = (int)cdiv(q.w, XTW), tiles_y = (int)cdiv(q.h, XTH);
  const int64_t total = (int64_t)q.n * tiles_x * tiles_y;
  int64_t per;
  const int64_t splits = conv3x3_wgrad_x2_splits(p, q, &per, bn != nullptr);
  const unsigned blocks = (unsigned)(co_tiles * ci_chunks * splits);
  const int kind = bn ? bn->kind : -1;
  SELUNET_REQUIRE(kind <= SELUNET_DA_TENSOR || bi == 64, "conv3x3_wgrad_x2: pool / heads dA sources need 64 columns");
  if (x2_wgrad_tile_queue()) {  // (co tile, ci chunk) groups take their pixel tiles from ticket counters
    unsigned* tq = tq_counters(st);
    if (tq == nullptr || co_tiles * ci_chunks > 64)
      return fail(SELUNET_ELAUNCH, "conv3x3_wgrad_x2: tile-queue counters unavailable (set SELUNET_OPT_TILE_QUEUE "
                                   "before capturing the step) or more than 64 (co tile, ci chunk) groups");
    auto k = bi == 128 ? (bn ? conv3x3_wgrad_x2_kernel<128, 1, true> : conv3x3_wgrad_x2_kernel<128, 0, true>)
             : kind == SELUNET_DA_POOL  ? conv3x3_wgrad_x2_kernel<64, 2, true>
             : kind == SELUNET_DA_HEADS ? conv3x3_wgrad_x2_kernel<64, 3, true>
             : (bn ? conv3x3_wgrad_x2_kernel<64, 1, true> : conv3x3_wgrad_x2_kernel<64, 0, true>);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, st, p, q, ldo, co_tiles, ci_chunks, per, tiles_x, tiles_y,
                       total, ws, (int64_t)p.K * ldo, amax_p, amax_q0, amax_q1, bn ? *bn : WgradBnArg{}, tq);
    return check_launch("conv3x3_wgrad_x2");
  }
  auto k = bi == 128 ? (bn ? conv3x3_wgrad_x2_kernel<128, 1> : conv3x3_wgrad_x2_kernel<128, 0>)
           : kind == SELUNET_DA_POOL  ? conv3x3_wgrad_x2_kernel<64, 2>
           : kind == SELUNET_DA_HEADS ? conv3x3_wgrad_x2_kernel<64, 3>
           : (bn ? conv3x3_wgrad_x2_kernel<64, 1> : conv3x3_wgrad_x2_kernel<64, 0>);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, st, p, q, ldo, co_tiles, ci_chunks, per, tiles_x, tiles_y, total,
                     ws, (int64_t)p.K * ldo, amax_p, amax_q0, amax_q1, bn ? *bn : WgradBnArg{}, nullptr);
  return check_launch("conv3x3_wgrad_x2");
}

bool conv3x3_wgrad_halo_eligible(const GatherArg& p, const GatherArg& q, int dtype) {
  if (dtype != SELUNET_BF16 && dtype != SELUNET_F32) return false;
  if (p.taps != 1 || p.nsrc != 1 || p.small || p.src[0].layout != 0 || p.K % 64 != 0) return false;
  if (q.taps != 9 || q.small || q.h < 8 || q.w < 16) return false;
  for (int s = 0; s < q.nsrc; ++s)
    if (q.src[s].C % 64 != 0 || q.src[s].layout != 0) return false;
  return true;
}

// pixel-tile splits of the halo weight gradient: ~512 workgroups over (co tile, ci chunk, split)
static void wgrad_tile(int dtype, int& th, int& tw) {
  th = dtype == SELUNET_F32 ? FTH : WTH;
  tw = dtype == SELUNET_F32 ? FTW : WTW;
}

int64_t conv3x3_wgrad_halo_splits(const GatherArg& p, const GatherArg& q, int dtype, int64_t* per_out) {
  const int ni = p.K;
  const int bi = ni % 128 == 0 ? 128 : 64;
  const int co_tiles = ni / bi, ci_chunks = q.Ctot / 64;
  int th, tw;
  wgrad_tile(dtype, th, tw);
  const int64_t total = (int64_t)q.n * cdiv(q.w, tw) * cdiv(q.h, th);
  // workgroup target over (co tile, ci chunk, pixel split); each split adds ni*ld*4 bytes of
  // partials for the fixed-order reduction to read. One workgroup per CU (256) measured best:
  // 6.53 vs 6.94 ms/step at 16 images/GPU (512: two per CU, twice the partials), 11.8 vs 12.2 at
  // 32, equal at 128; 128 and 384 lose (SELUNET_WGRAD_WGS overrides)
  const int64_t target = std::max<int64_t>(1, option(SELUNET_OPT_WGRAD_WGS, 256));
  const int64_t want = std::max<int64_t>(1, cdiv(target, (int64_t)co_tiles * ci_chunks));
  const int64_t per = cdiv(total, std::min(total, want));
  if (per_out) *per_out = per;
  return cdiv(total, per);
}

// ws == nullptr: fp32 atomics into out (zeroed by the caller). Otherwise every split writes its
// partial to ws[split][ni][ldo] (ws_stride = ni * ldo floats) and the caller reduces the splits.
int conv3x3_wgrad_halo_launch(const GatherArg& p, const GatherArg& q, float* out, int ldo, float* ws, int dtype,
                              hipStream_t st) {
  const int ni = p.K;
  const int bi = ni % 128 == 0 ? 128 : 64;
  const int co_tiles = ni / bi, ci_chunks = q.Ctot / 64;
  int th, tw;
  wgrad_tile(dtype, th, tw);
  const int tiles_x = (int)cdiv(q.w, tw), tiles_y = (int)cdiv(q.h, th);
  const int64_t total = (int64_t)q.n * tiles_x * tiles_y;
  int64_t per;
  const int64_t splits = conv3x3_wgrad_halo_splits(p, q, dtype, &per);
  const unsigned blocks = (unsigned)(co_tiles * ci_chunks * splits);
  const int64_t stride = (int64_t)ni * ldo;
  if (dtype == SELUNET_F32) {
    if (bi == 128)
      hipLaunchKernelGGL((conv3x3_wgrad_halo_f32_kernel<128, 64>), dim3(blocks), dim3(512), 0, st, p, q, out, ldo,
                         co_tiles, ci_chunks, per, tiles_x, tiles_y, total, ws, stride);
    else
      hipLaunchKernelGGL((conv3x3_wgrad_halo_f32_kernel<64, 32>), dim3(blocks), dim3(512), 0, st, p, q, out, ldo,
                         co_tiles, ci_chunks, per, tiles_x, tiles_y, total, ws, stride);
  } else if (bi == 128)
    hipLaunchKernelGGL(conv3x3_wgrad_halo_kernel<128>, dim3(blocks), dim3(512), 0, st, p, q, out, ldo, co_tiles,
                       ci_chunks, per, tiles_x, tiles_y, total, ws, stride);
  else
    hipLaunchKernelGGL(conv3x3_wgrad_halo_kernel<64>, dim3(blocks), dim3(512), 0, st, p, q, out, ldo, co_tiles,
                       ci_chunks, per, tiles_x, tiles_y, total, ws, stride);
  return check_launch("conv3x3_wgrad_halo");
}

bool conv3x3_halo_eligible(const GatherArg& g, int N, int dtype) {
  const int ck = dtype == SELUNET_F32 ? 32 : 64;
  if (g.taps != 9 || g.small || g.h < 16 || g.w < 16) return false;
  if (g.Ctot % ck != 0 || (g.nsrc > 1 && g.src[0].C % ck != 0)) return false;
  for (int s = 0; s < g.nsrc; ++s)
    if (g.src[s].layout != 0) return false;
  return N % 64 == 0;
}

int64_t conv3x3_halo_tiles(const GatherArg& g) {
  return (int64_t)g.n * cdiv(g.h, TH) * cdiv(g.w, TW);
}

// Workgroups (= CUs) the persistent multi-chunk kernel targets; a fixed constant rather than the
// device's CU count so that the statistics slab rows the host allocates never depend on the device.
constexpr int PERSIST_WGS_DEFAULT = 256;
static int PERSIST_WGS = PERSIST_WGS_DEFAULT;  // selunet_set_halo_workgroups

static bool persist_enabled() { return option(SELUNET_OPT_HALO_PERSIST, 1) != 0; }

// single-chunk layers (C = one 128-B chunk) run the non-persistent ONE_CHUNK kernel (two workgroups per CU;
// the persistent kernel measured 7 % slower on them, profiles/r04h_halo_persist_one_chunk.txt)
static bool halo_one_chunk(const GatherArg& g, int dtype) { return g.Ctot == (dtype == SELUNET_F32 ? 32 : 64); }
bool conv3x3_halo_one_chunk(const GatherArg& g, int dtype) { return halo_one_chunk(g, dtype); }

// output tiles per workgroup row of the persistent launch (= statistics slab rows): PERSIST_WGS
// workgroups at 128-column tiles; 64-column tiles (N % 128 != 0 or a split at 64) use twice the
// workgroups with the same rows, so the row count depends on the operand and N only
static int persist_rows(const GatherArg& g, int N) {
  const int64_t pt = conv3x3_halo_tiles(g);
  return (int)std::max<int64_t>(1, std::min<int64_t>(pt, PERSIST_WGS / std::max(1, N / 128)));
}

int64_t conv3x3_persist_rows(const GatherArg& g, int N) { return persist_rows(g, N); }
int conv3x3_persist_wgs() { return PERSIST_WGS; }

bool conv3x3_halo_persistent(const GatherArg& g, int dtype) { return !halo_one_chunk(g, dtype) && persist_enabled(); }

int64_t conv3x3_halo_stats_rows(const GatherArg& g, int N, int dtype) {
  if (halo_one_chunk(g, dtype) || !persist_enabled()) return conv3x3_halo_tiles(g);
  return persist_rows(g, N);
}

template <typename T, int BN>
static void launch_halo(const GatherArg& g, const void* b, int N, int k_pad, const EpiArg& ep, hipStream_t st) {
  const int tiles_x = (int)cdiv(g.w, TW), tiles_y = (int)cdiv(g.h, TH);
  const int n_tiles = N / BN;
  const int64_t blocks = conv3x3_halo_tiles(g) * n_tiles;
  const int dtype = sizeof(T) == 2 ? SELUNET_BF16 : SELUNET_F32;
  const bool one = halo_one_chunk(g, dtype);
  if (!one && persist_enabled()) {
    const int gp = (int)conv3x3_halo_stats_rows(g, N, dtype);
    auto k = conv3x3_halo_persist_kernel<T, BN, false>;
    hipLaunchKernelGGL(k, dim3((unsigned)(gp * n_tiles)), dim3(HTHREADS), 0, st, g, reinterpret_cast<const T*>(b), N,
                       k_pad, ep, n_tiles, tiles_x, tiles_y, (int)conv3x3_halo_tiles(g), gp, nullptr, nullptr, nullptr,
                       nullptr);
    return;
  }
  auto k = one ? conv3x3_halo_kernel<T, BN, true> : conv3x3_halo_kernel<T, BN, false>;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(HTHREADS), 0, st, g, reinterpret_cast<const T*>(b), N, k_pad,
                     ep, n_tiles, tiles_x, tiles_y);
}

static bool wino_enabled() { return option(SELUNET_OPT_WINO, 1) != 0; }

bool conv3x3_wino_shape_ok(int h, int w, int c_in, int c_src0, int n_cols) {
  return wino_enabled() && persist_enabled() && h >= TH && w >= TW && w % 2 == 0 && c_in % 32 == 0 &&
         c_src0 % 32 == 0 && c_in > 32 && n_cols % 64 == 0;
}

bool conv3x3_wino_eligible(const GatherArg& g, int N) {
  return conv3x3_halo_eligible(g, N, SELUNET_F32) && conv3x3_halo_persistent(g, SELUNET_F32) &&
         conv3x3_wino_shape_ok(g.h, g.w, g.Ctot, g.src[0].C, N);
}

template <int BN, int XS>
static void launch_wino(const GatherArg& g, const float* u, int N, const EpiArg& ep, hipStream_t st) {
  const int tiles_x = (int)cdiv(g.w, TW), tiles_y = (int)cdiv(g.h, TH);
  const int n_tiles = N / BN;
  const int gp = persist_rows(g, N);  // = the statistics slab rows of selunet_gemm_stats_rows
  hipLaunchKernelGGL((conv3x3_wino_persist_kernel<BN, XS>), dim3((unsigned)(gp * n_tiles)), dim3(HTHREADS), 0, st, g, u,
                     N, WINO_STEPS * g.Ctot, ep, n_tiles, tiles_x, tiles_y, (int)conv3x3_halo_tiles(g), gp);
}

bool conv3x3_wino_bn128(int N, const EpiArg& ep) {
  return N % 128 == 0 && !(ep.mode == SELUNET_EP_SPLIT && ep.split % 128 != 0);
}

int conv3x3_wino_launch(const GatherArg& g, const float* u, int N, const EpiArg& ep, hipStream_t st) {
  if (conv3x3_wino_bn128(N, ep)) launch_wino<128, 1>(g, u, N, ep, st);
  else launch_wino<64, 2>(g, u, N, ep, st);
  return check_launch("conv3x3_wino");
}

bool conv3x3_x2_shape_ok(int h, int w, int c_in, int c_src0, int n_cols) {
  return persist_enabled() && h >= TH && w >= TW && c_in % 32 == 0 && c_src0 % 32 == 0 && c_in > 32 &&
         n_cols % 64 == 0;
}

bool conv3x3_x2_eligible(const GatherArg& g, int N) {
  return conv3x3_halo_eligible(g, N, SELUNET_F32) && conv3x3_halo_persistent(g, SELUNET_F32) &&
         conv3x3_x2_shape_ok(g.h, g.w, g.Ctot, g.src[0].C, N);
}

// SELUNET_OPT_TILE_QUEUE: the split-fp16 persistent kernel takes its pixel tiles from a ticket counter
// (conv3x3_halo_persist_kernel, TQ) and flushes statistics per tile (slab rows = pixel tiles)
bool x2_tile_queue() { return (option(SELUNET_OPT_TILE_QUEUE, 0) & 1) != 0; }

// the queue's counters: [2][n_tiles <= 64] per device, zero between launches (each launch's last workgroups
// reset them). Allocated by selunet_set_option(SELUNET_OPT_TILE_QUEUE, > 0) on the current device — outside
// any stream capture — or on first use when the launch stream is not capturing. One launch in flight per
// device: the engine issues the persistent convolutions on one compute stream, so launches never overlap.
static unsigned* g_tq[64] = {};

int x2_tile_queue_prepare() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
  if (g_tq[dev] != nullptr) return 0;
  unsigned* p = nullptr;
  if (hipMalloc(&p, 128 * sizeof(unsigned)) != hipSuccess) return -1;
  if (hipMemset(p, 0, 128 * sizeof(unsigned)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    return -1;
  }
  g_tq[dev] = p;
  return 0;
}

static unsigned* tq_counters(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (g_tq[dev] == nullptr) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    if (x2_tile_queue_prepare() != 0) return nullptr;
  }
  return g_tq[dev];
}

// statistics slab rows of selunet_conv3x3_x2 (persistent kernel): workgroups per column tile, or pixel tiles
int64_t conv3x3_x2_persist_rows(const GatherArg& g, int N) {
  if (conv3x3_x2p_eligible(g, N)) return conv3x3_x2p_rows(g, N);
  return x2_tile_queue() ? conv3x3_halo_tiles(g) : persist_rows(g, N);
}

template <int BN>
static int launch_x2(const GatherArg& g, const float* w, int N, const EpiArg& ep, const float* amax0,
                     const float* amax1, hipStream_t st) {
  const int tiles_x = (int)cdiv(g.w, TW), tiles_y = (int)cdiv(g.h, TH);
  const int n_tiles = N / BN;
  const int gp = persist_rows(g, N);  // workgroups per column tile (static: = the statistics slab rows)
  const int k_pad = 9 * g.Ctot;
  // 16x16x32 MFMAs at BN = 64 (1-4 % faster per layer); at BN = 128 they cost 20-25 % (the extra
  // fragment registers spill: 180 B of scratch per lane against 44) — DESIGN.md §3
  if (x2_tile_queue()) {
    unsigned* tq = tq_counters(st);
    if (tq == nullptr || n_tiles > 64)
      return fail(SELUNET_ELAUNCH, "conv3x3_x2: tile-queue counters unavailable (set SELUNET_OPT_TILE_QUEUE "
                                   "before capturing the step)");
    hipLaunchKernelGGL((conv3x3_halo_persist_kernel<float, BN, true, BN == 64, true>), dim3((unsigned)(gp * n_tiles)),
                       dim3(HTHREADS), 0, st, g, w, N, k_pad, ep, n_tiles, tiles_x, tiles_y,
                       (int)conv3x3_halo_tiles(g), gp, w + (int64_t)N * k_pad, amax0, amax1, tq);
    return 0;
  }
  hipLaunchKernelGGL((conv3x3_halo_persist_kernel<float, BN, true, BN == 64>), dim3((unsigned)(gp * n_tiles)),
                     dim3(HTHREADS), 0, st, g, w, N, k_pad, ep, n_tiles, tiles_x, tiles_y, (int)conv3x3_halo_tiles(g),
                     gp, w + (int64_t)N * k_pad, amax0, amax1, nullptr);
  return 0;
}

// 128-column tiles whenever N allows: unlike the Winograd kernel's register output transform, the
// LDS-staged epilogue routes each column to its SPLIT output itself, so a tile may straddle the split
// (decoder_layer_1_2's data gradient, split at 64: one pass over its halo instead of two, 4.5 -> 3.x ms)
bool conv3x3_x2_bn128(int N, const EpiArg& ep) {
  return N % 128 == 0 && !(ep.mode == SELUNET_EP_SPLIT && ep.split % 8 != 0);
}

int conv3x3_x2_launch(const GatherArg& g, const float* w, int N, const EpiArg& ep, const float* amax0,
                      const float* amax1, hipStream_t st) {
  if (conv3x3_x2d_eligible(g, N)) return conv3x3_x2d_launch(g, w, ep, amax0, amax1, st);  // 64 columns
  if (conv3x3_x2p_eligible(g, N)) return conv3x3_x2p_launch(g, w, N, ep, amax0, amax1, st);  // 128, two per CU
  if (int rc = conv3x3_x2_bn128(N, ep) ? launch_x2<128>(g, w, N, ep, amax0, amax1, st)
                                       : launch_x2<64>(g, w, N, ep, amax0, amax1, st))
    return rc;
  return check_launch("conv3x3_x2");
}

int conv3x3_halo_launch(const GatherArg& g, const void* b, int N, int k_pad, const EpiArg& ep, int dtype,
                        hipStream_t st) {
  // single-chunk layers use 64-column tiles: LDS for two workgroups per CU
  const bool one = halo_one_chunk(g, dtype);
  const bool bn128 = !one && N % 128 == 0 && !(ep.mode == SELUNET_EP_SPLIT && ep.split % 128 != 0);
  if (dtype == SELUNET_F32) {
    if (bn128) launch_halo<float, 128>(g, b, N, k_pad, ep, st);
    else launch_halo<float, 64>(g, b, N, k_pad, ep, st);
  } else {
    if (bn128) launch_halo<__bf16, 128>(g, b, N, k_pad, ep, st);
    else launch_halo<__bf16, 64>(g, b, N, k_pad, ep, st);
  }
  return check_launch("conv3x3_halo");
}

}  // namespace selunet

extern "C" int32_t selunet_set_halo_workgroups(int32_t wgs) {
  const int prev = selunet::PERSIST_WGS;
  selunet::PERSIST_WGS = wgs > 0 ? wgs : selunet::PERSIST_WGS_DEFAULT;
  return prev;
}
