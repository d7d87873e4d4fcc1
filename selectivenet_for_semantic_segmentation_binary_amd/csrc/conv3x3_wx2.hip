// fp32 3x3 convolution (model.py:11) forward / data gradient on split-fp16 operands as a 1-D Winograd
// F(2,3) along x (selunet_conv3x3_wx2): for kernel row dy and the output pair (x, x+1)
//   y(x) = (M0 + M1) + M2,   y(x+1) = (M1 - M2) - M3,   M_xi = sum_c U_xi[dy][c] * V_xi[c]
// with V = (d0 - d2, d1 + d2, d2 - d1, d1 - d3) of the inputs d_j at x - 1 + j (row y + dy - 1) and
// U = (g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2) of the kernel row. Four products per pair and
// kernel row instead of six: 2/3 of the split-fp16 MFMAs of conv3x3_halo_persist_kernel<float, BN, X2>.
//
// Every V is formed once per (tile, 16-channel chunk) in fp32 from the BN+ReLU-transformed input,
// scaled by 2^e and split (h = fp16(v), l = fp16(v - h)) into LDS planes, so the MFMA loop reads
// ready fragments exactly as the direct kernel reads its halo; U comes split from
// selunet_pack_weights (SELUNET_PACK_CONV3X3_WX2). Each 32x32 accumulator takes three
// v_mfma_f32_32x32x16_f16 (h*l, l*h, h*h) per 16-channel step.
//
// Workgroup: 512 threads, one per CU, persistent over the output tiles prow, prow + gp, ... of one
// BN-column tile (as the direct kernel: statistics in registers, one slab row per workgroup). Tile
// 16 x 16 px = 128 output pairs. The 8 waves split plane groups x pairs x columns: wave w holds the
// accumulators of planes {0, 1} or {2, 3} (w & 1) for 64 pairs x 64 columns at BN = 128 (2 planes x
// 2 x 2 subtiles = 128 accumulator registers) or 32 pairs x 64 columns at BN = 64; the four planes
// of a pair meet in the LDS epilogue.
// A step is (kernel row dy, s): the waves of group wp multiply plane 2 wp + s, so a step stages the
// weights of two planes (16 KiB) and each wave reads 8 fragments for 12 MFMAs (the direct kernel's
// ratio); six steps per 16-channel chunk.
//
// Per chunk c of tile i (job J) the six steps t also stage job J + 1:
//   t = 0: the BN coefficients of job J + 1 (loaded into a register at the previous job's t = 3) -> LDS;
//   t = 2: the raw fp32 halo of job J + 1 (loaded into registers at the previous job's t = 3),
//          BN+ReLU applied, zero outside the image -> the raw LDS tile;
//   t = 3: the raw halo and coefficients of job J + 2 -> registers;
//   t = 4, 5: raw tile -> the four split V planes of job J + 1 (the other V buffer).
// The weights of step S + 1 are loaded during step S - 1 and stored to the other weight buffer after
// step S's MFMAs (one step of load distance left the MFMAs waiting for L2: 5-50 % slower than the direct
// kernel). At a tile's last chunk the V planes and weights of the next tile wait for the LDS-staged
// epilogue (which spans the V and weight buffers; the raw tile and coefficients sit above it).
#include "gemm_common.h"

namespace selunet {

constexpr int WX_TH = 16, WX_TW = 16;           // output tile (pixels)
constexpr int WX_HH = 18, WX_HW = 18;           // halo tile
constexpr int WX_HPIX = WX_HH * WX_HW;          // 324
constexpr int WX_THREADS = 512;
constexpr int WX_CK = 16;                       // channels per chunk
constexpr int WX_VROW = 64;                     // V row: 16 h + 16 l fp16 (four 16-B units)
constexpr int WX_VPLANE = WX_HH * 8 * WX_VROW;  // one plane: 18 halo rows x 8 pairs
constexpr int WX_VBUF = 4 * WX_VPLANE;          // four planes (36 KiB)
constexpr int WX_RAW = WX_HPIX * 64;            // raw fp32 halo of one chunk (20.25 KiB)
constexpr int WX_RAW_ROUNDS = (WX_HPIX * 4 + WX_THREADS - 1) / WX_THREADS;  // 16-B loads per thread: 3
constexpr int WX_SLOTS = WX_HH * 8 * 4;         // V-forming slots (halo row, pair, 4 channels): 576

// 16-B unit u of V row (hy, pair px2) lives at unit u ^ swizzle: the 16 lanes of a ds_read_b128 lane
// group (pairs of tile rows py..py+3, MFMA rows 0-3, 12-15, 20-27) then hit 16 distinct bank slots
__device__ __forceinline__ int wx_vswz(int hy, int px2) { return (2 * hy + (px2 >> 2)) & 3; }
// weight row (plane, column col): unit u at u ^ ((col >> 2) & 3), conflict-free for the B fragments
__device__ __forceinline__ int wx_bswz(int col) { return (col >> 2) & 3; }

template <int BN>
__global__ void __launch_bounds__(WX_THREADS, 1)
conv3x3_wx2_kernel(GatherArg g, const unsigned char* __restrict__ W, int N, EpiArg ep, int n_tiles, int tiles_x,
                   int tiles_y, int ptiles, int gp, const float* __restrict__ wcs, const float* __restrict__ amax0,
                   const float* __restrict__ amax1) {
  static_assert(BN == 128 || BN == 64, "64- or 128-column tiles");
  constexpr int WN_ = BN / 64;                  // column-wave groups
  constexpr int WM_ = 4 / WN_;                  // pair-wave groups
  constexpr int MT = 4 / WM_;                   // 32-pair subtiles per wave (2 at BN = 128)
  constexpr int STEPS = 6;                      // (dy, s) per chunk
  constexpr int BBUF = 2 * BN * WX_VROW;        // one step's weights: 2 planes x BN columns
  constexpr int B_ROUNDS = BBUF / 16 / WX_THREADS;
  static_assert(B_ROUNDS * 16 * WX_THREADS == BBUF, "weight rows split evenly over the threads");
  constexpr int OFF_B = 2 * WX_VBUF;
  constexpr int SMEM_EPI = WX_TH * WX_TW * (BN + 4) * 4;
  // statistics registers: fp32 at BN = 128 (as the direct kernel: fp64 ones would not fit its registers),
  // fp64 at BN = 64 (the full-resolution layers, ~128 tiles folded into each thread's sums)
  using Acc = std::conditional_t<BN == 128, float, double>;
  constexpr int FLUSH = stats_flush_bytes<BN, WX_THREADS, Acc>();
  constexpr int LOW = SMEM_EPI > FLUSH ? SMEM_EPI : FLUSH;  // the epilogue tile / statistics scratch
  constexpr int OFF_RAW = (OFF_B + 2 * BBUF > LOW ? OFF_B + 2 * BBUF : LOW);  // raw halo above both
  constexpr int OFF_SS = OFF_RAW + WX_RAW;
  constexpr int SMEM = OFF_SS + 4 * WX_CK * 4;  // (coefficients + a sink for the other threads' writes)
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  unsigned char* Vs = smem;
  unsigned char* Bs = smem + OFF_B;
  unsigned char* Raw = smem + OFF_RAW;
  float* Ss = reinterpret_cast<float*>(smem + OFF_SS);  // [16] scale, [16] shift of the staged chunk

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wp = wave & 1;                       // planes 2 wp, 2 wp + 1
  const int wm = (wave >> 1) % WM_, wn = (wave >> 1) / WM_;
  const int half = lane >> 5, l32 = lane & 31;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int n_tile = lb % n_tiles;
  const int prow = lb / n_tiles;
  const int n0 = n_tile * BN;
  const int ntl = prow < ptiles ? (ptiles - prow + gp - 1) / gp : 0;
  const int nchunks = g.Ctot / WX_CK;
  const int csteps = nchunks * STEPS;
  const int njobs = ntl * nchunks;
  const int64_t wrow = (int64_t)g.Ctot * 48;     // packed row bytes: 12 * Ctot values x (h, l)

  float xs, inv;
  {
    float am = amax0 ? amax0[0] : 0.0f;
    if (g.nsrc > 1 && amax1) am = fmaxf(am, amax1[0]);
    xs = x2_scale(am, &inv);
  }
  float cfac[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) cfac[b] = wcs[n0 + wn * 64 + b * 32 + l32] * inv;

  auto tile_xy = [&](int i, int& img, int& y0, int& x0) __attribute__((always_inline)) {
    const unsigned pt = (unsigned)(prow + i * gp);
    const unsigned r = pt / (unsigned)tiles_x;
    x0 = (int)(pt - r * (unsigned)tiles_x) * WX_TW;
    const unsigned r2 = r / (unsigned)tiles_y;
    y0 = (int)(r - r2 * (unsigned)tiles_y) * WX_TH;
    img = (int)r2;
  };
  auto chunk_src = [&](int chunk, int& c) -> SrcArg {
    c = chunk * WX_CK;
    const bool s1 = g.nsrc > 1 && c >= g.src[0].C;
    if (s1) c -= g.src[0].C;
    return pick_src(g, s1 ? 1 : 0);
  };

  // ---------------------------------------------------------------- weights
  // packed row: 16-channel block (chunk, dy) holds planes in the order 0, 2, 1, 3, so the two planes
  // of step (dy, s) — s (waves wp = 0) and 2 + s (wp = 1) — are 128 contiguous bytes at step * 128
  struct BRegs {
    uint4 v[B_ROUNDS];
  };
  // (staging address math is recomputed from an opaque copy of tid at every use: hoisted out of the
  // chunk loop it stays live through the MFMA steps and spills)
  auto b_load = [&](int st) __attribute__((always_inline)) {  // st: step within a tile (chunk * 6 + t)
    BRegs rb;
    int tq = tid;
    asm volatile("" : "+v"(tq));
#pragma unroll
    for (int r = 0; r < B_ROUNDS; ++r) {
      const int idx = r * WX_THREADS + tq;
      const int col = idx >> 3, u8 = idx & 7;
      rb.v[r] = *reinterpret_cast<const uint4*>(W + (int64_t)(n0 + col) * wrow + (int64_t)st * 128 + u8 * 16);
    }
    return rb;
  };
  auto b_store = [&](const BRegs& rb, int buf) __attribute__((always_inline)) {
    int tq = tid;
    asm volatile("" : "+v"(tq));
#pragma unroll
    for (int r = 0; r < B_ROUNDS; ++r) {
      const int idx = r * WX_THREADS + tq;
      const int col = idx >> 3, u8 = idx & 7;
      const int pl = u8 >> 2, u = u8 & 3;
      *reinterpret_cast<uint4*>(Bs + buf * BBUF + ((pl * BN + col) * 4 + (u ^ wx_bswz(col))) * 16) = rb.v[r];
    }
  };

  // ---------------------------------------------------------------- raw halo (16-B slice per round)
  // slice hidx = r * 512 + tid: halo pixel hidx >> 2, channels 4 (hidx & 3) .. + 3 (= 4 (tid & 3))
  const int rcc = tid & 3;
  struct RawRegs {
    uint4 v[WX_RAW_ROUNDS];
  };
  auto raw_load = [&](int job) __attribute__((always_inline)) {
    RawRegs rr;
    int img, y0, x0, c;
    tile_xy(job / nchunks, img, y0, x0);
    const SrcArg sa = chunk_src(job % nchunks, c);
    int tq = tid;
    asm volatile("" : "+v"(tq));
#pragma unroll
    for (int r = 0; r < WX_RAW_ROUNDS; ++r) {
      const int hp = min((r * WX_THREADS + tq) >> 2, WX_HPIX - 1);
      const int hy = hp / WX_HW, hx = hp - hy * WX_HW;
      const int ys = min(max(y0 - 1 + hy, 0), g.h - 1), xq = min(max(x0 - 1 + hx, 0), g.w - 1);
      rr.v[r] = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(sa.data) +
                                                (((int64_t)img * g.h + ys) * g.w + xq) * sa.C + c + (tq & 3) * 4);
    }
    return rr;
  };
  // BN + ReLU of the chunk's source (coefficients sc/sh for this thread's 4 channels, or none), zero
  // outside the image, to the raw LDS tile
  auto raw_store = [&](const RawRegs& rr, int job, bool tr, const float* sc, const float* sh, int relu)
      __attribute__((always_inline)) {
    int img, y0, x0;
    tile_xy(job / nchunks, img, y0, x0);
    int tq = tid;
    asm volatile("" : "+v"(tq));
    // branch-free (one basic block with the MFMAs of the step): slices past the halo repeat the last pixel
    // (the same value its owner writes); without a transform the coefficients are 1 / 0 (coef_load)
    const float lo = tr && relu ? 0.0f : -__builtin_huge_valf();
#pragma unroll
    for (int r = 0; r < WX_RAW_ROUNDS; ++r) {
      const int hp = min((r * WX_THREADS + tq) >> 2, WX_HPIX - 1);
      const int hy = hp / WX_HW, hx = hp - hy * WX_HW;
      const bool in = (unsigned)(y0 - 1 + hy) < (unsigned)g.h && (unsigned)(x0 - 1 + hx) < (unsigned)g.w;
      f32x4 v;
      __builtin_memcpy(&v, &rr.v[r], 16);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = in ? fmaxf(v[e] * sc[e] + sh[e], lo) : 0.0f;
      *reinterpret_cast<f32x4*>(Raw + hp * 64 + (tq & 3) * 16) = v;
    }
  };
  // raw LDS tile -> the four split V planes of V buffer vb (x2 scale xs): slots [s0, s1) of the 576
  auto form_v = [&](int vb, int s0, int s1) __attribute__((always_inline)) {
    int tq = tid;
    asm volatile("" : "+v"(tq));
    for (int s = s0 + tq; s < s1; s += WX_THREADS) {
      const int cg = s & 3, px2 = (s >> 2) & 7, hy = s >> 5;
      const unsigned char* rp = Raw + (hy * WX_HW + 2 * px2) * 64 + cg * 16;
      const f32x4 d0 = *reinterpret_cast<const f32x4*>(rp);
      const f32x4 d1 = *reinterpret_cast<const f32x4*>(rp + 64);
      const f32x4 d2 = *reinterpret_cast<const f32x4*>(rp + 128);
      const f32x4 d3 = *reinterpret_cast<const f32x4*>(rp + 192);
      f32x4 v[4];
      v[0] = d0 - d2;
      v[1] = d1 + d2;
      v[2] = d2 - d1;
      v[3] = d1 - d3;
      const int sw = wx_vswz(hy, px2);
      unsigned char* row = Vs + vb * WX_VBUF + (hy * 8 + px2) * WX_VROW + (cg & 1) * 8;
#pragma unroll
      for (int xi = 0; xi < 4; ++xi) {
        f16x4 h, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          _Float16 a, b;
          x2_split(v[xi][e] * xs, a, b);
          h[e] = a;
          l[e] = b;
        }
        *reinterpret_cast<f16x4*>(row + xi * WX_VPLANE + ((cg >> 1) ^ sw) * 16) = h;
        *reinterpret_cast<f16x4*>(row + xi * WX_VPLANE + ((2 + (cg >> 1)) ^ sw) * 16) = l;
      }
    }
  };

  auto form_slot = [&](int vb, int s) __attribute__((always_inline)) {
    const int cg = s & 3, px2 = (s >> 2) & 7, hy = s >> 5;
    const unsigned char* rp = Raw + (hy * WX_HW + 2 * px2) * 64 + cg * 16;
    const f32x4 d0 = *reinterpret_cast<const f32x4*>(rp);
    const f32x4 d1 = *reinterpret_cast<const f32x4*>(rp + 64);
    const f32x4 d2 = *reinterpret_cast<const f32x4*>(rp + 128);
    const f32x4 d3 = *reinterpret_cast<const f32x4*>(rp + 192);
    f32x4 v[4];
    v[0] = d0 - d2;
    v[1] = d1 + d2;
    v[2] = d2 - d1;
    v[3] = d1 - d3;
    const int sw = wx_vswz(hy, px2);
    unsigned char* row = Vs + vb * WX_VBUF + (hy * 8 + px2) * WX_VROW + (cg & 1) * 8;
#pragma unroll
    for (int xi = 0; xi < 4; ++xi) {
      f16x4 h, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        _Float16 a, b;
        x2_split(v[xi][e] * xs, a, b);
        h[e] = a;
        l[e] = b;
      }
      *reinterpret_cast<f16x4*>(row + xi * WX_VPLANE + ((cg >> 1) ^ sw) * 16) = h;
      *reinterpret_cast<f16x4*>(row + xi * WX_VPLANE + ((2 + (cg >> 1)) ^ sw) * 16) = l;
    }
  };
  const int wv = __builtin_amdgcn_readfirstlane(wave);

  // ---------------------------------------------------------------- MFMA step (dy, s)
  int vrow0[MT], vsw0[MT];
#pragma unroll
  for (int a = 0; a < MT; ++a) {
    const int pr = wm * 32 * MT + a * 32 + l32;  // the lane's pair (MFMA row) in subtile a
    const int py = pr >> 3, px2 = pr & 7;
    vrow0[a] = py * 8 + px2;
    vsw0[a] = wx_vswz(py, px2);
  }
  f32x16 acc[2][MT][2];  // (zeroed at each tile's first chunk)

  auto mma_step = [&](int vb, int bb, int t) __attribute__((always_inline)) {
    const int dy = t >> 1, sp = t & 1;
    const int xi = 2 * wp + sp;
    f16x8 ah[MT], al[MT], bh[2], bl[2];
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const unsigned char* r = Vs + vb * WX_VBUF + xi * WX_VPLANE + (vrow0[a] + dy * 8) * WX_VROW;
      const int sw = (vsw0[a] + 2 * dy) & 3;
      ah[a] = *reinterpret_cast<const f16x8*>(r + (half ^ sw) * 16);
      al[a] = *reinterpret_cast<const f16x8*>(r + ((2 + half) ^ sw) * 16);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int col = wn * 64 + b * 32 + l32;
      const unsigned char* r = Bs + bb * BBUF + (wp * BN + col) * WX_VROW;
      const int sw = wx_bswz(col);
      bh[b] = *reinterpret_cast<const f16x8*>(r + (half ^ sw) * 16);
      bl[b] = *reinterpret_cast<const f16x8*>(r + ((2 + half) ^ sw) * 16);
    }
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        f32x16& c = acc[sp][a][b];
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bl[b], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a], bh[b], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bh[b], c, 0, 0, 0);
      }
  };

  // coefficient register of job `job` (threads < 32: scale for tid < 16, shift above), 0 without BN
  auto coef_load = [&](int job) __attribute__((always_inline)) -> float {
    int c;
    const SrcArg sa = chunk_src(job % nchunks, c);
    const bool has = sa.scale != nullptr;
    const float* p = has ? ((tid & WX_CK) ? sa.shift : sa.scale) + c : wcs;  // (wcs: any valid address)
    const float v = p[tid & (WX_CK - 1)];
    return has ? v : ((tid & WX_CK) ? 0.0f : 1.0f);
  };

  // ---------------------------------------------------------------- prologue: job 0 -> V buffer 0
  if (njobs > 0) {
    int c0;
    const SrcArg sa = chunk_src(0, c0);
    float sc[4] = {1, 1, 1, 1}, sh[4] = {0, 0, 0, 0};
    if (sa.scale) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc[e] = sa.scale[c0 + rcc * 4 + e];
        sh[e] = sa.shift[c0 + rcc * 4 + e];
      }
    }
    raw_store(raw_load(0), 0, sa.scale != nullptr, sc, sh, sa.relu);
  }
  b_store(b_load(0), 0);
  BRegs rb_next = b_load(1);  // weights two steps ahead: loaded at step S - 1, stored after step S's MFMAs
  __syncthreads();
  if (njobs > 0) form_v(0, 0, WX_SLOTS);
  RawRegs ra = raw_load(njobs > 1 ? 1 : 0);
  float creg = coef_load(njobs > 1 ? 1 : 0);
  __syncthreads();

  Acc s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float amx = 0.0f;
  const TileStats ts = tile_stats(ep, prow, n0, N);
  float* tile = reinterpret_cast<float*>(smem);
  int J = 0, S = 0;
  for (int i = 0; i < ntl; ++i) {
    int img, y0, x0;
    tile_xy(i, img, y0, x0);
    BRegs rb_hold;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[p][a][b] = f32x16{};
    for (int c = 0; c < nchunks; ++c, ++J) {
      const bool has_next = J + 1 < njobs;
      const bool defer = c + 1 == nchunks && has_next;  // next job = next tile: V / weights after the epilogue
      int cn;
      const SrcArg sn = chunk_src((J + 1) % nchunks, cn);
#pragma unroll
      for (int t = 0; t < STEPS; ++t) {
        const int st = c * STEPS + t;
        const int st2 = st + 2;
        const BRegs rb_far = b_load(st2 < csteps ? st2 : st2 - csteps);  // (the next tile's steps wrap)
        // staging without branches (so the scheduler can place it among the step's MFMAs): past the
        // last job it stages harmless copies; at a tile's last chunk the V planes / weights it writes are
        // overwritten by the epilogue and staged again after it (rb_hold, form_v below)
        if (t == 0) Ss[tid < 2 * WX_CK ? tid : 2 * WX_CK + (tid & (2 * WX_CK - 1))] = creg;
        mma_step(J & 1, S & 1, t);
        if (t == 2) raw_store(ra, J + 1, sn.scale != nullptr, Ss + rcc * 4, Ss + WX_CK + rcc * 4, sn.relu);
        if (t == 3) {
          const int jn = J + 2 < njobs ? J + 2 : J;
          ra = raw_load(jn);
          creg = coef_load(jn);
        }
        // (slots 0-511 at t = 4, the last 64 — wave 7 — at t = 5)
        if (t == 4) form_slot((J + 1) & 1, tid);
        if (t == 5 && wv == 7) form_slot((J + 1) & 1, WX_THREADS + lane);
        if (t == STEPS - 1) rb_hold = rb_next;
        b_store(rb_next, (S + 1) & 1);
        __syncthreads();
        rb_next = rb_far;
        ++S;
      }
    }

    // ------------------------------------------------------------ epilogue of tile i
    // unscale, then the output transform across the two plane groups: waves of planes {0, 1} write
    // (M0 + M1, M1) at the pair's two pixels, waves of planes {2, 3} add M2 / subtract M2 and M3
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (wp == pass) {
#pragma unroll
        for (int a = 0; a < MT; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int col = wn * 64 + b * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int pr = wm * 32 * MT + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
              const int e = (pr >> 3) * WX_TW + 2 * (pr & 7);
              float* t0 = tile + e * (BN + 4) + col;
              float* t1 = t0 + (BN + 4);
              const float ma = acc[0][a][b][r] * cfac[b], mb = acc[1][a][b][r] * cfac[b];
              if (pass == 0) {
                *t0 = ma + mb;  // M0 + M1
                *t1 = mb;       // M1
              } else {
                *t0 = *t0 + ma;         // (M0 + M1) + M2
                *t1 = (*t1 - ma) - mb;  // (M1 - M2) - M3
              }
            }
          }
      }
      __syncthreads();
    }
    auto dst = [&](int pix, int cl) -> float* {
      const int y = y0 + pix / WX_TW, x = x0 + pix % WX_TW;
      if (y >= g.h || x >= g.w) return nullptr;
      const int64_t m = ((int64_t)img * g.h + y) * g.w + x;
      const int col = n0 + cl;
      if (ep.mode == SELUNET_EP_SPLIT)
        return col < ep.split ? reinterpret_cast<float*>(ep.out0) + m * ep.split + col
                              : reinterpret_cast<float*>(ep.out1) + m * (N - ep.split) + (col - ep.split);
      return reinterpret_cast<float*>(ep.out0) + m * N + col;
    };
    auto bias_col = [&](int cl) { return n0 + cl; };
    lds_tile_store_acc<float, WX_TH * WX_TW, BN, WX_THREADS>(tile, tid, dst, ep.bias, bias_col, ts, s1, s2, s3, amx);
    if (i + 1 < ntl) {
      __syncthreads();  // the tile has been read: LDS back to V planes / weights
      form_v(J & 1, 0, WX_SLOTS);  // (J is the next tile's first job; its raw halo was staged at t = 2)
      b_store(rb_hold, S & 1);
      __syncthreads();
    }
  }
  tile_stats_flush<BN, WX_THREADS>(tile, tid, ts, s1, s2, s3, amx);
}

int64_t conv3x3_persist_rows(const GatherArg& g, int N);

bool conv3x3_wx2_shape_ok(int h, int w, int c_in, int c_src0, int n_cols) {
  return h >= WX_TH && w >= WX_TW && w % 2 == 0 && c_in % WX_CK == 0 &&
         c_src0 % WX_CK == 0 && c_in >= 64 && c_in <= 512 && n_cols % 64 == 0;
}

int conv3x3_wx2_launch(const GatherArg& g, const float* w, int N, const EpiArg& ep, const float* amax0,
                       const float* amax1, hipStream_t st) {
  const int tiles_x = (int)cdiv(g.w, WX_TW), tiles_y = (int)cdiv(g.h, WX_TH);
  const bool bn128 = conv3x3_x2_bn128(N, ep);
  const int n_tiles = N / (bn128 ? 128 : 64);
  // = the statistics slab rows of selunet_conv3x3_x2_stats_rows
  const int gp = (int)(conv3x3_x2d_eligible(g, N) ? conv3x3_x2d_rows(g) : conv3x3_persist_rows(g, N));
  const int ptiles = (int)((int64_t)g.n * tiles_x * tiles_y);
  const int64_t kw = (int64_t)12 * g.Ctot;       // 32-bit words per packed row
  auto kern = bn128 ? conv3x3_wx2_kernel<128> : conv3x3_wx2_kernel<64>;
  hipLaunchKernelGGL(kern, dim3((unsigned)(gp * n_tiles)), dim3(WX_THREADS), 0, st, g,
                     reinterpret_cast<const unsigned char*>(w), N, ep, n_tiles, tiles_x, tiles_y, ptiles, gp,
                     w + (int64_t)N * kw, amax0, amax1);
  return check_launch("conv3x3_wx2");
}

}  // namespace selunet
