// fp32 3x3 convolution (model.py:11) forward / data gradient on split-fp16 operands for the 128-column layers
// (every CBR block from encoder_layer_2_1 to decoder_layer_2_1: K = 9 x 64 .. 9 x 512): the arithmetic of
// conv3x3_halo_persist_kernel<float, 128, X2> — the halo staged in LDS as fp16 high / low parts of the
// BN+ReLU-transformed, 2^e-scaled source, three v_mfma_f32_32x32x16_f16 (hl, lh, hh) per 32x32 subtile, tap and
// 16-channel k-step, k ascending — in a workgroup half its size, two per CU.
//
// The one-workgroup-per-CU kernel (8 waves, 64 x 64 per wave) leaves the MFMA pipe idle while all of its waves
// wait at the per-tap barriers, read their first fragments after each barrier, stage the next halo and run the
// LDS-staged epilogue (mfma_busy 0.57). Here:
//  * 256 threads = 4 waves, one per SIMD; wave w computes tile rows 4w..4w+3 (64 pixels) x all 128 columns:
//    2 x 4 subtiles, 128 accumulator registers; per k-step 4 halo and 8 weight fragment reads for 24 MFMAs
//    (0.5 ds_read_b128 per MFMA instead of 0.67: a quarter fewer LDS bytes per product);
//  * a job is (tile, 16-channel chunk); a step is (job, tap): one k-step, one barrier. 71 KB of LDS: two halo
//    buffers (324 x 64 B) and two weight buffers (128 x 64 B), both with their 16-B slots XOR-swizzled so
//    every ds_read_b128 lane group hits 16 distinct bank slots (halo: slot ^ (2 (hp >> 2) + hp / 18) & 3,
//    weights: slot ^ (row >> 2) & 3; found by search over the lane groups of the MI355X guide's LDS table and
//    the nine tap offsets) — two workgroups per CU, so one's barriers, staging and epilogue run under the
//    other's MFMAs;
//  * weights by LDS-DMA (global_load_lds_dwordx4, lane-linear images, the swizzle applied through the per-lane
//    source address), one step ahead; counted s_waitcnt vmcnt + raw s_barrier (no drain of the halo loads);
//  * the next job's halo, one 16-B slice per thread and tap over taps 0-5, is transformed, split and written to
//    the free halo buffer two taps after its load (the next tile's first job too: the epilogue leaves it alone);
//  * the epilogue stages the tile in four 32-column quarters (lds_tile_store_acc of the other kernels: statistics,
//    BN-backward sums, column sums, SPLIT outputs, range word); the per-tile statistics partials are reduced in
//    a fixed order into fp64 column accumulators in LDS (no statistics registers through the main loop).
// Persistent over the pixel tiles of its column tile (static walk prow, prow + gp, ...; slab rows = gp =
// min(tiles, 512 / column tiles), selunet_conv3x3_x2_stats_rows).
#include "gemm_common.h"

namespace selunet {

constexpr int XP_TH = 16, XP_TW = 16, XP_HW = 18, XP_HPIX = 324;
constexpr int XP_THREADS = 256;
constexpr int XP_BN = 128;
constexpr int XP_CK = 16;                                               // fp32 channels per job
constexpr int XP_ROWB = 64;                                             // halo / weight row bytes (h 32, l 32)
constexpr int XP_A_ROUNDS = (XP_HPIX * 4 + XP_THREADS - 1) / XP_THREADS;  // 16-B halo slices per thread: 6
constexpr int XP_HBUF = XP_HPIX * XP_ROWB;                              // 20736
constexpr int XP_BBUF = XP_BN * XP_ROWB;                                // 8192
constexpr int XP_NB = 3;                                                // weight buffers (DMA two steps ahead)
// [halo 0 | weights 0-2 | halo 1]: the halo buffer of a tile's last job and the weights are contiguous either
// way, and the epilogue stages its quarters there while the next tile's first halo waits in the other buffer
constexpr int XP_OFF_B = XP_HBUF;                                       // 20736
constexpr int XP_OFF_H1 = XP_OFF_B + XP_NB * XP_BBUF;                   // 45312
constexpr int XP_EPI_TC = 32;                                           // epilogue quarter: 32 columns
constexpr int XP_EPI = XP_TH * XP_TW * (XP_EPI_TC + 4) * 4;              // 36864
constexpr int XP_OFF_S = XP_OFF_H1 + XP_HBUF;                           // [2 jobs][scale 16, shift 16]
constexpr int XP_OFF_ACC = XP_OFF_S + 2 * 2 * XP_CK * 4;                // fp64 [3][128] column statistics
constexpr int XP_SMEM = XP_OFF_ACC + 3 * XP_BN * 8;                     // 69376
constexpr int XP_RS = XP_THREADS / (XP_EPI_TC / 8);                     // epilogue rows per pass: 64

// physical 16-B slot of logical slot s in halo row hp / weight row r (involutions)
__device__ __forceinline__ int xp_hslot(int hp, int s) { return s ^ ((2 * (hp >> 2) + hp / XP_HW) & 3); }
__device__ __forceinline__ int xp_wslot(int r, int s) { return s ^ ((r >> 2) & 3); }

__global__ void __launch_bounds__(XP_THREADS, 2)
conv3x3_x2p_kernel(GatherArg g, const float* __restrict__ B, int N, int k_pad, EpiArg ep, int n_tiles, int tiles_x,
                   int tiles_y, int ptiles, int gp, const float* __restrict__ wcs, const float* __restrict__ amax0,
                   const float* __restrict__ amax1) {
  static_assert(XP_EPI <= XP_HBUF + XP_NB * XP_BBUF, "the epilogue quarter fits a halo buffer and the weights");
  static_assert(XP_RS * XP_EPI_TC * 3 * 4 <= XP_EPI, "statistics partials exceed the tile");
  __shared__ __attribute__((aligned(16))) unsigned char smem[XP_SMEM];
  unsigned char* As = smem;
  unsigned char* Bs = smem + XP_OFF_B;
  float* Ss = reinterpret_cast<float*>(smem + XP_OFF_S);      // [2 jobs][scale 16, shift 16]
  double* Sacc = reinterpret_cast<double*>(smem + XP_OFF_ACC);  // [3][128]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = lane >> 5, l32 = lane & 31;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int n_tile = (int)(lb % (unsigned)n_tiles);
  const int prow = (int)(lb / (unsigned)n_tiles);
  const int n0 = n_tile * XP_BN;
  const int nchunks = g.Ctot / XP_CK;
  const int ntl = prow < ptiles ? (ptiles - prow + gp - 1) / gp : 0;
  const int csteps = nchunks * 9;
  const int njobs = ntl * nchunks;

  float xs, inv;
  {
    float am = amax0 ? amax0[0] : 0.0f;
    if (g.nsrc > 1 && amax1) am = fmaxf(am, amax1[0]);
    xs = x2_scale(am, &inv);
  }
  for (int e = tid; e < 3 * XP_BN; e += XP_THREADS) Sacc[e] = 0.0;

  auto tile_xy = [&](int i, int& img, int& y0, int& x0) __attribute__((always_inline)) {
    const unsigned pt = (unsigned)(prow + i * gp);
    const unsigned r = pt / (unsigned)tiles_x;
    x0 = (int)(pt - r * (unsigned)tiles_x) * XP_TW;
    const unsigned r2 = r / (unsigned)tiles_y;
    y0 = (int)(r - r2 * (unsigned)tiles_y) * XP_TH;
    img = (int)r2;
  };
  auto chunk_src = [&](int chunk, int& c) -> SrcArg {
    c = chunk * XP_CK;
    const bool s1 = g.nsrc > 1 && c >= g.src[0].C;
    if (s1) c -= g.src[0].C;
    return pick_src(g, s1 ? 1 : 0);
  };

  // ---------------------------------------------------------------- weights: LDS-DMA, two steps ahead
  typedef const __attribute__((address_space(1))) void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  // step st (chunk * 9 + tap) into buffer buf: wave w's two 1-KB DMA instructions fill rows 32w .. 32w + 31;
  // lane L of instruction i lands at row (2w + i) * 16 + L / 4, physical slot L % 4, and loads logical slot
  // xp_wslot(row, L % 4) of that row: slots 0 / 1 the high parts of channels 0-7 / 8-15 of the chunk, 2 / 3
  // the low parts (the pack stores each 32-k group as 32 high then 32 low fp16 parts)
  auto b_issue = [&](int st, int buf) __attribute__((always_inline)) {
    const int chunk = st / 9, tap = st - chunk * 9;
    const int k0 = tap * g.Ctot + (chunk >> 1) * 32;  // the pack's 32-k group (32 words)
    const int kh = (chunk & 1) * 2;                   // this chunk's first 16-B unit in the group's halves
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (wave * 2 + i) * 16 + (lane >> 2);
      const int s = xp_wslot(row, lane & 3);
      const float* p = B + (int64_t)(n0 + row) * k_pad + k0 + (s >> 1) * 16 + (kh + (s & 1)) * 4;
      __builtin_amdgcn_global_load_lds((gptr_t)p, (lptr_t)(Bs + buf * XP_BBUF + (wave * 2 + i) * 1024), 16, 0, 0);
    }
  };

  // ---------------------------------------------------------------- halo (raw fp32 -> split fp16)
  // slice r: hidx = r * 256 + tid -> halo pixel hidx >> 2, channels 4 (hidx & 3) .. + 3 (= 4 (tid & 3) .. + 3)
  uint4 ra[XP_A_ROUNDS];
  // a job's source and tile, resolved once per job (pick_src selects through a scalar branch, which inside the
  // unrolled taps would split them into blocks and cost the compiler's wait counts their precision)
  struct Job {
    SrcArg sa;
    int c, img, y0, x0;
  };
  auto job_of = [&](int job) __attribute__((always_inline)) {
    Job jb;
    tile_xy(job / nchunks, jb.img, jb.y0, jb.x0);
    jb.sa = chunk_src(job % nchunks, jb.c);
    return jb;
  };
  auto a_load = [&](const Job& jb, int r) __attribute__((always_inline)) {
    const SrcArg& sa = jb.sa;
    const int c = jb.c, img = jb.img, y0 = jb.y0, x0 = jb.x0;
    const int hp = min((r * XP_THREADS + tid) >> 2, XP_HPIX - 1);
    const int hy = hp / XP_HW, hx = hp - hy * XP_HW;
    const int ys = min(max(y0 - 1 + hy, 0), g.h - 1), xq = min(max(x0 - 1 + hx, 0), g.w - 1);
    ra[r] = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(sa.data) +
                                            (((int64_t)img * g.h + ys) * g.w + xq) * sa.C + c + (tid & 3) * 4);
  };
  // BN+ReLU of the source (sc / sh: this thread's 4 channels, or none), zero outside the image, 2^e, fp16
  // split: the slice's 16 B become 8 B of high parts (.x, .y) and 8 B of low parts (.z, .w)
  auto a_split = [&](const Job& jb, int r, const f32x4& sc, const f32x4& sh, float rlo)
      __attribute__((always_inline)) {
    const int y0 = jb.y0, x0 = jb.x0;
    const int hp = min((r * XP_THREADS + tid) >> 2, XP_HPIX - 1);
    const int hy = hp / XP_HW, hx = hp - hy * XP_HW;
    const bool in = (unsigned)(y0 - 1 + hy) < (unsigned)g.h && (unsigned)(x0 - 1 + hx) < (unsigned)g.w;
    f32x4 v;
    __builtin_memcpy(&v, &ra[r], 16);
    f16x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      // (sc = 1, sh = 0 for an untransformed source: exact; rlo = -inf without ReLU)
      float f = fmaxf(v[e] * sc[e] + sh[e], rlo);
      f = in ? f * xs : 0.0f;
      _Float16 a, b;
      x2_split(f, a, b);
      h[e] = a;
      l[e] = b;
    }
    uint4 o;
    __builtin_memcpy(&o, &h, 8);
    __builtin_memcpy(reinterpret_cast<unsigned char*>(&o) + 8, &l, 8);
    ra[r] = o;
  };
  // high parts of channel group cc = tid & 3 at logical slot cc >> 1 (+ 8 B for odd cc), low parts at 2 + (cc >> 1)
  auto a_store = [&](int hb, int r) __attribute__((always_inline)) {
    const int hidx = r * XP_THREADS + tid;
    if (hidx >= XP_HPIX * 4) return;
    const int hp = hidx >> 2, cc = tid & 3;
    unsigned char* base = As + hb * XP_OFF_H1 + hp * XP_ROWB + (cc & 1) * 8;
    // (inline ds_write_b64: the compiler cannot tell this halo buffer from the weight buffers an LDS-DMA is
    // writing, and before a plain LDS store it would wait for every DMA in flight — the next step's weights;
    // the step barrier's lgkmcnt(0) retires these stores)
    const unsigned ah = (unsigned)(uintptr_t)(base + (xp_hslot(hp, cc >> 1) << 4));
    const unsigned al = (unsigned)(uintptr_t)(base + (xp_hslot(hp, 2 + (cc >> 1)) << 4));
    const uint2 vh = make_uint2(ra[r].x, ra[r].y), vl = make_uint2(ra[r].z, ra[r].w);
    asm volatile("ds_write_b64 %0, %1" ::"v"(ah), "v"(vh));
    asm volatile("ds_write_b64 %0, %1" ::"v"(al), "v"(vl));
  };
  // ReLU floor of job j's source: 0, or -inf without ReLU (a max instead of a branch)
  auto a_rlo = [&](const Job& jb) __attribute__((always_inline)) -> float {
    return jb.sa.scale && jb.sa.relu ? 0.0f : -INFINITY;
  };
  // job j's transform for channel tid & 15 (scale for tid < 16, shift for 16 <= tid < 32; 1 / 0 without a
  // transform): every lane loads (the address stays valid), so no branch splits the tap
  auto coef_load = [&](const Job& jb) __attribute__((always_inline)) -> float {
    const SrcArg& sa = jb.sa;
    const int c = jb.c;
    const float* src = sa.scale ? ((tid & 16) ? sa.shift : sa.scale) + c : wcs;
    const float v = src[tid & 15];
    return sa.scale ? v : ((tid & 16) ? 0.0f : 1.0f);
  };

  // ---------------------------------------------------------------- MFMA step (32x32x16, 2 x 4 subtiles)
  f32x16 acc[2][4];
  // halo pixel of this lane's row of subtile a at tap (0, 0): tile row 4 wave + 2a + l32 / 16, column l32 % 16
  int hp0[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) hp0[a] = (wave * 4 + a * 2 + (l32 >> 4)) * XP_HW + (l32 & 15);
  const int wsw = (l32 >> 2) & 3;  // weight-row swizzle of this lane's rows (b * 32 + l32)
  auto mma_step = [&](int hbuf, int bbuf, int t) __attribute__((always_inline)) {
    const unsigned char* a_src = As + hbuf * XP_OFF_H1;
    const unsigned char* b_src = Bs + bbuf * XP_BBUF;
    const int dy = t / 3, dx = t - (t / 3) * 3;
    f16x8 ah[2], al[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      // (an opaque copy per step: hoisted out of the unrolled taps, the 36 row / slot offsets were spilled)
      int hp = hp0[a];
      asm volatile("" : "+v"(hp));
      hp += dy * XP_HW + dx;
      const unsigned char* p = a_src + hp * XP_ROWB;
      ah[a] = *reinterpret_cast<const f16x8*>(p + (xp_hslot(hp, half) << 4));
      al[a] = *reinterpret_cast<const f16x8*>(p + (xp_hslot(hp, 2 + half) << 4));
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const unsigned char* p = b_src + (b * 32 + l32) * XP_ROWB;
      const f16x8 bh = *reinterpret_cast<const f16x8*>(p + ((half ^ wsw) << 4));
      const f16x8 bl = *reinterpret_cast<const f16x8*>(p + (((2 + half) ^ wsw) << 4));
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bl, acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a], bh, acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a], bh, acc[a][b], 0, 0, 0);
      }
    }
  };
  // wait until this wave's vector-memory operations but the youngest `keep` (0 / 1 halo load, known per tap) are
  // done and its LDS writes have landed, then the workgroup barrier — never the vmcnt(0) drain of __syncthreads
  auto step_barrier = [&](int keep) __attribute__((always_inline)) {
    // (s_waitcnt through the builtin, which the compiler's wait-count pass understands: an inline-asm wait made it
    // drain every pending register load ahead of the asm, the halo slice in flight included; keep is a
    // compile-time constant per tap)
    if (keep >= 4) __builtin_amdgcn_s_waitcnt(0x0F74);
    else if (keep == 3) __builtin_amdgcn_s_waitcnt(0x0F73);
    else if (keep == 2) __builtin_amdgcn_s_waitcnt(0x0F72);
    else if (keep == 1) __builtin_amdgcn_s_waitcnt(0x0F71);
    else __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
  };
  auto lds_barrier = [&]() __attribute__((always_inline)) {  // LDS reads / writes only
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
  };

  // ---------------------------------------------------------------- prologue: job 0's halo, step 0's weights
  if (njobs > 0) {
    f32x4 sc = {1, 1, 1, 1}, sh = {0, 0, 0, 0};
    int c0;
    const SrcArg sa = chunk_src(0, c0);
    if (sa.scale) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc[e] = sa.scale[c0 + (tid & 3) * 4 + e];
        sh[e] = sa.shift[c0 + (tid & 3) * 4 + e];
      }
    }
    const Job j0 = job_of(0);
#pragma unroll
    for (int r = 0; r < XP_A_ROUNDS; ++r) a_load(j0, r);
#pragma unroll
    for (int r = 0; r < XP_A_ROUNDS; ++r) {
      a_split(j0, r, sc, sh, a_rlo(j0));
      a_store(0, r);
    }
    b_issue(0, 0);
    if (csteps > 1) b_issue(1, 1);
  }

  float amx = 0.0f;
  float creg = 0.0f;
  int J = 0, S = 0;
  for (int i = 0; i < ntl; ++i) {
    int img, y0, x0;
    tile_xy(i, img, y0, x0);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = f32x16{};
    for (int c = 0; c < nchunks; ++c, ++J) {
      // the next job (the last job's own data again at the end: every load stays valid and no branch splits the
      // taps, so the compiler's wait counts stay exact; the results go to the unused buffers)
      const Job jn = job_of(J + 1 < njobs ? J + 1 : J);
      const bool last_step_tile = c + 1 == nchunks;
      float* ssn = Ss + ((J + 1) & 1) * 2 * XP_CK;
      f32x4 nsc, nsh;
      float nrlo = 0.0f;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        // step S's weights (issued two steps ago) and the halo slice of tap t - 2 have landed everywhere (left in
        // flight: the two DMA instructions of step S + 1 and the slice of tap t - 1; the slice split at the end of
        // this tap is then known complete, so the compiler adds no wait of its own — with LDS-DMA and loads both
        // pending it could only wait for zero); at tap 8 everything (the tile's last job issues no DMA at tap 7,
        // which a per-tap constant cannot know); everyone is past step S - 1
        step_barrier(t == 8 ? 0 : 2 + (t >= 1 && t - 1 < XP_A_ROUNDS));
        // the next job's coefficients: issued before this step's DMA, so the next step's wait retires them
        if (t == 0) creg = coef_load(jn);
        if (t == 1 && tid < 2 * XP_CK) ssn[tid] = creg;  // visible from tap 2
        // slice t - 3 (split at the end of the last tap) to the free buffer — before this tap's DMA: an LDS write
        // behind an LDS-DMA in flight makes the compiler wait for the DMA
        if (t >= 3 && t - 3 < XP_A_ROUNDS) a_store((J + 1) & 1, t - 3);
        if (t < 7 || !last_step_tile) b_issue(c * 9 + t + 2, (S + 2) % XP_NB);  // (the next tile's: after the epilogue)
        if (t < XP_A_ROUNDS) a_load(jn, t);
        if (t == 2) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            nsc[e] = ssn[(tid & 3) * 4 + e];
            nsh[e] = ssn[XP_CK + (tid & 3) * 4 + e];
          }
          nrlo = a_rlo(jn);
        }
        mma_step(J & 1, S % XP_NB, t);
        if (t >= 2 && t - 2 < XP_A_ROUNDS) a_split(jn, t - 2, nsc, nsh, nrlo);  // slice t - 2, under the MFMAs
        ++S;
      }
    }

    // ------------------------------------------------------------ epilogue of tile i (four 32-column quarters)
    lds_barrier();  // every wave is done reading the last job's halo and the weights: the quarters take them
    float* tile = reinterpret_cast<float*>(smem + (((J - 1) & 1) ? XP_OFF_B : 0));
    auto dst = [&](int pix, int cl, int q) -> float* {
      const int y = y0 + pix / XP_TW, x = x0 + pix % XP_TW;
      if (y >= g.h || x >= g.w) return nullptr;
      const int64_t m = ((int64_t)img * g.h + y) * g.w + x;
      const int col = n0 + q * XP_EPI_TC + cl;
      if (ep.mode == SELUNET_EP_SPLIT)
        return col < ep.split ? reinterpret_cast<float*>(ep.out0) + m * ep.split + col
                              : reinterpret_cast<float*>(ep.out1) + m * (N - ep.split) + (col - ep.split);
      return reinterpret_cast<float*>(ep.out0) + m * N + col;
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q) lds_barrier();  // the previous quarter's partials have been reduced
      const float cf = wcs[n0 + q * 32 + l32] * inv;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          tile[(wave * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * half) * (XP_EPI_TC + 4) + l32] = acc[a][q][r] * cf;
      lds_barrier();
      float t1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      const TileStats ts = tile_stats(ep, prow, n0 + q * XP_EPI_TC, N);
      lds_tile_store_acc<float, XP_TH * XP_TW, XP_EPI_TC, XP_THREADS>(
          tile, tid, [&](int pix, int cl) { return dst(pix, cl, q); }, ep.bias,
          [&](int cl) { return n0 + q * XP_EPI_TC + cl; }, ts, t1, t2, t3, amx);
      // this tile's column partials -> fp64 accumulators, in a fixed order (row groups r0 = tid / 4 ascending)
      const int nst = ts.bnb.slab ? 3 : (ts.stats ? 2 : (ts.colsum ? 1 : 0));
      if (nst) {  // (uniform)
        lds_barrier();  // the quarter has been read: its space takes the partials [64 row groups][32 columns][3]
        const int cc = tid & 3, r0 = tid >> 2;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          tile[(r0 * XP_EPI_TC + cc * 8 + e) * 3 + 0] = t1[e];
          tile[(r0 * XP_EPI_TC + cc * 8 + e) * 3 + 1] = t2[e];
          tile[(r0 * XP_EPI_TC + cc * 8 + e) * 3 + 2] = t3[e];
        }
        lds_barrier();
        if (tid < XP_EPI_TC * nst) {
          const int col = tid % XP_EPI_TC, k = tid / XP_EPI_TC;
          float v = 0.0f;
#pragma unroll 8
          for (int r = 0; r < XP_RS; ++r) v += tile[(r * XP_EPI_TC + col) * 3 + k];
          Sacc[k * XP_BN + q * XP_EPI_TC + col] += (double)v;
        }
      }
    }
    if (i + 1 < ntl) {
      lds_barrier();  // the quarters have been read: the weights' space back to the next tile
      b_issue(0, S % XP_NB);
      if (csteps > 1) b_issue(1, (S + 1) % XP_NB);
    }
  }
  // this workgroup's slab row: the fp64 column accumulators, rounded once
  __syncthreads();
  {
    const TileStats ts = tile_stats(ep, prow, n0, N);
    const bool do_bn = ts.bnb.slab != nullptr, do_st = ts.stats != nullptr;
    const int nst = do_bn ? 3 : (do_st ? 2 : (ts.colsum ? 1 : 0));
    for (int e = tid; e < XP_BN * nst; e += XP_THREADS) {
      const int col = e % XP_BN, k = e / XP_BN;
      const float v = (float)Sacc[k * XP_BN + col];
      if (do_bn) ts.bnb.slab[k * ts.ld + col] = v;
      else if (do_st) ts.stats[k * ts.ld + col] = v;
      else if (ts.gcol0 + col < ts.colsum_cols) ts.colsum[col] = v;
    }
  }
  if (ep.amax) block_amax(ep.amax, amx, reinterpret_cast<float*>(smem));
}

// persistent workgroups (= statistics slab rows) per column tile: two per CU
int64_t conv3x3_x2p_rows(const GatherArg& g, int N) {
  const int64_t pt = (int64_t)g.n * cdiv(g.h, XP_TH) * cdiv(g.w, XP_TW);
  return std::max<int64_t>(1, std::min<int64_t>(pt, 2 * (int64_t)conv3x3_persist_wgs() / std::max(1, N / XP_BN)));
}

// SELUNET_OPT_X2P: the 128-column split-fp16 layers on this kernel (1) or on the one-workgroup-per-CU
// persistent kernel (0, default: this kernel measured 0-2 % slower on the deep-K forwards and 4-13 % on the data
// gradients and shallow layers, profiles/r06_x2p_ab.txt). Shape-only (the statistics-rows query knows no epilogue): multi-chunk inputs
// (C a multiple of 32, at least 64), N a multiple of 128, h, w >= 16; not with the tile queue.
bool conv3x3_x2p_eligible(const GatherArg& g, int N) {
  return option(SELUNET_OPT_X2P, 0) != 0 && !x2_tile_queue() && N % XP_BN == 0 && g.Ctot % 32 == 0 &&
         g.Ctot >= 2 * XP_CK && g.src[0].C % XP_CK == 0 && g.h >= XP_TH && g.w >= XP_TW;
}

int conv3x3_x2p_launch(const GatherArg& g, const float* w, int N, const EpiArg& ep, const float* amax0,
                       const float* amax1, hipStream_t st) {
  if (ep.mode == SELUNET_EP_SPLIT && ep.split % 8 != 0)
    return fail(SELUNET_EINVAL, "conv3x3_x2p: a SPLIT epilogue needs split %% 8 == 0 (got %d)", ep.split);
  if (ep.mode == SELUNET_EP_SCATTER2X) return fail(SELUNET_EINVAL, "conv3x3_x2p: scatter epilogue not supported");
  const int tiles_x = (int)cdiv(g.w, XP_TW), tiles_y = (int)cdiv(g.h, XP_TH);
  const int ptiles = (int)((int64_t)g.n * tiles_x * tiles_y);
  const int n_tiles = N / XP_BN;
  const int gp = (int)conv3x3_x2p_rows(g, N);
  const int k_pad = 9 * g.Ctot;
  hipLaunchKernelGGL(conv3x3_x2p_kernel, dim3((unsigned)(gp * n_tiles)), dim3(XP_THREADS), 0, st, g, w, N, k_pad, ep,
                     n_tiles, tiles_x, tiles_y, ptiles, gp, w + (int64_t)N * k_pad, amax0, amax1);
  return check_launch("conv3x3_x2p");
}

}  // namespace selunet
