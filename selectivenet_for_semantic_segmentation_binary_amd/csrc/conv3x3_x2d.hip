// fp32 3x3 convolution (model.py:11) forward / data gradient on split-fp16 operands for the 64-column
// layers (the full-resolution CBR blocks encoder_layer_1_2, decoder_layer_1_1 and decoder_layer_1_2's
// forward, encoder_layer_2_1's data gradient): the arithmetic of conv3x3_halo_persist_kernel<float, 64,
// X2, M16> (halo staged once per 32-channel chunk in LDS as fp16 high / low parts, three
// v_mfma_f32_16x16x32_f16 per 16x16 subtile and tap) in a smaller workgroup, two per CU.
//
// At 256x256 these layers have a short K loop (two or four channel chunks per 16 x 16 tile) and the
// one-workgroup-per-CU persistent kernel exposes what sits between the MFMA phases — each tile's
// LDS-staged epilogue, the halo and weight staging at chunk boundaries — as MFMA idle time (measured:
// mfma_busy 0.37-0.40, memory wait 0.41). Here a workgroup is 256 threads (4 waves, one per SIMD; wave
// w computes tile rows 4w..4w+3 x all 64 columns, 16 accumulator subtiles) with 72 KB of LDS: one halo
// buffer, two weight buffers. Two workgroups share a CU, so one's staging and epilogue run under the
// other's MFMAs. Persistent over the pixel tiles (512 workgroups = the statistics slab rows of
// selunet_conv3x3_x2_stats_rows, twice the one-per-CU kernels' target); per chunk the next job's halo is loaded into registers during the
// first taps, BN+ReLU-transformed and split during the last tap, and written after it; weights are
// double-buffered per tap and loaded two taps ahead.
#include "gemm_common.h"

namespace selunet {

constexpr int XD_TH = 16, XD_TW = 16, XD_HW = 18, XD_HPIX = 324;
constexpr int XD_THREADS = 256;
constexpr int XD_BN = 64;
constexpr int XD_CK = 32;                                            // fp32 channels per chunk
constexpr int XD_AROWB = 160;                                        // halo row bytes (128 used)
constexpr int XD_WROWB = 160;                                        // weight row bytes (128 used)
constexpr int XD_A_ROUNDS = (XD_HPIX * 8 + XD_THREADS - 1) / XD_THREADS;  // 16-B halo slices per thread: 11
constexpr int XD_B_ROUNDS = XD_BN * 8 / XD_THREADS;                  // 16-B weight slices per thread and tap: 2

__global__ void __launch_bounds__(XD_THREADS, 2)
conv3x3_x2d_kernel(GatherArg g, const float* __restrict__ B, int k_pad, EpiArg ep, int tiles_x, int tiles_y,
                   int ptiles, int gp, const float* __restrict__ wcs, const float* __restrict__ amax0,
                   const float* __restrict__ amax1) {
  constexpr int N = XD_BN;
  constexpr int OFF_B = XD_HPIX * XD_AROWB;                  // 51840
  constexpr int OFF_S = OFF_B + 2 * XD_BN * XD_WROWB;         // 72320
  constexpr int SMEM_EPI = XD_TH * XD_TW * (XD_BN + 4) * 4;   // 69632
  static_assert(SMEM_EPI <= OFF_S, "the epilogue tile must leave the coefficients alone");
  using Acc = double;  // (fp64 statistics registers across the ~64 tiles of a workgroup)
  static_assert(stats_flush_bytes<XD_BN, XD_THREADS, Acc>() <= OFF_S, "statistics scratch exceeds the tile");
  __shared__ __attribute__((aligned(16))) unsigned char smem[OFF_S + 2 * 2 * XD_CK * 4];
  unsigned char* As = smem;
  unsigned char* Bs = smem + OFF_B;
  float* Ss = reinterpret_cast<float*>(smem + OFF_S);  // [2 jobs][scale 32, shift 32]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, kg = lane >> 4;

  const unsigned lb = xcd_remap(blockIdx.x, gridDim.x);
  const int prow = (int)lb;
  const int ntl = prow < ptiles ? (ptiles - prow + gp - 1) / gp : 0;
  const int nchunks = g.Ctot / XD_CK;
  const int csteps = nchunks * 9;
  const int njobs = ntl * nchunks;

  float xs, inv;
  {
    float am = amax0 ? amax0[0] : 0.0f;
    if (g.nsrc > 1 && amax1) am = fmaxf(am, amax1[0]);
    xs = x2_scale(am, &inv);
  }
  float cfac[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) cfac[b] = wcs[b * 16 + l16] * inv;

  auto tile_xy = [&](int i, int& img, int& y0, int& x0) __attribute__((always_inline)) {
    const unsigned pt = (unsigned)(prow + i * gp);
    const unsigned r = pt / (unsigned)tiles_x;
    x0 = (int)(pt - r * (unsigned)tiles_x) * XD_TW;
    const unsigned r2 = r / (unsigned)tiles_y;
    y0 = (int)(r - r2 * (unsigned)tiles_y) * XD_TH;
    img = (int)r2;
  };
  auto chunk_src = [&](int chunk, int& c) -> SrcArg {
    c = chunk * XD_CK;
    const bool s1 = g.nsrc > 1 && c >= g.src[0].C;
    if (s1) c -= g.src[0].C;
    return pick_src(g, s1 ? 1 : 0);
  };

  // ---------------------------------------------------------------- weights ([64 rows][128 B] per step)
  struct BRegs {
    uint4 v[XD_B_ROUNDS];
  };
  auto b_load = [&](int st) __attribute__((always_inline)) {  // st: step within a tile (chunk * 9 + tap)
    const int chunk = st / 9, tap = st - chunk * 9;
    const int k0 = tap * g.Ctot + chunk * XD_CK;
    int tq = tid;
    asm volatile("" : "+v"(tq));
    BRegs rb;
#pragma unroll
    for (int r = 0; r < XD_B_ROUNDS; ++r) {
      const int idx = r * XD_THREADS + tq;
      const int row = idx >> 3, cc = idx & 7;
      rb.v[r] = *reinterpret_cast<const uint4*>(B + (int64_t)row * k_pad + k0 + cc * 4);
    }
    return rb;
  };
  auto b_store = [&](const BRegs& rb, int buf) __attribute__((always_inline)) {
    int tq = tid;
    asm volatile("" : "+v"(tq));
#pragma unroll
    for (int r = 0; r < XD_B_ROUNDS; ++r) {
      const int idx = r * XD_THREADS + tq;
      const int row = idx >> 3, cc = idx & 7;
      *reinterpret_cast<uint4*>(Bs + (buf * XD_BN + row) * XD_WROWB + cc * 16) = rb.v[r];
    }
  };

  // ---------------------------------------------------------------- halo (raw fp32 -> split fp16)
  // slice hidx = r * 256 + tid: halo pixel hidx >> 3, channels 4 (hidx & 3 ... tid & 7) .. + 3
  struct ARegs {
    uint4 v[XD_A_ROUNDS];
  };
  auto a_load = [&](ARegs& ra, int job, int r0, int r1) __attribute__((always_inline)) {
    int img, y0, x0, c;
    tile_xy(job / nchunks, img, y0, x0);
    const SrcArg sa = chunk_src(job % nchunks, c);
    int tq = tid;
    asm volatile("" : "+v"(tq));
#pragma unroll
    for (int r = 0; r < XD_A_ROUNDS; ++r) {
      if (r < r0 || r >= r1) continue;
      const int hp = min((r * XD_THREADS + tq) >> 3, XD_HPIX - 1);
      const int hy = hp / XD_HW, hx = hp - hy * XD_HW;
      const int ys = min(max(y0 - 1 + hy, 0), g.h - 1), xq = min(max(x0 - 1 + hx, 0), g.w - 1);
      ra.v[r] = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(sa.data) +
                                                (((int64_t)img * g.h + ys) * g.w + xq) * sa.C + c + (tq & 7) * 4);
    }
  };
  // in registers: BN+ReLU of the chunk's source (sc/sh for this thread's 4 channels, or none), zero
  // outside the image, scale 2^e, fp16 split: each 16-B slice becomes 8 B of high + 8 B of low parts
  auto a_split = [&](ARegs& ra, int job, bool tr, const float* sc, const float* sh, int relu)
      __attribute__((always_inline)) {
    int img, y0, x0;
    tile_xy(job / nchunks, img, y0, x0);
    int tq = tid;
    asm volatile("" : "+v"(tq));
#pragma unroll
    for (int r = 0; r < XD_A_ROUNDS; ++r) {
      const int hp = min((r * XD_THREADS + tq) >> 3, XD_HPIX - 1);
      const int hy = hp / XD_HW, hx = hp - hy * XD_HW;
      const bool in = (unsigned)(y0 - 1 + hy) < (unsigned)g.h && (unsigned)(x0 - 1 + hx) < (unsigned)g.w;
      f32x4 v;
      __builtin_memcpy(&v, &ra.v[r], 16);
      f16x4 h, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float f = v[e];
        if (tr) {
          f = f * sc[e] + sh[e];
          if (relu) f = fmaxf(f, 0.0f);
        }
        f = in ? f * xs : 0.0f;
        _Float16 a, b;
        x2_split(f, a, b);
        h[e] = a;
        l[e] = b;
      }
      uint4 o;
      __builtin_memcpy(&o, &h, 8);
      __builtin_memcpy(reinterpret_cast<unsigned char*>(&o) + 8, &l, 8);
      ra.v[r] = o;
    }
  };
  // the split slices to the halo tile: high parts of channel group cc at 16-B unit (cc >> 1), low parts at
  // 4 + (cc >> 1), both XOR the halo line's parity (conflict-free fragment reads, as halo_off)
  auto a_store = [&](const ARegs& ra) __attribute__((always_inline)) {
    int tq = tid;
    asm volatile("" : "+v"(tq));
    const int cc = tq & 7;
#pragma unroll
    for (int r = 0; r < XD_A_ROUNDS; ++r) {
      const int hidx = r * XD_THREADS + tq;
      if (hidx >= XD_HPIX * 8) continue;
      const int hp = hidx >> 3;
      const int par = (hp / XD_HW) & 1;
      unsigned char* base = As + hp * XD_AROWB + (cc & 1) * 8;
      *reinterpret_cast<uint2*>(base + (((cc >> 1) ^ par) << 4)) = make_uint2(ra.v[r].x, ra.v[r].y);
      *reinterpret_cast<uint2*>(base + (((4 + (cc >> 1)) ^ par) << 4)) = make_uint2(ra.v[r].z, ra.v[r].w);
    }
  };
  auto coef_load = [&](int job) __attribute__((always_inline)) -> float {
    int c;
    const SrcArg sa = chunk_src(job % nchunks, c);
    if (tid >= 2 * XD_CK || !sa.scale) return 0.0f;
    return tid < XD_CK ? sa.scale[c + tid] : sa.shift[c + tid - XD_CK];
  };

  // ---------------------------------------------------------------- MFMA tap (16x16x32)
  f32x4 acc[4][4];
  auto mma_tap = [&](int bbuf, int t) __attribute__((always_inline)) {
    const unsigned char* b_src = Bs + bbuf * XD_BN * XD_WROWB;
    const int dy = t / 3, dx = t - (t / 3) * 3;
    f16x8 bh[4], bl[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const unsigned char* p = b_src + (b * 16 + l16) * XD_WROWB + kg * 16;
      bh[b] = *reinterpret_cast<const f16x8*>(p);
      bl[b] = *reinterpret_cast<const f16x8*>(p + 64);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int hy = wave * 4 + a + dy;
      const unsigned char* p = As + (hy * XD_HW + l16 + dx) * XD_AROWB + ((kg ^ (hy & 1)) << 4);
      const f16x8 ah = *reinterpret_cast<const f16x8*>(p);
      const f16x8 al = *reinterpret_cast<const f16x8*>(p + 64);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[b], acc[a][b], 0, 0, 0);
      }
    }
  };

  // ---------------------------------------------------------------- prologue: job 0
  ARegs ra;
  if (njobs > 0) {
    a_load(ra, 0, 0, XD_A_ROUNDS);
    int c0;
    const SrcArg sa = chunk_src(0, c0);
    float sc[4] = {1, 1, 1, 1}, sh[4] = {0, 0, 0, 0};
    if (sa.scale) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc[e] = sa.scale[c0 + (tid & 7) * 4 + e];
        sh[e] = sa.shift[c0 + (tid & 7) * 4 + e];
      }
    }
    a_split(ra, 0, sa.scale != nullptr, sc, sh, sa.relu);
    a_store(ra);
  }
  b_store(b_load(0), 0);
  BRegs rb_next = b_load(1 % csteps);
  __syncthreads();

  Acc s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float amx = 0.0f;
  const TileStats ts = tile_stats(ep, prow, 0, N);
  float* tile = reinterpret_cast<float*>(smem);
  float creg = 0.0f;
  int J = 0, S = 0;
  for (int i = 0; i < ntl; ++i) {
    int img, y0, x0;
    tile_xy(i, img, y0, x0);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{};
    BRegs rb_hold;
    for (int c = 0; c < nchunks; ++c, ++J) {
      const bool has_next = J + 1 < njobs;
      const bool last_c = c + 1 == nchunks;
      int cn;
      const SrcArg sn = chunk_src((J + 1) % nchunks, cn);
      float* ssn = Ss + ((J + 1) & 1) * 2 * XD_CK;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int st2 = c * 9 + t + 2;
        const BRegs rb_far = b_load(st2 < csteps ? st2 : st2 - csteps);  // (the next tile's steps wrap)
        if (has_next) {
          if (t == 0) creg = coef_load(J + 1);
          // the next job's halo, two 16-B slices per tap from tap 0 (held in registers: one halo buffer)
          if (t < (XD_A_ROUNDS + 1) / 2) a_load(ra, J + 1, 2 * t, 2 * t + 2);
        }
        mma_tap(S & 1, t);
        if (t == 1 && has_next && tid < 2 * XD_CK) ssn[tid] = creg;
        if (t == 8 && has_next) {  // BN+ReLU, scale and split while the last tap's MFMAs run
          float sc[4] = {1, 1, 1, 1}, sh[4] = {0, 0, 0, 0};
          if (sn.scale) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              sc[e] = ssn[(tid & 7) * 4 + e];
              sh[e] = ssn[XD_CK + (tid & 7) * 4 + e];
            }
          }
          a_split(ra, J + 1, sn.scale != nullptr, sc, sh, sn.relu);
        }
        if (last_c && has_next && t == 8) rb_hold = rb_next;  // B(S + 1): stored after the epilogue
        else b_store(rb_next, (S + 1) & 1);
        __syncthreads();
        rb_next = rb_far;
        ++S;
      }
      if (!last_c) {  // the next chunk of this tile: halo -> LDS (every wave is past the last tap)
        a_store(ra);
        __syncthreads();
      }
    }

    // ------------------------------------------------------------ epilogue of tile i (LDS-staged)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          tile[((wave * 4 + a) * 16 + 4 * kg + e) * (N + 4) + b * 16 + l16] = acc[a][b][e] * cfac[b];
    __syncthreads();
    auto dst = [&](int pix, int cl) -> float* {
      const int y = y0 + pix / XD_TW, x = x0 + pix % XD_TW;
      if (y >= g.h || x >= g.w) return nullptr;
      const int64_t m = ((int64_t)img * g.h + y) * g.w + x;
      if (ep.mode == SELUNET_EP_SPLIT)
        return cl < ep.split ? reinterpret_cast<float*>(ep.out0) + m * ep.split + cl
                             : reinterpret_cast<float*>(ep.out1) + m * (N - ep.split) + (cl - ep.split);
      return reinterpret_cast<float*>(ep.out0) + m * N + cl;
    };
    auto bias_col = [&](int cl) { return cl; };
    lds_tile_store_acc<float, XD_TH * XD_TW, N, XD_THREADS>(tile, tid, dst, ep.bias, bias_col, ts, s1, s2, s3, amx);
    if (i + 1 < ntl) {
      __syncthreads();  // the tile has been read: LDS back to halo / weights
      a_store(ra);      // (the next tile's first chunk, split during the last tap)
      b_store(rb_hold, S & 1);
      __syncthreads();
    }
  }
  tile_stats_flush<N, XD_THREADS>(tile, tid, ts, s1, s2, s3, amx);
}

// persistent workgroups (= statistics slab rows) of the 64-column kernel: two per CU (twice the target of
// the one-per-CU persistent kernels, selunet_set_halo_workgroups)
int64_t conv3x3_x2d_rows(const GatherArg& g) {
  const int64_t pt = (int64_t)g.n * cdiv(g.h, XD_TH) * cdiv(g.w, XD_TW);
  return std::max<int64_t>(1, std::min<int64_t>(pt, 2 * (int64_t)conv3x3_persist_wgs()));
}

// Measured per layer against conv3x3_halo_persist_kernel<float, 64, X2> (tools/conv_bench.py --x2, same box,
// two runs each): forwards of 64-channel inputs 2-6 % faster, data gradients and the 128-channel inputs
// 1-4 % slower, hence the default (SELUNET_OPT_X2D 3: 64-channel inputs with a BN+ReLU source = forwards).
bool conv3x3_x2d_eligible(const GatherArg& g, int N) {
  const int64_t mode = option(SELUNET_OPT_X2D, 3);
  if (N != XD_BN || g.Ctot % XD_CK != 0 || mode <= 0) return false;
  if (mode == 1) return g.Ctot <= 1024;
  return g.Ctot <= 64 && (mode == 2 || g.src[0].scale != nullptr);
}

int conv3x3_x2d_launch(const GatherArg& g, const float* w, const EpiArg& ep, const float* amax0, const float* amax1,
                       hipStream_t st) {
  const int tiles_x = (int)cdiv(g.w, XD_TW), tiles_y = (int)cdiv(g.h, XD_TH);
  const int ptiles = (int)((int64_t)g.n * tiles_x * tiles_y);
  const int gp = (int)conv3x3_x2d_rows(g);
  const int k_pad = 9 * g.Ctot;
  hipLaunchKernelGGL(conv3x3_x2d_kernel, dim3((unsigned)gp), dim3(XD_THREADS), 0, st, g, w, k_pad, ep, tiles_x, tiles_y,
                     ptiles, gp, w + (int64_t)XD_BN * k_pad, amax0, amax1);
  return check_launch("conv3x3_x2d");
}

}  // namespace selunet
