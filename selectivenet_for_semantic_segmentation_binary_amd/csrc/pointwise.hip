// Memory-bound kernels of the SelectiveUNet_B step on gfx950: weight (un)packing, deterministic
// reductions, BatchNorm finalize/backward, MaxPool2d(2), the 1x1 heads, the selective / BCE
// losses and multi-tensor Adam. All NHWC loads are 4-channel vectors (16 B fp32 / 8 B bf16).
#include <cstdarg>
#include <cstdlib>
#include <cmath>

#include "common.h"

namespace selunet {

// ------------------------------------------------------------------ error state, options
static thread_local char g_err[512] = "";

int64_t g_options[SELUNET_OPT_COUNT] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
static_assert(SELUNET_OPT_COUNT == 17, "g_options initialiser: one -1 per option");

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(SELUNET_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
  return SELUNET_OK;
}

constexpr int TPB = 256;

// =========================================================================== packing
template <typename T>
__global__ void pack_conv3x3_kernel(const float* __restrict__ w, int co, int ci, int k_pad, T* fwd, T* dgrad) {
  const int64_t total_f = (int64_t)co * k_pad;
  const int64_t total_d = dgrad ? (int64_t)ci * 9 * co : 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total_f + total_d;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < total_f) {
      const int o = (int)(i / k_pad), k = (int)(i % k_pad);
      float v = 0.0f;
      if (k < 9 * ci) {
        const int tap = k / ci, c = k - tap * ci;
        v = w[((int64_t)o * ci + c) * 9 + tap];
      }
      fwd[i] = from_f<T>(v);
    } else {
      const int64_t j = i - total_f;
      const int c = (int)(j / (9 * co));
      const int k = (int)(j % (9 * co));
      const int tap = k / co, o = k - tap * co;
      dgrad[j] = from_f<T>(w[((int64_t)o * ci + c) * 9 + (8 - tap)]);
    }
  }
}

template <typename T>
__global__ void pack_convT_kernel(const float* __restrict__ w, int ci, int co, T* fwd, T* dgrad) {
  const int64_t total = (int64_t)ci * co * 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    // w[c][o][ab]
    const int ab = (int)(i & 3);
    const int64_t co_ci = i >> 2;
    const int o = (int)(co_ci % co), c = (int)(co_ci / co);
    const T v = from_f<T>(w[i]);
    if (fwd) fwd[((int64_t)ab * co + o) * ci + c] = v;
    if (dgrad) dgrad[(int64_t)c * 4 * co + ab * co + o] = v;
  }
}

__global__ void unpack_conv3x3_kernel(const float* __restrict__ packed, int co, int ci, int ld, float* out) {
  const int64_t total = (int64_t)co * ci * 9;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int tap = (int)(i % 9);
    const int64_t oc = i / 9;
    const int c = (int)(oc % ci), o = (int)(oc / ci);
    out[i] = packed[(int64_t)o * ld + tap * ci + c];
  }
}

__global__ void unpack_convT_kernel(const float* __restrict__ packed, int ci, int co, int ld, float* out) {
  const int64_t total = (int64_t)ci * co * 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ab = (int)(i & 3);
    const int64_t r = i >> 2;
    const int o = (int)(r % co), c = (int)(r / co);
    out[i] = packed[(int64_t)c * ld + ab * co + o];
  }
}

// All weight packs of a step in one launch (selunet_pack_weights): the list travels by value in
// the kernel arguments; block b serves the tensor whose element range [off, off + total) holds
// its first element, grid-striding over the concatenated element space.
template <typename T>
__global__ void pack_weights_kernel(selunet_pack_list l, int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int t = 0;
    while (t + 1 < l.n && i >= l.d[t + 1].offset) ++t;
    const selunet_pack_desc& d = l.d[t];
    const int64_t j = i - d.offset;
    const float* w = d.w;
    T* fwd = reinterpret_cast<T*>(d.fwd);
    T* dg = reinterpret_cast<T*>(d.dgrad);
    if (d.kind == SELUNET_PACK_CONV3X3) {  // as pack_conv3x3_kernel
      const int co = d.co, ci = d.ci, k_pad = d.k_pad;
      const int64_t total_f = (int64_t)co * k_pad;
      if (j < total_f) {
        const int o = (int)(j / k_pad), k = (int)(j % k_pad);
        float v = 0.0f;
        if (k < 9 * ci) {
          const int tap = k / ci, c = k - tap * ci;
          v = w[((int64_t)o * ci + c) * 9 + tap];
        }
        fwd[j] = from_f<T>(v);
      } else {
        const int64_t q = j - total_f;
        const int c = (int)(q / (9 * co));
        const int k = (int)(q % (9 * co));
        const int tap = k / co, o = k - tap * co;
        dg[q] = from_f<T>(w[((int64_t)o * ci + c) * 9 + (8 - tap)]);
      }
    } else if (d.kind == SELUNET_PACK_CONV3X3_WINO) {  // fp32 Winograd F(2,3) operands (conv3x3.hip)
      const int co = d.co, ci = d.ci;
      const int64_t total_f = (int64_t)co * 12 * ci;
      const bool fw = j < total_f;
      const int64_t q = fw ? j : j - total_f;
      const int rows_k = fw ? ci : co;  // k = (dy*4 + xi)*rows_k + c
      const int r = (int)(q / (12 * rows_k));
      const int k = (int)(q % (12 * rows_k));
      const int t = k / rows_k, c = k - t * rows_k;
      const int dy = t >> 2, xi = t & 3;
      // fwd: row o = r, input channel c, kernel row dy; dgrad: row = input channel r, column o = c,
      // flipped kernel (row 2 - dy, taps 2 - j)
      const float* gw = fw ? w + ((int64_t)r * ci + c) * 9 + dy * 3 : w + ((int64_t)c * ci + r) * 9 + (2 - dy) * 3;
      const double g0 = fw ? gw[0] : gw[2], g1 = gw[1], g2 = fw ? gw[2] : gw[0];
      const double u = xi == 0 ? g0 : xi == 1 ? 0.5 * (g0 + g1 + g2) : xi == 2 ? 0.5 * (g0 - g1 + g2) : g2;
      (fw ? fwd : dg)[q] = from_f<T>((float)u);
    } else if (d.kind == SELUNET_PACK_COPY) {  // fp32 values unchanged
      reinterpret_cast<float*>(d.fwd)[j] = w[j];
    } else {  // as pack_convT_kernel: w[c][o][ab]
      const int ci = d.ci, co = d.co;
      const int ab = (int)(j & 3);
      const int64_t co_ci = j >> 2;
      const int o = (int)(co_ci % co), c = (int)(co_ci / co);
      const T v = from_f<T>(w[j]);
      if (fwd) fwd[((int64_t)ab * co + o) * ci + c] = v;
      if (dg) dg[(int64_t)c * 4 * co + ab * co + o] = v;
    }
  }
}

// Split-fp16 ("x2") operands of the fp32 3x3 convolutions (SELUNET_PACK_CONV3X3_X2): one block per
// matrix row (fwd: output channel o, k = tap*ci + c; dgrad: input channel c, k = tap*co + o, taps
// flipped). The row is scaled by 2^e (max|w_row| * 2^e < 2^14, so both fp16 parts stay normal-range)
// and every 32-k group is stored as 32 fp16 high parts h = fp16(v) then 32 low parts
// l = fp16(v - h): v = h + l to 22 significant bits. The row's unscale factor 2^-e follows the
// matrix (fwd + co*9*ci, dgrad + ci*9*co). desc.offset = first block (row) of the entry.
__global__ void __launch_bounds__(256) pack_x2_kernel(selunet_pack_list l) {
  int t = 0;
  const int64_t b = blockIdx.x;
  while (t + 1 < l.n && b >= l.d[t + 1].offset) ++t;
  const selunet_pack_desc& d = l.d[t];
  const int co = d.co, ci = d.ci;
  const bool ct = d.kind == SELUNET_PACK_CONVT_X2;  // ConvTranspose2d [ci][co][2][2]
  const int fwd_rows = ct ? 4 * co : co;
  const int r = (int)(b - d.offset);
  const bool fw = r < fwd_rows;
  const int row = fw ? r : r - fwd_rows;
  const int len = ct ? (fw ? ci : 4 * co) : (fw ? 9 * ci : 9 * co);
  const float* w = d.w;
  // the row is gathered in SOURCE order (j walks the fp32 master's memory, contiguous runs of 9 taps
  // / 4 positions) into LDS at its packed position k, then max-reduced and written in k order
  __shared__ float rowv[9 * 512];
  __shared__ float red[256];
  float m = 0.0f;
  for (int j = threadIdx.x; j < len; j += 256) {
    int k;
    int64_t src;
    if (ct) {
      if (fw) {  // row (ab, o) = ab * co + o, k = c: w[c][o][ab] (stride 4 co)
        const int ab = row / co, o = row - ab * co;
        k = j;
        src = ((int64_t)j * co + o) * 4 + ab;
      } else {   // row c, k = ab * co + o: w[c][o][ab] contiguous over j = o * 4 + ab
        const int o = j >> 2, ab = j & 3;
        k = ab * co + o;
        src = (int64_t)row * 4 * co + j;
      }
    } else if (fw) {  // row o, k = tap * ci + c: w[o][c][tap] contiguous over j = c * 9 + tap
      const int c = j / 9, tap = j - c * 9;
      k = tap * ci + c;
      src = (int64_t)row * 9 * ci + j;
    } else {  // row c, k = tap * co + o (taps flipped): w[o][c][8 - tap], runs of 9 over j = o * 9 + tp
      const int o = j / 9, tp = j - o * 9;
      k = (8 - tp) * co + o;
      src = ((int64_t)o * ci + row) * 9 + tp;
    }
    const float v = w[src];
    rowv[k] = v;
    m = fmaxf(m, fabsf(v));
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  float* base = reinterpret_cast<float*>(fw ? d.fwd : d.dgrad);
  const int rows = fw ? fwd_rows : ci;
  float unscale;
  const float sc = x2_scale(red[0], &unscale);
  _Float16* out = reinterpret_cast<_Float16*>(base + (int64_t)row * len);
  constexpr int gsh = 5;  // k groups of 32 values: high parts, then low parts
  for (int k = threadIdx.x; k < len; k += 256) {
    const float v = rowv[k] * sc;
    const _Float16 h = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (float)h);
    const int grp = k >> gsh, j = k & ((1 << gsh) - 1);
    out[(grp << (gsh + 1)) + j] = h;
    out[(grp << (gsh + 1)) + (1 << gsh) + j] = lo;
  }
  if (threadIdx.x == 0) base[(int64_t)rows * len + row] = unscale;
}

__global__ void fill_u32_kernel(uint32_t* __restrict__ p, int64_t n, uint32_t v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

static unsigned grid_for(int64_t n, int64_t cap = 4096) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, TPB), cap));
}

// =========================================================================== reductions
constexpr int RED_SPLITS = 128;

__global__ void reduce_rows_l1(const float* __restrict__ slab, int64_t rows, int cols, int64_t chunk, double* ws) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane4 = threadIdx.x >> 6;
  const int64_t r0 = blockIdx.y * chunk;
  const int64_t r1 = std::min<int64_t>(rows, r0 + chunk);
  double acc = 0.0;
  if (col < cols)
    for (int64_t r = r0 + lane4; r < r1; r += 4) acc += (double)slab[r * cols + col];
  __shared__ double red[4][64];
  red[lane4][threadIdx.x & 63] = acc;
  __syncthreads();
  if (lane4 == 0 && col < cols)
    ws[(int64_t)blockIdx.y * cols + col] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// 4 split lanes x 64 columns per block; each lane sums every 4th split (8 independent loads in
// flight), then the 4 lane sums are added in a fixed order: deterministic, and latency-bound work
// spread over 4x the threads of a one-thread-per-column loop.
__global__ void reduce_rows_l2(const double* __restrict__ ws, int splits, int cols, double* out, float* out32) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sl = threadIdx.x >> 6;
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (col < cols) {
    int s = sl;
    for (; s + 28 < splits; s += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += ws[(int64_t)(s + 4 * u) * cols + col];
    }
    for (; s < splits; s += 4) acc[0] += ws[(int64_t)s * cols + col];
  }
  double t = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __shared__ double red[4][64];
  red[sl][threadIdx.x & 63] = t;
  __syncthreads();
  if (sl == 0 && col < cols) {
    const double v = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    if (out) out[col] = v;
    if (out32) out32[col] = (float)v;
  }
}

// up to 8192 blocks: at 8.4M pixels a pixel lane then folds 64 values (C = 64) sequentially in fp32
// before the fixed-order fp64 reduction of the slab (2048 blocks: 256 — the per-channel sums
// here, e.g. the BN-backward sum of dA, cancel, so long fp32 runs cost digits)
int64_t channel_slab_rows(int64_t m) { return std::max<int64_t>(1, std::min<int64_t>(cdiv(m, 256), 8192)); }
// rows (= blocks) of the centered second pass: after the first step it re-reads almost nothing (the shifted
// first pass flags few channels), so its launch is mostly blocks that write a zero row — 512 of them instead
// of up to 8192 (0.77 -> ~0.1 ms per bs=128 step); a re-read still streams at 8 waves per CU
int64_t bn_centered_rows(int64_t m) { return std::min<int64_t>(channel_slab_rows(m), 512); }

// Per-channel reduction skeleton over an NHWC [m][C] range: PL pixel lanes x (C/4) channel groups.
// C in {64,128,256,512}.
template <typename T, typename F>
__device__ inline void channel_loop(int64_t m, int C, F&& body) {
  const int CG = C >> 2;
  const int PL = TPB / CG;
  const int cg = threadIdx.x % CG, pl = threadIdx.x / CG;
  const int64_t rows = gridDim.x;
  const int64_t chunk = (m + rows - 1) / rows;
  const int64_t p0 = blockIdx.x * chunk;
  const int64_t p1 = std::min<int64_t>(m, p0 + chunk);
  for (int64_t p = p0 + pl; p < p1; p += PL) body(p, cg * 4);
}

// sum over the PL pixel lanes of a block for NV f32x4 accumulators -> slab row [NV][C]
template <int NV>
__device__ inline void channel_block_reduce(f32x4 (&acc)[NV], int C, float* slab_row) {
  __shared__ f32x4 red[TPB];
  const int CG = C >> 2;
  const int PL = TPB / CG;
  const int cg = threadIdx.x % CG, pl = threadIdx.x / CG;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    red[threadIdx.x] = acc[v];
    __syncthreads();
    for (int s = PL / 2; s > 0; s >>= 1) {
      if (pl < s) red[threadIdx.x] += red[threadIdx.x + s * CG];
      __syncthreads();
    }
    if (pl == 0) *reinterpret_cast<f32x4*>(slab_row + v * C + cg * 4) = red[threadIdx.x];
    __syncthreads();
  }
}

template <typename T>
__global__ void channel_sum_kernel(const T* __restrict__ x, int64_t m, int C, float* slab) {
  f32x4 acc[1] = {f32x4{0, 0, 0, 0}};
  channel_loop<T>(m, C, [&](int64_t p, int c) { acc[0] += Vec4<T>::load(x + p * C + c); });
  channel_block_reduce<1>(acc, C, slab + (int64_t)blockIdx.x * C);
}

// Second pass of the BatchNorm batch statistics: per-channel sums of d = y - center and d^2
// (center = the first pass's mean) -> slab [rows][2][C]. E[y^2] - mean^2 from the conv epilogue's
// sums loses ~eps * mean^2 / var of the variance (the first layer's invstd came out 14x further from
// the fp64 value than the reference's); the centered sums do not.
//
// Adaptive form (uvar != NULL, selunet_bn_centered_partials_adaptive): uvar = the first pass's
// unbiased variance n/(n-1) * (E[y^2] - mean^2). The first pass loses ~eps * (1 + mean^2/var) of
// the variance, so a group of 4 channels is re-read only if one of them has mean^2 > ratio * var;
// the others emit the sums that reproduce the first pass's variance exactly in the centered
// finalize (sum d = 0, sum d^2 = (n-1) * uvar, in slab row 0) — same outputs, no pass over y.
template <typename T>
__global__ void bn_centered_partials_kernel(const T* __restrict__ y, int64_t m, int C, const float* __restrict__ center,
                                            const float* __restrict__ uvar, float ratio, float* slab) {
  f32x4 acc[2] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
  const int c0 = (threadIdx.x % (C >> 2)) * 4;
  const f32x4 mu = *reinterpret_cast<const f32x4*>(center + c0);
  bool need = true;
  if (uvar) {
    const f32x4 uv = *reinterpret_cast<const f32x4*>(uvar + c0);
    need = false;
#pragma unroll
    for (int e = 0; e < 4; ++e) need |= !(mu[e] * mu[e] <= ratio * uv[e]);  // NaN / tiny var: re-read
    if (!need && blockIdx.x == 0 && threadIdx.x < (C >> 2)) acc[1] = uv * (float)(m - 1);
  }
  if (need) {
    channel_loop<T>(m, C, [&](int64_t p, int c) {
      const f32x4 d = Vec4<T>::load(y + p * C + c) - mu;
      acc[0] += d;
      acc[1] += d * d;
    });
  }
  channel_block_reduce<2>(acc, C, slab + (int64_t)blockIdx.x * 2 * C);
}

// =========================================================================== BatchNorm
// one channel of the BatchNorm finalize: batch statistics from the fp64 sums (training) or the
// running statistics (eval) -> mean (of the conv output without bias), invstd, folded scale/shift
struct BnFinArgs {
  int64_t count;
  const float* conv_bias;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  int64_t* nbt;
  float momentum, eps;
  int training;
  float *mean_o, *invstd_o, *scale_o, *shift_o;
  const float* center;  // non-NULL: s_sum / s_sq are sums of (y - center) and (y - center)^2
  // shifted first pass (selunet_bn_stats_finalize_shifted): uvar_flag_o = the unbiased variance, or -1
  // where (mean - center)^2 > flag_ratio * var (its one-pass variance is not exact enough: the
  // adaptive centered pass re-reads those channels); center_next_o = mean (the next step's center,
  // may alias center: read before written, per channel)
  float* uvar_flag_o;
  float flag_ratio;
  float* center_next_o;
  // bound_o (selunet_bn_stats_finalize_centered_bound): atomic max of (|gamma_c| * bound_sq + |beta_c|)
  // over the channels, the split-fp16 range word of relu(bn(y)) (see selunet_act_bound)
  float* bound_o;
  float bound_sq;
};

__device__ inline void bn_finalize_one(int c, double s_sum, double s_sq, const BnFinArgs& a) {
  const double b = a.conv_bias ? (double)a.conv_bias[c] : 0.0;
  double mean, var;
  if (a.training) {
    const double d = s_sum / (double)a.count;  // mean of y - center
    mean = (a.center ? (double)a.center[c] : 0.0) + d;
    var = s_sq / (double)a.count - d * d;      // centered: no cancellation against mean^2
    if (var < 0) var = 0;
    if (a.rmean) a.rmean[c] = (float)((1.0 - a.momentum) * a.rmean[c] + a.momentum * (mean + b));
    if (a.rvar)
      a.rvar[c] = (float)((1.0 - a.momentum) * a.rvar[c] + a.momentum * var * (double)a.count / (double)(a.count - 1));
  } else {
    mean = (double)a.rmean[c] - b;  // running stats track conv output *with* bias
    var = (double)a.rvar[c];
  }
  if (a.training && a.uvar_flag_o) {
    const double d = mean - (a.center ? (double)a.center[c] : 0.0);
    // the one-pass variance's error is ~eps_fp32 * (var + d^2); it feeds 1/sqrt(var + eps_bn) and the
    // running variance, which is compared raw (relative) with the reference's, so the criterion is on var
    // alone: a near-constant channel (var far below eps_bn) with a mean shift is re-read too
    a.uvar_flag_o[c] = d * d <= (double)a.flag_ratio * var
                           ? (float)(var * (double)a.count / (double)(a.count - 1)) : -1.0f;
  }
  // a non-finite batch mean is not carried into the next step's center (it would poison every later
  // shifted sum of this plan): the center falls back to 0, the unshifted statistics
  if (a.training && a.center_next_o) a.center_next_o[c] = isfinite(mean) ? (float)mean : 0.0f;
  const double inv = 1.0 / sqrt(var + (double)a.eps);
  const double sc = (double)a.gamma[c] * inv;
  a.mean_o[c] = (float)mean;
  a.invstd_o[c] = (float)inv;
  a.scale_o[c] = (float)sc;
  a.shift_o[c] = (float)((double)a.beta[c] - mean * sc);
}

__global__ void bn_finalize_kernel(const double* __restrict__ sums, int C, BnFinArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (a.training && a.nbt && c == 0) *a.nbt += 1;
  if (c >= C) return;
  bn_finalize_one(c, a.training ? sums[c] : 0.0, a.training ? sums[C + c] : 0.0, a);
}

template <typename T>
__global__ void bn_bwd_reduce_kernel(const T* __restrict__ dz, const T* __restrict__ y, int64_t m, int C,
                                     const float* __restrict__ scale, const float* __restrict__ shift,
                                     const float* __restrict__ mean, const float* __restrict__ invstd, float* slab) {
  f32x4 acc[3] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
  const int c0 = (threadIdx.x % (C >> 2)) * 4;
  const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c0);
  const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c0);
  const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + c0);
  const f32x4 is = *reinterpret_cast<const f32x4*>(invstd + c0);
  channel_loop<T>(m, C, [&](int64_t p, int c) {
    const f32x4 yv = Vec4<T>::load(y + p * C + c);
    const f32x4 g = Vec4<T>::load(dz + p * C + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float z = yv[e] * sc[e] + sh[e];
      const float da = z > 0.0f ? g[e] : 0.0f;
      const float xh = (yv[e] - mu[e]) * is[e];
      acc[0][e] += da;
      acc[1][e] += da * xh;
      acc[2][e] += xh;
    }
  });
  channel_block_reduce<3>(acc, C, slab + (int64_t)blockIdx.x * 3 * C);
}

struct BnbFinArgs {
  int64_t count;
  const float* gamma;
  const float* invstd;
  float *dgamma, *dbeta, *dbias, *coef;
  // selunet_bn_bwd_stats_finalize_bound: atomic max of an upper bound of |dy| over the channels into
  // *bound, from the exact max |dA| in *amax_da (the range word of the fused apply's dy operand)
  const float* amax_da;
  float* bound;
};

__device__ inline void bn_bwd_finalize_one(int c, int C, double sda, double sdax, double sx, const BnbFinArgs& a) {
  const double k0 = (double)a.gamma[c] * a.invstd[c];
  const double k1 = k0 * sda / (double)a.count;
  const double k2 = k0 * sdax / (double)a.count;
  if (a.dgamma) a.dgamma[c] = (float)sdax;
  if (a.dbeta) a.dbeta[c] = (float)sda;
  // sum over pixels of the conv-output gradient; analytically zero (BN removes the mean)
  if (a.dbias) a.dbias[c] = (float)(k0 * sda - (double)a.count * k1 - k2 * sx);
  a.coef[c] = (float)k0;
  a.coef[C + c] = (float)k1;
  a.coef[2 * C + c] = (float)k2;
  if (a.bound) {
    // dy = k0 da - k1 - k2 xhat with |da| <= |dA| <= amax_da and |xhat| <= sqrt(count - 1) (Samuelson:
    // batch statistics; the fp32 mean / invstd and the rounding of dy are covered by the 1.25 margin).
    // The split-fp16 operand needs an upper bound only: a loose one costs precision below 2^-17 of it
    // (absolute error <= 2^-39 of the bound), far under fp32 rounding of the products it feeds
    const double bnd = fabs(k0) * (double)a.amax_da[0] + fabs(k1) + fabs(k2) * sqrt((double)a.count);
    atomicMax(reinterpret_cast<unsigned*>(a.bound), __float_as_uint((float)(1.25 * bnd)));
  }
}

__global__ void bn_bwd_finalize_kernel(const double* __restrict__ sums, int C, BnbFinArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  bn_bwd_finalize_one(c, C, sums[c], sums[C + c], sums[2 * C + c], a);
}

// Column sums of a [rows][SETS][C] slab (fp32 partials, or the fp64 first-level split sums) in
// fp64, followed in the same launch by the per-channel BatchNorm finalize (forward, SETS = 2) or
// BatchNorm-backward finalize (SETS = 3): one launch where reduce_rows + *_finalize took three.
// 1024 threads = 16 row lanes x 64 channels; every lane keeps 8 rows x SETS loads in flight, the
// 16 lane sums are added in a fixed order (deterministic).
constexpr int RF_LANES = 16, RF_U = 8;
template <typename S, int SETS>
__global__ void __launch_bounds__(1024) reduce_finalize_kernel(const S* __restrict__ src, int64_t rows, int C,
                                                               double* __restrict__ sums_out, BnFinArgs fa,
                                                               BnbFinArgs ba) {
  const int cl = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int64_t cols = (int64_t)SETS * C;
  double acc[SETS];
#pragma unroll
  for (int s = 0; s < SETS; ++s) acc[s] = 0.0;
  if (c < C) {
    int64_t r = lane;
    for (; r + (RF_U - 1) * RF_LANES < rows; r += RF_U * RF_LANES) {
      S v[RF_U][SETS];
#pragma unroll
      for (int u = 0; u < RF_U; ++u)
#pragma unroll
        for (int s = 0; s < SETS; ++s) v[u][s] = src[(r + u * RF_LANES) * cols + s * C + c];
#pragma unroll
      for (int u = 0; u < RF_U; ++u)
#pragma unroll
        for (int s = 0; s < SETS; ++s) acc[s] += (double)v[u][s];
    }
    for (; r < rows; r += RF_LANES)
#pragma unroll
      for (int s = 0; s < SETS; ++s) acc[s] += (double)src[r * cols + s * C + c];
  }
  __shared__ double red[SETS][RF_LANES][64];
#pragma unroll
  for (int s = 0; s < SETS; ++s) red[s][lane][cl] = acc[s];
  __syncthreads();
  if (SETS == 2 && fa.nbt && threadIdx.x == 0 && blockIdx.x == 0) *fa.nbt += 1;
  if (lane != 0) return;  // (wave-uniform: wave 0 stays whole for the wave-wide range-word max below)
  float bound = 0.0f;      // lanes c >= C contribute 0
  if (c < C) {
    double t[SETS];
#pragma unroll
    for (int s = 0; s < SETS; ++s) {
      double x = 0.0;
#pragma unroll
      for (int l = 0; l < RF_LANES; ++l) x += red[s][l][cl];
      t[s] = x;
      if (sums_out) sums_out[s * C + c] = x;
    }
    if constexpr (SETS == 2) {
      bn_finalize_one(c, t[0], t[1], fa);
      if (fa.bound_o) bound = (fabsf(fa.gamma[c]) * fa.bound_sq + fabsf(fa.beta[c])) * 1.0001f;
    } else {
      bn_bwd_finalize_one(c, C, t[0], t[1], t[2], ba);
    }
  }
  if (SETS == 2 && fa.bound_o) atomic_amax(fa.bound_o, bound);
}

// rows up to which the fused reductions read the fp32 slab in one launch; above it a first level
// (reduce_rows_l1) cuts the rows to <= RED_SPLITS fp64 split sums first (SELUNET_RF_SINGLE)
static int64_t rf_single_rows() { return option(SELUNET_OPT_RF_SINGLE, 1024); }

// slab [rows][SETS][c] fp32 -> launches of the fused reduce + finalize (ws: >= selunet_reduce_ws_bytes(SETS*c))
template <int SETS>
static void launch_reduce_finalize(const float* slab, int64_t rows, int c, double* ws, double* sums,
                                   const BnFinArgs& fa, const BnbFinArgs& ba, hipStream_t st) {
  const unsigned blocks = (unsigned)cdiv(c, 64);
  if (rows <= rf_single_rows()) {
    hipLaunchKernelGGL((reduce_finalize_kernel<float, SETS>), dim3(blocks), dim3(1024), 0, st, slab, rows, c, sums,
                       fa, ba);
    return;
  }
  const int cols = SETS * c;
  const int splits = (int)std::min<int64_t>(RED_SPLITS, cdiv(rows, 16));
  const int64_t chunk = cdiv(rows, splits);
  hipLaunchKernelGGL(reduce_rows_l1, dim3((unsigned)cdiv(cols, 64), splits), dim3(TPB), 0, st, slab, rows, cols, chunk,
                     ws);
  hipLaunchKernelGGL((reduce_finalize_kernel<double, SETS>), dim3(blocks), dim3(1024), 0, st, ws, (int64_t)splits, c,
                     sums, fa, ba);
}

// dy = k0*dA - k1 - k2*xhat = k0*dA - (k1 - k2*mean*invstd) - (k2*invstd)*y. Each thread owns a fixed
// group of 8 channels (coefficients in registers) and strides over pixels: 16-B bf16 / 32-B fp32
// vectors, one pass over dz and y, one write of dy.
template <typename T, int U = 4>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ dz, const T* __restrict__ y, int64_t m, int C,
                                    const float* __restrict__ scale, const float* __restrict__ shift,
                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                    const float* __restrict__ coef, T* __restrict__ dy, float* amax) {
  const int CG = C >> 3;
  const int cg = threadIdx.x % CG, pl = threadIdx.x / CG;
  const int PL = TPB / CG;
  const int c = cg * 8;
  float sc[8], sh[8], k0[8], a[8], b[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[c + e];
    sh[e] = shift[c + e];
    k0[e] = coef[c + e];
    const float k2i = coef[2 * C + c + e] * invstd[c + e];
    a[e] = k2i;
    b[e] = coef[C + c + e] - k2i * mean[c + e];
  }
  // U pixels per thread and iteration, all loads issued before any use (loads in flight per wave)
  const int64_t stride = (int64_t)gridDim.x * PL;
  float am = 0.0f;
  auto one = [&](const f32x4& y0, const f32x4& y1, const f32x4& g0, const f32x4& g1, int64_t off) {
    f32x4 o0, o1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o0[e] = (y0[e] * sc[e] + sh[e] > 0.0f ? k0[e] * g0[e] : 0.0f) - b[e] - a[e] * y0[e];
      o1[e] = (y1[e] * sc[e + 4] + sh[e + 4] > 0.0f ? k0[e + 4] * g1[e] : 0.0f) - b[e + 4] - a[e + 4] * y1[e];
    }
    if (amax) {
#pragma unroll
      for (int e = 0; e < 4; ++e) am = fmaxf(am, fmaxf(fabsf(o0[e]), fabsf(o1[e])));
    }
    Vec4<T>::store(dy + off, o0);
    Vec4<T>::store(dy + off + 4, o1);
  };
  int64_t p = blockIdx.x * (int64_t)PL + pl;
  for (; p + (U - 1) * stride < m; p += U * stride) {
    f32x4 y0[U], y1[U], g0[U], g1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (p + u * stride) * C + c;
      y0[u] = Vec4<T>::load(y + off);
      y1[u] = Vec4<T>::load(y + off + 4);
      g0[u] = Vec4<T>::load(dz + off);
      g1[u] = Vec4<T>::load(dz + off + 4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(y0[u], y1[u], g0[u], g1[u], (p + u * stride) * C + c);
  }
  for (; p < m; p += stride) {
    const int64_t off = p * C + c;
    one(Vec4<T>::load(y + off), Vec4<T>::load(y + off + 4), Vec4<T>::load(dz + off), Vec4<T>::load(dz + off + 4),
        off);
  }
  __shared__ float wred[TPB / 64];
  if (amax) block_amax(amax, am, wred);
}

// The same with 4 channels per thread, lanes of a wave on consecutive 16-B (fp32) vectors: C / 4 lanes per
// pixel, so each load / store instruction covers 64 x 16 contiguous bytes (the 8-channel form above
// reads two interleaved halves of every 32-B segment per instruction); U pixels per thread in flight.
template <typename T, int U>
__global__ void bn_bwd_apply4_kernel(const T* __restrict__ dz, const T* __restrict__ y, int64_t m, int C,
                                     const float* __restrict__ scale, const float* __restrict__ shift,
                                     const float* __restrict__ mean, const float* __restrict__ invstd,
                                     const float* __restrict__ coef, T* __restrict__ dy, float* amax) {
  const int CG = C >> 2;
  const int cg = threadIdx.x % CG, pl = threadIdx.x / CG;
  const int PL = TPB / CG;
  const int c = cg * 4;
  float sc[4], sh[4], k0[4], a[4], b[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    sc[e] = scale[c + e];
    sh[e] = shift[c + e];
    k0[e] = coef[c + e];
    const float k2i = coef[2 * C + c + e] * invstd[c + e];
    a[e] = k2i;
    b[e] = coef[C + c + e] - k2i * mean[c + e];
  }
  const int64_t stride = (int64_t)gridDim.x * PL;
  float am = 0.0f;
  auto one = [&](const f32x4& yv, const f32x4& g, int64_t off) {
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (yv[e] * sc[e] + sh[e] > 0.0f ? k0[e] * g[e] : 0.0f) - b[e] - a[e] * yv[e];
    if (amax) {
#pragma unroll
      for (int e = 0; e < 4; ++e) am = fmaxf(am, fabsf(o[e]));
    }
    Vec4<T>::store(dy + off, o);
  };
  int64_t p = blockIdx.x * (int64_t)PL + pl;
  for (; p + (U - 1) * stride < m; p += U * stride) {
    f32x4 yv[U], g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (p + u * stride) * C + c;
      yv[u] = Vec4<T>::load(y + off);
      g[u] = Vec4<T>::load(dz + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(yv[u], g[u], (p + u * stride) * C + c);
  }
  for (; p < m; p += stride) one(Vec4<T>::load(y + p * C + c), Vec4<T>::load(dz + p * C + c), p * C + c);
  __shared__ float wred[TPB / 64];
  if (amax) block_amax(amax, am, wred);
}

// selunet_act_bound: max_c |gamma_c| * sqrt(count) + max_c |beta_c| (one block)
__global__ void __launch_bounds__(256) act_bound_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        int C, float sq, float* out) {
  float g = 0.0f, b = 0.0f;
  for (int c = threadIdx.x; c < C; c += 256) {
    g = fmaxf(g, fabsf(gamma[c]));
    b = fmaxf(b, fabsf(beta[c]));
  }
  __shared__ float red[2][256];
  red[0][threadIdx.x] = g;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[0][threadIdx.x] = fmaxf(red[0][threadIdx.x], red[0][threadIdx.x + s]);
      red[1][threadIdx.x] = fmaxf(red[1][threadIdx.x], red[1][threadIdx.x + s]);
    }
    __syncthreads();
  }
  // rounded up a little: the bound must hold for the fp32 values the loaders compute
  if (threadIdx.x == 0) out[0] = (red[0][0] * sq + red[1][0]) * 1.0001f;
}

// =========================================================================== first-layer im2col
// x NCHW fp32 [n][c][h][w] -> out [n*h*w][k_pad] (dtype), column tap*c + ci of a 3x3 pad-1 window,
// zero beyond 9c. Lets the C_in = 3 layer (model.py:29) run as a dense GEMM (forward and weight
// gradient) instead of an element-wise gather.
template <typename T>
__global__ void im2col3x3_kernel(const float* __restrict__ x, int n, int c, int h, int w, int k_pad,
                                 T* __restrict__ out) {
  const int64_t M = (int64_t)n * h * w;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < M; p += (int64_t)gridDim.x * blockDim.x) {
    const int xx = (int)(p % w);
    const int64_t t = p / w;
    const int yy = (int)(t % h);
    const int64_t img = t / h;
    T* row = out + p * k_pad;
    for (int k0 = 0; k0 < k_pad; k0 += 8) {
      T v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + e;
        float f = 0.0f;
        if (k < 9 * c) {
          const int tap = k / c, ci = k - tap * c;
          const int ys = yy + tap / 3 - 1, xs = xx + tap % 3 - 1;
          if ((unsigned)ys < (unsigned)h && (unsigned)xs < (unsigned)w)
            f = x[((img * c + ci) * h + ys) * (int64_t)w + xs];
        }
        v[e] = from_f<T>(f);
      }
      if constexpr (sizeof(T) == 2) {
        uint4 o;
        __builtin_memcpy(&o, v, 16);
        *reinterpret_cast<uint4*>(row + k0) = o;
      } else {
        *reinterpret_cast<f32x4*>(row + k0) = f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
        *reinterpret_cast<f32x4*>(row + k0 + 4) = f32x4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
      }
    }
  }
}

// =========================================================================== MaxPool2d(2)
template <typename T>
__device__ inline f32x4 bn_relu4(const T* p, const float* scale, const float* shift, int c) {
  f32x4 v = Vec4<T>::load(p);
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] * scale[c + e] + shift[c + e], 0.0f);
  return v;
}

template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ y, int n, int h, int w, int C, const float* scale,
                                   const float* shift, T* __restrict__ out) {
  const int ho = h >> 1, wo = w >> 1;
  const int64_t nv = (int64_t)n * ho * wo * (C / 4);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % (C / 4)) * 4;
    int64_t p = i / (C / 4);
    const int xo = (int)(p % wo);
    p /= wo;
    const int yo = (int)(p % ho);
    const int64_t img = p / ho;
    const T* b = y + ((img * h + 2 * yo) * w + 2 * xo) * C + c;
    f32x4 best = bn_relu4(b, scale, shift, c);
    const f32x4 v1 = bn_relu4(b + C, scale, shift, c);
    const f32x4 v2 = bn_relu4(b + (int64_t)w * C, scale, shift, c);
    const f32x4 v3 = bn_relu4(b + (int64_t)w * C + C, scale, shift, c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (v1[e] > best[e]) best[e] = v1[e];
      if (v2[e] > best[e]) best[e] = v2[e];
      if (v3[e] > best[e]) best[e] = v3[e];
    }
    Vec4<T>::store(out + i * 4, best);
  }
}

// BN-backward partial sums of dA (channel group c of 4): sum da, sum da*xhat, sum xhat with
// da = dA*[y*scale+shift > 0] (see selunet_bn_bwd_stats)
struct BnbAcc {
  f32x4 acc[3] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
  __device__ inline void add(const f32x4& y, const f32x4& da_raw, const f32x4& sc, const f32x4& sh, const f32x4& mu,
                             const f32x4& is) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float da = y[e] * sc[e] + sh[e] > 0.0f ? da_raw[e] : 0.0f;
      const float xh = (y[e] - mu[e]) * is[e];
      acc[0][e] += da;
      acc[1][e] += da * xh;
      acc[2][e] += xh;
    }
  }
};

// dz = route(dp) + dskip per 2x2 window; with bnb, the BN-backward sums of dz (as stored) too.
// Each thread keeps one 4-channel group (the grid stride is a multiple of C/4), so its sums are
// reduced per block into slab row blockIdx.x.
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ y, int n, int h, int w, int C, const float* scale,
                                   const float* shift, const T* __restrict__ dp, const T* __restrict__ dskip,
                                   T* __restrict__ dz, const float* mean, const float* invstd, float* bn_slab,
                                   float* da_amax) {
  const int ho = h >> 1, wo = w >> 1;
  const int CG = C >> 2;
  const int64_t nv = (int64_t)n * ho * wo * CG;
  const int c = (int)(threadIdx.x % CG) * 4;
  const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c);
  const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c);
  f32x4 mu = f32x4{0, 0, 0, 0}, is = f32x4{0, 0, 0, 0};
  if (bn_slab) {
    mu = *reinterpret_cast<const f32x4*>(mean + c);
    is = *reinterpret_cast<const f32x4*>(invstd + c);
  }
  BnbAcc bn;
  float am = 0.0f;  // da_amax: max |dA| as stored
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned p = (unsigned)(i / CG);  // output pixel (< 2^31: checked on the host)
    const unsigned xo = p % (unsigned)wo, t = p / (unsigned)wo;
    const unsigned yo = t % (unsigned)ho, img = t / (unsigned)ho;
    const int64_t base = (((int64_t)img * h + 2 * yo) * w + 2 * xo) * C + c;
    const int64_t off[4] = {base, base + C, base + (int64_t)w * C, base + (int64_t)w * C + C};
    f32x4 yr[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) yr[q] = Vec4<T>::load(y + off[q]);
    int arg[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float best = fmaxf(yr[0][e] * sc[e] + sh[e], 0.0f);
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const float v = fmaxf(yr[q][e] * sc[e] + sh[e], 0.0f);
        if (v > best) {  // first maximum in row-major window order (ATen, strict >)
          best = v;
          arg[e] = q;
        }
      }
    }
    const f32x4 g = Vec4<T>::load(dp + i * 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 o = dskip ? Vec4<T>::load(dskip + off[q]) : f32x4{0, 0, 0, 0};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (arg[e] == q) o[e] += g[e];
      if (dz) Vec4<T>::store(dz + off[q], o);  // (null: the sums only, selunet_bn_bwd_apply_pool forms dz)
      if (bn_slab || da_amax) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = to_f(from_f<T>(o[e]));  // as stored
        if (bn_slab) bn.add(yr[q], o, sc, sh, mu, is);
#pragma unroll
        for (int e = 0; e < 4; ++e) am = fmaxf(am, fabsf(o[e]));
      }
    }
  }
  if (bn_slab) channel_block_reduce<3>(bn.acc, C, bn_slab + (int64_t)blockIdx.x * 3 * C);
  __shared__ float wred[TPB / 64];
  if (da_amax) block_amax(da_amax, am, wred);
}

// =========================================================================== 1x1 heads (C = 64)
// 16 lanes per pixel, 4 channels per lane; 4 pixels per wave instruction.
constexpr int HU = 4;

// Sum over each 16-lane row of the wave, in every lane of the row, by DPP moves (VALU): quad xor 1,
// quad xor 2, half-row mirror, row mirror. A __shfl_xor butterfly compiles to ds_bpermute through the
// LDS crossbar, each waited on in turn (12 per pixel group in heads_fwd).
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));  // row_mirror
  return v;
}
template <typename T>
__global__ void heads_fwd_kernel(const T* __restrict__ y, int64_t m, const float* __restrict__ scale,
                                 const float* __restrict__ shift, const float* __restrict__ w,
                                 const float* __restrict__ b, int nh, float* o0, float* o1, float* o2) {
  const int sub = threadIdx.x & 15;
  const int c = sub * 4;
  const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c);
  const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c);
  f32x4 wv[3];
  for (int h = 0; h < 3; ++h) wv[h] = h < nh ? *reinterpret_cast<const f32x4*>(w + h * 64 + c) : f32x4{0, 0, 0, 0};
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x >> 4);
  auto one = [&](f32x4 z, int64_t p) {
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = fmaxf(z[e] * sc[e] + sh[e], 0.0f);
    float acc[3];
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      acc[h] = row16_sum(z[0] * wv[h][0] + z[1] * wv[h][1] + z[2] * wv[h][2] + z[3] * wv[h][3]);
    }
    if (sub == 0) {
      o0[p] = acc[0] + b[0];
      if (nh > 1) {
        o1[p] = acc[1] + b[1];
        o2[p] = acc[2] + b[2];
      }
    }
  };
  // HU pixels per lane group and iteration, loads issued before any use
  int64_t p = blockIdx.x * (int64_t)(blockDim.x >> 4) + (threadIdx.x >> 4);
  for (; p + (HU - 1) * stride < m; p += HU * stride) {
    f32x4 z[HU];
#pragma unroll
    for (int u = 0; u < HU; ++u) z[u] = Vec4<T>::load(y + (p + u * stride) * 64 + c);
#pragma unroll
    for (int u = 0; u < HU; ++u) one(z[u], p + u * stride);
  }
  for (; p < m; p += stride) one(Vec4<T>::load(y + p * 64 + c), p);
}

template <typename T>
__global__ void heads_bwd_kernel(const T* __restrict__ y, int64_t m, const float* __restrict__ scale,
                                 const float* __restrict__ shift, const float* __restrict__ w, int nh,
                                 const float* __restrict__ g0, const float* __restrict__ g1,
                                 const float* __restrict__ g2, T* __restrict__ dz, float* slab,
                                 const float* __restrict__ mean, const float* __restrict__ invstd, float* bn_slab,
                                 float* da_amax) {
  const int sub = threadIdx.x & 15;
  const int c = sub * 4;
  const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c);
  const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c);
  f32x4 wv[3];
  for (int h = 0; h < 3; ++h) wv[h] = h < nh ? *reinterpret_cast<const f32x4*>(w + h * 64 + c) : f32x4{0, 0, 0, 0};
  f32x4 dw[3] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
  float db[3] = {0, 0, 0};
  f32x4 mu = f32x4{0, 0, 0, 0}, is = f32x4{0, 0, 0, 0};
  if (bn_slab) {
    mu = *reinterpret_cast<const f32x4*>(mean + c);
    is = *reinterpret_cast<const f32x4*>(invstd + c);
  }
  BnbAcc bn;
  float am = 0.0f;  // da_amax: max |dA| as stored
  const int64_t rows = gridDim.x;
  const int64_t chunk = (m + rows - 1) / rows;
  const int64_t p0 = blockIdx.x * chunk, p1 = std::min<int64_t>(m, p0 + chunk);
  auto one = [&](const f32x4& yv, const float* g, int64_t p) {
    f32x4 z;
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = fmaxf(yv[e] * sc[e] + sh[e], 0.0f);
    f32x4 d = wv[0] * g[0] + wv[1] * g[1] + wv[2] * g[2];  // (as bn_bwd_apply_heads_kernel forms it)
    if (dz) Vec4<T>::store(dz + p * 64 + c, d);  // (null: the sums only, selunet_bn_bwd_apply_heads forms dz)
    if (bn_slab || da_amax) {
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = to_f(from_f<T>(d[e]));  // as stored
      if (bn_slab) bn.add(yv, d, sc, sh, mu, is);
#pragma unroll
      for (int e = 0; e < 4; ++e) am = fmaxf(am, fabsf(d[e]));
    }
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      dw[h] += z * g[h];
      db[h] += g[h];
    }
  };
  int64_t p = p0 + (threadIdx.x >> 4);
  constexpr int PS = TPB >> 4;
  for (; p + (HU - 1) * PS < p1; p += HU * PS) {
    f32x4 yv[HU];
    float g[HU][3];
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const int64_t q = p + u * PS;
      yv[u] = Vec4<T>::load(y + q * 64 + c);
      g[u][0] = g0[q];
      g[u][1] = nh > 1 ? g1[q] : 0.0f;
      g[u][2] = nh > 1 ? g2[q] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < HU; ++u) one(yv[u], g[u], p + u * PS);
  }
  for (; p < p1; p += PS) {
    const float g[3] = {g0[p], nh > 1 ? g1[p] : 0.0f, nh > 1 ? g2[p] : 0.0f};
    one(Vec4<T>::load(y + p * 64 + c), g, p);
  }
  // block reduce: 16 pixel lanes per channel group
  __shared__ float red[TPB][13];
  for (int h = 0; h < 3; ++h) {
    red[threadIdx.x][h * 4 + 0] = dw[h][0];
    red[threadIdx.x][h * 4 + 1] = dw[h][1];
    red[threadIdx.x][h * 4 + 2] = dw[h][2];
    red[threadIdx.x][h * 4 + 3] = dw[h][3];
  }
  __syncthreads();
  float* row = slab + (int64_t)blockIdx.x * nh * 65;
  if (threadIdx.x < 16) {
    for (int h = 0; h < nh; ++h)
      for (int e = 0; e < 4; ++e) {
        float s = 0.0f;
        for (int q = 0; q < 16; ++q) s += red[q * 16 + threadIdx.x][h * 4 + e];
        row[h * 65 + threadIdx.x * 4 + e] = s;
      }
  }
  __syncthreads();
  // bias: each pixel is seen by 16 lanes; the sub == 0 lane carries its g
  for (int h = 0; h < nh; ++h) {
    red[threadIdx.x][12] = (sub == 0) ? db[h] : 0.0f;
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.0f;
      for (int q = 0; q < TPB; q += 16) s += red[q][12];
      row[h * 65 + 64] = s;
    }
    __syncthreads();
  }
  if (bn_slab) channel_block_reduce<3>(bn.acc, 64, bn_slab + (int64_t)blockIdx.x * 3 * 64);
  __shared__ float wred[TPB / 64];
  if (da_amax) block_amax(da_amax, am, wred);
}

// =========================================================================== BN-backward apply with dA formed
// on the fly. Two producers of a layer's dA are cheap to recompute: the 1x1 heads' backward (dA = sum_h
// g_h w_h, three fp32 planes) and the max-pool backward (dA = route(dP) + dskip). Their kernels then run
// in sums-only mode (dz = null: the BN-backward sums of dA as it would be stored, no write), and the
// apply forms dA again from (g planes | y, dP, dskip) instead of reading it: the heads path saves dA's
// write and re-read (2 x M x 64 x esz), the pool path dA's write (its re-read becomes the dskip read).
// dy = (y sc + sh > 0 ? k0 dA : 0) - b - a y exactly as bn_bwd_apply_kernel, dA rounded to T first (as
// stored in the unfused path).
struct ApplyCoef {
  f32x4 sc, sh, k0, a, b;
};
__device__ inline ApplyCoef apply_coef(const float* scale, const float* shift, const float* mean, const float* invstd,
                                       const float* coef, int C, int c) {
  ApplyCoef q;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    q.sc[e] = scale[c + e];
    q.sh[e] = shift[c + e];
    q.k0[e] = coef[c + e];
    const float k2i = coef[2 * C + c + e] * invstd[c + e];
    q.a[e] = k2i;
    q.b[e] = coef[C + c + e] - k2i * mean[c + e];
  }
  return q;
}
__device__ inline f32x4 apply4(const ApplyCoef& q, const f32x4& y, const f32x4& g) {
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = (y[e] * q.sc[e] + q.sh[e] > 0.0f ? q.k0[e] * g[e] : 0.0f) - q.b[e] - q.a[e] * y[e];
  return o;
}
template <typename T>
__device__ inline f32x4 as_stored(f32x4 v) {
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = to_f(from_f<T>(v[e]));
  return v;
}

// heads (C = 64): 16 lanes per pixel, 4 channels per lane, HU pixels per lane group in flight
template <typename T>
__global__ void bn_bwd_apply_heads_kernel(const T* __restrict__ y, int64_t m, const float* __restrict__ scale,
                                          const float* __restrict__ shift, const float* __restrict__ mean,
                                          const float* __restrict__ invstd, const float* __restrict__ coef,
                                          const float* __restrict__ w, int nh, const float* __restrict__ g0,
                                          const float* __restrict__ g1, const float* __restrict__ g2,
                                          T* __restrict__ dy, float* amax) {
  const int sub = threadIdx.x & 15;
  const int c = sub * 4;
  const ApplyCoef q = apply_coef(scale, shift, mean, invstd, coef, 64, c);
  f32x4 wv[3];
  for (int h = 0; h < 3; ++h) wv[h] = h < nh ? *reinterpret_cast<const f32x4*>(w + h * 64 + c) : f32x4{0, 0, 0, 0};
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x >> 4);
  float am = 0.0f;
  auto one = [&](const f32x4& yv, const float* g, int64_t p) {
    const f32x4 d = as_stored<T>(wv[0] * g[0] + wv[1] * g[1] + wv[2] * g[2]);
    const f32x4 o = apply4(q, yv, d);
    if (amax) {
#pragma unroll
      for (int e = 0; e < 4; ++e) am = fmaxf(am, fabsf(o[e]));
    }
    Vec4<T>::store(dy + p * 64 + c, o);
  };
  int64_t p = blockIdx.x * (int64_t)(blockDim.x >> 4) + (threadIdx.x >> 4);
  for (; p + (HU - 1) * stride < m; p += HU * stride) {
    f32x4 yv[HU];
    float g[HU][3];
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const int64_t r = p + u * stride;
      yv[u] = Vec4<T>::load(y + r * 64 + c);
      g[u][0] = g0[r];
      g[u][1] = nh > 1 ? g1[r] : 0.0f;
      g[u][2] = nh > 1 ? g2[r] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < HU; ++u) one(yv[u], g[u], p + u * stride);
  }
  for (; p < m; p += stride) {
    const float g[3] = {g0[p], nh > 1 ? g1[p] : 0.0f, nh > 1 ? g2[p] : 0.0f};
    one(Vec4<T>::load(y + p * 64 + c), g, p);
  }
  __shared__ float wred[TPB / 64];
  if (amax) block_amax(amax, am, wred);
}

// max-pool: one 2x2 window x 4 channels per thread and iteration (maxpool_bwd_kernel's decomposition; each
// thread keeps one channel group, the grid stride is a multiple of C/4)
template <typename T>
__global__ void bn_bwd_apply_pool_kernel(const T* __restrict__ y, int n, int h, int w, int C,
                                         const float* __restrict__ scale, const float* __restrict__ shift,
                                         const float* __restrict__ mean, const float* __restrict__ invstd,
                                         const float* __restrict__ coef, const T* __restrict__ dp,
                                         const T* __restrict__ dskip, T* __restrict__ dy, float* amax) {
  const int ho = h >> 1, wo = w >> 1;
  const int CG = C >> 2;
  const int64_t nv = (int64_t)n * ho * wo * CG;
  const int c = (int)(threadIdx.x % CG) * 4;
  const ApplyCoef q = apply_coef(scale, shift, mean, invstd, coef, C, c);
  float am = 0.0f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned p = (unsigned)(i / CG);  // output pixel (< 2^31: checked on the host)
    const unsigned xo = p % (unsigned)wo, t = p / (unsigned)wo;
    const unsigned yo = t % (unsigned)ho, img = t / (unsigned)ho;
    const int64_t base = (((int64_t)img * h + 2 * yo) * w + 2 * xo) * C + c;
    const int64_t off[4] = {base, base + C, base + (int64_t)w * C, base + (int64_t)w * C + C};
    f32x4 yr[4], sk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      yr[k] = Vec4<T>::load(y + off[k]);
      sk[k] = dskip ? Vec4<T>::load(dskip + off[k]) : f32x4{0, 0, 0, 0};
    }
    const f32x4 g = Vec4<T>::load(dp + i * 4);
    int arg[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float best = fmaxf(yr[0][e] * q.sc[e] + q.sh[e], 0.0f);
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const float v = fmaxf(yr[k][e] * q.sc[e] + q.sh[e], 0.0f);
        if (v > best) {  // first maximum in row-major window order (ATen, strict >), as maxpool_bwd_kernel
          best = v;
          arg[e] = k;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x4 d = sk[k];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (arg[e] == k) d[e] += g[e];
      const f32x4 o = apply4(q, yr[k], as_stored<T>(d));
      if (amax) {
#pragma unroll
        for (int e = 0; e < 4; ++e) am = fmaxf(am, fabsf(o[e]));
      }
      Vec4<T>::store(dy + off[k], o);
    }
  }
  __shared__ float wred[TPB / 64];
  if (amax) block_amax(amax, am, wred);
}

// =========================================================================== losses
int64_t loss_slab_rows(int64_t p) { return std::max<int64_t>(1, std::min<int64_t>(cdiv(p, 4096), 1024)); }

template <int NV>
__device__ inline void block_sum_store(float (&v)[NV], float* dst) {
  __shared__ float red[NV][TPB / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float s = wave_sum(v[k]);
    if (lane == 0) red[k][wv] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    float s = 0.0f;
    for (int q = 0; q < TPB / 64; ++q) s += red[threadIdx.x][q];
    dst[threadIdx.x] = s;
  }
}

// HARD (hard_selection=True, selective_loss.py:74-77): the risk numerator weights each pixel by the
// detached hard selection [sigmoid(g) > 0.5] instead of sigmoid(g); the coverage stays the soft mean.
template <bool HARD>
__global__ void selective_partials_kernel(const float* __restrict__ out, const float* __restrict__ sel,
                                          const float* __restrict__ tgt, int64_t P, float* slab) {
  const int64_t rows = gridDim.x;
  const int64_t chunk = (P + rows - 1) / rows;
  const int64_t p0 = blockIdx.x * chunk, p1 = std::min<int64_t>(P, p0 + chunk);
  float acc[2] = {0.0f, 0.0f};
  for (int64_t i = p0 + threadIdx.x; i < p1; i += TPB) {
    const float s = sigmoidf_(sel[i]);
    const float x = out[i], t = tgt[i];
    const float ell = t * softplusf_(-x) + (1.0f - t) * softplusf_(x);
    acc[0] += s;
    acc[1] += ell * (HARD ? (s > 0.5f ? 1.0f : 0.0f) : s);
  }
  block_sum_store<2>(acc, slab + blockIdx.x * 2);
}

__global__ void selective_finalize_kernel(const double* sums, double P, float lamb, float tc, float* loss,
                                          float* coverage, float* state) {
  const double S0 = sums[0], S1 = sums[1];
  const double cov = S0 / P;
  const double R = S1 / S0;
  const double d = fmax((double)tc - cov, 0.0);
  loss[0] = (float)(R + (double)lamb * d * d);
  coverage[0] = (float)cov;
  state[0] = (float)S0;
  state[1] = (float)R;
  state[2] = (float)d;
  state[3] = (float)P;
}

// HARD: selection and coverage are detached (selective_loss.py:75-76), so d_sel = 0 and the
// output gradient carries the hard weight over the (constant) soft selection sum.
template <bool HARD>
__global__ void selective_bwd_kernel(const float* __restrict__ out, const float* __restrict__ sel,
                                     const float* __restrict__ tgt, int64_t P, const float* state, float lamb,
                                     const float* g_loss, const float* g_cov, float* d_out, float* d_sel) {
  const float S0 = state[0], R = state[1], d = state[2], Pg = state[3];
  const float gl = g_loss ? g_loss[0] : 1.0f;
  const float gc = g_cov ? g_cov[0] : 0.0f;
  const float inv_s0 = 1.0f / S0;
  const float cterm = (gc - gl * 2.0f * lamb * d) / Pg;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    const float s = sigmoidf_(sel[i]);
    const float x = out[i], t = tgt[i];
    const float px = sigmoidf_(x);
    if constexpr (HARD) {
      d_out[i] = gl * (s > 0.5f ? 1.0f : 0.0f) * (px - t) * inv_s0;
      d_sel[i] = 0.0f;
    } else {
      const float ell = t * softplusf_(-x) + (1.0f - t) * softplusf_(x);
      d_out[i] = gl * s * (px - t) * inv_s0;
      d_sel[i] = s * (1.0f - s) * (gl * (ell - R) * inv_s0 + cterm);
    }
  }
}

__global__ void bce_partials_kernel(const float* __restrict__ a, const float* __restrict__ t, int64_t P, float* slab) {
  const int64_t rows = gridDim.x;
  const int64_t chunk = (P + rows - 1) / rows;
  const int64_t p0 = blockIdx.x * chunk, p1 = std::min<int64_t>(P, p0 + chunk);
  float acc[1] = {0.0f};
  for (int64_t i = p0 + threadIdx.x; i < p1; i += TPB) {
    const float x = a[i], y = t[i];
    acc[0] += (1.0f - y) * x + softplusf_(-x);  // = -[y log s(x) + (1-y) log(1-s(x))]
  }
  block_sum_store<1>(acc, slab + blockIdx.x);
}

__global__ void bce_finalize_kernel(const double* sums, double P, float* loss) { loss[0] = (float)(sums[0] / P); }

__global__ void bce_bwd_kernel(const float* __restrict__ a, const float* __restrict__ t, int64_t P, float inv_p,
                               const float* g_loss, float* d) {
  const float g = g_loss ? g_loss[0] : 1.0f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = g * (sigmoidf_(a[i]) - t[i]) * inv_p;
}

// =========================================================================== N-output heads
// The CE UNet's heads (model.py:170,174-175; 2 + 2 + 2 outputs for n_cls = 2) on relu(bn(y)):
// 16 lanes per pixel (4 channels each), one 16-lane shuffle reduction per output. Outputs go to
// per-output planes with an image stride, so NCHW logits are written in place.
struct HeadPlanesArg {
  int n, hw;
  float* plane[8];
  int64_t img_stride[8];
  int w_off[8], b_off[8];
  int row_len;
};

template <typename T>
__global__ void heads_n_fwd_kernel(const T* __restrict__ y, int64_t m, const float* __restrict__ scale,
                                   const float* __restrict__ shift, const float* __restrict__ w,
                                   const float* __restrict__ b, HeadPlanesArg hp) {
  const int sub = threadIdx.x & 15;
  const int c = sub * 4;
  const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c);
  const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c);
  f32x4 wv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) wv[k] = k < hp.n ? *reinterpret_cast<const f32x4*>(w + k * 64 + c) : f32x4{0, 0, 0, 0};
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x >> 4);
  for (int64_t p = blockIdx.x * (int64_t)(blockDim.x >> 4) + (threadIdx.x >> 4); p < m; p += stride) {
    f32x4 z = Vec4<T>::load(y + p * 64 + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = fmaxf(z[e] * sc[e] + sh[e], 0.0f);
    const int64_t img = p / hp.hw, q = p - img * hp.hw;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < hp.n) {
        const float a = row16_sum(z[0] * wv[k][0] + z[1] * wv[k][1] + z[2] * wv[k][2] + z[3] * wv[k][3]);
        if (sub == 0) hp.plane[k][img * hp.img_stride[k] + q] = a + b[k];
      }
    }
  }
}

template <typename T>
__global__ void heads_n_bwd_kernel(const T* __restrict__ y, int64_t m, const float* __restrict__ scale,
                                   const float* __restrict__ shift, const float* __restrict__ w, HeadPlanesArg hp,
                                   T* __restrict__ dz, float* slab, const float* __restrict__ mean,
                                   const float* __restrict__ invstd, float* bn_slab) {
  const int sub = threadIdx.x & 15;
  const int c = sub * 4;
  const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c);
  const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c);
  f32x4 wv[8], dw[8];
  float db[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wv[k] = k < hp.n ? *reinterpret_cast<const f32x4*>(w + k * 64 + c) : f32x4{0, 0, 0, 0};
    dw[k] = f32x4{0, 0, 0, 0};
    db[k] = 0.0f;
  }
  f32x4 mu = f32x4{0, 0, 0, 0}, is = f32x4{0, 0, 0, 0};
  if (bn_slab) {
    mu = *reinterpret_cast<const f32x4*>(mean + c);
    is = *reinterpret_cast<const f32x4*>(invstd + c);
  }
  BnbAcc bn;
  const int64_t rows = gridDim.x;
  const int64_t chunk = (m + rows - 1) / rows;
  const int64_t p0 = blockIdx.x * chunk, p1 = std::min<int64_t>(m, p0 + chunk);
  for (int64_t p = p0 + (threadIdx.x >> 4); p < p1; p += (TPB >> 4)) {
    const f32x4 yv = Vec4<T>::load(y + p * 64 + c);
    f32x4 z;
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = fmaxf(yv[e] * sc[e] + sh[e], 0.0f);
    const int64_t img = p / hp.hw, q = p - img * hp.hw;
    f32x4 d = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < hp.n) {
        const float g = hp.plane[k][img * hp.img_stride[k] + q];
        d += wv[k] * g;
        dw[k] += z * g;
        db[k] += g;
      }
    }
    if (dz) Vec4<T>::store(dz + p * 64 + c, d);  // (null: the sums only, selunet_bn_bwd_apply_heads_planes forms dz)
    if (bn_slab) {
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = to_f(from_f<T>(d[e]));  // as stored
      bn.add(yv, d, sc, sh, mu, is);
    }
  }
  // block reduce: the 16 pixel lanes of each channel group, then the weight/bias sums per output
  __shared__ f32x4 red[TPB];
  __shared__ float redb[TPB];
  float* row = slab + (int64_t)blockIdx.x * hp.row_len;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k < hp.n) {  // (block-uniform)
      red[threadIdx.x] = dw[k];
      redb[threadIdx.x] = sub == 0 ? db[k] : 0.0f;  // each pixel's g is carried by its sub == 0 lane
      __syncthreads();
      if (threadIdx.x < 16) {
        f32x4 s = f32x4{0, 0, 0, 0};
        for (int q = 0; q < TPB / 16; ++q) s += red[q * 16 + threadIdx.x];
#pragma unroll
        for (int e = 0; e < 4; ++e) row[hp.w_off[k] + threadIdx.x * 4 + e] = s[e];  // (any offset)
      }
      if (threadIdx.x == 16) {
        float s = 0.0f;
        for (int q = 0; q < TPB; q += 16) s += redb[q];
        row[hp.b_off[k]] = s;
      }
      __syncthreads();
    }
  }
  if (bn_slab) channel_block_reduce<3>(bn.acc, 64, bn_slab + (int64_t)blockIdx.x * 3 * 64);
}

// the N-output heads of the CE UNet (up to 8 gradient planes, selunet_head_planes): dA = sum_k g_k w_k,
// formed in the order of heads_n_bwd_kernel
template <typename T>
__global__ void bn_bwd_apply_heads_planes_kernel(const T* __restrict__ y, int64_t m, const float* __restrict__ scale,
                                                 const float* __restrict__ shift, const float* __restrict__ mean,
                                                 const float* __restrict__ invstd, const float* __restrict__ coef,
                                                 const float* __restrict__ w, HeadPlanesArg hp, T* __restrict__ dy,
                                                 float* amax) {
  const int sub = threadIdx.x & 15;
  const int c = sub * 4;
  const ApplyCoef q = apply_coef(scale, shift, mean, invstd, coef, 64, c);
  f32x4 wv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) wv[k] = k < hp.n ? *reinterpret_cast<const f32x4*>(w + k * 64 + c) : f32x4{0, 0, 0, 0};
  float am = 0.0f;
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x >> 4);
  for (int64_t p = blockIdx.x * (int64_t)(blockDim.x >> 4) + (threadIdx.x >> 4); p < m; p += stride) {
    const f32x4 yv = Vec4<T>::load(y + p * 64 + c);
    const int64_t img = p / hp.hw, qq = p - img * hp.hw;
    f32x4 d = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < hp.n) d += wv[k] * hp.plane[k][img * hp.img_stride[k] + qq];
    }
    const f32x4 o = apply4(q, yv, as_stored<T>(d));
    if (amax) {
#pragma unroll
      for (int e = 0; e < 4; ++e) am = fmaxf(am, fabsf(o[e]));
    }
    Vec4<T>::store(dy + p * 64 + c, o);
  }
  __shared__ float wred[TPB / 64];
  if (amax) block_amax(amax, am, wred);
}


// =========================================================================== cross-entropy losses
// logits NCHW [N][C][hw]; lse over C <= 8 classes (max-shifted), ell = lse - x[t]
__device__ __forceinline__ float ce_pixel(const float* __restrict__ x, int64_t base, int64_t hw, int C, int t,
                                          float (&e)[8], float& inv_se) {
  float xv[8];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    xv[c] = c < C ? x[base + c * hw] : -INFINITY;
    mx = fmaxf(mx, xv[c]);
  }
  float se = 0.0f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    e[c] = c < C ? __expf(xv[c] - mx) : 0.0f;
    se += e[c];
  }
  inv_se = 1.0f / se;
  float xt = t < 0 ? __builtin_nanf("") : xv[0];
#pragma unroll
  for (int c = 1; c < 8; ++c) xt = c == t ? xv[c] : xt;
  return mx + __logf(se) - xt;
}

// class index of pixel i, or -1 outside [0, C): such a target (e.g. torch's ignore_index -100, or
// an unconverted 0/255 mask) makes the pixel's loss term and gradients NaN — torch's
// CrossEntropyLoss and the reference's scatter_ one-hot reject it — instead of being trained as
// a clamped class
__device__ __forceinline__ int ce_target(const int64_t* tgt, int64_t i, int C) {
  const int64_t t = tgt[i];
  return (t < 0 || t >= C) ? -1 : (int)t;
}
__device__ __forceinline__ float ce_onehot(int c, int t) { return t < 0 ? __builtin_nanf("") : (c == t ? 1.0f : 0.0f); }

template <bool HARD>
__global__ void ce_selective_partials_kernel(const float* __restrict__ out, const float* __restrict__ sel,
                                             const int64_t* __restrict__ tgt, int64_t P, int C, int64_t hw,
                                             float* slab) {
  const int64_t rows = gridDim.x;
  const int64_t chunk = (P + rows - 1) / rows;
  const int64_t p0 = blockIdx.x * chunk, p1 = std::min<int64_t>(P, p0 + chunk);
  float acc[2] = {0.0f, 0.0f};
  for (int64_t i = p0 + threadIdx.x; i < p1; i += TPB) {
    const int64_t img = i / hw, q = i - img * hw;
    const float s = sigmoidf_(sel[(img * 2 + 1) * hw + q] - sel[img * 2 * hw + q]);  // softmax(.)[:, 1]
    float e[8], inv_se;
    const float ell = ce_pixel(out, img * C * hw + q, hw, C, ce_target(tgt, i, C), e, inv_se);
    acc[0] += s;
    acc[1] += ell * (HARD ? (s > 0.5f ? 1.0f : 0.0f) : s);
  }
  block_sum_store<2>(acc, slab + blockIdx.x * 2);
}

template <bool HARD>
__global__ void ce_selective_bwd_kernel(const float* __restrict__ out, const float* __restrict__ sel,
                                        const int64_t* __restrict__ tgt, int64_t P, int C, int64_t hw,
                                        const float* state, float lamb, const float* g_loss, const float* g_cov,
                                        float* d_out, float* d_sel) {
  const float S0 = state[0], R = state[1], d = state[2], Pg = state[3];
  const float gl = g_loss ? g_loss[0] : 1.0f;
  const float gc = g_cov ? g_cov[0] : 0.0f;
  const float inv_s0 = 1.0f / S0;
  const float cterm = (gc - gl * 2.0f * lamb * d) / Pg;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t img = i / hw, q = i - img * hw;
    const int64_t s0i = img * 2 * hw + q, s1i = s0i + hw;
    const float s = sigmoidf_(sel[s1i] - sel[s0i]);
    const int t = ce_target(tgt, i, C);
    const int64_t base = img * C * hw + q;
    float e[8], inv_se;
    const float ell = ce_pixel(out, base, hw, C, t, e, inv_se);
    const float k = gl * (HARD ? (s > 0.5f ? 1.0f : 0.0f) : s) * inv_s0;
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (c < C) d_out[base + c * hw] = k * (e[c] * inv_se - ce_onehot(c, t));
    const float ds = HARD ? 0.0f : s * (1.0f - s) * (gl * (ell - R) * inv_s0 + cterm);
    d_sel[s1i] = ds;
    d_sel[s0i] = -ds;
  }
}

__global__ void ce_partials_kernel(const float* __restrict__ a, const int64_t* __restrict__ tgt, int64_t P, int C,
                                   int64_t hw, float* slab) {
  const int64_t rows = gridDim.x;
  const int64_t chunk = (P + rows - 1) / rows;
  const int64_t p0 = blockIdx.x * chunk, p1 = std::min<int64_t>(P, p0 + chunk);
  float acc[1] = {0.0f};
  for (int64_t i = p0 + threadIdx.x; i < p1; i += TPB) {
    const int64_t img = i / hw, q = i - img * hw;
    float e[8], inv_se;
    acc[0] += ce_pixel(a, img * C * hw + q, hw, C, ce_target(tgt, i, C), e, inv_se);
  }
  block_sum_store<1>(acc, slab + blockIdx.x);
}

__global__ void ce_bwd_kernel(const float* __restrict__ a, const int64_t* __restrict__ tgt, int64_t P, int C,
                              int64_t hw, float inv_p, const float* g_loss, float* d) {
  const float g = (g_loss ? g_loss[0] : 1.0f) * inv_p;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t img = i / hw, q = i - img * hw;
    const int64_t base = img * C * hw + q;
    const int t = ce_target(tgt, i, C);
    float e[8], inv_se;
    ce_pixel(a, base, hw, C, t, e, inv_se);
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (c < C) d[base + c * hw] = g * (e[c] * inv_se - ce_onehot(c, t));
  }
}

// =========================================================================== Adam
__global__ void adam_kernel(const selunet_adam_tensor* __restrict__ list, int n, float lr_bc1, float beta1,
                            float beta2, float eps, float wd, float bc2_sqrt) {
  const int64_t chunk = blockIdx.x;
  int t = 0;
  while (t + 1 < n && list[t + 1].chunk_begin <= chunk) ++t;
  const selunet_adam_tensor T = list[t];
  const int64_t base = (chunk - T.chunk_begin) * SELUNET_ADAM_CHUNK;
  const int64_t end = std::min<int64_t>(T.numel, base + SELUNET_ADAM_CHUNK);
  for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) {
    float g = T.grad[i];
    float p = T.param[i];
    if (wd != 0.0f) g += wd * p;
    float m = T.exp_avg[i];
    m = m + (1.0f - beta1) * (g - m);  // exp_avg.lerp_(grad, 1 - beta1)
    float v = T.exp_avg_sq[i] * beta2 + (1.0f - beta2) * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p - lr_bc1 * (m / denom);
    T.exp_avg[i] = m;
    T.exp_avg_sq[i] = v;
    T.param[i] = p;
  }
}

}  // namespace selunet

using namespace selunet;

#define DISPATCH_T(dtype, ...)                                                      \
  do {                                                                              \
    if ((dtype) == SELUNET_F32) {                                                   \
      using T = float;                                                              \
      __VA_ARGS__;                                                                  \
    } else if ((dtype) == SELUNET_BF16) {                                           \
      using T = __bf16;                                                             \
      __VA_ARGS__;                                                                  \
    } else {                                                                        \
      return fail(SELUNET_EINVAL, "dtype must be SELUNET_F32 or SELUNET_BF16");    \
    }                                                                               \
  } while (0)

static bool ok_channels(int32_t c) { return c == 64 || c == 128 || c == 256 || c == 512; }

extern "C" {

const char* selunet_last_error(void) { return g_err; }
int32_t selunet_version(void) { return 1; }

int64_t selunet_set_option(int32_t key, int64_t value) {
  if (key < 0 || key >= SELUNET_OPT_COUNT) {
    set_error("selunet_set_option: unknown key %d", key);
    return INT64_MIN;
  }
  const int64_t prev = g_options[key];
  if (key == SELUNET_OPT_TILE_QUEUE && value > 0 && x2_tile_queue_prepare() != 0) {
    set_error("selunet_set_option: tile-queue counters could not be allocated on the current device");
    return INT64_MIN;
  }
  g_options[key] = value < 0 ? -1 : value;
  return prev;
}

int selunet_pack_conv3x3(const float* w, int32_t co, int32_t ci, int32_t k_pad, void* fwd, void* dgrad,
                         int32_t dtype, void* stream) {
  SELUNET_REQUIRE(w && fwd && co > 0 && ci > 0 && k_pad >= 9 * ci, "pack_conv3x3: bad arguments");
  const int64_t total = (int64_t)co * k_pad + (dgrad ? (int64_t)ci * 9 * co : 0);
  DISPATCH_T(dtype, hipLaunchKernelGGL(pack_conv3x3_kernel<T>, dim3(grid_for(total)), dim3(TPB), 0, as_stream(stream),
                                       w, co, ci, k_pad, (T*)fwd, (T*)dgrad));
  return check_launch("pack_conv3x3");
}

int selunet_pack_convT(const float* w, int32_t ci, int32_t co, void* fwd, void* dgrad, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(w && (fwd || dgrad) && co > 0 && ci > 0, "pack_convT: bad arguments");
  DISPATCH_T(dtype, hipLaunchKernelGGL(pack_convT_kernel<T>, dim3(grid_for((int64_t)ci * co * 4)), dim3(TPB), 0,
                                       as_stream(stream), w, ci, co, (T*)fwd, (T*)dgrad));
  return check_launch("pack_convT");
}

int selunet_pack_weights(const selunet_pack_list* list, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(list && list->n > 0 && list->n <= SELUNET_PACK_MAX, "pack_weights: bad list");
  selunet_pack_list l = *list;
  selunet_pack_list lx = *list;  // the split-fp16 entries, one block per matrix row
  lx.n = 0;
  int64_t off = 0, xrows = 0;
  for (int t = 0; t < l.n; ++t) {
    selunet_pack_desc& d = l.d[t];
    SELUNET_REQUIRE(d.w && (d.fwd || d.dgrad) && d.co > 0 && d.ci > 0, "pack_weights: bad entry %d", t);
    d.offset = off;
    if (d.kind == SELUNET_PACK_CONV3X3_X2 || d.kind == SELUNET_PACK_CONVT_X2) {
      const bool ct = d.kind == SELUNET_PACK_CONVT_X2;
      SELUNET_REQUIRE(dtype == SELUNET_F32 && d.fwd && d.k_pad == (ct ? d.ci : 9 * d.ci) && d.ci % 32 == 0 &&
                          d.co % 32 == 0,
                      "pack_weights: split-fp16 entry %d needs fp32, fwd, k_pad = %s and ci, co multiples of 32", t,
                      ct ? "ci" : "9*ci");
      SELUNET_REQUIRE(ct ? (d.ci <= 4608 && 4 * d.co <= 4608) : (d.ci <= 512 && d.co <= 512),
                      "pack_weights: split-fp16 entry %d: a packed row is staged in LDS (<= 4608 values)", t);
      lx.d[lx.n] = d;
      lx.d[lx.n].offset = xrows;
      ++lx.n;
      xrows += (ct ? 4 * d.co : d.co) + (d.dgrad ? d.ci : 0);
    } else if (d.kind == SELUNET_PACK_CONV3X3) {
      SELUNET_REQUIRE(d.fwd && d.k_pad >= 9 * d.ci, "pack_weights: bad conv3x3 entry %d", t);
      off += (int64_t)d.co * d.k_pad + (d.dgrad ? (int64_t)d.ci * 9 * d.co : 0);
    } else if (d.kind == SELUNET_PACK_CONV3X3_WINO) {
      SELUNET_REQUIRE(dtype == SELUNET_F32 && d.fwd && d.k_pad == 12 * d.ci,
                      "pack_weights: Winograd entry %d needs fp32, fwd and k_pad = 12*ci", t);
      off += (int64_t)d.co * 12 * d.ci + (d.dgrad ? (int64_t)d.ci * 12 * d.co : 0);
    } else if (d.kind == SELUNET_PACK_COPY) {
      SELUNET_REQUIRE(d.fwd && !d.dgrad, "pack_weights: copy entry %d needs fwd only", t);
      off += (int64_t)d.co * d.ci;
    } else {
      SELUNET_REQUIRE(d.kind == SELUNET_PACK_CONVT, "pack_weights: bad kind in entry %d", t);
      off += (int64_t)d.ci * d.co * 4;
    }
  }
  if (off > 0)
    DISPATCH_T(dtype, hipLaunchKernelGGL(pack_weights_kernel<T>, dim3(grid_for(off, 8192)), dim3(TPB), 0,
                                         as_stream(stream), l, off));
  if (xrows > 0) hipLaunchKernelGGL(pack_x2_kernel, dim3((unsigned)xrows), dim3(256), 0, as_stream(stream), lx);
  return check_launch("pack_weights");
}

int selunet_unpack_conv3x3_grad(const float* packed, int32_t co, int32_t ci, int32_t ld, float* out, void* stream) {
  SELUNET_REQUIRE(packed && out && co > 0 && ci > 0 && ld >= 9 * ci, "unpack_conv3x3_grad: bad arguments");
  hipLaunchKernelGGL(unpack_conv3x3_kernel, dim3(grid_for((int64_t)co * ci * 9)), dim3(TPB), 0, as_stream(stream),
                     packed, co, ci, ld, out);
  return check_launch("unpack_conv3x3_grad");
}

int selunet_unpack_convT_grad(const float* packed, int32_t ci, int32_t co, float* out, void* stream) {
  SELUNET_REQUIRE(packed && out && co > 0 && ci > 0, "unpack_convT_grad: bad arguments");
  const int ld = selunet_wgrad_ld(4 * co);
  hipLaunchKernelGGL(unpack_convT_kernel, dim3(grid_for((int64_t)co * ci * 4)), dim3(TPB), 0, as_stream(stream),
                     packed, ci, co, ld, out);
  return check_launch("unpack_convT_grad");
}

int selunet_memset(void* dst, int32_t value, int64_t bytes, void* stream) {
  SELUNET_REQUIRE(dst && bytes >= 0, "memset: bad arguments");
  if (bytes && reinterpret_cast<uintptr_t>(dst) % 4 == 0 && bytes % 4 == 0) {
    // a kernel, not hipMemsetAsync: inside captured HIP graphs small memset nodes were seen to leave the
    // target unwritten on the second launch of the graph (tests/test_gpu_graphs.py)
    const uint32_t v = (uint32_t)(value & 0xff) * 0x01010101u;
    const int64_t n = bytes / 4;
    hipLaunchKernelGGL(fill_u32_kernel, dim3(grid_for(n, 4096)), dim3(TPB), 0, as_stream(stream),
                       reinterpret_cast<uint32_t*>(dst), n, v);
    return check_launch("memset");
  }
  if (bytes && hipMemsetAsync(dst, value, (size_t)bytes, as_stream(stream)) != hipSuccess)
    return fail(SELUNET_ELAUNCH, "hipMemsetAsync failed");
  return 0;
}

int selunet_memcpy(void* dst, const void* src, int64_t bytes, void* stream) {
  SELUNET_REQUIRE(dst && src && bytes >= 0, "memcpy: bad arguments");
  if (bytes && hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, as_stream(stream)) != hipSuccess)
    return fail(SELUNET_ELAUNCH, "hipMemcpyAsync failed");
  return 0;
}

int selunet_stream_create(void** out) {
  SELUNET_REQUIRE(out, "stream_create: bad arguments");
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    return fail(SELUNET_ELAUNCH, "hipStreamCreateWithFlags failed");
  *out = s;
  return 0;
}

int selunet_stream_destroy(void* s) {
  if (s && hipStreamDestroy(as_stream(s)) != hipSuccess) return fail(SELUNET_ELAUNCH, "hipStreamDestroy failed");
  return 0;
}

int selunet_graph_capture_begin(void* stream) {
  SELUNET_REQUIRE(stream, "graph_capture_begin: capture needs a created (non-default) stream");
  if (hipStreamBeginCapture(as_stream(stream), hipStreamCaptureModeThreadLocal) != hipSuccess)
    return fail(SELUNET_ELAUNCH, "hipStreamBeginCapture failed");
  return 0;
}

int selunet_graph_capture_end(void* stream, void** exec) {
  SELUNET_REQUIRE(stream && exec, "graph_capture_end: bad arguments");
  *exec = nullptr;
  hipGraph_t g = nullptr;
  if (hipStreamEndCapture(as_stream(stream), &g) != hipSuccess || !g)
    return fail(SELUNET_ELAUNCH, "hipStreamEndCapture failed");
  hipGraphExec_t e = nullptr;
  const hipError_t rc = hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (rc != hipSuccess) return fail(SELUNET_ELAUNCH, "hipGraphInstantiate failed");
  *exec = e;
  return 0;
}

int selunet_graph_launch(void* exec, void* stream) {
  SELUNET_REQUIRE(exec, "graph_launch: bad arguments");
  if (hipGraphLaunch((hipGraphExec_t)exec, as_stream(stream)) != hipSuccess)
    return fail(SELUNET_ELAUNCH, "hipGraphLaunch failed");
  return 0;
}

int selunet_graph_destroy(void* exec) {
  if (exec && hipGraphExecDestroy((hipGraphExec_t)exec) != hipSuccess)
    return fail(SELUNET_ELAUNCH, "hipGraphExecDestroy failed");
  return 0;
}

int64_t selunet_reduce_ws_bytes(int32_t cols) { return (int64_t)RED_SPLITS * cols * (int64_t)sizeof(double); }

int selunet_reduce_rows(const float* slab, int64_t rows, int32_t cols, double* ws, double* out, float* out32,
                        void* stream) {
  SELUNET_REQUIRE(slab && ws && (out || out32) && rows > 0 && cols > 0, "reduce_rows: bad arguments");
  const int splits = (int)std::min<int64_t>(RED_SPLITS, cdiv(rows, 16));
  const int64_t chunk = cdiv(rows, splits);
  hipLaunchKernelGGL(reduce_rows_l1, dim3((unsigned)cdiv(cols, 64), splits), dim3(TPB), 0, as_stream(stream), slab,
                     rows, cols, chunk, ws);
  hipLaunchKernelGGL(reduce_rows_l2, dim3((unsigned)cdiv(cols, 64)), dim3(TPB), 0, as_stream(stream), ws, splits,
                     cols, out, out32);
  return check_launch("reduce_rows");
}

int64_t selunet_channel_slab_rows(int64_t m) { return channel_slab_rows(m); }
int64_t selunet_bn_centered_rows(int64_t m) { return bn_centered_rows(m); }

int selunet_channel_sum(const void* x, int64_t m, int32_t c, float* slab, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(x && slab && m > 0 && ok_channels(c), "channel_sum: bad arguments (C=%d)", c);
  DISPATCH_T(dtype, hipLaunchKernelGGL(channel_sum_kernel<T>, dim3((unsigned)channel_slab_rows(m)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)x, m, c, slab));
  return check_launch("channel_sum");
}

int selunet_bn_finalize(const double* sums, int64_t count, int32_t c, const float* conv_bias, const float* gamma,
                        const float* beta, float* running_mean, float* running_var, int64_t* num_batches,
                        float momentum, float eps, int32_t training, float* mean, float* invstd, float* scale,
                        float* shift, void* stream) {
  SELUNET_REQUIRE(gamma && beta && mean && invstd && scale && shift && c > 0, "bn_finalize: bad arguments");
  if (training) {
    SELUNET_REQUIRE(sums != nullptr, "bn_finalize: sums is NULL");
    SELUNET_REQUIRE(count > 1, "Expected more than 1 value per channel when training (got %lld)", (long long)count);
  } else {
    SELUNET_REQUIRE(running_mean && running_var, "bn_finalize(eval): running stats are NULL");
  }
  const BnFinArgs a{count, conv_bias, gamma, beta, running_mean, running_var, num_batches, momentum, eps, training,
                    mean, invstd, scale, shift};
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)cdiv(c, TPB)), dim3(TPB), 0, as_stream(stream), sums, c, a);
  return check_launch("bn_finalize");
}

int selunet_bn_stats_finalize(const float* slab, int64_t rows, double* ws, double* sums, int64_t count, int32_t c,
                              const float* conv_bias, const float* gamma, const float* beta, float* running_mean,
                              float* running_var, int64_t* num_batches, float momentum, float eps, float* mean,
                              float* invstd, float* scale, float* shift, void* stream) {
  SELUNET_REQUIRE(slab && ws && rows > 0 && gamma && beta && mean && invstd && scale && shift && c > 0,
                  "bn_stats_finalize: bad arguments");
  SELUNET_REQUIRE(count > 1, "Expected more than 1 value per channel when training (got %lld)", (long long)count);
  const BnFinArgs fa{count, conv_bias, gamma, beta, running_mean, running_var, num_batches, momentum, eps, 1,
                     mean, invstd, scale, shift};
  launch_reduce_finalize<2>(slab, rows, c, ws, sums, fa, BnbFinArgs{}, as_stream(stream));
  return check_launch("bn_stats_finalize");
}

int selunet_bn_stats_finalize_shifted(const float* slab, int64_t rows, double* ws, int64_t count, int32_t c,
                                      float* center, const float* conv_bias, const float* gamma, const float* beta,
                                      float ratio, float* mean, float* uvar_flag, float* invstd, float* scale,
                                      float* shift, void* stream) {
  SELUNET_REQUIRE(slab && ws && rows > 0 && center && gamma && beta && mean && uvar_flag && invstd && scale && shift &&
                      c > 0 && ratio >= 0.0f,
                  "bn_stats_finalize_shifted: bad arguments");
  SELUNET_REQUIRE(count > 1, "Expected more than 1 value per channel when training (got %lld)", (long long)count);
  BnFinArgs fa{count, conv_bias, gamma, beta, nullptr, nullptr, nullptr, 0.0f, 1e-5f, 1,
               mean, invstd, scale, shift, center};
  fa.uvar_flag_o = uvar_flag;
  fa.flag_ratio = ratio;
  fa.center_next_o = center;
  launch_reduce_finalize<2>(slab, rows, c, ws, nullptr, fa, BnbFinArgs{}, as_stream(stream));
  return check_launch("bn_stats_finalize_shifted");
}

int selunet_bn_centered_partials(const void* y, int64_t m, int32_t c, const float* center, float* slab, int32_t dtype,
                                 void* stream) {
  SELUNET_REQUIRE(y && center && slab && m > 0 && ok_channels(c), "bn_centered_partials: bad arguments (C=%d)", c);
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_centered_partials_kernel<T>, dim3((unsigned)bn_centered_rows(m)), dim3(TPB),
                                       0, as_stream(stream), (const T*)y, m, c, center, nullptr, 0.0f, slab));
  return check_launch("bn_centered_partials");
}

int selunet_bn_centered_partials_adaptive(const void* y, int64_t m, int32_t c, const float* center, const float* uvar,
                                          float ratio, float* slab, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(y && center && uvar && slab && m > 1 && ok_channels(c) && ratio >= 0.0f,
                  "bn_centered_partials_adaptive: bad arguments (C=%d)", c);
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_centered_partials_kernel<T>, dim3((unsigned)bn_centered_rows(m)), dim3(TPB),
                                       0, as_stream(stream), (const T*)y, m, c, center, uvar, ratio, slab));
  return check_launch("bn_centered_partials_adaptive");
}

int selunet_bn_stats_finalize_centered_bound(const float* slab, int64_t rows, double* ws, double* sums,
                                             int64_t count, int32_t c, const float* center, const float* conv_bias,
                                             const float* gamma, const float* beta, float* running_mean,
                                             float* running_var, int64_t* num_batches, float momentum, float eps,
                                             float* mean, float* invstd, float* scale, float* shift, float* bound,
                                             void* stream) {
  SELUNET_REQUIRE(slab && ws && rows > 0 && center && gamma && beta && mean && invstd && scale && shift && c > 0,
                  "bn_stats_finalize_centered: bad arguments");
  SELUNET_REQUIRE(count > 1, "Expected more than 1 value per channel when training (got %lld)", (long long)count);
  BnFinArgs fa{count, conv_bias, gamma, beta, running_mean, running_var, num_batches, momentum, eps, 1,
               mean, invstd, scale, shift, center};
  fa.bound_o = bound;
  fa.bound_sq = (float)std::sqrt((double)count);
  launch_reduce_finalize<2>(slab, rows, c, ws, sums, fa, BnbFinArgs{}, as_stream(stream));
  return check_launch("bn_stats_finalize_centered");
}

int selunet_bn_stats_finalize_centered(const float* slab, int64_t rows, double* ws, double* sums, int64_t count,
                                       int32_t c, const float* center, const float* conv_bias, const float* gamma,
                                       const float* beta, float* running_mean, float* running_var,
                                       int64_t* num_batches, float momentum, float eps, float* mean, float* invstd,
                                       float* scale, float* shift, void* stream) {
  return selunet_bn_stats_finalize_centered_bound(slab, rows, ws, sums, count, c, center, conv_bias, gamma, beta,
                                                  running_mean, running_var, num_batches, momentum, eps, mean, invstd,
                                                  scale, shift, nullptr, stream);
}

int selunet_bn_bwd_stats_finalize(const float* slab, int64_t rows, double* ws, double* sums, int64_t count,
                                  int32_t c, const float* gamma, const float* invstd, float* dgamma, float* dbeta,
                                  float* dbias, float* coef, void* stream) {
  SELUNET_REQUIRE(slab && ws && rows > 0 && gamma && invstd && coef && c > 0 && count > 0,
                  "bn_bwd_stats_finalize: bad arguments");
  const BnbFinArgs ba{count, gamma, invstd, dgamma, dbeta, dbias, coef};
  launch_reduce_finalize<3>(slab, rows, c, ws, sums, BnFinArgs{}, ba, as_stream(stream));
  return check_launch("bn_bwd_stats_finalize");
}

int selunet_bn_bwd_stats_finalize_bound(const float* slab, int64_t rows, double* ws, double* sums, int64_t count,
                                        int32_t c, const float* gamma, const float* invstd, float* dgamma, float* dbeta,
                                        float* dbias, float* coef, const float* amax_da, float* bound, void* stream) {
  SELUNET_REQUIRE(slab && ws && rows > 0 && gamma && invstd && coef && c > 0 && count > 0 && amax_da && bound,
                  "bn_bwd_stats_finalize_bound: bad arguments");
  BnbFinArgs ba{count, gamma, invstd, dgamma, dbeta, dbias, coef};
  ba.amax_da = amax_da;
  ba.bound = bound;
  launch_reduce_finalize<3>(slab, rows, c, ws, sums, BnFinArgs{}, ba, as_stream(stream));
  return check_launch("bn_bwd_stats_finalize_bound");
}

int selunet_bn_bwd_reduce(const void* dz, const void* y, int64_t m, int32_t c, const float* scale, const float* shift,
                          const float* mean, const float* invstd, float* slab, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(dz && y && scale && shift && mean && invstd && slab && m > 0 && ok_channels(c),
                  "bn_bwd_reduce: bad arguments");
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_bwd_reduce_kernel<T>, dim3((unsigned)channel_slab_rows(m)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)dz, (const T*)y, m, c, scale, shift, mean, invstd,
                                       slab));
  return check_launch("bn_bwd_reduce");
}

int selunet_bn_bwd_finalize(const double* sums, int64_t count, int32_t c, const float* gamma, const float* invstd,
                            float* dgamma, float* dbeta, float* dbias, float* coef, void* stream) {
  SELUNET_REQUIRE(sums && gamma && invstd && coef && c > 0 && count > 0, "bn_bwd_finalize: bad arguments");
  const BnbFinArgs a{count, gamma, invstd, dgamma, dbeta, dbias, coef};
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((unsigned)cdiv(c, TPB)), dim3(TPB), 0, as_stream(stream), sums, c, a);
  return check_launch("bn_bwd_finalize");
}

int selunet_bn_bwd_apply(const void* dz, const void* y, int64_t m, int32_t c, const float* scale, const float* shift,
                         const float* mean, const float* invstd, const float* coef, void* dy, int32_t dtype,
                         void* stream) {
  return selunet_bn_bwd_apply_amax(dz, y, m, c, scale, shift, mean, invstd, coef, dy, nullptr, dtype, stream);
}

int selunet_act_bound(const float* gamma, const float* beta, int32_t c, int64_t count, float* out, void* stream) {
  SELUNET_REQUIRE(gamma && beta && out && c > 0 && c <= 4096 && count > 0, "act_bound: bad arguments");
  hipLaunchKernelGGL(act_bound_kernel, dim3(1), dim3(256), 0, as_stream(stream), gamma, beta, c,
                     (float)std::sqrt((double)count), out);
  return check_launch("act_bound");
}

int selunet_bn_bwd_apply_amax(const void* dz, const void* y, int64_t m, int32_t c, const float* scale,
                              const float* shift, const float* mean, const float* invstd, const float* coef, void* dy,
                              float* amax, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(dz && y && scale && shift && mean && invstd && coef && dy && m > 0 && c % 4 == 0,
                  "bn_bwd_apply: bad arguments");
  SELUNET_REQUIRE(ok_channels(c), "bn_bwd_apply: C must be 64, 128, 256 or 512 (got %d)", c);
  const int64_t form = option(SELUNET_OPT_APPLY_U8, 0);  // 0: 8 channels x 4 pixels, 1: x 8 pixels, 2 / 3: the
                                                           // 4-channel contiguous form with 8 / 16 pixels in flight
  const bool u8 = form == 1;
  const int64_t gcap = std::max<int64_t>(1, option(SELUNET_OPT_APPLY_GRID, 1024));
  if (form == 2 || form == 3) {
    const unsigned b4 = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(m, TPB / (c / 4)), gcap));
    if (form == 2)
      DISPATCH_T(dtype, hipLaunchKernelGGL((bn_bwd_apply4_kernel<T, 8>), dim3(b4), dim3(TPB), 0, as_stream(stream),
                                           (const T*)dz, (const T*)y, m, c, scale, shift, mean, invstd, coef, (T*)dy,
                                           amax));
    else
      DISPATCH_T(dtype, hipLaunchKernelGGL((bn_bwd_apply4_kernel<T, 16>), dim3(b4), dim3(TPB), 0, as_stream(stream),
                                           (const T*)dz, (const T*)y, m, c, scale, shift, mean, invstd, coef, (T*)dy,
                                           amax));
    return check_launch("bn_bwd_apply");
  }
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(m, TPB / (c / 8)), gcap));
  if (u8) {
    DISPATCH_T(dtype, hipLaunchKernelGGL((bn_bwd_apply_kernel<T, 8>), dim3(blocks), dim3(TPB), 0, as_stream(stream),
                                         (const T*)dz, (const T*)y, m, c, scale, shift, mean, invstd, coef, (T*)dy,
                                         amax));
    return check_launch("bn_bwd_apply");
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(blocks), dim3(TPB), 0,
                                       as_stream(stream), (const T*)dz, (const T*)y, m, c, scale, shift, mean, invstd,
                                       coef, (T*)dy, amax));
  return check_launch("bn_bwd_apply");
}

int selunet_im2col3x3(const float* x, int32_t n, int32_t c, int32_t h, int32_t w, int32_t k_pad, void* out,
                      int32_t dtype, void* stream) {
  SELUNET_REQUIRE(x && out && n > 0 && c > 0 && h > 0 && w > 0 && k_pad >= 9 * c && k_pad % 8 == 0,
                  "im2col3x3: bad arguments");
  const int64_t M = (int64_t)n * h * w;
  DISPATCH_T(dtype, hipLaunchKernelGGL(im2col3x3_kernel<T>, dim3(grid_for(M, 8192)), dim3(TPB), 0, as_stream(stream),
                                       x, n, c, h, w, k_pad, (T*)out));
  return check_launch("im2col3x3");
}

int selunet_maxpool2_fwd(const void* y, int32_t n, int32_t h, int32_t w, int32_t c, const float* scale,
                         const float* shift, void* out, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(y && out && scale && shift && n > 0 && h > 1 && w > 1 && c % 4 == 0, "maxpool2_fwd: bad arguments");
  SELUNET_REQUIRE(h % 2 == 0 && w % 2 == 0, "maxpool2_fwd: H and W must be even (got %d x %d)", h, w);
  const int64_t nv = (int64_t)n * (h / 2) * (w / 2) * (c / 4);
  DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_fwd_kernel<T>, dim3(grid_for(nv, 8192)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)y, n, h, w, c, scale, shift, (T*)out));
  return check_launch("maxpool2_fwd");
}

int64_t selunet_maxpool2_bwd_slab_rows(int32_t n, int32_t h, int32_t w, int32_t c) {
  // at least 8 windows per thread (a block's reduction and slab row amortised: at 16 images one window per thread
  // cost 0.33 ms/step against 0.19 for 1/8 of the 128-image work) and at least 1024 blocks where there is work
  const int64_t nv = (int64_t)n * (h / 2) * (w / 2) * (c / 4);
  const int64_t want = std::max<int64_t>(cdiv(nv, (int64_t)TPB * 8), std::min<int64_t>(cdiv(nv, TPB), 1024));
  return std::max<int64_t>(1, std::min<int64_t>(want, 8192));
}

int selunet_maxpool2_bwd(const void* y, int32_t n, int32_t h, int32_t w, int32_t c, const float* scale,
                         const float* shift, const void* dpool, const void* dskip, void* dz,
                         const selunet_bn_bwd_stats* bnb, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(y && dpool && (dz || (bnb && bnb->slab)) && scale && shift && n > 0 && h % 2 == 0 && w % 2 == 0 &&
                      ok_channels(c),
                  "maxpool2_bwd: bad arguments");
  SELUNET_REQUIRE((int64_t)n * (h / 2) * (w / 2) < (int64_t(1) << 31), "maxpool2_bwd: grid too large");
  const float *mean = nullptr, *invstd = nullptr;
  float* bslab = nullptr;
  if (bnb && bnb->slab) {
    SELUNET_REQUIRE(bnb->y == y && bnb->scale == scale && bnb->shift == shift && bnb->mean && bnb->invstd,
                    "maxpool2_bwd: bnb must describe the pooled layer (same y/scale/shift) with mean/invstd");
    mean = bnb->mean;
    invstd = bnb->invstd;
    bslab = bnb->slab;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3((unsigned)selunet_maxpool2_bwd_slab_rows(n, h, w, c)),
                                       dim3(TPB), 0, as_stream(stream), (const T*)y, n, h, w, c, scale, shift,
                                       (const T*)dpool, (const T*)dskip, (T*)dz, mean, invstd, bslab,
                                       bnb ? bnb->amax : nullptr));
  return check_launch("maxpool2_bwd");
}

int selunet_heads_fwd(const void* y, int64_t m, const float* scale, const float* shift, const float* w,
                      const float* b, int32_t nh, float* out0, float* out1, float* out2, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(y && scale && shift && w && b && out0 && m > 0 && (nh == 1 || nh == 3), "heads_fwd: bad arguments");
  SELUNET_REQUIRE(nh == 1 || (out1 && out2), "heads_fwd: out1/out2 required for 3 heads");
  DISPATCH_T(dtype, hipLaunchKernelGGL(heads_fwd_kernel<T>, dim3(grid_for(m * 16, 8192)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)y, m, scale, shift, w, b, nh, out0, out1, out2));
  return check_launch("heads_fwd");
}

int selunet_heads_bwd(const void* y, int64_t m, const float* scale, const float* shift, const float* w, int32_t nh,
                      const float* g0, const float* g1, const float* g2, void* dz, float* slab,
                      const selunet_bn_bwd_stats* bnb, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(y && scale && shift && w && g0 && (dz || (bnb && bnb->slab)) && slab && m > 0 && (nh == 1 || nh == 3),
                  "heads_bwd: bad arguments");
  SELUNET_REQUIRE(nh == 1 || (g1 && g2), "heads_bwd: g1/g2 required for 3 heads");
  const float *mean = nullptr, *invstd = nullptr;
  float* bslab = nullptr;
  if (bnb && bnb->slab) {
    SELUNET_REQUIRE(bnb->y == y && bnb->scale == scale && bnb->shift == shift && bnb->mean && bnb->invstd,
                    "heads_bwd: bnb must describe the heads' input layer (same y/scale/shift) with mean/invstd");
    mean = bnb->mean;
    invstd = bnb->invstd;
    bslab = bnb->slab;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(heads_bwd_kernel<T>, dim3((unsigned)channel_slab_rows(m)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)y, m, scale, shift, w, nh, g0, g1, g2, (T*)dz,
                                       slab, mean, invstd, bslab, bnb ? bnb->amax : nullptr));
  return check_launch("heads_bwd");
}

int selunet_bn_bwd_apply_heads(const void* y, int64_t m, const float* scale, const float* shift, const float* mean,
                               const float* invstd, const float* coef, const float* w, int32_t nh, const float* g0,
                               const float* g1, const float* g2, void* dy, float* amax, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(y && scale && shift && mean && invstd && coef && w && g0 && dy && m > 0 && (nh == 1 || nh == 3),
                  "bn_bwd_apply_heads: bad arguments");
  SELUNET_REQUIRE(nh == 1 || (g1 && g2), "bn_bwd_apply_heads: g1/g2 required for 3 heads");
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_bwd_apply_heads_kernel<T>, dim3(grid_for(m * 16 / HU, 2048)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)y, m, scale, shift, mean, invstd, coef, w, nh, g0,
                                       g1, g2, (T*)dy, amax));
  return check_launch("bn_bwd_apply_heads");
}

int selunet_bn_bwd_apply_pool(const void* y, int32_t n, int32_t h, int32_t w, int32_t c, const float* scale,
                              const float* shift, const float* mean, const float* invstd, const float* coef,
                              const void* dpool, const void* dskip, void* dy, float* amax, int32_t dtype,
                              void* stream) {
  SELUNET_REQUIRE(y && dpool && dy && scale && shift && mean && invstd && coef && n > 0 && h % 2 == 0 && w % 2 == 0 &&
                      ok_channels(c),
                  "bn_bwd_apply_pool: bad arguments");
  SELUNET_REQUIRE((int64_t)n * (h / 2) * (w / 2) < (int64_t(1) << 31), "bn_bwd_apply_pool: grid too large");
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_bwd_apply_pool_kernel<T>,
                                       dim3((unsigned)selunet_maxpool2_bwd_slab_rows(n, h, w, c)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)y, n, h, w, c, scale, shift, mean, invstd, coef,
                                       (const T*)dpool, (const T*)dskip, (T*)dy, amax));
  return check_launch("bn_bwd_apply_pool");
}

int64_t selunet_loss_slab_rows(int64_t p) { return loss_slab_rows(p); }

static int selective_partials(bool hard, const float* out, const float* sel, const float* target, int64_t p,
                              float* slab, void* stream) {
  SELUNET_REQUIRE(out && sel && target && slab && p > 0, "selective_partials: bad arguments");
  hipLaunchKernelGGL(hard ? selective_partials_kernel<true> : selective_partials_kernel<false>,
                     dim3((unsigned)loss_slab_rows(p)), dim3(TPB), 0, as_stream(stream), out, sel, target, p, slab);
  return check_launch("selective_partials");
}
int selunet_selective_partials(const float* out, const float* sel, const float* target, int64_t p, float* slab,
                               void* stream) {
  return selective_partials(false, out, sel, target, p, slab, stream);
}
int selunet_selective_partials_hard(const float* out, const float* sel, const float* target, int64_t p, float* slab,
                                    void* stream) {
  return selective_partials(true, out, sel, target, p, slab, stream);
}

int selunet_selective_finalize(const double* sums, double p_global, float lamb, float target_coverage, float* loss,
                               float* coverage, float* state, void* stream) {
  SELUNET_REQUIRE(sums && loss && coverage && state && p_global > 0, "selective_finalize: bad arguments");
  hipLaunchKernelGGL(selective_finalize_kernel, dim3(1), dim3(1), 0, as_stream(stream), sums, p_global, lamb,
                     target_coverage, loss, coverage, state);
  return check_launch("selective_finalize");
}

static int selective_bwd(bool hard, const float* out, const float* sel, const float* target, int64_t p,
                         const float* state, float lamb, const float* g_loss, const float* g_coverage, float* d_out,
                         float* d_sel, void* stream) {
  SELUNET_REQUIRE(out && sel && target && state && d_out && d_sel && p > 0, "selective_bwd: bad arguments");
  hipLaunchKernelGGL(hard ? selective_bwd_kernel<true> : selective_bwd_kernel<false>, dim3(grid_for(p, 8192)),
                     dim3(TPB), 0, as_stream(stream), out, sel, target, p, state, lamb, g_loss, g_coverage, d_out,
                     d_sel);
  return check_launch("selective_bwd");
}
int selunet_selective_bwd(const float* out, const float* sel, const float* target, int64_t p, const float* state,
                          float lamb, const float* g_loss, const float* g_coverage, float* d_out, float* d_sel,
                          void* stream) {
  return selective_bwd(false, out, sel, target, p, state, lamb, g_loss, g_coverage, d_out, d_sel, stream);
}
int selunet_selective_bwd_hard(const float* out, const float* sel, const float* target, int64_t p,
                               const float* state, const float* g_loss, float* d_out, float* d_sel, void* stream) {
  return selective_bwd(true, out, sel, target, p, state, 0.0f, g_loss, nullptr, d_out, d_sel, stream);
}

int selunet_bce_partials(const float* logit, const float* target, int64_t p, float* slab, void* stream) {
  SELUNET_REQUIRE(logit && target && slab && p > 0, "bce_partials: bad arguments");
  hipLaunchKernelGGL(bce_partials_kernel, dim3((unsigned)loss_slab_rows(p)), dim3(TPB), 0, as_stream(stream), logit,
                     target, p, slab);
  return check_launch("bce_partials");
}

int selunet_bce_finalize(const double* sums, double p_global, float* loss, void* stream) {
  SELUNET_REQUIRE(sums && loss && p_global > 0, "bce_finalize: bad arguments");
  hipLaunchKernelGGL(bce_finalize_kernel, dim3(1), dim3(1), 0, as_stream(stream), sums, p_global, loss);
  return check_launch("bce_finalize");
}

int selunet_bce_bwd(const float* logit, const float* target, int64_t p, double p_global, const float* g_loss,
                    float* d_logit, void* stream) {
  SELUNET_REQUIRE(logit && target && d_logit && p > 0 && p_global > 0, "bce_bwd: bad arguments");
  hipLaunchKernelGGL(bce_bwd_kernel, dim3(grid_for(p, 8192)), dim3(TPB), 0, as_stream(stream), logit, target, p,
                     (float)(1.0 / p_global), g_loss, d_logit);
  return check_launch("bce_bwd");
}

int selunet_adam_step(const selunet_adam_tensor* list, int32_t n, int64_t total_chunks, float lr, float beta1,
                      float beta2, float eps, float weight_decay, int64_t step, void* stream) {
  SELUNET_REQUIRE(list && n > 0 && total_chunks > 0 && step > 0, "adam_step: bad arguments");
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)total_chunks), dim3(TPB), 0, as_stream(stream), list, n,
                     (float)(lr / bc1), beta1, beta2, eps, weight_decay, (float)std::sqrt(bc2));
  return check_launch("adam_step");
}

static int head_planes_arg(const selunet_head_planes* a, HeadPlanesArg& h, bool bwd) {
  SELUNET_REQUIRE(a != nullptr && a->n >= 1 && a->n <= 8 && a->hw > 0, "head planes: need 1..8 outputs and hw > 0");
  std::memset(&h, 0, sizeof(h));
  h.n = a->n;
  h.hw = a->hw;
  h.row_len = a->row_len;
  for (int k = 0; k < a->n; ++k) {
    SELUNET_REQUIRE(a->plane[k] != nullptr && a->img_stride[k] >= a->hw, "head planes: plane %d missing/bad stride", k);
    h.plane[k] = a->plane[k];
    h.img_stride[k] = a->img_stride[k];
    h.w_off[k] = a->w_off[k];
    h.b_off[k] = a->b_off[k];
    if (bwd)
      SELUNET_REQUIRE(a->w_off[k] >= 0 && a->w_off[k] + 64 <= a->row_len && a->b_off[k] >= 0 &&
                          a->b_off[k] < a->row_len,
                      "head planes: slab offsets of output %d outside row_len %d", k, a->row_len);
  }
  return 0;
}

int selunet_heads_fwd_planes(const void* y, int64_t m, const float* scale, const float* shift, const float* w,
                             const float* b, const selunet_head_planes* out, int32_t dtype, void* stream) {
  SELUNET_REQUIRE(y && scale && shift && w && b && m > 0, "heads_fwd_planes: bad arguments");
  HeadPlanesArg h;
  if (int rc = head_planes_arg(out, h, false)) return rc;
  SELUNET_REQUIRE(m % h.hw == 0, "heads_fwd_planes: m (%lld) must be a multiple of hw (%d)", (long long)m, h.hw);
  DISPATCH_T(dtype, hipLaunchKernelGGL(heads_n_fwd_kernel<T>, dim3(grid_for(m * 16, 8192)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)y, m, scale, shift, w, b, h));
  return check_launch("heads_fwd_planes");
}

int selunet_heads_bwd_planes(const void* y, int64_t m, const float* scale, const float* shift, const float* w,
                             const selunet_head_planes* grads, void* dz, float* slab, const selunet_bn_bwd_stats* bnb,
                             int32_t dtype, void* stream) {
  SELUNET_REQUIRE(y && scale && shift && w && (dz || (bnb && bnb->slab)) && slab && m > 0, "heads_bwd_planes: bad arguments");
  HeadPlanesArg h;
  if (int rc = head_planes_arg(grads, h, true)) return rc;
  SELUNET_REQUIRE(m % h.hw == 0, "heads_bwd_planes: m (%lld) must be a multiple of hw (%d)", (long long)m, h.hw);
  const float *mean = nullptr, *invstd = nullptr;
  float* bslab = nullptr;
  if (bnb && bnb->slab) {
    SELUNET_REQUIRE(bnb->y == y && bnb->scale == scale && bnb->shift == shift && bnb->mean && bnb->invstd,
                    "heads_bwd_planes: bnb must describe the heads' input layer (same y/scale/shift)");
    mean = bnb->mean;
    invstd = bnb->invstd;
    bslab = bnb->slab;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(heads_n_bwd_kernel<T>, dim3((unsigned)channel_slab_rows(m)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)y, m, scale, shift, w, h, (T*)dz, slab, mean,
                                       invstd, bslab));
  return check_launch("heads_bwd_planes");
}

int selunet_bn_bwd_apply_heads_planes(const void* y, int64_t m, const float* scale, const float* shift,
                                      const float* mean, const float* invstd, const float* coef, const float* w,
                                      const selunet_head_planes* grads, void* dy, float* amax, int32_t dtype,
                                      void* stream) {
  SELUNET_REQUIRE(y && scale && shift && mean && invstd && coef && w && dy && m > 0,
                  "bn_bwd_apply_heads_planes: bad arguments");
  HeadPlanesArg h;
  if (int rc = head_planes_arg(grads, h, true)) return rc;
  SELUNET_REQUIRE(m % h.hw == 0, "bn_bwd_apply_heads_planes: m (%lld) must be a multiple of hw (%d)", (long long)m,
                  h.hw);
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_bwd_apply_heads_planes_kernel<T>, dim3(grid_for(m * 16, 2048)), dim3(TPB), 0,
                                       as_stream(stream), (const T*)y, m, scale, shift, mean, invstd, coef, w, h,
                                       (T*)dy, amax));
  return check_launch("bn_bwd_apply_heads_planes");
}


static int ce_selective_partials(bool hard, const float* out, const float* sel, const int64_t* target, int64_t n,
                                 int32_t c, int64_t hw, float* slab, void* stream) {
  SELUNET_REQUIRE(out && sel && target && slab && n > 0 && hw > 0 && c >= 1 && c <= 8,
                  "ce_selective_partials: bad arguments (n_cls must be 1..8)");
  const int64_t p = n * hw;
  hipLaunchKernelGGL(hard ? ce_selective_partials_kernel<true> : ce_selective_partials_kernel<false>,
                     dim3((unsigned)loss_slab_rows(p)), dim3(TPB), 0, as_stream(stream), out, sel, target, p, c, hw,
                     slab);
  return check_launch("ce_selective_partials");
}
int selunet_ce_selective_partials(const float* out, const float* sel, const int64_t* target, int64_t n, int32_t c,
                                  int64_t hw, float* slab, void* stream) {
  return ce_selective_partials(false, out, sel, target, n, c, hw, slab, stream);
}
int selunet_ce_selective_partials_hard(const float* out, const float* sel, const int64_t* target, int64_t n,
                                       int32_t c, int64_t hw, float* slab, void* stream) {
  return ce_selective_partials(true, out, sel, target, n, c, hw, slab, stream);
}

static int ce_selective_bwd(bool hard, const float* out, const float* sel, const int64_t* target, int64_t n,
                            int32_t c, int64_t hw, const float* state, float lamb, const float* g_loss,
                            const float* g_coverage, float* d_out, float* d_sel, void* stream) {
  SELUNET_REQUIRE(out && sel && target && state && d_out && d_sel && n > 0 && hw > 0 && c >= 1 && c <= 8,
                  "ce_selective_bwd: bad arguments");
  const int64_t p = n * hw;
  hipLaunchKernelGGL(hard ? ce_selective_bwd_kernel<true> : ce_selective_bwd_kernel<false>, dim3(grid_for(p, 8192)),
                     dim3(TPB), 0, as_stream(stream), out, sel, target, p, c, hw, state, lamb, g_loss, g_coverage,
                     d_out, d_sel);
  return check_launch("ce_selective_bwd");
}
int selunet_ce_selective_bwd(const float* out, const float* sel, const int64_t* target, int64_t n, int32_t c,
                             int64_t hw, const float* state, float lamb, const float* g_loss, const float* g_coverage,
                             float* d_out, float* d_sel, void* stream) {
  return ce_selective_bwd(false, out, sel, target, n, c, hw, state, lamb, g_loss, g_coverage, d_out, d_sel, stream);
}
int selunet_ce_selective_bwd_hard(const float* out, const float* sel, const int64_t* target, int64_t n, int32_t c,
                                  int64_t hw, const float* state, const float* g_loss, float* d_out, float* d_sel,
                                  void* stream) {
  return ce_selective_bwd(true, out, sel, target, n, c, hw, state, 0.0f, g_loss, nullptr, d_out, d_sel, stream);
}

int selunet_ce_partials(const float* logit, const int64_t* target, int64_t n, int32_t c, int64_t hw, float* slab,
                        void* stream) {
  SELUNET_REQUIRE(logit && target && slab && n > 0 && hw > 0 && c >= 1 && c <= 8, "ce_partials: bad arguments");
  const int64_t p = n * hw;
  hipLaunchKernelGGL(ce_partials_kernel, dim3((unsigned)loss_slab_rows(p)), dim3(TPB), 0, as_stream(stream), logit,
                     target, p, c, hw, slab);
  return check_launch("ce_partials");
}

int selunet_ce_bwd(const float* logit, const int64_t* target, int64_t n, int32_t c, int64_t hw, double p_global,
                   const float* g_loss, float* d_logit, void* stream) {
  SELUNET_REQUIRE(logit && target && d_logit && n > 0 && hw > 0 && c >= 1 && c <= 8 && p_global > 0,
                  "ce_bwd: bad arguments");
  const int64_t p = n * hw;
  hipLaunchKernelGGL(ce_bwd_kernel, dim3(grid_for(p, 8192)), dim3(TPB), 0, as_stream(stream), logit, target, p, c, hw,
                     (float)(1.0 / p_global), g_loss, d_logit);
  return check_launch("ce_bwd");
}

}  // extern "C"
