/*
 * selunet.h — C-ABI of the MI355X (gfx950) SelectiveUNet_B training path.
 *
 * The reference has no FFI: its boundary is the Python API of `model.UNet_B`
 * (model.py:18-103), `selective_loss.calc_selective_risk_image_b`
 * (selective_loss.py:58-85), `torch.nn.BCEWithLogitsLoss` (train.py:78,195) and
 * `torch.optim.Adam` (train.py:90,209). Every ATen op those dispatch to on the
 * hot path is replaced by one of the entry points below; the Python host layer
 * (selectivenet_for_semantic_segmentation_binary_amd/) binds them with ctypes and
 * keeps the reference's module/function signatures. Each entry point notes the
 * reference call it replaces.
 *
 * Conventions
 *  - Plain device pointers, sizes and a `hipStream_t` passed as `void*` (the
 *    caller's current stream). No allocation, no synchronisation, no host copies
 *    inside any call: all workspaces are caller-owned, so every call is graph-
 *    capturable.
 *  - Activations are NHWC (channels contiguous), element type `dtype`
 *    (SELUNET_F32 or SELUNET_BF16); statistics, losses, weight gradients and
 *    optimizer state are fp32 (reductions fp64 where noted).
 *  - Return 0 on success, otherwise a nonzero code; `selunet_last_error()` gives
 *    the message of the last failing call on this thread.
 */
#ifndef SELUNET_H
#define SELUNET_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { SELUNET_F32 = 0, SELUNET_BF16 = 1 };

enum {
  SELUNET_OK = 0,
  SELUNET_EINVAL = 1,  /* bad argument (null pointer, size, alignment, unsupported shape) */
  SELUNET_ELAUNCH = 2, /* HIP launch error */
};

/* Kernel-selection and tuning options (selunet_set_option). The library reads no environment
 * variables; every value < 0 selects the built-in default. Selection options take 0/1. */
enum {
  SELUNET_OPT_HALO = 0,           /* 3x3 convolutions on the LDS halo kernels (1) or the gather GEMM (0) */
  SELUNET_OPT_HALO_PERSIST,       /* persistent halo kernel for multi-chunk layers: 0 off, 1 on (1) */
  SELUNET_OPT_WINO,               /* exact-fp32 3x3 fwd/dgrad as 1-D Winograd F(2,3) (1) or direct (0) */
  SELUNET_OPT_WINO_WGRAD,         /* exact-fp32 3x3 weight gradient as the Winograd transpose (1) */
  SELUNET_OPT_WINO_WGRAD_TW,      /* its tile width: 16 (default) or 8 pixels */
  SELUNET_OPT_WINO_WGRAD_WAVES,   /* its waves per workgroup: 12 (default) or 8 */
  SELUNET_OPT_WGRAD_WGS,          /* workgroup target of the halo / Winograd weight gradients (256) */
  SELUNET_OPT_X2_WGRAD_WGS,       /* workgroup target of the split-fp16 3x3 weight gradient (256) */
  SELUNET_OPT_GEMM_WGRAD_WGS,     /* workgroup target of the generic weight gradient (512) */
  SELUNET_OPT_GATHER_WGS,         /* resident gather-GEMM workgroups (512; 0 = one tile each) */
  SELUNET_OPT_RF_SINGLE,          /* slab rows reduced in one launch by the fused reductions (1024) */
  SELUNET_OPT_APPLY_U8,           /* BN-backward apply form: 0 8 ch x 4 px, 1 8 ch x 8 px, 2/3 4 contiguous ch x 8/16 px (0) */
  SELUNET_OPT_APPLY_GRID,         /* BN-backward apply: grid cap (1024) */
  SELUNET_OPT_X2D,                /* 64-column split-fp16 3x3 layers on the two-workgroups-per-CU kernel: 0 never,
                                   * 1 every eligible layer, 2 inputs of at most 64 channels, 3 (default) those of
                                   * them whose source carries a BN+ReLU transform (the forwards) */
  SELUNET_OPT_TILE_QUEUE,         /* bit mask (robustness to a concurrent all-reduce), 0 = static walks
                                   * (default). Bit 0: the split-fp16 persistent 3x3 kernel takes its pixel tiles from
                                   * a ticket counter and writes statistics per tile (selunet_conv3x3_x2_stats_rows
                                   * follows it). Bit 1: so do the split-fp16 weight gradients' (co tile, ci chunk)
                                   * groups (each partial then sums the tiles its workgroup took: the weight gradient
                                   * is not bit-reproducible run to run) */
  SELUNET_OPT_X2P,                /* 128-column split-fp16 3x3 layers (multi-chunk inputs) on the kernel with two
                                   * 256-thread workgroups per CU and LDS-DMA weights (1) or on the
                                   * one-workgroup-per-CU persistent kernel (0, default: measured faster);
                                   * selunet_conv3x3_x2_stats_rows follows it */
  SELUNET_OPT_CONVT_RING,         /* ConvTranspose2d forward / data gradient on 256-column blocks (fp32: K >= 256;
                                   * bf16: K >= 512): the LDS-DMA ring kernels with the forward on 8 x 1 waves (2,
                                   * default) or, fp32, 4 x 2 waves (1), or the resident-weight / staged kernels (0);
                                   * selunet_gemm_gather_x2_stats_rows / selunet_gemm_stats_rows follow it */
  SELUNET_OPT_COUNT
};
/* Sets option `key` to `value` (< 0: default); returns the previous setting, or INT64_MIN for an
 * unknown key. Changes apply to later calls (the stats-slab row counts of selunet_gemm_stats_rows
 * follow SELUNET_OPT_HALO_PERSIST / GATHER_WGS). Not thread-safe; set before enqueuing work. */
int64_t selunet_set_option(int32_t key, int64_t value);

/* Rows of the GEMM output tile (pixels per workgroup); stats slabs have ceil(M/128) rows. */
#define SELUNET_GEMM_BM 128

/* One source tensor of an implicit-GEMM operand. The transform
 * v -> relu?(v*scale[c] + shift[c]) is the folded BatchNorm of the producing
 * CBR block (model.py:12-13), applied on load; padded positions read 0 after it. */
typedef struct selunet_source {
  const void* data;    /* NHWC [n][hs][ws][channels] (layout 0) or NCHW fp32 (layout 1) */
  const float* scale;  /* per-channel, NULL = identity */
  const float* shift;
  int32_t channels;
  int32_t relu;        /* clamp at 0 after the affine */
  int32_t layout;      /* 0 NHWC, 1 NCHW (network input only, fp32) */
  int32_t reserved;
} selunet_source;

/* A gathered ("im2col without materialisation") matrix G[M][K]:
 *   row m = (img*h + y)*w + x over an n x h x w pixel grid,
 *   column k = tap*(C0+C1) + c, c < C0 from src[0] else src[1] (torch.cat((up, skip), 1),
 *   model.py:83,87,91). taps: 1 = the pixel itself; 9 = 3x3 neighbourhood, zero padded
 *   (conv 3x3 pad 1, model.py:11); 4 = the 2x2 block (2y+a, 2x+b) of a (2h)x(2w) source grid
 *   (ConvTranspose2d k2 s2 backward, model.py:44,51,57). */
typedef struct selunet_gather {
  int32_t n, h, w;
  int32_t taps;
  int32_t nsrc;
  int32_t reserved;
  selunet_source src[2];
} selunet_gather;

enum { SELUNET_EP_PLAIN = 0, SELUNET_EP_SPLIT = 1, SELUNET_EP_SCATTER2X = 2 };

/* Epilogue of selunet_gemm_gather. PLAIN: out0[M][N]; SPLIT: columns < split go to
 * out0[M][split], the rest to out1[M][N-split] (backward of torch.cat); SCATTER2X:
 * column (a*2+b)*Cq + c of row (img,y,x) goes to out0[img][2y+a][2x+b][c], Cq = N/4
 * (ConvTranspose2d k2 s2 forward). bias (fp32, per output channel) is added when
 * non-NULL. stats (fp32 [selunet_gemm_stats_rows(a, N, dtype)][2][N]): per-workgroup column
 * sum and sum of squares of the fp32 accumulators (BatchNorm batch statistics, model.py:12). */
/* BatchNorm-backward partial sums of a freshly written data gradient dA of a CBR block (fused into
 * the kernel that produces dA instead of re-reading it): per workgroup and channel,
 * sum(da), sum(da*xhat), sum(xhat) with da = dA*[y*scale+shift > 0], xhat = (y-mean)*invstd,
 * dA rounded to the activation dtype first (as stored). slab = NULL disables it. */
typedef struct selunet_bn_bwd_stats {
  const void* y;       /* the block's pre-BN conv output, same [M][C] layout as dA */
  const float* scale;  /* folded BN + ReLU of the forward pass */
  const float* shift;
  const float* mean;   /* batch statistics of the forward pass */
  const float* invstd;
  float* slab;         /* [rows][3][C] */
  float* amax;         /* nullable: atomic max of |dA| as stored (float bits; zeroed by the caller) — read by
                        * selunet_maxpool2_bwd and selunet_heads_bwd only, whose sums-only mode never stores
                        * dA: the range word selunet_bn_bwd_stats_finalize_bound needs for a fused apply */
} selunet_bn_bwd_stats;

typedef struct selunet_epilogue {
  void* out0;
  void* out1;
  const float* bias;
  float* stats;
  int32_t mode;
  int32_t split;
  /* SPLIT only (nullable): [stats_rows][split] per-workgroup column sums of the out0 part (the
   * ConvTranspose2d bias gradient of the up-sampled half of a torch.cat, model.py:44,51,57). */
  float* colsum;
  /* PLAIN only: BatchNorm-backward sums of the written tile, slab [stats_rows][3][N]. */
  selunet_bn_bwd_stats bnb;
  /* nullable: max |stored value| folded into *amax with an atomic max (float bits; the caller zeroes
   * it): the range word of a split-fp16 operand (selunet_conv3x3_x2) read by the next layer. */
  float* amax;
  /* nullable, with stats: per-column shift c (the previous step's batch mean): stats then hold the sums
   * of (v - c) and (v - c)^2, which selunet_bn_stats_finalize_shifted turns into the mean and a
   * one-pass variance that loses ~eps * (mean - c)^2 / var instead of ~eps * mean^2 / var. */
  const float* stats_center;
} selunet_epilogue;

const char* selunet_last_error(void);
int32_t selunet_version(void);
/* Fingerprint (SHA-256 prefix) of the kernel sources, headers and flags this library was built from. */
const char* selunet_build_id(void);

/* ---- weight repacking (fp32 master weights -> GEMM operands, dtype) ---------------- */
/* conv3x3 weight [co][ci][3][3] -> fwd [co][k_pad] (k = tap*ci + c, zero pad to k_pad) and,
 * if dgrad != NULL, dgrad [ci][9*co] with the taps flipped (k = tap*co + o). */
int selunet_pack_conv3x3(const float* w, int32_t co, int32_t ci, int32_t k_pad, void* fwd,
                         void* dgrad, int32_t dtype, void* stream);
/* ConvTranspose2d weight [ci][co][2][2] -> fwd [4*co][ci] (row (a*2+b)*co+o) and
 * dgrad [ci][4*co]. */
int selunet_pack_convT(const float* w, int32_t ci, int32_t co, void* fwd, void* dgrad,
                       int32_t dtype, void* stream);
/* packed fp32 grads -> reference layouts (accumulated into out when accumulate != 0) */
int selunet_unpack_conv3x3_grad(const float* packed, int32_t co, int32_t ci, int32_t k_pad,
                                float* out, void* stream);
int selunet_unpack_convT_grad(const float* packed, int32_t ci, int32_t co, float* out, void* stream);

/* ---- implicit GEMMs (MFMA) ------------------------------------------------------------ */
/* out = G_a[M][K] * B^T, B = [n_cols][k_pad] in dtype. Replaces conv2d 3x3 forward and
 * data-gradient, conv_transpose2d forward and data-gradient (model.py:11,44,51,57). */
int selunet_gemm_gather(const selunet_gather* a, const void* b, int32_t n_cols, int32_t k_pad,
                        const selunet_epilogue* ep, int32_t dtype, void* stream);
/* fp32 3x3 conv forward / data gradient (model.py:11; the reference's conv2d and its input
 * gradient) as a 1-D Winograd F(2,3) along x: per output pair and kernel row, four fp32 MFMA passes
 * over transformed operands (V = d0-d2, d1+d2, d2-d1, d1-d3; U = g0, (g0+g1+g2)/2, (g0-g1+g2)/2,
 * g2) instead of six direct ones. u = [n_cols][12*C] (k = (dy*4 + xi)*C + c), written by
 * selunet_pack_weights with kind SELUNET_PACK_CONV3X3_WINO. Same operands, epilogues and
 * statistics slab rows (selunet_gemm_stats_rows) as selunet_gemm_gather on the same 3x3 gather;
 * selunet_conv3x3_wino_ok tells from the shapes whether a layer can take it (fp32 multi-chunk
 * halo layers: h, w >= 16, w even, C a multiple of 32 and > 32, n_cols a multiple of 64). */
int32_t selunet_conv3x3_wino_ok(int32_t h, int32_t w, int32_t c_in, int32_t c_src0, int32_t n_cols);
int selunet_conv3x3_wino(const selunet_gather* a, const float* u, int32_t n_cols,
                         const selunet_epilogue* ep, void* stream);
const char* selunet_conv3x3_wino_kernel_name(int32_t n_cols, int32_t mode, int32_t split);
/* fp32 3x3 conv forward / data gradient (model.py:11 and its input gradient) on the fp16 matrix
 * cores: each fp32 operand is split into two fp16 parts, v*2^e = h + l (22 significant bits,
 * 2^e a power of two that keeps the operand below 2^14), and every product is summed as
 * h_a*h_b + h_a*l_b + l_a*h_b in fp32 accumulators (three v_mfma_f32_32x32x16_f16 per 16-channel
 * step; the dropped l_a*l_b is below 2^-22 of the product). Measured relative RMS error against
 * fp64 at K = 576..4608 is at or below the exact fp32 MFMA's (tools/split_probe.hip). Operand
 * ranges: amax0 / amax1 (device words, amax1 only for a two-source gather) bound |source value
 * after its BN+ReLU transform|: selunet_act_bound for a BN+ReLU source, the producing kernel's
 * atomic max (selunet_epilogue.amax, selunet_bn_bwd_apply) otherwise. w: a
 * SELUNET_PACK_CONV3X3_X2 pack ([n_cols][9*C] + n_cols row unscale factors). Same gathers,
 * epilogues and statistics slab rows as selunet_gemm_gather; selunet_conv3x3_x2_ok tells whether a
 * layer can take it (h, w >= 16, C and c_src0 multiples of 32, C > 32, n_cols a multiple of 64). */
/* selunet_gemm_gather on split-fp16 operands (ConvTranspose2d forward / data gradient in fp32 training,
 * model.py:44,51,57): w a split-fp16 pack (SELUNET_PACK_CONVT_X2 rows, k_pad == K, K a multiple of 32),
 * amax0 / amax1 the sources' range words; any gather taps and epilogue of selunet_gemm_gather. Its
 * statistics slabs have selunet_gemm_gather_x2_stats_rows rows (256-row persistent tiles). */
int selunet_gemm_gather_x2(const selunet_gather* a, const float* w, int32_t n_cols, int32_t k_pad,
                           const selunet_epilogue* ep, const float* amax0, const float* amax1, void* stream);
int64_t selunet_gemm_gather_x2_stats_rows(const selunet_gather* a, int32_t n_cols);
/* selunet_gemm_wgrad_ws_to on split-fp16 operands (the ConvTranspose2d weight gradient in fp32 training,
 * layout SELUNET WG_CONVT = 2, or a Conv2d one, layout 1): vector gathers, K_p and K_q multiples of 64;
 * amax_p0/p1, amax_q0/q1 the sources' range words (p1 / q1 only for two-source gathers). Partials in
 * ws (>= selunet_gemm_wgrad_x2_ws_bytes), summed in a fixed order into out. */
int64_t selunet_gemm_wgrad_x2_ws_bytes(const selunet_gather* p, const selunet_gather* q);
int selunet_gemm_wgrad_x2(const selunet_gather* p, const selunet_gather* q, float* ws, int64_t ws_bytes, int32_t layout,
                          float* out, const float* amax_p0, const float* amax_p1, const float* amax_q0,
                          const float* amax_q1, void* stream);
int32_t selunet_conv3x3_x2_ok(int32_t h, int32_t w, int32_t c_in, int32_t c_src0, int32_t n_cols);
/* fp32 3x3 weight gradient (autograd of model.py:11's weight) on split-fp16 operands, the same
 * arithmetic as selunet_conv3x3_x2: p = dY (1 tap, [M][co]), q = the layer input (3x3 gather, BN+ReLU
 * transforms of its sources); amax_p / amax_q0 / amax_q1 their range words. Pixel-split partials in
 * ws (>= selunet_conv3x3_wgrad_x2_ws_bytes) are summed in a fixed order straight into out, the
 * Conv2d weight layout [co][ci][3][3] (deterministic). -1 bytes: operands not eligible (q: h >= 8,
 * w >= 16, channels multiples of 64; co a multiple of 64). */
int64_t selunet_conv3x3_wgrad_x2_ws_bytes(const selunet_gather* p, const selunet_gather* q);
int selunet_conv3x3_wgrad_x2(const selunet_gather* p, const selunet_gather* q, float* ws, int64_t ws_bytes,
                             float* out, const float* amax_p, const float* amax_q0, const float* amax_q1,
                             void* stream);
/* selunet_conv3x3_wgrad_x2 with the layer's BN-backward apply fused into its dY staging (replaces
 * selunet_bn_bwd_apply_amax + selunet_conv3x3_wgrad_x2; model.py:12-13's backward): p gathers dA (one
 * source, no transform), bnb the forward's y / scale / shift / mean / invstd (slab unused), coef the
 * [3][C] coefficients of selunet_bn_bwd_stats_finalize; the kernel forms
 * dy = (y*scale+shift > 0 ? k0*dA : 0) - k1 - k2*invstd*(y - mean) exactly as selunet_bn_bwd_apply,
 * stages it split-fp16 with the range word amax_p (an upper bound of |dy|:
 * selunet_bn_bwd_stats_finalize_bound), and writes dy [M][C] (fp32, nullable) with its exact max |dy|
 * into *dy_amax (atomic max; zeroed by the caller) for the layer's data gradient. */
int selunet_conv3x3_wgrad_x2_bn(const selunet_gather* p, const selunet_gather* q, float* ws, int64_t ws_bytes,
                                float* out, const float* amax_p, const float* amax_q0, const float* amax_q1,
                                const selunet_bn_bwd_stats* bnb, const float* coef, float* dy, float* dy_amax,
                                void* stream);
/* Where selunet_conv3x3_wgrad_x2_bn_src's dY staging takes dA from. TENSOR: p's source (as
 * selunet_conv3x3_wgrad_x2_bn). POOL: the layer feeds a 2x2 max-pool (model.py:30,60-61's encoder
 * blocks): dA = route(pooled) + skip, pooled [n][h/2][w/2][C] the pool output's gradient routed to
 * the first maximum of relu(y*scale+shift) in row-major window order, skip [M][C] (nullable) added to
 * every pixel — selunet_bn_bwd_apply_pool's dA. HEADS: the layer feeds the 1x1 heads (model.py:62-66):
 * dA[m][c] = sum_h head_w[h][c] * g[h][m] over nh = 1 or 3 heads, C = 64 — selunet_bn_bwd_apply_heads's
 * dA. For POOL / HEADS p only gives the grid and C (its data is not read) and C must be 64. */
enum { SELUNET_DA_TENSOR = 0, SELUNET_DA_POOL = 1, SELUNET_DA_HEADS = 2 };
typedef struct selunet_da_source {
  int32_t kind;
  int32_t nh;
  const float* pooled;
  const float* skip;
  const float* head_w;
  const float* g[3];
} selunet_da_source;
/* selunet_conv3x3_wgrad_x2_bn with dA formed from `src` (NULL: TENSOR): the fused pool / heads applies
 * (selunet_bn_bwd_apply_pool / _heads) move into the weight gradient's staging like the plain one. */
int selunet_conv3x3_wgrad_x2_bn_src(const selunet_gather* p, const selunet_gather* q, float* ws, int64_t ws_bytes,
                                    float* out, const float* amax_p, const float* amax_q0, const float* amax_q1,
                                    const selunet_bn_bwd_stats* bnb, const float* coef, const selunet_da_source* src,
                                    float* dy, float* dy_amax, void* stream);
int selunet_conv3x3_x2(const selunet_gather* a, const float* w, int32_t n_cols, const selunet_epilogue* ep,
                       const float* amax0, const float* amax1, void* stream);
const char* selunet_conv3x3_x2_kernel_name(const selunet_gather* a, int32_t n_cols, int32_t mode, int32_t split);
/* Statistics slab rows (stats / colsum / BN-backward sums of the epilogue) selunet_conv3x3_x2 and
 * write for this operand: the layers SELUNET_OPT_X2D sends to the 64-column kernel
 * with two 256-thread workgroups per CU have min(16x16 tiles, 512) rows, others as
 * selunet_gemm_stats_rows. selunet_conv3x3_x2_kernel_name names the kernel a call would run. */
int64_t selunet_conv3x3_x2_stats_rows(const selunet_gather* a, int32_t n_cols);
/* Range word of a training-mode BatchNorm+ReLU output relu(gamma*xhat + beta) over `count` values
 * per channel: |xhat| <= sqrt(count - 1) for batch statistics (Samuelson's inequality), so
 * *out = max_c |gamma_c| * sqrt(count) + max_c |beta_c| bounds every element (max-pooled copies
 * included). One block; c <= 4096. */
int selunet_act_bound(const float* gamma, const float* beta, int32_t c, int64_t count, float* out, void* stream);
/* Rows of the stats slab selunet_gemm_gather writes for this operand (workgroup rows of the
 * kernel it dispatches to: 16x16 halo tiles for single-chunk 3x3 operands, the persistent
 * workgroups of the multi-chunk halo kernel, else 128-row tiles); -1 on error. */
int64_t selunet_gemm_stats_rows(const selunet_gather* a, int32_t n_cols, int32_t dtype);
/* Tuning/testing knob: workgroups the persistent multi-chunk 3x3 kernel targets (default 256, one
 * per MI355X CU; wgs <= 0 restores the default). Returns the previous value. The stats-slab row
 * count depends on it: query selunet_gemm_stats_rows after changing it. Not thread-safe. */
int32_t selunet_set_halo_workgroups(int32_t wgs);
/* Tuning/testing knob: workgroups the persistent generic gather GEMM (ConvTranspose2d forward and
 * data gradient, 3x3 layers the halo kernels do not take) targets: default 512 (two per CU), 0 = one
 * output tile per workgroup, < 0 restores the default. Returns the previous value. Changes the
 * stats-slab row count like selunet_set_halo_workgroups. Not thread-safe. */
int32_t selunet_set_gather_workgroups(int32_t wgs);
/* Name of the kernel a selunet_gemm_gather (q == NULL; mode = epilogue mode) or
 * selunet_gemm_wgrad (q = the Q operand) call with these operands dispatches to. */
const char* selunet_gemm_kernel_name(const selunet_gather* a, const selunet_gather* q, int32_t n_cols,
                                     int32_t mode, int32_t dtype);
/* out[ni][nj] += sum_m G_p[m][i] * G_q[m][j] (fp32 atomics; out zeroed by the caller).
 * Replaces the weight-gradient of conv2d / conv_transpose2d (train.py:208 backward). */
int selunet_gemm_wgrad(const selunet_gather* p, const selunet_gather* q, float* out,
                       int32_t dtype, void* stream);
/* Deterministic variant: the pixel splits write their partial sums to the workspace `ws`
 * (selunet_gemm_wgrad_ws_bytes bytes; fp32 [splits][ni][ld]) and a reduction kernel sums them in
 * a fixed order into out, which is overwritten (no zeroing needed; pad columns become 0). Operands
 * without a split-partials path (fp32) report 0 bytes; out is then zeroed and accumulated with
 * atomics inside the call. Removes the fp32 atomic traffic (~150 MB per 3x3 layer) of
 * selunet_gemm_wgrad. */
int64_t selunet_gemm_wgrad_ws_bytes(const selunet_gather* p, const selunet_gather* q, int32_t dtype);
int selunet_gemm_wgrad_ws(const selunet_gather* p, const selunet_gather* q, float* out, float* ws,
                          int64_t ws_bytes, int32_t dtype, void* stream);
/* selunet_gemm_wgrad_ws with the result written in the reference parameter layout by the split
 * reduction itself: layout 1 = Conv2d weight [co][ci][3][3] (P = dY, Q = the 3x3 input taps),
 * layout 2 = ConvTranspose2d weight [ci][co][2][2] (P = the input, Q = the 4 output taps) — the
 * .grad of model.py:11 / model.py:44,51,57 weights. `packed` ([ni][selunet_wgrad_ld] fp32) is
 * scratch used only by operands without a split-partials path (may be NULL otherwise). */
int selunet_gemm_wgrad_ws_to(const selunet_gather* p, const selunet_gather* q, float* packed,
                             float* ws, int64_t ws_bytes, int32_t layout, float* out, int32_t dtype,
                             void* stream);
/* Row stride of the packed wgrad output for a Q operand with kq columns (kq rounded up to
 * the column tile); `out` must be [ni][selunet_wgrad_ld(kq)], the pad columns are garbage-free
 * zeros when out was zeroed. */
int32_t selunet_wgrad_ld(int32_t kq);

/* Every weight pack of a step in one launch: conv3x3 entries as selunet_pack_conv3x3 (fwd
 * required, dgrad optional), ConvTranspose2d entries as selunet_pack_convT (w [ci][co][2][2]).
 * `offset` is computed by the call. Replaces the per-tensor loop over model.py's conv/unpool
 * parameters (model.py:11,44,51,57) that casting fp32 masters to the compute operands needs. */
#define SELUNET_PACK_MAX 32
/* SELUNET_PACK_CONV3X3_WINO (fp32): fwd = [co][12*ci] and dgrad = [ci][12*co] Winograd weight
 * operands of selunet_conv3x3_wino (k_pad = 12*ci; dgrad from the flipped/transposed kernel). */
/* SELUNET_PACK_CONV3X3_X2 (fp32): split-fp16 operands of selunet_conv3x3_x2, k_pad = 9*ci; fwd =
 * [co][9*ci] and dgrad = [ci][9*co] 32-bit words (taps flipped), each row scaled by 2^e_row
 * (max|w_row| * 2^e_row < 2^14) and every 32-k group (one tap, 32 channels) stored as 32 fp16 high
 * parts h = fp16(v) then 32 low parts l = fp16(v - h); the row unscale factors 2^-e_row follow the
 * matrix: fwd + co*9*ci (co floats), dgrad + ci*9*co (ci floats). ci, co multiples of 32. */
/* SELUNET_PACK_CONVT_X2 (fp32): the same split-fp16 format for a ConvTranspose2d weight [ci][co][2][2]:
 * fwd = [4*co][ci] (row (a*2+b)*co + o, k_pad = ci) + 4*co unscale factors, dgrad = [ci][4*co] + ci. */
/* SELUNET_PACK_COPY (any dtype): co*ci fp32 values w -> fwd unchanged (dgrad unused) — the heads'
 * current weights and biases (model.py:62,65,66) gathered into the contiguous [heads][64] / [heads]
 * operands of selunet_heads_fwd in the same launch. */
enum {
  SELUNET_PACK_CONV3X3 = 0,
  SELUNET_PACK_CONVT = 1,
  SELUNET_PACK_CONV3X3_WINO = 2,
  SELUNET_PACK_CONV3X3_X2 = 3,
  SELUNET_PACK_CONVT_X2 = 4,
  SELUNET_PACK_COPY = 5
};
typedef struct selunet_pack_desc {
  const float* w;
  void* fwd;
  void* dgrad;
  int32_t kind, co, ci, k_pad;
  int64_t offset;
} selunet_pack_desc;
typedef struct selunet_pack_list {
  int32_t n, _pad;
  selunet_pack_desc d[SELUNET_PACK_MAX];
} selunet_pack_list;
int selunet_pack_weights(const selunet_pack_list* list, int32_t dtype, void* stream);

/* ---- reductions ----------------------------------------------------------------------- */
/* out[c] = sum_r slab[r][c] in fp64, deterministic order, written as fp64 (out) and/or fp32
 * (out32), either may be NULL; ws: >= selunet_reduce_ws_bytes(cols). */
int64_t selunet_reduce_ws_bytes(int32_t cols);
int selunet_reduce_rows(const float* slab, int64_t rows, int32_t cols, double* ws, double* out,
                        float* out32, void* stream);
/* per-channel sums of an NHWC tensor: slab [selunet_channel_slab_rows(M)][C] */
int64_t selunet_channel_slab_rows(int64_t m);
int selunet_channel_sum(const void* x, int64_t m, int32_t c, float* slab, int32_t dtype, void* stream);

/* ---- BatchNorm2d (model.py:12; eps 1e-5, momentum 0.1) ------------------------------- */
/* From fp64 sums [2][C] (sum, sumsq of conv output without bias) over `count` pixels:
 * training: mean/invstd of the batch, running stats updated (unbiased var), *num_batches += 1;
 * eval (training == 0): running stats. Writes mean (of conv output w/o bias), invstd, and the
 * folded scale = gamma*invstd, shift = beta - mean*scale used by consumers' loaders. */
int selunet_bn_finalize(const double* sums, int64_t count, int32_t c, const float* conv_bias,
                        const float* gamma, const float* beta, float* running_mean,
                        float* running_var, int64_t* num_batches, float momentum, float eps,
                        int32_t training, float* mean, float* invstd, float* scale, float* shift,
                        void* stream);
/* slab [selunet_channel_slab_rows(M)][3][C]: sum(dA), sum(dA*xhat), sum(xhat), dA = dz*[z>0],
 * z = relu(y*scale+shift), xhat = (y-mean)*invstd. */
int selunet_bn_bwd_reduce(const void* dz, const void* y, int64_t m, int32_t c, const float* scale,
                          const float* shift, const float* mean, const float* invstd, float* slab,
                          int32_t dtype, void* stream);
/* From fp64 sums [3][C]: dgamma, dbeta, dbias (pre-BN conv bias), coef [3][C]. */
int selunet_bn_bwd_finalize(const double* sums, int64_t count, int32_t c, const float* gamma,
                            const float* invstd, float* dgamma, float* dbeta, float* dbias,
                            float* coef, void* stream);
/* Fused forms used by the training step: the column sums of the statistics slab the producer
 * wrote ([rows][2][C] sum/sumsq for the forward, [rows][3][C] for the backward) reduced in fp64
 * (fixed order) and finalized in one launch (two above SELUNET_RF_SINGLE rows, default 1024).
 * Same results as selunet_reduce_rows + selunet_bn_finalize(training = 1) /
 * selunet_bn_bwd_finalize up to the fp64 summation order. ws: >= selunet_reduce_ws_bytes(2*C or
 * 3*C); sums (fp64 [2|3][C]) may be NULL. Replace BatchNorm2d's batch-statistics pass
 * (model.py:12) and its backward (autograd of model.py:12). */
int selunet_bn_stats_finalize(const float* slab, int64_t rows, double* ws, double* sums, int64_t count,
                              int32_t c, const float* conv_bias, const float* gamma, const float* beta,
                              float* running_mean, float* running_var, int64_t* num_batches,
                              float momentum, float eps, float* mean, float* invstd, float* scale,
                              float* shift, void* stream);
/* Second (centered) pass of the batch statistics, fp32 parity configuration: slab [rows][2][c] of
 * per-channel sums of (y - center) and (y - center)^2 over y [m][c] (center = the first pass's
 * batch mean; rows = selunet_bn_centered_rows(m)); then selunet_bn_stats_finalize_centered
 * reduces it like selunet_bn_stats_finalize (mean = center + E[y - center], var = E[(y - center)^2]
 * - E[y - center]^2) and writes the same outputs — `mean` may alias `center`. Same role as
 * selunet_bn_stats_finalize (model.py:12 BatchNorm2d batch statistics), numerically two-pass. */
int64_t selunet_bn_centered_rows(int64_t m);
int selunet_bn_centered_partials(const void* y, int64_t m, int32_t c, const float* center, float* slab,
                                 int32_t dtype, void* stream);
/* Adaptive second pass: uvar[c] = the first pass's unbiased variance (selunet_bn_stats_finalize with
 * running_var = a zeroed scratch, running_mean = NULL, momentum 1). A group of 4 channels is re-read
 * (as selunet_bn_centered_partials) only if one of them has center^2 > ratio * uvar — where
 * E[y^2] - mean^2 loses digits; the others write the sums that make the centered finalize return
 * the first pass's variance. Same slab layout and finalize. */
int selunet_bn_centered_partials_adaptive(const void* y, int64_t m, int32_t c, const float* center,
                                          const float* uvar, float ratio, float* slab, int32_t dtype,
                                          void* stream);
/* First pass of the fp32 batch statistics from a slab of SHIFTED sums (selunet_epilogue.stats_center =
 * center, the previous step's batch mean): mean = center + E[y - center]; uvar_flag[c] = the unbiased
 * one-pass variance, or -1 where (mean - center)^2 > ratio * var (there it loses digits); center is
 * then overwritten with mean (the next step's center). invstd / scale / shift are provisional (eps
 * 1e-5, no running-statistic update). Followed by selunet_bn_centered_partials_adaptive(center = mean,
 * uvar = uvar_flag, ratio = +inf: re-reads exactly the flagged channel groups) and
 * selunet_bn_stats_finalize_centered, whose outputs are final. In training the previous batch mean
 * differs from the current one by a small fraction of the standard deviation, so after the first
 * step almost no channel group is re-read. */
int selunet_bn_stats_finalize_shifted(const float* slab, int64_t rows, double* ws, int64_t count, int32_t c,
                                      float* center, const float* conv_bias, const float* gamma,
                                      const float* beta, float ratio, float* mean, float* uvar_flag,
                                      float* invstd, float* scale, float* shift, void* stream);
int selunet_bn_stats_finalize_centered(const float* slab, int64_t rows, double* ws, double* sums,
                                       int64_t count, int32_t c, const float* center,
                                       const float* conv_bias, const float* gamma, const float* beta,
                                       float* running_mean, float* running_var, int64_t* num_batches,
                                       float momentum, float eps, float* mean, float* invstd,
                                       float* scale, float* shift, void* stream);
/* selunet_bn_stats_finalize_centered that also folds the split-fp16 range word of relu(bn(y)) into
 * *bound (zeroed by the caller before the step): atomic max over the channels of
 * (|gamma_c| * sqrt(count) + |beta_c|) * 1.0001 — the per-channel form of selunet_act_bound's
 * Samuelson bound (never larger), without its separate launch. bound may be NULL. */
int selunet_bn_stats_finalize_centered_bound(const float* slab, int64_t rows, double* ws, double* sums,
                                             int64_t count, int32_t c, const float* center,
                                             const float* conv_bias, const float* gamma, const float* beta,
                                             float* running_mean, float* running_var, int64_t* num_batches,
                                             float momentum, float eps, float* mean, float* invstd,
                                             float* scale, float* shift, float* bound, void* stream);
int selunet_bn_bwd_stats_finalize(const float* slab, int64_t rows, double* ws, double* sums,
                                  int64_t count, int32_t c, const float* gamma, const float* invstd,
                                  float* dgamma, float* dbeta, float* dbias, float* coef,
                                  void* stream);
/* selunet_bn_bwd_stats_finalize that also folds an upper bound of |dy| into *bound (zeroed by the
 * caller; atomic max over the channels of 1.25 * (|k0| amax_da + |k1| + |k2| sqrt(count)), amax_da the
 * exact max |dA| its producer recorded): the range word selunet_conv3x3_wgrad_x2_bn stages dy with
 * before dy exists. */
int selunet_bn_bwd_stats_finalize_bound(const float* slab, int64_t rows, double* ws, double* sums,
                                        int64_t count, int32_t c, const float* gamma, const float* invstd,
                                        float* dgamma, float* dbeta, float* dbias, float* coef,
                                        const float* amax_da, float* bound, void* stream);
/* dy = coef0*dA - coef1 - coef2*xhat (the conv-output gradient). */
int selunet_bn_bwd_apply(const void* dz, const void* y, int64_t m, int32_t c, const float* scale,
                         const float* shift, const float* mean, const float* invstd,
                         const float* coef, void* dy, int32_t dtype, void* stream);
/* The same with max|dy| folded into *amax (atomic max on the float bits; zeroed by the caller):
 * the range word of dy as a split-fp16 operand (selunet_conv3x3_x2, split-fp16 weight gradient). */
int selunet_bn_bwd_apply_amax(const void* dz, const void* y, int64_t m, int32_t c, const float* scale,
                              const float* shift, const float* mean, const float* invstd,
                              const float* coef, void* dy, float* amax, int32_t dtype, void* stream);

/* Stream-ordered device memset / device-to-device copy (hipMemsetAsync / hipMemcpyAsync):
 * zeroing atomic-accumulation targets and gathering small parameter vectors inside a recorded
 * launch plan, without host synchronisation. */
int selunet_memset(void* dst, int32_t value, int64_t bytes, void* stream);
int selunet_memcpy(void* dst, const void* src, int64_t bytes, void* stream);

/* ---- HIP graphs of recorded launch plans ---------------------------------------------------
 * A replayed launch plan (a whole forward or backward pass, ~100 launches) is captured once into
 * a hipGraph and afterwards issued with one selunet_graph_launch instead of one host call per
 * kernel. Capture runs on a private non-blocking stream (the default stream cannot capture);
 * the instantiated graph is then launched on the caller's stream. */
int selunet_stream_create(void** out);
int selunet_stream_destroy(void* stream);
int selunet_graph_capture_begin(void* stream);
int selunet_graph_capture_end(void* stream, void** exec);
int selunet_graph_launch(void* exec, void* stream);
int selunet_graph_destroy(void* exec);

/* ---- first layer (C_in = 3 or 2, model.py:24-29) --------------------------------------- */
/* x NCHW fp32 -> out [n*h*w][k_pad] in dtype: column tap*c + ci of the 3x3 pad-1 window, zero
 * for columns >= 9c. The first conv then runs as selunet_gemm_gather with taps = 1. */
int selunet_im2col3x3(const float* x, int32_t n, int32_t c, int32_t h, int32_t w, int32_t k_pad, void* out,
                      int32_t dtype, void* stream);
/* encoder_layer_1_1's conv (model.py:29) straight from the NCHW fp32 input x [n][cin][h][w]
 * (cin <= 3) to y [n*h*w][64] in dtype, no bias (it cancels in training-mode BN), with the BN
 * column statistics of selunet_gemm_gather (stats [selunet_first_conv_rows][2][64], nullable).
 * wpack: the conv weight from selunet_pack_conv3x3 with k_pad = 32. */
int64_t selunet_first_conv_rows(int32_t n, int32_t h, int32_t w);
/* selunet_first_conv_fwd with its statistics shifted by center (selunet_epilogue.stats_center). */
int selunet_first_conv_fwd_centered(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w,
                                    const void* wpack, void* y, float* stats, const float* center,
                                    int32_t dtype, void* stream);
int selunet_first_conv_fwd(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, const void* wpack,
                           void* y, float* stats, int32_t dtype, void* stream);
/* Its weight gradient: slab [selunet_first_conv_wgrad_rows][64][32] of per-workgroup partial sums
 * of dY^T im2col(x) (column k = tap*cin + c); reduce the rows (selunet_reduce_rows) to the packed
 * [64][32] gradient, then selunet_unpack_conv3x3_grad(.., ld = 32). */
int64_t selunet_first_conv_wgrad_rows(int32_t n, int32_t h, int32_t w);
int selunet_first_conv_wgrad(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, const void* dy,
                             float* slab, int32_t dtype, void* stream);
/* The same weight gradient with encoder_layer_1_1's BatchNorm+ReLU backward fused into the staging:
 * dz = dA of the layer, y its conv output, scale/shift/mean/invstd its BN, coef [3][64] from
 * selunet_bn_bwd_stats_finalize; dy = (y*scale+shift > 0 ? k0*dz : 0) - b - a*y exactly as
 * selunet_bn_bwd_apply forms it, never written (replaces selunet_bn_bwd_apply + selunet_first_conv_wgrad,
 * whose dy has no other reader: the input needs no gradient, model.py:29 / train.py:207). */
int selunet_first_conv_wgrad_bn(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, const void* dz,
                                const void* y, const float* scale, const float* shift, const float* mean,
                                const float* invstd, const float* coef, float* slab, int32_t dtype, void* stream);

/* ---- MaxPool2d(2) on relu(bn(y)) (model.py:31,35,39) ---------------------------------- */
int selunet_maxpool2_fwd(const void* y, int32_t n, int32_t h, int32_t w, int32_t c,
                         const float* scale, const float* shift, void* out, int32_t dtype,
                         void* stream);
/* dz = route(dpool to the first max of each window, row-major, strict >) + dskip (nullable).
 * bnb (nullable; bnb->y must be y): BatchNorm-backward sums of dz, slab
 * [selunet_maxpool2_bwd_slab_rows(n, h, w, c)][3][c]. dz may be NULL when bnb is given: the sums only
 * (selunet_bn_bwd_apply_pool then forms dz itself). */
int selunet_maxpool2_bwd(const void* y, int32_t n, int32_t h, int32_t w, int32_t c,
                         const float* scale, const float* shift, const void* dpool,
                         const void* dskip, void* dz, const selunet_bn_bwd_stats* bnb, int32_t dtype,
                         void* stream);
int64_t selunet_maxpool2_bwd_slab_rows(int32_t n, int32_t h, int32_t w, int32_t c);

/* ---- 1x1 heads conv1x1 / conv_select / conv_aux on relu(bn(y)), C = 64 (model.py:62-66) */
int selunet_heads_fwd(const void* y, int64_t m, const float* scale, const float* shift,
                      const float* w, const float* b, int32_t nh, float* out0, float* out1,
                      float* out2, int32_t dtype, void* stream);
/* dz[m][c] = sum_h g_h[m] w_h[c]; slab [selunet_channel_slab_rows(M)][nh][65]: per head
 * sum g*z (weight grad, 64) and sum g (bias grad). bnb (nullable; bnb->y must be y):
 * BatchNorm-backward sums of dz, slab [selunet_channel_slab_rows(M)][3][64]. */
int selunet_heads_bwd(const void* y, int64_t m, const float* scale, const float* shift,
                      const float* w, int32_t nh, const float* g0, const float* g1,
                      const float* g2, void* dz, float* slab, const selunet_bn_bwd_stats* bnb,
                      int32_t dtype, void* stream);
/* BatchNorm-backward apply (as selunet_bn_bwd_apply_amax; amax nullable) with dA formed on the fly
 * instead of read, for the two producers whose dA is cheap to recompute — their kernels then run in
 * sums-only mode (dz = NULL), so dA is never written:
 *  _heads: dA[m][c] = sum_h g_h[m] w_h[c] (C = 64; the arguments of selunet_heads_bwd);
 *  _pool:  dA = route(dpool) + dskip (the arguments of selunet_maxpool2_bwd).
 * dA is rounded to dtype before use, as the stored tensor of the unfused path. Replaces the
 * selunet_heads_bwd / selunet_maxpool2_bwd write + selunet_bn_bwd_apply read of dA for decoder_layer_1_1
 * and encoder_layer_{1,2,3}_2 (model.py:62-66, 31/35/39, the backward of CBR_2D model.py:12-13). */
int selunet_bn_bwd_apply_heads(const void* y, int64_t m, const float* scale, const float* shift,
                               const float* mean, const float* invstd, const float* coef,
                               const float* w, int32_t nh, const float* g0, const float* g1,
                               const float* g2, void* dy, float* amax, int32_t dtype, void* stream);
int selunet_bn_bwd_apply_pool(const void* y, int32_t n, int32_t h, int32_t w, int32_t c,
                              const float* scale, const float* shift, const float* mean,
                              const float* invstd, const float* coef, const void* dpool,
                              const void* dskip, void* dy, float* amax, int32_t dtype, void* stream);

/* ---- N-output 1x1 heads (the CE `UNet`, model.py:106-191: conv1x1 64->n_cls, conv_select
 * 64->2, conv_aux 64->n_cls) on relu(bn(y)), C = 64. Output k (k < n <= 8) is an fp32 plane
 * set: pixel q of image i at plane[k][i * img_stride[k] + q] (q < hw), so the channels of
 * NCHW [N, C, H, W] logits are planes base + c*hw with img_stride C*hw. */
typedef struct selunet_head_planes {
  int32_t n;               /* outputs (<= 8) */
  int32_t hw;              /* pixels per image */
  float* plane[8];         /* fwd: written; bwd: the incoming gradients (read) */
  int64_t img_stride[8];
  int32_t w_off[8];        /* bwd: slab column of output k's 64 weight grads */
  int32_t b_off[8];        /*      and of its bias grad */
  int32_t row_len;         /*      slab row length (the heads' segment of the gradient buffer) */
} selunet_head_planes;
/* w fp32 [n][64], b fp32 [n] */
int selunet_heads_fwd_planes(const void* y, int64_t m, const float* scale, const float* shift,
                             const float* w, const float* b, const selunet_head_planes* out,
                             int32_t dtype, void* stream);
/* dz[m][c] = sum_k g_k[m] w_k[c]; slab [selunet_channel_slab_rows(M)][row_len]: per output the
 * sums g*z (64, at w_off) and g (at b_off); bnb as selunet_heads_bwd. */
int selunet_heads_bwd_planes(const void* y, int64_t m, const float* scale, const float* shift,
                             const float* w, const selunet_head_planes* grads, void* dz, float* slab,
                             const selunet_bn_bwd_stats* bnb, int32_t dtype, void* stream);
/* selunet_bn_bwd_apply_heads for the N-output heads: dA[m][c] = sum_k g_k[m] w_k[c] from the gradient
 * planes of selunet_heads_bwd_planes (which then runs with dz = NULL: the sums only). */
int selunet_bn_bwd_apply_heads_planes(const void* y, int64_t m, const float* scale, const float* shift,
                                      const float* mean, const float* invstd, const float* coef,
                                      const float* w, const selunet_head_planes* grads, void* dy,
                                      float* amax, int32_t dtype, void* stream);

/* ---- losses ----------------------------------------------------------------------------- */
/* calc_selective_risk_image_b (selective_loss.py:58-85), numerically stable form.
 * partials slab [selunet_loss_slab_rows(P)][2]: sum sigmoid(g), sum ell*sigmoid(g). */
int64_t selunet_loss_slab_rows(int64_t p);
int selunet_selective_partials(const float* out, const float* sel, const float* target,
                               int64_t p, float* slab, void* stream);
/* sums[2] global (after any cross-rank all-reduce), p_global pixels -> loss, coverage,
 * and state[4] = {S0, R, d, P} for the backward. */
int selunet_selective_finalize(const double* sums, double p_global, float lamb,
                               float target_coverage, float* loss, float* coverage,
                               float* state, void* stream);
int selunet_selective_bwd(const float* out, const float* sel, const float* target, int64_t p,
                          const float* state, float lamb, const float* g_loss,
                          const float* g_coverage, float* d_out, float* d_sel, void* stream);
/* hard_selection=True (selective_loss.py:74-77): the risk numerator weights pixels by the detached
 * hard selection [sigmoid(g) > 0.5] (slab column 1 = sum ell*[sigmoid(g) > 0.5]; column 0 stays
 * sum sigmoid(g), the coverage); finalized by selunet_selective_finalize. Selection and coverage are
 * detached in the reference, so the backward writes d_sel = 0 and
 * d_out = g_loss * [sigmoid(g) > 0.5] * (sigmoid(x) - t) / sum sigmoid(g). */
int selunet_selective_partials_hard(const float* out, const float* sel, const float* target,
                                    int64_t p, float* slab, void* stream);
int selunet_selective_bwd_hard(const float* out, const float* sel, const float* target, int64_t p,
                               const float* state, const float* g_loss, float* d_out, float* d_sel,
                               void* stream);
/* BCEWithLogitsLoss() mean (train.py:78): slab [selunet_loss_slab_rows(P)][1]. */
int selunet_bce_partials(const float* logit, const float* target, int64_t p, float* slab,
                         void* stream);
int selunet_bce_finalize(const double* sums, double p_global, float* loss, void* stream);
int selunet_bce_bwd(const float* logit, const float* target, int64_t p, double p_global,
                    const float* g_loss, float* d_logit, void* stream);
/* Cross-entropy forms (CE `UNet`, n_cls = C <= 8): logits NCHW fp32 [N][C][hw], selection NCHW
 * [N][2][hw], target int64 class indices [N][hw] (a value outside [0, C) makes that pixel's loss
 * term and gradients NaN, as torch rejects it).
 * calc_selective_risk_image (selective_loss.py:24-56): s = softmax(selection)[:, 1],
 * ell = -log_softmax(output)[target]; partials slab [selunet_loss_slab_rows(N*hw)][2] = sum s,
 * sum ell*s — finalized by selunet_selective_finalize exactly as the BCE form. */
int selunet_ce_selective_partials(const float* out, const float* sel, const int64_t* target, int64_t n,
                                  int32_t c, int64_t hw, float* slab, void* stream);
int selunet_ce_selective_bwd(const float* out, const float* sel, const int64_t* target, int64_t n, int32_t c,
                             int64_t hw, const float* state, float lamb, const float* g_loss,
                             const float* g_coverage, float* d_out, float* d_sel, void* stream);
/* hard_selection=True of the CE form (selective_loss.py:43-48), as the _hard BCE entry points. */
int selunet_ce_selective_partials_hard(const float* out, const float* sel, const int64_t* target, int64_t n,
                                       int32_t c, int64_t hw, float* slab, void* stream);
int selunet_ce_selective_bwd_hard(const float* out, const float* sel, const int64_t* target, int64_t n,
                                  int32_t c, int64_t hw, const float* state, const float* g_loss,
                                  float* d_out, float* d_sel, void* stream);
/* torch.nn.CrossEntropyLoss() mean (train.py:80): slab [selunet_loss_slab_rows(N*hw)][1] = sum ell,
 * finalized by selunet_bce_finalize (sum / P). */
int selunet_ce_partials(const float* logit, const int64_t* target, int64_t n, int32_t c, int64_t hw,
                        float* slab, void* stream);
int selunet_ce_bwd(const float* logit, const int64_t* target, int64_t n, int32_t c, int64_t hw, double p_global,
                   const float* g_loss, float* d_logit, void* stream);

/* ---- torch.optim.Adam (train.py:90,209), multi-tensor ---------------------------------- */
typedef struct selunet_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
  int64_t chunk_begin; /* prefix sum of ceil(numel / SELUNET_ADAM_CHUNK) */
} selunet_adam_tensor;
#define SELUNET_ADAM_CHUNK 4096
/* list: device array of n entries. step: the 1-based step count after increment. */
int selunet_adam_step(const selunet_adam_tensor* list, int32_t n, int64_t total_chunks, float lr,
                      float beta1, float beta2, float eps, float weight_decay, int64_t step,
                      void* stream);

/* ---- training-loop I/O ------------------------------------- */
/* Pre-decoded patches -> network input and BCE target, replacing PatchDataset.__getitem__'s
 * numpy transforms (utils/data_utils.py:94-125,160-168,220-221; train.py:189-191).
 * img: uint8 NHWC [n][h][w][cin] (cin = 3, RGB); lab: uint8 [n][h][w] raw mask values (only 255
 * maps to 1); flips: uint8 [n] (bit 0 = np.fliplr, bit 1 = np.flipud; NULL = none).
 * x: fp32 NCHW [n][3][h][w] = (float32(v/255.0) - 0.5)/0.5; target: fp32 [n][h][w] in {0,1}.
 * cin = 2: input_type 'GH' (utils/data_utils.py:13-27): x [n][2][h][w] = normalised (cv2 gray,
 * skimage hematoxylin stain min-max scaled with the reference's constants). */
int selunet_prep_batch(const uint8_t* img, const uint8_t* lab, const uint8_t* flips, int32_t n,
                       int32_t h, int32_t w, int32_t cin, float* x, float* target, void* stream);
/* The same by input_type: mode 0 'RGB', 1 'GH', 2 'H_RGB' (utils/data_utils.py:29-41: the
 * hematoxylin stain recombined alone by skimage.color.combine_stains; x [n][3][h][w]). */
int selunet_prep_batch_mode(const uint8_t* img, const uint8_t* lab, const uint8_t* flips, int32_t n,
                            int32_t h, int32_t w, int32_t mode, float* x, float* target, void* stream);
/* Per-batch metrics of train.py:211-238 / eval.py:218-246 accumulated on the device:
 * counts[6] (uint64, caller-zeroed, accumulated across calls) = {cm[0][0], cm[0][1], cm[1][0],
 * cm[1][1], selected, total} with cm[label][pred] = Evaluator.confusion_matrix
 * (utils/compute_metric.py:10-26) over pixels whose selection logit >= t_sel (all pixels when
 * sel is NULL); pred = out >= t_out. t_out / t_sel: the smallest fp32 logit the reference's
 * host rule (sigmoid in fp64 or fp32, then > cut_off) maps to 1. */
int selunet_seg_metrics(const float* out, const float* sel, const float* target, int64_t p,
                        float t_out, float t_sel, unsigned long long* counts, void* stream);

/* ---- multi-GPU overlap probe (bench/tools only, not on the training path) ------
 * Stand-in for one bucketed RCCL all-reduce kernel on a single GPU: n_wg workgroups of 256 threads
 * reduce-copy dst[i] += src[i] over their slices of [0, n) (n % 4 == 0, 16-B aligned), repeatedly,
 * until `us` microseconds of GPU wall clock have passed since each workgroup started — holding
 * n_wg CUs' worth of waves the way a ring all-reduce holds its channels. Issued on a side stream at
 * GradBucketer's bucket points by tools/overlap_emulation.py. */
int selunet_cu_hold(const float* src, float* dst, int64_t n, int32_t n_wg, float us, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SELUNET_H */
