/*
 * sdmi.h — C ABI of the MI355X (gfx950) latent-diffusion denoising path.
 *
 * The reference (wangze22/StableDiffusion-PyTorch) has no native library: its boundary is the
 * PyTorch nn.Module surface (models/unet_cond_base.py:15,124; models/blocks.py; scheduler/
 * linear_noise_scheduler.py:13,26,50) over aten kernels. Each entry point below replaces the aten
 * op(s) the reference's modules call at the cited line; the Python mirror in
 * stablediffusion-pytorch_amd/sdmi/ binds them with ctypes.
 *
 * Conventions
 *  - Every pointer is a device pointer owned by the caller; kernels never allocate. Scratch that an
 *    op needs is sized by its *_workspace query and passed in.
 *  - Activations are NHWC ("pixel-major, channel-contiguous") bf16 (raw uint16 bits); a row stride
 *    (ld, in elements) lets a tensor be a channel slice of a wider buffer (skip concatenation).
 *  - Statistics, accumulators, master weights and gradients are fp32.
 *  - All work is enqueued on `stream` (a hipStream_t); no entry point synchronises.
 *  - Return value: 0 = ok, <0 = rejected arguments (nothing launched), >0 = hipError_t.
 */
#ifndef SDMI_H
#define SDMI_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* sdmi_stream_t; /* hipStream_t */

/* ---------------------------------------------------------------------------------------------
 * MFMA GEMM family:  C[m][n] = epilogue( sum_k A[m][k] * B[k][n] )
 *
 * Replaces aten conv2d / conv_transpose2d (fwd, dgrad, wgrad) called by nn.Conv2d at
 * models/blocks.py:48-53,67-72,102-109 and nn.ConvTranspose2d at models/blocks.py:457-459, and
 * aten addmm/mm called by nn.Linear (blocks.py:58-61, :89, :97; unet_cond_base.py:86-90) and by
 * nn.MultiheadAttention's packed in/out projections (blocks.py:83,94).
 * ------------------------------------------------------------------------------------------- */
enum {
  SDMI_A_ROWMAJOR = 0, /* A[m][k] = A[m*lda + k]                                   */
  SDMI_A_CONV = 1,     /* A[m][k] = im2col gather of an NHWC tensor (see geometry)  */
  SDMI_A_COLMAJOR = 2  /* A[m][k] = A[k*lda + m]                                   */
};
enum {
  SDMI_B_NK = 0,      /* B[k][n] = B[n*ldb + k]  (nn.Linear / packed conv weight)   */
  SDMI_B_KN = 1,      /* B[k][n] = B[k*ldb + n]                                   */
  SDMI_B_KN_CONV = 2  /* B[k][n] = im2col gather: k = pixel, n = (tap, channel)    */
};

typedef struct sdmi_conv_geom {
  /* gathered NHWC input: pixel (b, iy, ix) channel c at x[((b*ih + iy)*iw + ix)*ldx + c] */
  int ih, iw, cin, ldx;
  int kh, kw;           /* taps */
  int oh, ow;           /* GEMM pixel grid (any size) used to decompose a pixel index m   */
  int sy, sx, oy0, ox0; /* iy = oy*sy + ty + oy0, ix = ox*sx + tx + ox0 (zero outside)      */
} sdmi_conv_geom;

typedef struct sdmi_gemm_desc {
  int m, n, k;
  int a_mode, b_mode;
  const void* a; int lda; /* bf16 */
  const void* b; int ldb; /* bf16 */
  sdmi_conv_geom geom;    /* used by SDMI_A_CONV / SDMI_B_KN_CONV */
  /* epilogue: v = alpha*acc + bias[n] + rowbias[(m / rb_div)*rb_ld + n] + resid[orow*ldr + n];
   *           v = act(v); C[orow*ldc + ocol] = v   (orow = row remap of m, ocol = col permute of n) */
  void* c; int ldc; int c_f32;
  const float* bias;          /* fp32 [n] or NULL      */
  const void* rowbias;        /* bf16 or NULL           */
  int rb_ld, rb_div;          /* rb_div 0 or 1: one rowbias row per output row */
  const void* resid; int ldr; /* bf16 or NULL           */
  float alpha;
  int act;                    /* 0 none, 1 SiLU, 2 ReLU, 3 ReLU-gradient mask (aux) */
  /* row remap (stride-2 sub-pixel phases of a transposed conv): m -> (b, oy, ox) on a
   * (r_gh x r_gw) grid, orow = (b*r_oh + oy*r_sy + r_oy)*r_ow + ox*r_sx + r_ox */
  int remap, r_gh, r_gw, r_oh, r_ow, r_sy, r_sx, r_oy, r_ox;
  /* column permute (weight-gradient layouts): n = tap*p_cin + c  ->  ocol = c*p_taps + tap (perm 1, torch
   * conv weight layout) or tap*p_cvalid + c (perm 2, tap-major Linear layout of a patch embedding), stored
   * only for c < p_cvalid (0 = all): gradients of zero-padded input channels are dropped */
  int perm, p_cin, p_taps, p_cvalid;
  /* store limits (0 = m / n): rows >= m_store and columns >= n_store are computed but not stored,
   * and the bias is read only for stored columns (zero-padded output channels) */
  int m_store, n_store;
  /* second A source (SDMI_A_CONV only): columns k >= k_split read a2[m*lda2 + (k - k_split)] (bf16, row-major,
   * same pixel grid) -- fuses a 1x1 conv of another tensor into the same GEMM by K-concatenation */
  const void* a2; int lda2; int k_split;
  const float* bias2; /* second fp32 [n] bias added in the epilogue, or NULL */
  /* rowbias row index = (m / rb_div) % rb_mod when rb_mod > 0: a per-token table shared by every
   * sample (the DiT patch position embedding, models/patch_embed.py:93-95) */
  int rb_mod;
  /* act 3 (ReLU backward, models/transformer_layer.py:38-42 / transformer.py:107-111): v is kept where
   * aux[orow*ld_aux + n] > 0 (aux = the saved bf16 ReLU output), else 0 */
  const void* aux; int ld_aux;
  /* split-K slices requested by the caller (0 = built-in heuristic); clamped to >= 1 k-tile per slice and to
   * 32-bit slab offsets. Used with the measured per-shape table of sdmi/tuned_gemm.json. */
  int splits_hint;
  /* column-tile width request (0 = by occupancy: 192 when N % 192 == 0 fills the 512 workgroup slots in fewer
   * rounds; 128 / 192 = that width where the 192-wide tile applies: B_NK, row-major or implicit-conv A) */
  int tile_n_hint;
  /* reduction outputs of a col-major-A GEMM (SDMI_A_COLMAJOR: A = dY^T of a weight gradient), computed in the same
   * launch by extra synthesised B columns: sum_out[m] (and sum_out2[m]) = sum_k A[m][k] -- the bias gradient,
   * replacing a separate column-sum pass over dY -- and gsum_out[g*gsum_ld + m] (bf16) = sum over k in
   * [g*sum_group, (g+1)*sum_group) of A[m][k] -- per-sample sums, the time-embedding bias gradient
   * (models/blocks.py:117-118). NULL = not computed. Rows >= m_store are not stored. */
  float* sum_out;
  float* sum_out2;
  void* gsum_out;
  int gsum_ld;
  int sum_group;
  /* mainloop request (0 = built-in choice): 1 register-staged operands; LDS-DMA rings: 2 / 3 stages of 64-deep k
   * (128 x {64..192} tiles), 4 = 8-wave 128 x {256, 384} tiles, 5 = 3 stages of 32-deep k, 6 = 4 stages of 64-deep k
   * (128 x 128), 7 / 8 = 64 x 64 / 64 x 128 tiles with 6 stages of 64-deep k, 9 / 10 = 64 x 128 tiles with 3 / 2
   * stages (7-10: K-contiguous A and B only, the low-resolution GEMMs). Downgraded where the mode does not support it.
   * Used with the measured
   * per-shape table of sdmi/tuned_gemm.json. */
  int variant_hint;
  /* GroupNorm-backward statistics of the output (SDMI_GN_PART): the GEMM produces dy, the gradient of a
   * [SiLU(]GroupNorm(x)[)] output (models/blocks.py:45-47, 64-66, 124-126, 137-139; unet_cond_base.py:179-180), and also
   * writes, per segment of gn_rb rows (gn_rb in {16, 32, 64} divides gn_P, the rows per sample) and output column j,
   * gn_part[2*(seg*n + j)] = sum dz, gn_part[2*(seg*n + j) + 1] = sum dz*xhat over the segment's rows, where
   * dz = bf16(dy) [* SiLU'(x*a + s)], xhat = (x - mean)*rstd, x = gn_x[row*gn_ldx + j] (bf16) and {a, s, mean, rstd} =
   * gn_tab[(row / gn_P)*n + j] (the float4 forward table of sdmi_gn_fwd). Unsplit launches need gn_rb | 64, split-K
   * launches gn_rb % 8 == 0. Plain epilogue only (alpha; no bias / rowbias / resid / act / remap / perm / reductions;
   * bf16 16-B aligned output). gn_part NULL = off. sdmi_gn_bwd_part consumes the partials. */
  const void* gn_x; int gn_ldx;
  const float* gn_tab;
  float* gn_part;
  int gn_P, gn_rb, gn_silu;
} sdmi_gemm_desc;

/* Split-K plan: how many K slices the launcher will use and the fp32 workspace bytes it needs. */
/* mainloop variant (0 register-staged, 2 / 3 LDS-DMA stages) and column-tile width (128 / 192) a launch of d
 * uses; host-only, for profiling attribution */
int sdmi_gemm_kernel_info(const sdmi_gemm_desc* d, int* variant, int* tile_n);
int sdmi_gemm_plan(const sdmi_gemm_desc* d, int* splits, size_t* workspace_bytes);
int sdmi_gemm(const sdmi_gemm_desc* d, void* workspace, size_t workspace_bytes, sdmi_stream_t stream);

/* Grouped launch: ngroups (<= SDMI_GEMM_GROUP_MAX) independent problems d[0..ngroups) that are identical in every
 * descriptor field but the a / b / c / sum_out pointers (e.g. the same-shape weight gradients of one UNet block's
 * attention projections), in ONE launch (and one split-K reducer launch): the grid's z dimension runs over
 * (problem, split). No bias / resid / rowbias / aux / second A source / sum_out2 / gsum_out. The split count is the
 * single problem's (tuned, via splits_hint, or heuristic) divided by ngroups; per problem the result is bitwise the
 * single launch's at that split count. */
#define SDMI_GEMM_GROUP_MAX 8
int sdmi_gemm_grouped_plan(const sdmi_gemm_desc* d, int ngroups, int* splits, size_t* workspace_bytes);
int sdmi_gemm_grouped(const sdmi_gemm_desc* d, int ngroups, void* workspace, size_t workspace_bytes,
                      sdmi_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Fused multi-head attention (flash-style), bf16 in/out, fp32 softmax statistics.
 * Replaces the core of torch nn.MultiheadAttention as called at models/blocks.py:128 (self) and
 * :140 (cross, kv = context_proj(context)): softmax((q / sqrt(d)) k^T) v per head, head h in columns
 * [h*d, h*d+d) of row-major [batch*len][ld] buffers; d % 8 == 0, d <= 64; S (keys) may differ from N.
 * lse: fp32 [B*H][N], base 2: log2 sum_j 2^(s_ij log2 e) (saved for the backward).  Backward: dq, dk, dv (no atomics); delta_ws fp32 [B*H*N].
 * ------------------------------------------------------------------------------------------- */
int sdmi_attn_fwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* out, int ldo,
                  float* lse, int B, int H, int N, int S, int d, sdmi_stream_t stream);
int sdmi_attn_bwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, const void* o, int ldo,
                  const void* dout, int lddo, const float* lse, float* delta_ws, void* dq, int lddq, void* dk,
                  int lddk, void* dv, int lddv, int B, int H, int N, int S, int d, sdmi_stream_t stream);
/* The same backward as ONE pass over the keys (P and dS computed once per score; dQ from a transposed dS image in
 * LDS): one key block (S <= 128) stores dQ directly, more key blocks sum fp32 dQ partials (ws, at least
 * sdmi_attn_bwd_workspace bytes) in a fixed key-block order -- deterministic, no float atomics. delta_ws as above. */
size_t sdmi_attn_bwd_workspace(int B, int H, int N, int S, int d);
int sdmi_attn_bwd_fused(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, const void* o, int ldo,
                        const void* dout, int lddo, const float* lse, float* delta_ws, void* ws, size_t ws_bytes,
                        void* dq, int lddq, void* dk, int lddk, void* dv, int lddv, int B, int H, int N, int S, int d,
                        sdmi_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * GroupNorm (+ fused SiLU) on NHWC bf16 x[b][p][c] = x[(b*P + p)*ld + c]; fp32 statistics.
 * Replaces nn.GroupNorm -> nn.SiLU (models/blocks.py:45-47, 64-66; unet_cond_base.py:179-180) and the
 * attention pre-norms on the (B, C, HW) view (blocks.py:124-126, 137-139).  ws: sdmi_chan_reduce_workspace
 * bytes (unused by sdmi_gn_stats).  Each reduction is one launch; batch sums (dgamma/dbeta, per-c sums) are
 * finished in-kernel by the last workgroup of each channel strip.
 * sdmi_gn_bwd: dx (+= addend if given), dgamma/dbeta (fp32, both or neither), table2_ws fp32 [B*C*4].
 * sdmi_chan_sum: per-(b,c) pixel sums (bf16, row stride ld_bc) and per-channel sums (fp32; c < c_store),
 * i.e. the bias and time-embedding-bias gradients of the convs at blocks.py:48-61, 102-107.
 * ------------------------------------------------------------------------------------------- */
size_t sdmi_chan_reduce_workspace(int B, int P, int C);
/* table: fp32 float4 [B][C] = {a = rstd*gamma, s = beta - mean*a, mean, rstd} (per (b, c); the group
 * statistics folded with the affine), produced by sdmi_gn_stats and consumed by apply / backward. */
int sdmi_gn_stats(const void* x, int ldx, int B, int P, int C, int G, float eps, const float* gamma, const float* beta,
                  float* ws, float* table, sdmi_stream_t stream);
/* stats + apply in one call (a single pass over x for small images); table as sdmi_gn_stats */
int sdmi_gn_fwd(const void* x, int ldx, void* y, int ldy, int B, int P, int C, int G, float eps, const float* gamma,
                const float* beta, int silu, float* ws, float* table, sdmi_stream_t stream);
int sdmi_gn_apply(const void* x, int ldx, void* y, int ldy, const float* table, int B, int P, int C, int silu,
                  sdmi_stream_t stream);
int sdmi_gn_bwd(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                const float* gamma, int B, int P, int C, int G, int silu, float* ws, float* table2_ws, float* dgamma,
                float* dbeta, const void* addend, int ldadd, sdmi_stream_t stream);
/* GroupNorm (+SiLU) backward whose reductions were produced by the data-gradient GEMM that wrote dy
 * (sdmi_gemm_desc::gn_part, rb rows per segment, part = float2 [B * P / rb][C]): one streaming launch per GroupNorm
 * (dx = a*dz + q*x + o + addend; dgamma / dbeta) instead of the single-pass kernel's load / reduce / apply phases.
 * ws: sdmi_chan_reduce_workspace. Same arithmetic as sdmi_gn_bwd up to the fp32 summation order of the partials. */
int sdmi_gn_bwd_part(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                     const float* gamma, int B, int P, int C, int G, int silu, const float* part, int rb, float* ws,
                     float* dgamma, float* dbeta, const void* addend, int ldadd, sdmi_stream_t stream);

/* The two GroupNorm backward forms with dgamma / dbeta deferred: rows [B][C][2] receives the per-(batch row, channel)
 * sums {sum dz, sum dz*xhat} and the launch has no batch tail; sdmi_gn_rows_sum then writes dbeta[c] = sum_b rows[b][c][0]
 * and dgamma[c] = sum_b rows[b][c][1] (in batch order; the fused forms' batch tail may group the rows differently, so
 * the two agree to fp32 summation order) -- e.g. on a side stream, off the data-gradient chain. */
int sdmi_gn_bwd_rows(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                     const float* gamma, int B, int P, int C, int G, int silu, float* ws, float* table2_ws, float* rows,
                     const void* addend, int ldadd, sdmi_stream_t stream);
int sdmi_gn_bwd_part_rows(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                          const float* gamma, int B, int P, int C, int G, int silu, const float* part, int rb, float* ws,
                          float* rows, const void* addend, int ldadd, sdmi_stream_t stream);
int sdmi_gn_rows_sum(const float* rows, int B, int C, float* dgamma, float* dbeta, sdmi_stream_t stream);
/* Up to SDMI_GN_ROWS_GROUP_MAX rows buffers summed in ONE launch (each job exactly as sdmi_gn_rows_sum, bitwise): the
 * deferred GroupNorm sums of one UNet block are issued together at its weight-gradient flush. */
#define SDMI_GN_ROWS_GROUP_MAX 16
typedef struct {
  const float* rows;
  float* dgamma;
  float* dbeta;
  int B, C;
} sdmi_gn_rows_job;
int sdmi_gn_rows_sum_grouped(const sdmi_gn_rows_job* jobs, int njobs, sdmi_stream_t stream);


int sdmi_chan_sum(const void* dy, int lddy, int B, int P, int C, float* ws, void* per_bc, int ld_bc, float* per_c,
                  float* per_c2, int c_store, sdmi_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Input / output staging, scheduler, loss, time embedding, elementwise.
 *  sdmi_prep_input   : unet_cond_base.py:131-140 -- x NCHW fp32 -> NHWC bf16 (cpad channels) with the
 *                      nearest-resized mask (F.interpolate default) through the 1x1 cond_conv_in
 *                      (no bias) in channels cx..cx+cmo-1; keep[b] (optional) = cond-drop multiplier
 *                      (utils/diffusion_utils.py:31-37) applied at gather time.
 *  sdmi_cond_wgrad   : gradient of cond_conv_in.weight.
 *  sdmi_prep_input_cmap / sdmi_cond_wgrad_cmap : the same with the mask given as a uint8 class map
 *                      (B,MH,MW) instead of the (B,cmi,MH,MW) fp32 one-hot that dataset/celeb_dataset.py:164-175
 *                      builds (clamp(0,cmi) -> one_hot(cmi+1) -> drop background); bit-identical results.
 *  sdmi_add_noise    : scheduler/linear_noise_scheduler.py:26-48 (bit-exact fp32 mul/mul/add).
 *  sdmi_mse          : nn.MSELoss (train_ddpm_cond_celebhq_multi_gpu.py:267,346) + its gradient times
 *                      the loss scale (gscale or *gscale_dev, GradScaler :269,362).
 *  sdmi_time_embedding: models/blocks.py:5-24 (t stride 0 broadcasts one timestep).
 * ------------------------------------------------------------------------------------------- */
int sdmi_prep_input(const float* x, int B, int cx, int H, int W, const float* mask, int cmi, int MH, int MW,
                    const float* wcond, int cmo, void* out, int cpad, const float* keep, sdmi_stream_t stream);
int sdmi_cond_wgrad(const void* dxin, int ld, int cx, int B, int H, int W, const float* mask, int cmi, int MH, int MW,
                    int cmo, float* dw, const float* keep, sdmi_stream_t stream);
int sdmi_prep_input_cmap(const float* x, int B, int cx, int H, int W, const unsigned char* cmap, int cmi, int MH,
                         int MW, const float* wcond, int cmo, void* out, int cpad, const float* keep,
                         sdmi_stream_t stream);
int sdmi_cond_wgrad_cmap(const void* dxin, int ld, int cx, int B, int H, int W, const unsigned char* cmap, int cmi,
                         int MH, int MW, int cmo, float* dw, const float* keep, sdmi_stream_t stream);
int sdmi_nhwc_to_nchw(const void* src, int src_f32, int ld, int B, int C, int HW, float* dst, sdmi_stream_t stream);
int sdmi_nchw_to_nhwc_bf16(const float* src, int B, int C, int HW, void* dst, int ld, sdmi_stream_t stream);
int sdmi_add_noise(const float* x0, const float* eps, const long long* t, const float* sqrt_abar,
                   const float* sqrt_one_minus_abar, int B, long long per_sample, float* out, sdmi_stream_t stream);
size_t sdmi_mse_workspace(void);
int sdmi_mse(const float* pred, int ld, const float* target, int B, int C, int HW, float gscale,
             const float* gscale_dev, void* grad, float* ws, float* loss, sdmi_stream_t stream);
int sdmi_time_embedding(const long long* t, int tstride, int B, int dim, void* out, int ld, float* out_f32,
                        sdmi_stream_t stream);
int sdmi_silu(const void* x, const void* dy, void* y, long long n, sdmi_stream_t stream);
/* fp32 ReLU (dy NULL) or its backward dx = dy * (x > 0) (the leaf path's nn.ReLU, transformer.py:72,80) */
int sdmi_relu(const float* x, const float* dy, float* y, long long n, sdmi_stream_t stream);
int sdmi_copy_slice(const void* src, int lds, void* dst, int ldd, long long P, int C, int accumulate,
                    sdmi_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * DiT row kernels (models/transformer.py:153-213, transformer_layer.py:80-106). Tokens are row-major bf16
 * [B*N][ld] (N tokens per sample, C = hidden size, C % 8 == 0, C <= 512, 16-B aligned rows). The adaLN
 * tables shift / scale / gate are bf16 [B][ld_mod] column slices of the one GEMM that evaluates every
 * layer's adaptive_norm_layer.
 *  sdmi_ln_mod_fwd : [xo = x + gate*v (gate NULL: ungated)] -> LayerNorm(no affine, eps) -> y = xhat*(1+scale)
 *                    + shift (shift = scale = NULL: plain LayerNorm); mean / rstd fp32 [rows] saved.
 *                    x_f32: the residual stream x / xo is fp32 (more precise than the reference's bf16
 *                    autocast stream; v, gate, shift, scale, y stay bf16).
 *  sdmi_ln_mod_bwd : dx = dres + LayerNorm'(dy*(1+scale)); partial dshift / dscale rows (fp32, one per
 *                    (sample, token chunk of sdmi_ln_chunk_rows(N)), row stride ws_ld); with gate: the gate
 *                    backward of the branch that produced x, dv = gate*dx and partial dgate = sum dx*v.
 *                    x_f32: x, dres and dx are fp32; dx16 (optional) receives a bf16 copy of dx.
 *  sdmi_mod_finalize: out[b][c] = bf16(sum over the chunk partial rows) -- fixed order, no atomics.
 *  sdmi_tokens_to_nchw / sdmi_nchw_to_tokens_bf16 : '(nh nw) (ph pw c)' token layout <-> NCHW fp32
 *                    (the reference's einops rearranges, transformer.py:209-212, patch_embed.py:88-89).
 *  sdmi_mse_patch  : nn.MSELoss with pred in token layout, target NCHW (p = 1: NHWC pred, as sdmi_mse).
 * ------------------------------------------------------------------------------------------- */
int sdmi_ln_chunk_rows(int N);
int sdmi_ln_mod_fwd(const void* x, int ldx, const void* v, int ldv, const void* gate, void* xo, int ldxo,
                    const void* shift, const void* scale, int ld_mod, void* y, int ldy, float* mean, float* rstd,
                    int rows, int C, int N, float eps, int x_f32, sdmi_stream_t stream);
int sdmi_ln_mod_bwd(const void* x, int ldx, const float* mean, const float* rstd, const void* dy, int lddy,
                    const void* scale, int ld_mod, const void* dres, int lddres, void* dx, int lddx, float* psh,
                    float* psc, int ws_ld, const void* gate, const void* v, int ldv, void* dv, int lddv, float* pg,
                    int rows, int C, int N, int x_f32, void* dx16, int ld16, sdmi_stream_t stream);
int sdmi_mod_finalize(const float* ws, int B, int chunks, int ws_ld, int W, void* out, int ldo, sdmi_stream_t stream);
int sdmi_tokens_to_nchw(const void* src, int src_f32, int ld, int B, int C, int H, int W, int p, float* dst,
                        sdmi_stream_t stream);
int sdmi_nchw_to_tokens_bf16(const float* src, int B, int C, int H, int W, int p, void* dst, int ld,
                             sdmi_stream_t stream);
int sdmi_mse_patch(const float* pred, int ld, const float* target, int B, int C, int H, int W, int p, float gscale,
                   const float* gscale_dev, void* grad, float* ws, float* loss, sdmi_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * VQVAE latent interface (models/vqvae.py:93-153).
 *  sdmi_vq_quantize : pre_quant_conv (1x1, fp32; w = NULL: identity) of the encoder output z (NHWC fp32 [P][ldz],
 *                     C <= 8 valid channels), nearest codebook row by torch.cdist's mm form sqrt(max(|x|^2 + |e|^2
 *                     - 2 x.e, 0)) with first-minimum argmin, straight-through output zq = x + (q - x) (NCHW fp32),
 *                     int64 indices (B*H*W), optional pre-quantisation latent xq (NCHW fp32) and the codebook /
 *                     commitment loss mean((q - x)^2). ws: sdmi_vq_workspace(B*HW) bytes.
 *  sdmi_pointwise_in: post_quant_conv (1x1, fp32) of an NCHW fp32 latent into NHWC bf16 [P][ld] (tail zeroed).
 * ------------------------------------------------------------------------------------------- */
/*  sdmi_vq_bwd      : training backward of the latent interface (train_vqvae_celebhq.py:405-430, recon + codebook
 *                     + commitment terms; LPIPS / GAN out of scope): from dzin (gradient of post_quant_conv's output,
 *                     NHWC bf16) -> post_quant_conv dW/db, the straight-through gradient of the pre-quantisation
 *                     latent plus commitment_beta * 2 (x - q) / n, pre_quant_conv dW/db and dz_enc (NHWC bf16
 *                     gradient of encoder_conv_out's output), and the codebook gradient codebook_weight * 2 (q - x) / n
 *                     scattered to the selected rows (deterministic, no atomics). ws: sdmi_vq_bwd_workspace() bytes.
 *                     dzq_add (nullable, NCHW fp32): an extra gradient of the quantised latent (the module's returned
 *                     z); loss_w (nullable, device {codebook, commitment}): multiplies the two host weights (the
 *                     autograd gradients of the two loss outputs, read on the device). */
size_t sdmi_vq_workspace(long long pixels);
size_t sdmi_vq_bwd_workspace(void);
int sdmi_vq_bwd(const void* dzin, int ld_dzin, const float* zq, const float* w_post, const float* xq, const long long* idx,
                const float* codebook, int K, const float* z_enc, int ldz, const float* w_pre, int B, int HW, int C,
                float commitment_beta, float codebook_weight, void* dz_enc, int ld_out, float* ws, float* dw_post,
                float* db_post, float* dw_pre, float* db_pre, float* demb, const float* dzq_add, const float* loss_w,
                sdmi_stream_t stream);
int sdmi_vq_quantize(const float* z, int ldz, const float* w, const float* b, const float* codebook, int K, int B,
                     int HW, int C, float* zq, long long* idx, float* xq, float* ws, float* loss, sdmi_stream_t stream);
int sdmi_pointwise_in(const float* z, int B, int C, int HW, const float* w, const float* b, int cout, void* out,
                      int ld, sdmi_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Sampling steps (scheduler/linear_noise_scheduler.py), fp32 elementwise, bit-exact to the reference given the
 * same noise (correctly rounded fp32 div / sqrt, no FMA contraction).
 *  sdmi_ddpm_prev : LinearNoiseScheduler.sample_prev_timestep (:50-78); timestep read from device memory
 *                   (t_dev), z unused at t == 0, x0 (clamped prediction) optional; decrement_t: t_dev -= 1 after
 *                   the step (capturable sampling loop, no host round trip per step).
 *  sdmi_ddim_prev : DDIMSampler.sample_one_step (:164-182) for alpha_t = abar[t], alpha_prev = abar[t_prev].
 *  sdmi_ddim_prev_dev: the same DDIM step with the pair read on the device: i = *idx, alpha_t = abar[ts[i]],
 *                   alpha_prev = abar[tp[i]] (DDIMSampler.forward's time_steps / time_steps_prev, :231-242); advance:
 *                   afterwards *idx -= 1 and *t_dev = ts[*idx] (the model's timestep) -- a capturable DDIM loop.
 *  sdmi_affine_step: DDPMSampler.sample_one_step (:111-124): out = (c1 x - c2 eps) + sqrt(var) z (z NULL: + 0).
 * ------------------------------------------------------------------------------------------- */
int sdmi_ddpm_prev(const float* xt, const float* eps, const float* z, long long n, long long* t_dev, const float* betas,
                   const float* alphas, const float* abar, const float* s1m, float* prev, float* x0, int decrement_t,
                   sdmi_stream_t stream);
int sdmi_ddim_prev(const float* xt, const float* eps, const float* noise, long long n, float alpha_t, float alpha_prev,
                   float eta, float* out, sdmi_stream_t stream);
int sdmi_ddim_prev_dev(const float* xt, const float* eps, const float* noise, long long n, const long long* ts,
                       const long long* tp, long long* idx, long long* t_dev, const float* abar, float eta, float* out,
                       int advance, sdmi_stream_t stream);
int sdmi_affine_step(const float* x, const float* eps, const float* z, long long n, float c1, float c2, float var,
                     float* out, sdmi_stream_t stream);

/* Device standard-normal noise (captured sampling loops): out[i] ~ N(0,1), Philox4x32-10(seed, i / 4, *offset_dev)
 * + Box-Muller; advance != 0 increments *offset_dev after the draw (the next replay draws fresh noise). Replaces
 * the host torch.randn of LinearNoiseScheduler.sample_prev_timestep (scheduler/linear_noise_scheduler.py:72). */
int sdmi_randn(float* out, long long n, unsigned long long seed, unsigned long long* offset_dev, int advance,
               sdmi_stream_t stream);

/* Every random draw of one training step in ONE launch (train_ddpm_cond_celebhq_multi_gpu.py:299-330 /
 * diffusion_utils.py:21-37 draw them with torch.randn / randint / rand + where): noise[n] ~ N(0,1), t[b] uniform in
 * [0, T), txt[b] = (u < p_text) ? empty : text[b] (rows of row_elems fp32; txt == NULL skips the text drop),
 * keep[b] = (u > p_keep) ? 1 : 0 (keep == NULL skips it). Philox4x32-10 keyed by seed at draw offset `offset`
 * (the caller advances it every step). */
int sdmi_step_draw(float* noise, long long n, long long* t, int B, int T, const float* text, const float* empty,
                   float* txt, long long row_elems, float p_text, float* keep, float p_keep, unsigned long long seed,
                   unsigned long long offset, sdmi_stream_t stream);

/* bf16 GEMM-layout weight packing (the per-step fp32 -> bf16 cast that autocast performs,
 * train_ddpm_cond_celebhq_multi_gpu.py:281-283, fused with the layout change):
 * dst[o][a][b][i] = bf16(src[o*so + i*si + (kh_off + kh_mul*a)*skh + (kw_off + kw_mul*b)*skw]), 0 for i >= I. */
typedef struct sdmi_pack_desc {
  const float* src;
  void* dst;
  long long so, si, skh, skw;
  int O, I, Ipad, KH, KW, kh_off, kh_mul, kw_off, kw_mul;
  int dst_ld; /* row stride of dst in elements (0 = KH*KW*Ipad): packs into a column slice of a wider matrix */
} sdmi_pack_desc;
/* Work split: one workgroup packs max(1, sdmi_pack_chunk() / (KH*KW*Ipad)) consecutive destination rows;
 * bmap_dev holds one int2 (descriptor index, first row) per workgroup. KH*KW*(Ipad+8) <= 16384. */
int sdmi_pack_chunk(void);
int sdmi_pack_weights(const sdmi_pack_desc* descs_dev, const void* bmap_dev, int nblocks, sdmi_stream_t stream);

/* Transposed weight layouts derived from already-packed bf16 ones (the dgrad layout of a conv is its forward
 * layout transposed per tap with the taps flipped; sub-pixel phase layouts select 4 of 16 taps):
 * dst[i*dst_ld + t*dst_tap + o] = src[o*src_ld + smap[t]*src_tap + i] for o < O, i < I, t < taps.
 * Work split: one workgroup per 64 (o) x 64 (i) tile of one tap; bmap_dev holds one int4 (descriptor, first i,
 * first o, tap) per workgroup. src / dst 16-byte aligned rows; I and O multiples of 8 within the padded views. */
typedef struct sdmi_tpack_desc {
  const void* src;
  void* dst;
  int O, I, taps;
  int src_ld, src_tap, dst_ld, dst_tap;
  signed char smap[16];
} sdmi_tpack_desc;
int sdmi_pack_transpose(const sdmi_tpack_desc* descs_dev, const void* bmap_dev, int nblocks, sdmi_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Optimizer step over flat fp32 buffers (train_ddpm_cond_celebhq_multi_gpu.py:362-378):
 * GradScaler.unscale_ + clip_grad_norm_(max_norm) + non-finite skip + scaler.update (state on device:
 * float[8] = {norm, coef, scale, growth, step, skip, loss, dp_loss_flag}), then Adam (torch defaults) + EMA.
 * grad_div = data-parallel world size (gradients arrive summed). growth_interval <= 0: no loss scaler (the
 * plain fp32 VQVAE trainer, train_vqvae_celebhq.py:466): the scale in state[2] is left as is (keep it 1).
 * skip_if_loss_nonfinite: 0 ignore the loss; 1 a non-finite state[6] skips the step WITHOUT scaler.update()
 * (:348-352); 2 the same decided by state[7] != 0 (data parallel: the all-reduced sum of every rank's flag, so every
 * replica skips together). A non-finite gradient norm skips the step and backs the scale off (:366-371).
 * sdmi_loss_flag: mode 0 *dst = !isfinite(*src) (a rank's flag, e.g. into the all-reduced gradient tail);
 * mode 1 *dst = (*src != 0) (the summed flag into state[7]).
 * ------------------------------------------------------------------------------------------- */
size_t sdmi_optim_workspace(void);
int sdmi_clip_unscale(const float* grads, long long n, float max_norm, float* state, float* ws, int growth_interval,
                      int skip_if_loss_nonfinite, float grad_div, sdmi_stream_t stream);
/* any n: ws holds sdmi_optim_workspace_for(n) bytes (one fp32 partial per 128 Ki-gradient block; -3 if ws_bytes is
 * smaller). sdmi_clip_unscale is this call with ws_bytes = sdmi_optim_workspace() (n up to ~268 M). */
size_t sdmi_optim_workspace_for(long long n);
int sdmi_clip_unscale_ws(const float* grads, long long n, float max_norm, float* state, float* ws, size_t ws_bytes,
                         int growth_interval, int skip_if_loss_nonfinite, float grad_div, sdmi_stream_t stream);
int sdmi_loss_flag(const float* src, float* dst, int mode, sdmi_stream_t stream);
/* sdmi_clip_finalize reduces the first n block partials (double accumulation, index order) and applies the clip /
 * skip / scaler update above. */
int sdmi_clip_finalize(const float* partial, int n, float max_norm, float* state, int growth_interval,
                       int skip_if_loss_nonfinite, float grad_div, sdmi_stream_t stream);
/* ema_alpha: the fp32 value of (1 - ema_decay) as the caller computes it (the reference passes alpha = 1 - 0.9999
 * from Python doubles, :376-378) */
int sdmi_adam_ema(float* params, const float* grads, float* m, float* v, float* ema, long long n, const float* state,
                  float lr, float b1, float b2, float eps, float ema_decay, float ema_alpha, sdmi_stream_t stream);
/* The same step also writing params_bf16[i] = bf16(params[i]) (round to nearest even; untouched on a skipped step):
 * the autocast weight cast folded into the optimizer pass. The trainer keeps a bf16 image of the flat parameter
 * buffer this way, and every weight whose GEMM layout is its flat layout is read from it directly (no repack). */
int sdmi_adam_ema_bf16(float* params, const float* grads, float* m, float* v, float* ema, long long n,
                       const float* state, float lr, float b1, float b2, float eps, float ema_decay, float ema_alpha,
                       void* params_bf16, sdmi_stream_t stream);
/* dst[i] = bf16(src[i]) over n elements (src 16-B, dst 8-B aligned): the initial bf16 parameter image */
int sdmi_cast_bf16(const float* src, void* dst, long long n, sdmi_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Leaf-path glue (sdmi/leaf.py; fp32 torch layouts): what the reference computes with aten between its layers.
 * sdmi_resize_nearest: F.interpolate(mode='nearest') of BC planes IHxIW -> OHxOW (unet_cond_base.py:132,
 *   transformer.py:169): src = min(floor(dst * (float)in / out), in - 1).
 * sdmi_chan_copy: NCHW channel slab dst[b][dst_c0 + c][p] = src[b][src_c0 + c][p] (torch.cat along dim 1 and the
 *   split of its gradient, unet_cond_base.py:136, transformer.py:170).
 * sdmi_modulate_fwd / _bwd: y = r + x * (alpha + s[b][c]) + t[b][c] over (B, N, C) rows (s, t row stride ls; r, t
 *   optional): the DiT's adaLN modulation (alpha 1, transformer_layer.py:86-88, :97-99, transformer.py:205-207) and
 *   gated residual (alpha 0, r = the stream, transformer_layer.py:89, :100); backward dx = dy * (alpha + s),
 *   ds = sum_n dy * x, dt = sum_n dy (each output optional; dr = dy is the caller's).
 * sdmi_attn_map: the attention weights an MHA returns for need_weights=True (multihead_attention.py:107-118):
 *   softmax(q_h k_h^T * scaling) per head from fp32 rows q [B*N][ldq], k [B*S][ldk] (head h at columns h*d..),
 *   averaged over heads into out (B, N, S), or per head into (B, H, N, S); S <= 4096.
 * ------------------------------------------------------------------------------------------- */
int sdmi_resize_nearest(const float* in, int BC, int IH, int IW, float* out, int OH, int OW, sdmi_stream_t stream);
int sdmi_chan_copy(const float* src, int src_c, int src_c0, float* dst, int dst_c, int dst_c0, int B, int C,
                   long long P, sdmi_stream_t stream);
int sdmi_modulate_fwd(const float* x, const float* r, const float* s, const float* t, int ls, float alpha, float* y,
                      int B, int N, int C, sdmi_stream_t stream);
int sdmi_modulate_bwd(const float* x, const float* dy, const float* s, int ls, float alpha, float* dx, float* ds,
                      float* dt, int B, int N, int C, sdmi_stream_t stream);
int sdmi_attn_map(const float* q, int ldq, const float* k, int ldk, int B, int H, int N, int S, int d, float scaling,
                  int average, float* out, sdmi_stream_t stream);


/* ---------------------------------------------------------------------------------------------
 * Launch plans (host side of a training / sampling step, no reference counterpart: the reference issues every
 * aten op from Python per step, train_ddpm_cond_celebhq_multi_gpu.py:299-378). Between sdmi_plan_begin and
 * sdmi_plan_end every kernel launch of this library executes AND is recorded (kernel, grid, LDS bytes, stream,
 * a copy of its arguments); the caller notes the event record / stream wait edges it issues itself and numbered
 * callouts (work outside the library: RCCL collectives, torch copies). sdmi_plan_replay re-issues the recorded
 * ops from op index `start` until the next callout (*callout = its id, *next = the op after it) or the end
 * (*callout = -1). Pointers, grids and streams are replayed verbatim: the caller keeps every recorded buffer,
 * stream and event alive and refills inputs in place. One recorder per process (not re-entrant).
 * ------------------------------------------------------------------------------------------- */
int sdmi_plan_begin(void);
int sdmi_plan_end(void** plan);
int sdmi_plan_recording(void);
int sdmi_plan_note_event(void* event, sdmi_stream_t stream);
int sdmi_plan_note_wait(sdmi_stream_t stream, void* event);
int sdmi_plan_note_callout(int id);
int sdmi_plan_info(const void* plan, int* ops, int* launches);
int sdmi_plan_replay(void* plan, int start, int* callout, int* next);
int sdmi_plan_destroy(void* plan);
/* profiling: op kind (0 launch, 1 event record, 2 stream wait, 3 callout, 4 all-reduce), kernel name, grid[3], block,
 * LDS bytes;
 * and the average device time of launch op i re-issued alone (iters times after warm untimed issues). */
int sdmi_plan_op_info(const void* plan, int i, int* kind, const char** name, int* grid, int* block, int* shmem);
int sdmi_plan_op_stream(const void* plan, int i, sdmi_stream_t* stream); /* the stream op i was recorded on */
int sdmi_plan_time_op(void* plan, int i, int warm, int iters, float* us);

/* ---------------------------------------------------------------------------------------------
 * Gradient all-reduce through RCCL, issued by the library on the caller's stream (replaces the DDP bucket hook's
 * NCCL all-reduce, train_ddpm_cond_celebhq_multi_gpu.py:257-263 -> torch DDP, and this package's earlier
 * torch.distributed callouts). sdmi_comm_load binds the RCCL shared library the process already uses (path: torch's
 * bundled librccl.so, or any RCCL) by dlopen -- libsdmi.so does not link RCCL. Rank 0 makes the unique id
 * (NCCL_UNIQUE_ID_BYTES = 128 bytes), the caller broadcasts it, every rank calls sdmi_comm_init (collective, blocking)
 * with the device current. sdmi_allreduce: in-place sum of count elements (dtype 0 fp32, 1 bf16) on `stream`;
 * while a plan records it is recorded and replayed natively (no callout). Status: 0 ok, 1000 + ncclResult_t on an
 * RCCL error, negative on bad arguments / RCCL not loaded.
 * ------------------------------------------------------------------------------------------- */
int sdmi_comm_load(const char* rccl_path);
int sdmi_comm_unique_id(unsigned char* id);
int sdmi_comm_init(const unsigned char* id, int nranks, int rank, void** comm);
int sdmi_allreduce(void* comm, void* buf, long long count, int dtype, sdmi_stream_t stream);
int sdmi_comm_destroy(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* SDMI_H */
