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
  int oh_log2, ow_log2; /* GEMM pixel grid (power-of-two) used to decompose a pixel index  */
  int sy, sx, oy0, ox0; /* iy = oy*sy + ty + oy0, ix = ox*sx + tx + ox0 (zero outside)      */
} sdmi_conv_geom;

typedef struct sdmi_gemm_desc {
  int m, n, k;
  int a_mode, b_mode;
  const void* a; int lda; /* bf16 */
  const void* b; int ldb; /* bf16 */
  sdmi_conv_geom geom;    /* used by SDMI_A_CONV / SDMI_B_KN_CONV */
  /* epilogue: v = alpha*acc + bias[n] + rowbias[(m >> rb_shift)*rb_ld + n] + resid[orow*ldr + n];
   *           v = act(v); C[orow*ldc + ocol] = v   (orow = row remap of m, ocol = col permute of n) */
  void* c; int ldc; int c_f32;
  const float* bias;          /* fp32 [n] or NULL      */
  const void* rowbias;        /* bf16 or NULL           */
  int rb_ld, rb_shift;
  const void* resid; int ldr; /* bf16 or NULL           */
  float alpha;
  int act;                    /* 0 none, 1 SiLU         */
  /* row remap (stride-2 sub-pixel phases of a transposed conv): m -> (b, oy, ox) on a
   * (2^r_gh_log2 x 2^r_gw_log2) grid, orow = (b*r_oh + oy*r_sy + r_oy)*r_ow + ox*r_sx + r_ox */
  int remap, r_gh_log2, r_gw_log2, r_oh, r_ow, r_sy, r_sx, r_oy, r_ox;
  /* column permute (weight-gradient layouts): n = tap*p_cin + c  ->  ocol = c*p_taps + tap, stored only
   * for c < p_cvalid (0 = all): gradients of zero-padded input channels are dropped */
  int perm, p_cin, p_taps, p_cvalid;
  /* store limits (0 = m / n): rows >= m_store and columns >= n_store are computed but not stored,
   * and the bias is read only for stored columns (zero-padded output channels) */
  int m_store, n_store;
} sdmi_gemm_desc;

/* Split-K plan: how many K slices the launcher will use and the fp32 workspace bytes it needs. */
int sdmi_gemm_plan(const sdmi_gemm_desc* d, int* splits, size_t* workspace_bytes);
int sdmi_gemm(const sdmi_gemm_desc* d, void* workspace, size_t workspace_bytes, sdmi_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SDMI_H */
