// VQVAE latent-interface kernels for gfx950 (reference models/vqvae.py).
//
//  vq_quantize : pre_quant_conv (1x1, fp32) of the encoder output, nearest-codebook search and the
//                straight-through output of VQVAE.quantize (vqvae.py:93-126). Distances follow torch.cdist's
//                matrix-product form (|x|^2 + |e|^2 - 2 x.e, clamped at 0, square-rooted) and the FIRST
//                minimum wins, like torch.argmin. Codebook (K x C fp32) rows are read with wave-uniform
//                addresses (scalar loads, one row per half-wave); a 1024-thread workgroup owns 32 pixels and its
//                16 waves scan 16 disjoint codebook slices (each half-wave one half of its slice), merged with a
//                lowest-index tie-break; the codes' |e|^2 come from an LDS table built once per workgroup.
//                Outputs: z_q = x + (q - x) in NCHW fp32 (the STE forward value), int64 indices, and the
//                (codebook == commitment) loss mean((q - x)^2).
//  pointwise_in: post_quant_conv (1x1, fp32) of an NCHW fp32 latent straight into the NHWC bf16 operand of
//                decoder_conv_in (vqvae.py:141-144), zero-padding the channel tail.
//  vq_bwd      : the training backward of the latent interface (train_vqvae_celebhq.py:405-430 without the
//                LPIPS / GAN terms): post_quant_conv backward, the straight-through estimator (dL/dx += dL/dz_q),
//                the commitment term beta * mean((sg[q] - x)^2), pre_quant_conv backward into the bf16 NHWC
//                gradient of encoder_conv_out; the 1x1-conv weight / bias gradients as per-block partials summed in
//                a fixed order (deterministic). vq_codebook_grad: the codebook term w * mean((q - sg[x])^2) into the
//                embedding rows (index_select backward): 64 codes per workgroup, the pixels streamed through LDS and
//                split over 8 waves, per-wave partial sums in pixel order added in wave order (deterministic).
#include "common.h"
#include "../../include/sdmi.h"
#include <algorithm>

namespace {

constexpr int VQ_NT = 1024, VQ_WAVES = VQ_NT / 64, MAXC = 8;
constexpr int VQ_EN_MAX = 16384;  // codes whose |e|^2 table fits the quantize kernel's LDS (64 KiB)

struct VqArgs {
  const float* z; int ldz;  // encoder_conv_out output, NHWC fp32 [P][ldz], channels < C valid
  const float* w; const float* b;  // pre_quant_conv weight (C, C, 1, 1) and bias (C), or null (identity)
  const float* codebook; int K;
  int B, HW, C;
  float* zq;  // NCHW fp32 (B, C, H, W)
  long long* idx;  // (B*HW)
  float* xq;  // optional NCHW fp32 pre-quantisation latent (after pre_quant_conv)
  float* partial;  // per-workgroup sum of (q - x)^2
};

// |e_k|^2 of one code, in the order the distance loop has always summed it (c ascending)
__device__ __forceinline__ float code_norm(const float* e, int C) {
  float en = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c < C) {
      const float ec = e[c];
      en += ec * ec;
    }
  }
  return en;
}

// Nearest code per pixel (torch.cdist mm form + argmin, first minimum). A workgroup takes 32 pixels; wave w scans
// code slice w of 16, its lanes 0-31 the first half of the slice and lanes 32-63 the second half for the same 32
// pixels, and the halves merge with a strict < (the first minimum, as one ascending scan would keep). 32 pixels per
// workgroup instead of 64 puts the 8192-pixel latent of a B = 8, 256^2 batch on 256 workgroups (was 128: half the
// CUs idle); EN: the codes' |e|^2 precomputed once per workgroup into LDS instead of per (pixel, code).
template <bool EN>
__global__ __launch_bounds__(VQ_NT) void vq_quantize_kernel(const VqArgs a) {
  extern __shared__ float sen[];  // EN: |e_k|^2 of every code
  __shared__ float sd[VQ_WAVES][32];
  __shared__ int si[VQ_WAVES][32];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, pl = lane & 31;
  const long long P = (long long)a.B * a.HW;
  const long long pix = (long long)blockIdx.x * 32 + pl;
  const bool on = pix < P;
  const int C = a.C;
  if constexpr (EN) {
    for (int k = threadIdx.x; k < a.K; k += VQ_NT) sen[k] = code_norm(a.codebook + (long long)k * C, C);
    __syncthreads();
  }
  float x[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) x[c] = 0.f;
  if (on) {
    float zin[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) zin[c] = c < C ? a.z[pix * a.ldz + c] : 0.f;
    if (a.w) {
#pragma unroll
      for (int co = 0; co < MAXC; ++co) {
        if (co >= C) break;
        float s = a.b ? a.b[co] : 0.f;
#pragma unroll
        for (int ci = 0; ci < MAXC; ++ci)
          if (ci < C) s = fmaf(a.w[co * C + ci], zin[ci], s);
        x[co] = s;
      }
    } else {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) x[c] = zin[c];
    }
  }
  // |x|^2 and -2x, as cdist's mm form builds them
  float xn = 0.f, m2[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c < C) xn += x[c] * x[c];
    m2[c] = -2.f * x[c];
  }
  const int per = (a.K + VQ_WAVES - 1) / VQ_WAVES;
  const int w0 = wave * per, w1 = min(a.K, w0 + per);
  const int wm = min(w1, w0 + (per + 1) / 2);
  // step j: lanes 0-31 code w0 + j, lanes 32-63 code wm + j -- both loads wave-uniform (scalar), selected per half
  const int n0 = wm - w0;
  float best = INFINITY;
  int bi = half ? wm : w0;
#pragma unroll 4
  for (int j = 0; j < n0; ++j) {
    const int ka = w0 + j, kb = wm + j;
    const int kbl = min(kb, a.K - 1);  // (in bounds; the update below is masked when kb is past the slice)
    const float* ea = a.codebook + (long long)ka * C;
    const float* eb = a.codebook + (long long)kbl * C;
    float en = 0.f, dot = 0.f;
    if constexpr (EN) {
      en = sen[half ? kbl : ka];
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
        if (c < C) dot = fmaf(m2[c], half ? eb[c] : ea[c], dot);
    } else {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        if (c < C) {
          const float ec = half ? eb[c] : ea[c];
          en += ec * ec;
          dot = fmaf(m2[c], ec, dot);
        }
      }
    }
    const float d = sqrtf(fmaxf(dot + xn + en, 0.f));
    if ((!half || kb < w1) && d < best) {
      best = d;
      bi = half ? kb : ka;
    }
  }
  {  // the second half's codes all follow the first half's: take them only when strictly nearer
    const float d2 = __shfl_xor(best, 32);
    const int i2 = __shfl_xor(bi, 32);
    if (!half && d2 < best) {
      best = d2;
      bi = i2;
    }
  }
  if (!half) {
    sd[wave][pl] = best;
    si[wave][pl] = bi;
  }
  __syncthreads();
  if (wave == 0) {
    float bd = INFINITY;
    int bk = 0;
    float loss = 0.f;
    if (!half) {
      bd = sd[0][pl];
      bk = si[0][pl];
      for (int w = 1; w < VQ_WAVES; ++w) {  // slices are in ascending k order: strict < keeps the first minimum
        const float d = sd[w][pl];
        if (d < bd) {
          bd = d;
          bk = si[w][pl];
        }
      }
    }
    if (on && !half) {
      const float* q = a.codebook + (long long)bk * C;
      const long long b = pix / a.HW, p = pix - b * a.HW;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        if (c < C) {
          const float diff = q[c] - x[c];
          loss += diff * diff;
          const long long o = (b * C + c) * a.HW + p;
          a.zq[o] = x[c] + diff;  // straight-through forward value x + (q - x) (vqvae.py:121)
          if (a.xq) a.xq[o] = x[c];
        }
      }
      a.idx[pix] = bk;
    }
    loss = wave_sum(loss);
    if (lane == 0) a.partial[blockIdx.x] = loss;
  }
}

__global__ void vq_loss_kernel(const float* partial, int n, float scale, float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = (red[0] + red[1] + red[2] + red[3]) * scale;
}

__global__ void pointwise_in_kernel(const float* z, int B, int C, int HW, const float* w, const float* b, int cout,
                                    bf16_t* out, int ld) {
  const long long P = (long long)B * HW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < P * ld; i += (long long)gridDim.x * blockDim.x) {
    const long long pix = i / ld;
    const int co = (int)(i - pix * ld);
    float v = 0.f;
    if (co < cout) {
      const long long bb = pix / HW, p = pix - bb * HW;
      v = b ? b[co] : 0.f;
      for (int ci = 0; ci < C; ++ci) v = fmaf(w[co * C + ci], z[(bb * C + ci) * HW + p], v);
    }
    out[i] = f2bf(v);
  }
}

constexpr int VQB_NT = 256;
constexpr int VQB_PART = 2 * MAXC * MAXC + 2 * MAXC;  // dW_post, dW_pre, db_post, db_pre partials per block

struct VqBwdArgs {
  const bf16_t* dzin; int ld_dzin;      // gradient of decoder_conv_in's input, NHWC bf16 [P][ld] (post_quant output)
  const float* zq;                      // quantised latent (NCHW fp32): post_quant_conv input
  const float* w_post;                  // post_quant_conv weight (C, C)
  const float* xq;                      // pre-quantisation latent (NCHW fp32)
  const long long* idx;                 // code per pixel
  const float* codebook;                // (K, C)
  const float* z_enc; int ldz;          // encoder_conv_out output, NHWC fp32 [P][ldz]: pre_quant_conv input
  const float* w_pre;                   // pre_quant_conv weight (C, C)
  int B, HW, C;
  float g_commit;                       // commitment_beta * 2 / (P * C)
  const float* dzq_add;                 // optional extra gradient of the quantised latent (NCHW fp32), or null
  const float* loss_w;                  // optional device loss weights {codebook, commitment} (scale the host ones)
  bf16_t* dz_enc; int ld_out;           // gradient of encoder_conv_out's output, NHWC bf16 [P][ld_out]
  float* partial;                       // [blocks][VQB_PART]
};

__global__ __launch_bounds__(VQB_NT) void vq_bwd_kernel(const VqBwdArgs a) {
  __shared__ float red[VQB_NT / 64][VQB_PART];
  const int C = a.C;
  const long long P = (long long)a.B * a.HW;
  const float g_commit = a.loss_w ? a.g_commit * a.loss_w[1] : a.g_commit;
  float acc[VQB_PART];
#pragma unroll
  for (int i = 0; i < VQB_PART; ++i) acc[i] = 0.f;
  for (long long pix = (long long)blockIdx.x * VQB_NT + threadIdx.x; pix < P; pix += (long long)gridDim.x * VQB_NT) {
    const long long bb = pix / a.HW, p = pix - bb * a.HW;
    float dzin[MAXC], zq[MAXC], x[MAXC], q[MAXC], ze[MAXC], dzq[MAXC], dx[MAXC];
    const long long k = a.idx[pix];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const bool on = c < C;
      dzin[c] = on ? bf2f(a.dzin[pix * a.ld_dzin + c]) : 0.f;
      zq[c] = on ? a.zq[(bb * C + c) * a.HW + p] : 0.f;
      x[c] = on ? a.xq[(bb * C + c) * a.HW + p] : 0.f;
      q[c] = on ? a.codebook[k * C + c] : 0.f;
      ze[c] = on ? a.z_enc[pix * a.ldz + c] : 0.f;
    }
    // post_quant_conv backward: dzq = W_post^T dzin (the straight-through gradient of x), dW_post, db_post
#pragma unroll
    for (int ci = 0; ci < MAXC; ++ci) {
      float s = 0.f;
#pragma unroll
      for (int co = 0; co < MAXC; ++co)
        if (co < C && ci < C) s = fmaf(a.w_post[co * C + ci], dzin[co], s);
      if (a.dzq_add && ci < C) s += a.dzq_add[(bb * C + ci) * a.HW + p];
      dzq[ci] = s;
    }
#pragma unroll
    for (int co = 0; co < MAXC; ++co) {
#pragma unroll
      for (int ci = 0; ci < MAXC; ++ci) acc[co * MAXC + ci] = fmaf(dzin[co], zq[ci], acc[co * MAXC + ci]);
      acc[2 * MAXC * MAXC + co] += dzin[co];
    }
    // STE + commitment: dL/dx = dzq + beta * 2 (x - q) / n
#pragma unroll
    for (int c = 0; c < MAXC; ++c) dx[c] = fmaf(g_commit, x[c] - q[c], dzq[c]);
    // pre_quant_conv backward
#pragma unroll
    for (int co = 0; co < MAXC; ++co) {
#pragma unroll
      for (int ci = 0; ci < MAXC; ++ci)
        acc[MAXC * MAXC + co * MAXC + ci] = fmaf(dx[co], ze[ci], acc[MAXC * MAXC + co * MAXC + ci]);
      acc[2 * MAXC * MAXC + MAXC + co] += dx[co];
    }
    for (int ci = 0; ci < a.ld_out; ++ci) {
      float s = 0.f;
      if (ci < C)
        for (int co = 0; co < C; ++co) s = fmaf(a.w_pre[co * C + ci], dx[co], s);
      a.dz_enc[pix * a.ld_out + ci] = f2bf(s);
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < VQB_PART; ++i) {
    const float v = wave_sum(acc[i]);
    if (lane == 0) red[wave][i] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < VQB_PART; i += VQB_NT) {
    float v = 0.f;
    for (int w = 0; w < VQB_NT / 64; ++w) v += red[w][i];
    a.partial[(long long)blockIdx.x * VQB_PART + i] = v;
  }
}

// sum the per-block partials in block order and scatter them to the four gradient tensors (C x C, C x C, C, C)
__global__ void vq_bwd_finish_kernel(const float* partial, int blocks, int C, float* dw_post, float* db_post,
                                     float* dw_pre, float* db_pre) {
  for (int i = threadIdx.x; i < VQB_PART; i += blockDim.x) {
    float v = 0.f;
    for (int b = 0; b < blocks; ++b) v += partial[(long long)b * VQB_PART + i];
    if (i < MAXC * MAXC) {
      const int co = i / MAXC, ci = i % MAXC;
      if (co < C && ci < C && dw_post) dw_post[co * C + ci] = v;
    } else if (i < 2 * MAXC * MAXC) {
      const int j = i - MAXC * MAXC, co = j / MAXC, ci = j % MAXC;
      if (co < C && ci < C && dw_pre) dw_pre[co * C + ci] = v;
    } else if (i < 2 * MAXC * MAXC + MAXC) {
      const int co = i - 2 * MAXC * MAXC;
      if (co < C && db_post) db_post[co] = v;
    } else {
      const int co = i - 2 * MAXC * MAXC - MAXC;
      if (co < C && db_pre) db_pre[co] = v;
    }
  }
}

// demb[k] = g_codebook * sum over pixels p with idx[p] == k of (q_k - x_p). A workgroup owns 64 codes (one per
// lane) and streams the index list and the pre-quantisation latent through LDS, 1024 pixels per round; each of its 8
// waves scans one eighth of every round (four indices per LDS load, a wave-uniform address: broadcast) and
// accumulates its matches branch-free from LDS, in pixel order; the waves' partial sums are then added in wave order
// (a fixed order: deterministic). At random init most pixels pick a few codes: the first form (one thread per code
// scanning every pixel, x_p from global memory per match) serialised those codes' threads on global round trips and
// took 1.3-1.7 ms of the 256^2 VQVAE training step. Padding entries are -1 and never match a code.
constexpr int CB_WAVES = 8;
__global__ __launch_bounds__(64 * CB_WAVES) void vq_codebook_grad_kernel(const long long* idx, const float* xq,
                                                                        const float* codebook, int K, int B, int HW,
                                                                        int C, float g_codebook, const float* loss_w,
                                                                        float* demb) {
  __shared__ int4 sidx4[256];
  __shared__ float4 sxa[1024], sxb[1024];  // x_p channels 0-3 and 4-7 of the round's pixels
  __shared__ float red[CB_WAVES][MAXC + 1][64];
  int* sidx = (int*)sidx4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  const long long P = (long long)B * HW;
  float acc[MAXC];
  int cnt = 0;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) acc[c] = 0.f;
  for (long long p0 = 0; p0 < P; p0 += 1024) {
    __syncthreads();
    for (int j = threadIdx.x; j < 1024; j += 64 * CB_WAVES) {
      const long long pix = p0 + j;
      int v = -1;
      float xv[MAXC];
#pragma unroll
      for (int c = 0; c < MAXC; ++c) xv[c] = 0.f;
      if (pix < P) {
        v = (int)idx[pix];
        const long long bb = pix / HW, p = pix - bb * HW;
#pragma unroll
        for (int c = 0; c < MAXC; ++c)
          if (c < C) xv[c] = xq[(bb * C + c) * HW + p];
      }
      sidx[j] = v;
      sxa[j] = make_float4(xv[0], xv[1], xv[2], xv[3]);
      sxb[j] = make_float4(xv[4], xv[5], xv[6], xv[7]);
    }
    __syncthreads();
#pragma unroll 2
    for (int j4 = wave * 32; j4 < wave * 32 + 32; ++j4) {
      const int4 v = sidx4[j4];
      if (v.x != k && v.y != k && v.z != k && v.w != k) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool m = (e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w))) == k;
        const float4 xa = sxa[4 * j4 + e];
        cnt += m;
        acc[0] -= m ? xa.x : 0.f;
        acc[1] -= m ? xa.y : 0.f;
        acc[2] -= m ? xa.z : 0.f;
        acc[3] -= m ? xa.w : 0.f;
        if (C > 4) {
          const float4 xb = sxb[4 * j4 + e];
          acc[4] -= m ? xb.x : 0.f;
          acc[5] -= m ? xb.y : 0.f;
          acc[6] -= m ? xb.z : 0.f;
          acc[7] -= m ? xb.w : 0.f;
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) red[wave][c][lane] = acc[c];
  red[wave][MAXC][lane] = (float)cnt;  // exact: counts <= 2^24
  __syncthreads();
  if (wave != 0 || k >= K) return;
  float tc = 0.f;
  for (int c = 0; c < MAXC; ++c) acc[c] = 0.f;
  for (int w = 0; w < CB_WAVES; ++w) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) acc[c] += red[w][c][lane];
    tc += red[w][MAXC][lane];
  }
  if (loss_w) g_codebook *= loss_w[0];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
    if (c < C) demb[(long long)k * C + c] = g_codebook * fmaf(tc, codebook[(long long)k * C + c], acc[c]);
}

}  // namespace

// one loss partial per quantize workgroup (32 pixels)
extern "C" size_t sdmi_vq_workspace(long long pixels) { return (size_t)((pixels + 31) / 32) * sizeof(float); }

extern "C" int sdmi_vq_quantize(const float* z, int ldz, const float* w, const float* b, const float* codebook, int K,
                                int B, int HW, int C, float* zq, long long* idx, float* xq, float* ws, float* loss,
                                sdmi_stream_t stream) {
  if (!z || !codebook || !zq || !idx || !ws || !loss || K <= 0 || B <= 0 || HW <= 0 || C <= 0 || C > MAXC || ldz < C)
    return -1;
  VqArgs a;
  a.z = z; a.ldz = ldz; a.w = w; a.b = b; a.codebook = codebook; a.K = K; a.B = B; a.HW = HW; a.C = C;
  a.zq = zq; a.idx = idx; a.xq = xq; a.partial = ws;
  const long long P = (long long)B * HW;
  const int blocks = (int)((P + 31) / 32);
  if (K <= VQ_EN_MAX)
    sdmi_rt::launch(vq_quantize_kernel<true>, dim3(blocks), dim3(VQ_NT), (size_t)K * sizeof(float), (hipStream_t)stream, a);
  else
    sdmi_rt::launch(vq_quantize_kernel<false>, dim3(blocks), dim3(VQ_NT), 0, (hipStream_t)stream, a);
  SDMI_CHECK_LAUNCH();
  sdmi_rt::launch(vq_loss_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, ws, blocks, 1.0f / (float)(P * C),
                     loss);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_pointwise_in(const float* z, int B, int C, int HW, const float* w, const float* b, int cout,
                                 void* out, int ld, sdmi_stream_t stream) {
  if (!z || !out || B <= 0 || C <= 0 || HW <= 0 || cout <= 0 || ld < cout) return -1;
  const long long total = (long long)B * HW * ld;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
  sdmi_rt::launch(pointwise_in_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, z, B, C, HW, w, b, cout,
                     (bf16_t*)out, ld);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" size_t sdmi_vq_bwd_workspace(void) { return (size_t)512 * VQB_PART * sizeof(float); }

extern "C" int sdmi_vq_bwd(const void* dzin, int ld_dzin, const float* zq, const float* w_post, const float* xq,
                           const long long* idx, const float* codebook, int K, const float* z_enc, int ldz,
                           const float* w_pre, int B, int HW, int C, float commitment_beta, float codebook_weight,
                           void* dz_enc, int ld_out, float* ws, float* dw_post, float* db_post, float* dw_pre,
                           float* db_pre, float* demb, const float* dzq_add, const float* loss_w,
                           sdmi_stream_t stream) {
  if (!dzin || !zq || !w_post || !xq || !idx || !codebook || !z_enc || !w_pre || !dz_enc || !ws || !demb ||
      C <= 0 || C > MAXC || ld_out < C || ldz < C || ld_dzin < C || B <= 0 || HW <= 0 || K <= 0)
    return -1;
  const long long P = (long long)B * HW;
  const float n = (float)(P * C);
  VqBwdArgs a;
  a.dzin = (const bf16_t*)dzin; a.ld_dzin = ld_dzin; a.zq = zq; a.w_post = w_post; a.xq = xq; a.idx = idx;
  a.codebook = codebook; a.z_enc = z_enc; a.ldz = ldz; a.w_pre = w_pre; a.B = B; a.HW = HW; a.C = C;
  a.g_commit = commitment_beta * 2.0f / n;
  a.dzq_add = dzq_add; a.loss_w = loss_w;
  a.dz_enc = (bf16_t*)dz_enc; a.ld_out = ld_out; a.partial = ws;
  const int blocks = (int)std::min<long long>(512, (P + VQB_NT - 1) / VQB_NT);
  sdmi_rt::launch(vq_bwd_kernel, dim3(blocks), dim3(VQB_NT), 0, (hipStream_t)stream, a);
  SDMI_CHECK_LAUNCH();
  sdmi_rt::launch(vq_bwd_finish_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, (const float*)ws, blocks, C,
                  dw_post, db_post, dw_pre, db_pre);
  SDMI_CHECK_LAUNCH();
  sdmi_rt::launch(vq_codebook_grad_kernel, dim3((K + 63) / 64), dim3(64 * CB_WAVES), 0, (hipStream_t)stream, idx, xq,
                  codebook, K, B, HW, C, codebook_weight * 2.0f / n, loss_w, demb);
  SDMI_CHECK_LAUNCH();
  return 0;
}
