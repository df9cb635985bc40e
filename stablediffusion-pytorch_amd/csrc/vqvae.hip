// VQVAE latent-interface kernels for gfx950 (reference models/vqvae.py).
//
//  vq_quantize : pre_quant_conv (1x1, fp32) of the encoder output, nearest-codebook search and the
//                straight-through output of VQVAE.quantize (vqvae.py:93-126). Distances follow torch.cdist's
//                matrix-product form (|x|^2 + |e|^2 - 2 x.e, clamped at 0, square-rooted) and the FIRST
//                minimum wins, like torch.argmin. Codebook (K x C fp32) rows are read with wave-uniform
//                addresses (broadcast loads); a 1024-thread workgroup owns 64 pixels (one per lane) and its
//                16 waves scan 16 disjoint codebook slices, merged in LDS with lowest-index tie-break.
//                Outputs: z_q = x + (q - x) in NCHW fp32 (the STE forward value), int64 indices, and the
//                (codebook == commitment) loss mean((q - x)^2).
//  pointwise_in: post_quant_conv (1x1, fp32) of an NCHW fp32 latent straight into the NHWC bf16 operand of
//                decoder_conv_in (vqvae.py:141-144), zero-padding the channel tail.
#include "common.h"
#include "../../include/sdmi.h"
#include <algorithm>

namespace {

constexpr int VQ_NT = 1024, VQ_WAVES = VQ_NT / 64, MAXC = 8;

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

__global__ __launch_bounds__(VQ_NT) void vq_quantize_kernel(const VqArgs a) {
  __shared__ float sd[VQ_WAVES][64];
  __shared__ int si[VQ_WAVES][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long P = (long long)a.B * a.HW;
  const long long pix = (long long)blockIdx.x * 64 + lane;
  const bool on = pix < P;
  const int C = a.C;
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
  const int k0 = wave * per, k1 = min(a.K, k0 + per);
  float best = INFINITY;
  int bi = k0;
#pragma unroll 1
  for (int k = k0; k < k1; ++k) {
    const float* e = a.codebook + (long long)k * C;  // wave-uniform address
    float en = 0.f, dot = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < C) {
        const float ec = e[c];
        en += ec * ec;
        dot = fmaf(m2[c], ec, dot);
      }
    }
    const float d = sqrtf(fmaxf(dot + xn + en, 0.f));
    if (d < best) {
      best = d;
      bi = k;
    }
  }
  sd[wave][lane] = best;
  si[wave][lane] = bi;
  __syncthreads();
  if (wave == 0) {
    float bd = sd[0][lane];
    int bk = si[0][lane];
    for (int w = 1; w < VQ_WAVES; ++w) {  // slices are in ascending k order: strict < keeps the first minimum
      const float d = sd[w][lane];
      if (d < bd) {
        bd = d;
        bk = si[w][lane];
      }
    }
    float loss = 0.f;
    if (on) {
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

}  // namespace

extern "C" size_t sdmi_vq_workspace(long long pixels) { return (size_t)((pixels + 63) / 64) * sizeof(float); }

extern "C" int sdmi_vq_quantize(const float* z, int ldz, const float* w, const float* b, const float* codebook, int K,
                                int B, int HW, int C, float* zq, long long* idx, float* xq, float* ws, float* loss,
                                sdmi_stream_t stream) {
  if (!z || !codebook || !zq || !idx || !ws || !loss || K <= 0 || B <= 0 || HW <= 0 || C <= 0 || C > MAXC || ldz < C)
    return -1;
  VqArgs a;
  a.z = z; a.ldz = ldz; a.w = w; a.b = b; a.codebook = codebook; a.K = K; a.B = B; a.HW = HW; a.C = C;
  a.zq = zq; a.idx = idx; a.xq = xq; a.partial = ws;
  const long long P = (long long)B * HW;
  const int blocks = (int)((P + 63) / 64);
  sdmi_rt::launch(vq_quantize_kernel, dim3(blocks), dim3(VQ_NT), 0, (hipStream_t)stream, a);
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
