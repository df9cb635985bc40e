// Elementwise / reduction glue of the leaf-module path (sdmi/leaf.py) that the reference writes as aten ops between
// its layers, so a model whose leaves were swapped (and therefore runs leaf by leaf) still computes on HIP:
//   * nearest interpolation of the mask condition (F.interpolate default mode, unet_cond_base.py:132,
//     transformer.py:169) and channel concatenation / its split (torch.cat, unet_cond_base.py:136);
//   * the DiT adaLN modulation  y = r + x * (alpha + s[b, c]) + t[b, c]  and its backward -- LayerNorm output
//     modulation (transformer_layer.py:86-88, :97-99; transformer.py:205-207, alpha = 1, s = scale, t = shift) and the
//     gated residual (transformer_layer.py:89, :100, r = stream, alpha = 0, s = gate);
//   * the attention map that nn.MultiheadAttention-style modules return for need_weights=True
//     (multihead_attention.py:107-118): softmax(q k^T * scaling) per head, averaged over heads or not.
// All fp32 (the leaf path's tensors), row-major / NCHW exactly as torch lays them out; reductions are per-workgroup
// in a fixed order (deterministic, no atomics).
#include "common.h"
#include "../../include/sdmi.h"

namespace {
constexpr int NT = 256;

long long grid_of(long long work) {
  long long g = (work + NT - 1) / NT;
  return g < 1 ? 1 : g > 65535 * 8 ? 65535 * 8 : g;
}

// out[b][c][y][x] = in[b][c][floor(y * IH / OH)][floor(x * IW / OW)]  (aten's nearest: src = floor(dst * scale),
// scale = in / out as float, clamped to in - 1)
__global__ void resize_nearest_kernel(const float* in, int BC, int IH, int IW, float* out, int OH, int OW) {
  const long long total = (long long)BC * OH * OW;
  const float sy = (float)IH / (float)OH, sx = (float)IW / (float)OW;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int x = (int)(i % OW);
    const long long r = i / OW;
    const int y = (int)(r % OH);
    const long long bc = r / OH;
    int iy = (int)floorf((float)y * sy), ix = (int)floorf((float)x * sx);
    iy = iy < IH - 1 ? iy : IH - 1;
    ix = ix < IW - 1 ? ix : IW - 1;
    out[i] = in[(bc * IH + iy) * IW + ix];
  }
}

// dst[b][dc0 + c][p] = src[b][sc0 + c][p] for c < C, p < P (NCHW channel-slab copy: concatenation and its split)
__global__ void chan_copy_kernel(const float* src, int sC, int sc0, float* dst, int dC, int dc0, int B, int C,
                                 long long P) {
  const long long per = (long long)C * P, total = (long long)B * per;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long b = i / per, r = i - b * per;
    dst[(b * dC + dc0) * P + r] = src[(b * sC + sc0) * P + r];
  }
}

// y[b][n][c] = (r ? r[b][n][c] : 0) + x[b][n][c] * (alpha + s[b*ls + c]) + (t ? t[b*ls + c] : 0)
__global__ void modulate_fwd_kernel(const float* x, const float* r, const float* s, const float* t, int ls, float alpha,
                                    float* y, int B, int N, int C) {
  const long long total = (long long)B * N * C;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const int b = (int)(i / ((long long)N * C));
    float v = x[i] * (alpha + s[(long long)b * ls + c]);
    if (t) v += t[(long long)b * ls + c];
    if (r) v += r[i];
    y[i] = v;
  }
}

// backward of modulate_fwd: dx = dy * (alpha + s); ds[b][c] = sum_n dy * x; dt[b][c] = sum_n dy. One workgroup per
// (b, 64-column strip): 4 row lanes of 64 columns, partial sums merged in LDS in a fixed order.
__global__ void modulate_bwd_kernel(const float* x, const float* dy, const float* s, int ls, float alpha, float* dx,
                                    float* ds, float* dt, int N, int C) {
  __shared__ float rs[2][4][64];
  const int b = blockIdx.y, c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  float as = 0.f, at = 0.f;
  if (c < C) {
    const float m = alpha + s[(long long)b * ls + c];
    for (int n = rl; n < N; n += 4) {
      const long long i = ((long long)b * N + n) * C + c;
      const float g = dy[i];
      if (dx) dx[i] = g * m;
      as = fmaf(g, x[i], as);
      at += g;
    }
  }
  rs[0][rl][threadIdx.x & 63] = as;
  rs[1][rl][threadIdx.x & 63] = at;
  __syncthreads();
  if (rl == 0 && c < C) {
    const int l = threadIdx.x & 63;
    const float S = ((rs[0][0][l] + rs[0][1][l]) + rs[0][2][l]) + rs[0][3][l];
    const float T = ((rs[1][0][l] + rs[1][1][l]) + rs[1][2][l]) + rs[1][3][l];
    if (ds) ds[(long long)b * ls + c] = S;
    if (dt) dt[(long long)b * ls + c] = T;
  }
}

// Attention map: one workgroup per (b, query row n). For every head: scores over the S keys (fp32 dot products over
// d), the row max and sum of exp (workgroup reductions in a fixed order), p = exp(score - max) / sum; averaged over
// heads into out[b][n][s] (avg) or written per head into out[b][h][n][s].
constexpr int AMAP_SMAX = 4096;
__global__ void attn_map_kernel(const float* q, int ldq, const float* k, int ldk, int B, int H, int N, int S, int d,
                                float scaling, int avg, float* out) {
  __shared__ float red[NT / 64];
  __shared__ float bcast;
  const int n = blockIdx.x, b = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int PER = AMAP_SMAX / NT;  // keys per thread
  float acc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) acc[j] = 0.f;
  const float* qrow = q + ((long long)b * N + n) * ldq;
  for (int h = 0; h < H; ++h) {
    float sc[PER];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int s = threadIdx.x + j * NT;
      sc[j] = -INFINITY;
      if (s < S) {
        const float* krow = k + ((long long)b * S + s) * ldk + h * d;
        float dot = 0.f;
        for (int e = 0; e < d; ++e) dot = fmaf(qrow[h * d + e], krow[e], dot);
        sc[j] = dot * scaling;
        mx = fmaxf(mx, sc[j]);
      }
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    if (threadIdx.x == 0) bcast = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    const float M = bcast;
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      sc[j] = threadIdx.x + j * NT < S ? expf(sc[j] - M) : 0.f;
      sum += sc[j];
    }
    sum = wave_sum(sum);
    __syncthreads();
    if (lane == 0) red[wave] = sum;
    __syncthreads();
    if (threadIdx.x == 0) bcast = ((red[0] + red[1]) + red[2]) + red[3];
    __syncthreads();
    const float inv = 1.f / bcast;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int s = threadIdx.x + j * NT;
      if (s >= S) continue;
      if (avg) acc[j] += sc[j] * inv;
      else out[(((long long)b * H + h) * N + n) * S + s] = sc[j] * inv;
    }
    __syncthreads();
  }
  if (avg) {
    const float invH = 1.f / (float)H;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int s = threadIdx.x + j * NT;
      if (s < S) out[((long long)b * N + n) * S + s] = acc[j] * invH;
    }
  }
}
}  // namespace

extern "C" int sdmi_resize_nearest(const float* in, int BC, int IH, int IW, float* out, int OH, int OW,
                                   sdmi_stream_t stream) {
  if (!in || !out || BC <= 0 || IH <= 0 || IW <= 0 || OH <= 0 || OW <= 0) return -1;
  sdmi_rt::launch(resize_nearest_kernel, dim3((unsigned)grid_of((long long)BC * OH * OW)), dim3(NT), 0,
                  (hipStream_t)stream, in, BC, IH, IW, out, OH, OW);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_chan_copy(const float* src, int src_c, int src_c0, float* dst, int dst_c, int dst_c0, int B, int C,
                              long long P, sdmi_stream_t stream) {
  if (!src || !dst || B <= 0 || C <= 0 || P <= 0 || src_c0 < 0 || dst_c0 < 0 || src_c0 + C > src_c ||
      dst_c0 + C > dst_c)
    return -1;
  sdmi_rt::launch(chan_copy_kernel, dim3((unsigned)grid_of((long long)B * C * P)), dim3(NT), 0, (hipStream_t)stream,
                  src, src_c, src_c0, dst, dst_c, dst_c0, B, C, P);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_modulate_fwd(const float* x, const float* r, const float* s, const float* t, int ls, float alpha,
                                 float* y, int B, int N, int C, sdmi_stream_t stream) {
  if (!x || !s || !y || B <= 0 || N <= 0 || C <= 0 || ls < C) return -1;
  sdmi_rt::launch(modulate_fwd_kernel, dim3((unsigned)grid_of((long long)B * N * C)), dim3(NT), 0, (hipStream_t)stream,
                  x, r, s, t, ls, alpha, y, B, N, C);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_modulate_bwd(const float* x, const float* dy, const float* s, int ls, float alpha, float* dx,
                                 float* ds, float* dt, int B, int N, int C, sdmi_stream_t stream) {
  if (!x || !dy || !s || B <= 0 || N <= 0 || C <= 0 || ls < C) return -1;
  sdmi_rt::launch(modulate_bwd_kernel, dim3((unsigned)((C + 63) / 64), (unsigned)B), dim3(NT), 0, (hipStream_t)stream,
                  x, dy, s, ls, alpha, dx, ds, dt, N, C);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_attn_map(const float* q, int ldq, const float* k, int ldk, int B, int H, int N, int S, int d,
                             float scaling, int average, float* out, sdmi_stream_t stream) {
  if (!q || !k || !out || B <= 0 || H <= 0 || N <= 0 || S <= 0 || S > AMAP_SMAX || d <= 0 || ldq < H * d ||
      ldk < H * d || N > 65535 * 32)
    return -1;
  sdmi_rt::launch(attn_map_kernel, dim3((unsigned)N, (unsigned)B), dim3(NT), 0, (hipStream_t)stream, q, ldq, k, ldk, B,
                  H, N, S, d, scaling, average, out);
  SDMI_CHECK_LAUNCH();
  return 0;
}
