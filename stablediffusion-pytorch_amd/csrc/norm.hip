// GroupNorm (+ fused SiLU) forward/backward and per-(batch, channel) pixel reductions on NHWC bf16.
//
// Replaces nn.GroupNorm(32, C) -> nn.SiLU() (models/blocks.py:45-47, 64-66 and the Mid/Up copies),
// the attention pre-norms on the (B, C, HW) view (blocks.py:124-126, 137-139: same statistics as
// 4-D) and unet_cond_base.py:179-180. Statistics are fp32 (partials) / fp64 (final merge), eps 1e-5.
//
// All kernels see an activation as x[b][p][c] = x[(b*P + p)*ld + c], P = H*W pixels.
//  1. sdmi_chan_reduce  : per (b, c) partial sums over a pixel slice (grid = B x splits):
//        mode 0: (sum x, sum x^2)                                   -> GN statistics
//        mode 1: (sum dz, sum dz*xhat), dz = dy [* silu'(z)]          -> GN backward
//        mode 2: (sum dy, 0)                                         -> bias / time-embedding grads
//  2. finalize kernels turn partials into mean/rstd, GN backward coefficients, dgamma/dbeta, bias grads.
//  3. sdmi_gn_apply / sdmi_gn_bwd_apply : vectorised elementwise passes (8 channels per lane).
#include "common.h"
#include "../../include/sdmi.h"

namespace {

constexpr int NT = 256;

struct RedArgs {
  const bf16_t* x; int ldx;   // GN input
  const bf16_t* dy; int ldy;  // upstream grad (modes 1, 2)
  const float4* tab;          // mode 1: per-(b,c) {a = rstd*gamma, s = beta - mean*a, mean, rstd}
  int B, P, C, G, silu, mode, splits;
  float* part;  // [B][splits][C][2]
};

__global__ __launch_bounds__(NT) void chan_reduce_kernel(RedArgs a) {
  const int b = blockIdx.x, sp = blockIdx.y;
  const int C8 = a.C >> 3;
  const int rows = NT / C8;  // pixel rows processed per iteration
  const int t = threadIdx.x;
  const int col = t % C8, r = t / C8;
  const bool active = r < rows;
  const int p_per = (a.P + a.splits - 1) / a.splits;
  const int p0 = sp * p_per, p1 = min(a.P, p0 + p_per);
  const int c0 = col * 8;
  const int Cg = a.C / a.G;

  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  float4 tb[8];
  if (a.mode == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) tb[e] = a.tab[(long long)b * a.C + c0 + e];
  }
  (void)Cg;
  if (active) {
    for (int p = p0 + r; p < p1; p += rows) {
      long long pix = (long long)b * a.P + p;
      float xv[8], gv[8];
      if (a.mode == 0) {
        unpack8(*(const uint4*)(a.x + pix * a.ldx + c0), xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) { s1[e] += xv[e]; s2[e] += xv[e] * xv[e]; }
      } else if (a.mode == 1) {
        unpack8(*(const uint4*)(a.x + pix * a.ldx + c0), xv);
        unpack8(*(const uint4*)(a.dy + pix * a.ldy + c0), gv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float xh = (xv[e] - tb[e].z) * tb[e].w;
          float dz = gv[e];
          if (a.silu) dz *= silu_grad_f(fmaf(xv[e], tb[e].x, tb[e].y));
          s1[e] += dz;
          s2[e] += dz * xh;
        }
      } else {
        unpack8(*(const uint4*)(a.dy + pix * a.ldy + c0), gv);
#pragma unroll
        for (int e = 0; e < 8; ++e) s1[e] += gv[e];
      }
    }
  }
  // reduce across the `rows` threads sharing a column
  __shared__ float red[NT][17];
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[t][e] = s1[e]; red[t][8 + e] = s2[e]; }
  __syncthreads();
  // thread j < C (channel) sums over rows
  for (int ch = t; ch < a.C; ch += NT) {
    int cc = ch >> 3, e = ch & 7;
    float u = 0.f, v = 0.f;
    for (int rr = 0; rr < rows; ++rr) {
      u += red[rr * C8 + cc][e];
      v += red[rr * C8 + cc][8 + e];
    }
    float* o = a.part + (((long long)b * a.splits + sp) * a.C + ch) * 2;
    o[0] = u;
    o[1] = v;
  }
}

// ---- finalize kernels: partials [B][splits][C][2] -> per-(b,c) / per-(b,g) / per-c results ----

// column sums over all (b, split) rows for 64 channels [c0, c0+64): 256 threads = 64 channels x 4 row groups
__device__ __forceinline__ void colsum64(const float* part, int rows, int C, int c0, float& u, float& v, bool& own) {
  __shared__ float red[4][64][2];
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int c = c0 + cx;
  float a = 0.f, b = 0.f;
  if (c < C) {
    int r = ry;
    for (; r + 28 < rows; r += 32) {  // 8 independent loads in flight per lane
      float2 v2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v2[j] = *(const float2*)(part + ((long long)(r + 4 * j) * C + c) * 2);
#pragma unroll
      for (int j = 0; j < 8; ++j) { a += v2[j].x; b += v2[j].y; }
    }
    for (; r < rows; r += 4) {
      const float2 v2 = *(const float2*)(part + ((long long)r * C + c) * 2);
      a += v2.x;
      b += v2.y;
    }
  }
  red[ry][cx][0] = a;
  red[ry][cx][1] = b;
  __syncthreads();
  own = ry == 0 && c < C;
  u = red[0][cx][0] + red[1][cx][0] + red[2][cx][0] + red[3][cx][0];
  v = red[0][cx][1] + red[1][cx][1] + red[2][cx][1] + red[3][cx][1];
}

// per-channel totals of one batch row b over the splits, into LDS (C <= 2048)
__device__ __forceinline__ void batch_totals(const float* part, int b, int splits, int C, float2* tot) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, d = 0.f;
    for (int sp = 0; sp < splits; ++sp) {
      const float2 v2 = *(const float2*)(part + (((long long)b * splits + sp) * C + c) * 2);
      a += v2.x;
      d += v2.y;
    }
    tot[c] = make_float2(a, d);
  }
  __syncthreads();
}

// mean/rstd per (b, g): one block per b
__global__ __launch_bounds__(256) void gn_stats_finalize_kernel(const float* part, int B, int splits, int C, int G,
                                                                int P, float eps, const float* gamma,
                                                                const float* beta, float4* tab) {
  __shared__ float2 tot[2048];
  __shared__ float2 grp[2048];
  const int b = blockIdx.x;
  batch_totals(part, b, splits, C, tot);
  const int Cg = C / G;
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    double s1 = 0, s2 = 0;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      s1 += tot[c].x;
      s2 += tot[c].y;
    }
    double n = (double)P * Cg;
    double mu = s1 / n;
    double var = s2 / n - mu * mu;
    if (var < 0) var = 0;
    grp[g] = make_float2((float)mu, (float)(1.0 / sqrt(var + (double)eps)));
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float2 mr = grp[c / Cg];
    float a = mr.y * gamma[c];
    tab[(long long)b * C + c] = make_float4(a, beta[c] - mr.x * a, mr.x, mr.y);
  }
}

// GN backward: blocks [0, B): coef[b][g] = (sum_c gamma_c S1[b,c], sum_c gamma_c S2[b,c]);
// blocks [B, B + ceil(C/64)): dbeta[c] = sum_b S1, dgamma[c] = sum_b S2.
// dx = rstd*(dz*gamma - A/n - xhat*Bc/n) = a*dz + q*x + o with q = -rstd^2 Bc/n, o = rstd^2 mean Bc/n - rstd A/n
__global__ __launch_bounds__(256) void gn_bwd_finalize_kernel(const float* part, int B, int splits, int C, int G,
                                                              int P, const float* gamma, const float4* tab,
                                                              float4* tab2, float* dgamma, float* dbeta) {
  if ((int)blockIdx.x < B) {
    __shared__ float2 tot[2048];
    __shared__ float2 grp[2048];
    const int b = blockIdx.x;
    batch_totals(part, b, splits, C, tot);
    const int Cg = C / G;
    const float inv_n = 1.0f / ((float)P * Cg);
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
      float A = 0.f, Bc = 0.f;
      for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
        A += gamma[c] * tot[c].x;
        Bc += gamma[c] * tot[c].y;
      }
      float4 t = tab[(long long)b * C + g * Cg];
      float r = t.w, mu = t.z;
      grp[g] = make_float2(-r * r * Bc * inv_n, r * r * mu * Bc * inv_n - r * A * inv_n);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float4 t = tab[(long long)b * C + c];
      float2 qo = grp[c / Cg];
      tab2[(long long)b * C + c] = make_float4(t.x, t.y, qo.x, qo.y);
    }
    return;
  }
  float u, v;
  bool own;
  const int c0 = ((int)blockIdx.x - B) * 64;
  colsum64(part, B * splits, C, c0, u, v, own);
  if (own && dgamma) {
    dbeta[c0 + (threadIdx.x & 63)] = u;
    dgamma[c0 + (threadIdx.x & 63)] = v;
  }
}

// per-(b,c) sums (mode 2): blocks [0, nbc) write per_bc[b*ld + c] (bf16); blocks [nbc, nbc + ceil(C/64)) write
// per_c[c] = per_c2[c] = sum_b for c < c_store (fp32)
__global__ __launch_bounds__(256) void chan_sum_finalize_kernel(const float* part, int B, int splits, int C,
                                                                bf16_t* per_bc, int ld, float* per_c, float* per_c2,
                                                                int c_store, int nbc) {
  if ((int)blockIdx.x < nbc) {
    int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx < B * C) {
      int b = idx / C, c = idx - b * C;
      float u = 0.f;
      for (int sp = 0; sp < splits; ++sp) u += part[(((long long)b * splits + sp) * C + c) * 2];
      per_bc[(long long)b * ld + c] = f2bf(u);
    }
    return;
  }
  float u, v;
  bool own;
  const int c0 = ((int)blockIdx.x - nbc) * 64;
  colsum64(part, B * splits, C, c0, u, v, own);
  const int c = c0 + (threadIdx.x & 63);
  if (own && c < c_store) {
    if (per_c) per_c[c] = u;
    if (per_c2) per_c2[c] = u;
  }
}

struct ApplyArgs {
  const bf16_t* x; int ldx;
  bf16_t* y; int ldy;
  const bf16_t* dy; int lddy;
  bf16_t* dx; int lddx;
  const float4* tab;  // apply: {a, s, -, -}; backward: {a, s, q, o}
  const bf16_t* add; int ldadd;
  int B, P, C, silu;
};

// y = act(x*a + s)
__global__ __launch_bounds__(NT) void gn_apply_kernel(ApplyArgs a) {
  const int C8 = a.C >> 3;
  long long total = (long long)a.B * a.P * C8;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    long long pix = i / C8;
    int c0 = (int)(i - pix * C8) * 8;
    int b = (int)(pix / a.P);
    const float4* t = a.tab + (long long)b * a.C + c0;
    float xv[8], yv[8];
    unpack8(*(const uint4*)(a.x + pix * a.ldx + c0), xv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float4 te = t[e];
      float z = fmaf(xv[e], te.x, te.y);
      yv[e] = a.silu ? silu_f(z) : z;
    }
    *(uint4*)(a.y + pix * a.ldy + c0) = pack8(yv);
  }
}

// dx = a*dz + q*x + o (+ addend), dz = dy [* silu'(x*a + s)]
__global__ __launch_bounds__(NT) void gn_bwd_apply_kernel(ApplyArgs a) {
  const int C8 = a.C >> 3;
  long long total = (long long)a.B * a.P * C8;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    long long pix = i / C8;
    int c0 = (int)(i - pix * C8) * 8;
    int b = (int)(pix / a.P);
    const float4* t = a.tab + (long long)b * a.C + c0;
    float xv[8], gv[8], ov[8], av[8];
    unpack8(*(const uint4*)(a.x + pix * a.ldx + c0), xv);
    unpack8(*(const uint4*)(a.dy + pix * a.lddy + c0), gv);
    if (a.add) unpack8(*(const uint4*)(a.add + pix * a.ldadd + c0), av);
    else for (int e = 0; e < 8; ++e) av[e] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float4 te = t[e];
      float dz = gv[e];
      if (a.silu) dz *= silu_grad_f(fmaf(xv[e], te.x, te.y));
      ov[e] = av[e] + fmaf(te.x, dz, fmaf(te.z, xv[e], te.w));
    }
    *(uint4*)(a.dx + pix * a.lddx + c0) = pack8(ov);
  }
}

int pick_splits(int B, int P) {
  int s = 1;
  while (B * s < 1024 && P / (s * 2) >= 16) s *= 2;
  return s;
}

int grid_for(long long work) {
  long long g = (work + NT - 1) / NT;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" size_t sdmi_chan_reduce_workspace(int B, int P, int C) {
  return (size_t)B * pick_splits(B, P) * C * 2 * sizeof(float);
}

// stats -> per-(b,c) table {a = rstd*gamma, s = beta - mean*a, mean, rstd} (fp32 float4 [B][C])
extern "C" int sdmi_gn_stats(const void* x, int ldx, int B, int P, int C, int G, float eps, const float* gamma,
                             const float* beta, float* ws, float* table, sdmi_stream_t stream) {
  if (C % 8 || C > 8 * NT || G <= 0 || C % G) return -1;
  hipStream_t s = (hipStream_t)stream;
  RedArgs a = {};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.B = B; a.P = P; a.C = C; a.G = G; a.mode = 0;
  a.splits = pick_splits(B, P); a.part = ws;
  hipLaunchKernelGGL(chan_reduce_kernel, dim3(B, a.splits), dim3(NT), 0, s, a);
  SDMI_CHECK_LAUNCH();
  hipLaunchKernelGGL(gn_stats_finalize_kernel, dim3(B), dim3(256), 0, s, ws, B, a.splits, C, G, P, eps, gamma, beta,
                     (float4*)table);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_gn_apply(const void* x, int ldx, void* y, int ldy, const float* table, int B, int P, int C,
                             int silu, sdmi_stream_t stream) {
  if (C % 8) return -1;
  ApplyArgs a = {};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.y = (bf16_t*)y; a.ldy = ldy;
  a.tab = (const float4*)table; a.B = B; a.P = P; a.C = C; a.silu = silu;
  hipLaunchKernelGGL(gn_apply_kernel, dim3(grid_for((long long)B * P * C / 8)), dim3(NT), 0, (hipStream_t)stream, a);
  SDMI_CHECK_LAUNCH();
  return 0;
}

// table: forward table from sdmi_gn_stats; table2_ws: float4 [B][C] scratch
extern "C" int sdmi_gn_bwd(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                           const float* gamma, int B, int P, int C, int G, int silu, float* ws, float* table2_ws,
                           float* dgamma, float* dbeta, const void* addend, int ldadd, sdmi_stream_t stream) {
  if (C % 8 || C > 8 * NT || C % G) return -1;
  hipStream_t s = (hipStream_t)stream;
  RedArgs r = {};
  r.x = (const bf16_t*)x; r.ldx = ldx; r.dy = (const bf16_t*)dy; r.ldy = lddy; r.tab = (const float4*)table;
  r.B = B; r.P = P; r.C = C; r.G = G; r.silu = silu; r.mode = 1; r.splits = pick_splits(B, P); r.part = ws;
  hipLaunchKernelGGL(chan_reduce_kernel, dim3(B, r.splits), dim3(NT), 0, s, r);
  SDMI_CHECK_LAUNCH();
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(B + (dgamma ? (C + 63) / 64 : 0)), dim3(256), 0, s, ws, B, r.splits,
                     C, G, P, gamma, (const float4*)table, (float4*)table2_ws, dgamma, dbeta);
  SDMI_CHECK_LAUNCH();
  ApplyArgs a = {};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.dy = (const bf16_t*)dy; a.lddy = lddy; a.dx = (bf16_t*)dx; a.lddx = lddx;
  a.tab = (const float4*)table2_ws; a.add = (const bf16_t*)addend; a.ldadd = ldadd;
  a.B = B; a.P = P; a.C = C; a.silu = silu;
  hipLaunchKernelGGL(gn_bwd_apply_kernel, dim3(grid_for((long long)B * P * C / 8)), dim3(NT), 0, s, a);
  SDMI_CHECK_LAUNCH();
  return 0;
}

// per-(b, c) and per-c sums of dy over pixels (bias and time-embedding-bias gradients)
extern "C" int sdmi_chan_sum(const void* dy, int lddy, int B, int P, int C, float* ws, void* per_bc, int ld_bc,
                             float* per_c, float* per_c2, int c_store, sdmi_stream_t stream) {
  if (c_store <= 0 || c_store > C) c_store = C;
  if (C % 8 || C > 8 * NT) return -1;
  hipStream_t s = (hipStream_t)stream;
  RedArgs r = {};
  r.dy = (const bf16_t*)dy; r.ldy = lddy; r.B = B; r.P = P; r.C = C; r.G = 1; r.mode = 2;
  r.splits = pick_splits(B, P); r.part = ws;
  hipLaunchKernelGGL(chan_reduce_kernel, dim3(B, r.splits), dim3(NT), 0, s, r);
  SDMI_CHECK_LAUNCH();
  int nbc = per_bc ? (B * C + 255) / 256 : 0;
  int ncol = (per_c || per_c2) ? (C + 63) / 64 : 0;
  if (nbc + ncol == 0) return 0;
  hipLaunchKernelGGL(chan_sum_finalize_kernel, dim3(nbc + ncol), dim3(256), 0, s, ws, B, r.splits, C, (bf16_t*)per_bc,
                     ld_bc, per_c, per_c2, c_store, nbc);
  SDMI_CHECK_LAUNCH();
  return 0;
}
