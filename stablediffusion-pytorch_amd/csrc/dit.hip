// DiT (models/transformer.py, transformer_layer.py) row kernels for gfx950.
//
// Token activations are row-major bf16 [B*N][ld] (N tokens per sample, C = hidden size channels). The
// adaLN modulation tables (shift / scale / gate per (sample, channel)) are bf16 column slices of the ONE
// GEMM that evaluates every layer's adaptive_norm_layer at once ([B][ld_mod]).
//
//  ln_mod_fwd : [x += gate * v  (gated residual of the previous sub-block, stored)] ->
//               LayerNorm(no affine, eps) -> y = xhat * (1 + scale) + shift                (bf16)
//               transformer_layer.py:89-91, 94-103, 104-106; transformer.py:205-207
//  ln_mod_bwd : dx = dres + LN'(dy * (1 + scale)); per-(sample, channel) partial sums of dy (dshift) and
//               dy * xhat (dscale) for this workgroup's token chunk; optionally the gate backward of the
//               residual branch that produced x (dv = gate * dx, partial sums of dx * v = dgate) fused in,
//               since it reads the same rows.
//  mod_finalize: sums the token-chunk partials in fixed order (deterministic, no atomics) into the bf16
//               gradient of the modulation table, consumed by the adaLN weight-gradient GEMM.
//  patch helpers: NCHW fp32 <-> token-major '(nh nw) (ph pw c)' (transformer.py:209-212,
//               patch_embed.py:88-89) and the MSE loss read straight from the token layout.
//
// One 64-lane wave owns one token row at a time; lane l holds channels [8l, 8l+8) (C % 8 == 0, C <= 512),
// so row statistics are wave reductions and every global access is a 16-byte vector.
#include <cstdlib>

#include "common.h"
#include "../../include/sdmi.h"
#include <algorithm>

namespace {

constexpr int NT = 256;
constexpr int WAVES = NT / 64;
constexpr int RPW = 1;  // rows per wave in the forward kernel (measured on DiT-12L: 4 -> 1 = -0.05 ms/step)

struct LnFwdArgs {
  const void* x; int ldx;  // residual stream (bf16, or fp32 when the kernel's F32)
  const bf16_t* v; int ldv;
  const bf16_t* gate;
  void* xo; int ldxo;
  const bf16_t* shift; const bf16_t* scale; int ld_mod;
  bf16_t* y; int ldy;
  float* mean; float* rstd;
  int rpw;  // rows per wave (RPW)
  int rows, C, N;
  float eps;
};

__device__ __forceinline__ void load8(const bf16_t* p, float* f) { unpack8(*(const uint4*)p, f); }

// residual-stream rows: bf16 or fp32 (F32) -- 8 consecutive channels
template <bool F32>
__device__ __forceinline__ void sload8(const void* base, long long off, float* f) {
  if (F32) {
    const float4 a = *(const float4*)((const float*)base + off), b = *(const float4*)((const float*)base + off + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  } else {
    unpack8(*(const uint4*)((const bf16_t*)base + off), f);
  }
}
template <bool F32>
__device__ __forceinline__ void sstore8(void* base, long long off, const float* f) {
  if (F32) {
    *(float4*)((float*)base + off) = make_float4(f[0], f[1], f[2], f[3]);
    *(float4*)((float*)base + off + 4) = make_float4(f[4], f[5], f[6], f[7]);
  } else {
    *(uint4*)((bf16_t*)base + off) = pack8(f);
  }
}

template <bool F32>
__global__ __launch_bounds__(NT) void ln_mod_fwd_kernel(const LnFwdArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool on = lane < (a.C >> 3);
  const int c0 = lane * 8;
  const float inv_c = 1.0f / (float)a.C;
#pragma unroll 1
  for (int i = 0; i < a.rpw; ++i) {
    const int row = (blockIdx.x * WAVES + wave) * a.rpw + i;
    if (row >= a.rows) return;
    const int b = row / a.N;
    float xv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (on) {
      sload8<F32>(a.x, (long long)row * a.ldx + c0, xv);
      if (a.v) {
        float vv[8], gv[8];
        load8(a.v + (long long)row * a.ldv + c0, vv);
        if (a.gate) {
          load8(a.gate + (long long)b * a.ld_mod + c0, gv);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) gv[e] = 1.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] += gv[e] * vv[e];
        if (!F32) {  // a bf16 residual stream: normalise the rounded value
          const uint4 packed = pack8(xv);
          unpack8(packed, xv);
        }
        sstore8<F32>(a.xo, (long long)row * a.ldxo + c0, xv);
      }
    }
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += xv[e];
    const float mu = wave_sum(s) * inv_c;
    float q = 0.f;
    if (on) {
#pragma unroll
      for (int e = 0; e < 8; ++e) q += (xv[e] - mu) * (xv[e] - mu);
    }
    const float rs = rsqrtf(wave_sum(q) * inv_c + a.eps);
    if (on) {
      float yv[8], sh[8], sc[8];
      if (a.scale) {
        load8(a.scale + (long long)b * a.ld_mod + c0, sc);
        load8(a.shift + (long long)b * a.ld_mod + c0, sh);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) { sc[e] = 0.f; sh[e] = 0.f; }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) yv[e] = (xv[e] - mu) * rs * (1.f + sc[e]) + sh[e];
      *(uint4*)(a.y + (long long)row * a.ldy + c0) = pack8(yv);
    }
    if (lane == 0) {
      a.mean[row] = mu;
      a.rstd[row] = rs;
    }
  }
}

struct LnBwdArgs {
  const void* x; int ldx;  // LayerNorm input (the residual stream; fp32 when F32, as dres / dx)
  const float* mean; const float* rstd;
  const bf16_t* dy; int lddy;
  const bf16_t* scale; int ld_mod;  // null: plain LayerNorm (no modulation, no dshift/dscale)
  const void* dres; int lddres;
  void* dx; int lddx;
  bf16_t* dx16; int ld16;  // optional bf16 copy of dx (GEMM operand of the patch-embedding backward)
  float* psh; float* psc; int ws_ld;  // partial rows (b*chunks + chunk) of the modulation gradient
  // fused gate backward of the branch that produced x: dv = gate * dx, partial dgate = sum dx * v
  const bf16_t* gate; const bf16_t* v; int ldv; bf16_t* dv; int lddv; float* pg;
  int rows, C, N, R;  // R tokens per workgroup (N % R == 0)
};

template <bool F32>
__global__ __launch_bounds__(NT) void ln_mod_bwd_kernel(const LnBwdArgs a) {
  __shared__ float red[WAVES][3][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool on = lane < (a.C >> 3);
  const int c0 = lane * 8;
  const float inv_c = 1.0f / (float)a.C;
  const int chunks = a.N / a.R;
  const int b = blockIdx.x / chunks, chunk = blockIdx.x - b * chunks;
  const int r0 = b * a.N + chunk * a.R;
  float sc[8], gv[8];
  float ash[8], asc[8], ag[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sc[e] = 0.f; gv[e] = 0.f; ash[e] = 0.f; asc[e] = 0.f; ag[e] = 0.f; }
  if (on && a.scale) load8(a.scale + (long long)b * a.ld_mod + c0, sc);
  if (on && a.gate) load8(a.gate + (long long)b * a.ld_mod + c0, gv);
#pragma unroll 1
  for (int r = wave; r < a.R; r += WAVES) {
    const int row = r0 + r;
    const float mu = a.mean[row], rs = a.rstd[row];
    float xh[8], dyv[8], dxh[8];
    float s1 = 0.f, s2 = 0.f;
    if (on) {
      sload8<F32>(a.x, (long long)row * a.ldx + c0, xh);
      load8(a.dy + (long long)row * a.lddy + c0, dyv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xh[e] = (xh[e] - mu) * rs;
        dxh[e] = dyv[e] * (1.f + sc[e]);
        ash[e] += dyv[e];
        asc[e] += dyv[e] * xh[e];
        s1 += dxh[e];
        s2 += dxh[e] * xh[e];
      }
    }
    s1 = wave_sum(s1) * inv_c;
    s2 = wave_sum(s2) * inv_c;
    if (on) {
      float dxv[8], rr[8];
      if (a.dres) {
        sload8<F32>(a.dres, (long long)row * a.lddres + c0, rr);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) rr[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) dxv[e] = rr[e] + rs * (dxh[e] - s1 - xh[e] * s2);
      if (!F32) {  // bf16 gradient stream: the gate backward reads the stored (rounded) value
        const uint4 packed = pack8(dxv);
        unpack8(packed, dxv);
      }
      sstore8<F32>(a.dx, (long long)row * a.lddx + c0, dxv);
      if (a.dx16) *(uint4*)(a.dx16 + (long long)row * a.ld16 + c0) = pack8(dxv);
      if (a.pg) {
        float vv[8], dvv[8];
        load8(a.v + (long long)row * a.ldv + c0, vv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          dvv[e] = gv[e] * dxv[e];
          ag[e] += dxv[e] * vv[e];
        }
        *(uint4*)(a.dv + (long long)row * a.lddv + c0) = pack8(dvv);
      }
    }
  }
  // cross-wave reduction of the per-channel partial sums of this token chunk
  if (on) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[wave][0][c0 + e] = ash[e];
      red[wave][1][c0 + e] = asc[e];
      red[wave][2][c0 + e] = ag[e];
    }
  }
  __syncthreads();
  const long long prow = (long long)blockIdx.x * a.ws_ld;
  for (int c = threadIdx.x; c < a.C; c += NT) {
    float t0 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
      t0 += red[w][0][c];
      t1 += red[w][1][c];
      t2 += red[w][2][c];
    }
    if (a.psh) a.psh[prow + c] = t0;
    if (a.psc) a.psc[prow + c] = t1;
    if (a.pg) a.pg[prow + c] = t2;
  }
}

__global__ void mod_finalize_kernel(const float* ws, int B, int chunks, int ws_ld, int W, bf16_t* out, int ldo) {
  const long long total = (long long)B * W;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / W), c = (int)(i - (long long)b * W);
    const float* p = ws + (long long)b * chunks * ws_ld + c;
    float s = 0.f;
#pragma unroll 8  // (independent loads in flight; the sum stays in chunk order)
    for (int k = 0; k < chunks; ++k) s += p[(long long)k * ws_ld];
    out[(long long)b * ldo + c] = f2bf(s);
  }
}

// token-major element (row = b*N + nh*nw_cnt + nw, col = (ph*p + pw)*C + c)  <->  NCHW (b, c, nh*p+ph, nw*p+pw)
__device__ __forceinline__ long long nchw_index(long long row, int col, int C, int H, int W, int p) {
  const int nw_cnt = W / p, N = (H / p) * nw_cnt;
  const long long b = row / N;
  const int n = (int)(row - b * N);
  const int nh = n / nw_cnt, nw = n - nh * nw_cnt;
  const int tap = col / C, c = col - tap * C;
  const int ph = tap / p, pw = tap - ph * p;
  return ((b * C + c) * H + nh * p + ph) * (long long)W + nw * p + pw;
}

__global__ void tokens_to_nchw_kernel(const void* src, int src_f32, int ld, int B, int C, int H, int W, int p,
                                      float* dst) {
  const int K = p * p * C;
  const long long total = (long long)B * (H / p) * (W / p) * K;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / K;
    const int col = (int)(i - row * K);
    const float v = src_f32 ? ((const float*)src)[row * ld + col] : bf2f(((const bf16_t*)src)[row * ld + col]);
    dst[nchw_index(row, col, C, H, W, p)] = v;
  }
}

__global__ void nchw_to_tokens_kernel(const float* src, int B, int C, int H, int W, int p, bf16_t* dst, int ld) {
  const int K = p * p * C;
  const long long total = (long long)B * (H / p) * (W / p) * ld;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / ld;
    const int col = (int)(i - row * ld);
    dst[i] = col < K ? f2bf(src[nchw_index(row, col, C, H, W, p)]) : (bf16_t)0;
  }
}

__global__ void mse_patch_kernel(const float* pred, int ld, const float* target, int B, int C, int H, int W, int p,
                                 float gscale, const float* gscale_dev, bf16_t* grad, float* partial) {
  if (gscale_dev) gscale = *gscale_dev;
  const int K = p * p * C;
  const long long total = (long long)B * (H / p) * (W / p) * ld;
  const float n = (float)((long long)B * C * H * W);
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long row = i / ld;
    const int col = (int)(i - row * ld);
    float g = 0.f;
    if (col < K) {
      const float d = pred[i] - target[nchw_index(row, col, C, H, W, p)];
      acc += d * d;
      g = 2.f * d / n * gscale;
    }
    if (grad) grad[i] = f2bf(g);
  }
  __shared__ float red[NT / 64];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < NT / 64; ++w) s += red[w];
    partial[blockIdx.x] = s;
  }
}

__global__ void sum_rows_kernel(const float* partial, int n, float scale, float* out) {
  __shared__ float red[NT / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += NT) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    *out = t * scale;
  }
}

int grid_for(long long total, int per = 256) { return (int)std::min<long long>((total + per - 1) / per, 8192); }

bool vec_ok(const void* p, int ld) { return p == nullptr || ((uintptr_t)p % 16 == 0 && ld % 8 == 0); }

}  // namespace

// token rows per backward workgroup (= per shift/scale/gate partial chunk): the largest power of two <= the cap
// dividing N. Each wave walks its rows serially (two dependent load round trips per row), so a smaller cap buys
// workgroups: cap 8 (32 -> 8 measured -0.16 ms per DiT-12L step).
extern "C" int sdmi_ln_chunk_rows(int N) {
  for (int r = 8; r > 1; r >>= 1)
    if (N % r == 0) return r;
  return 1;
}

extern "C" int sdmi_ln_mod_fwd(const void* x, int ldx, const void* v, int ldv, const void* gate, void* xo, int ldxo,
                               const void* shift, const void* scale, int ld_mod, void* y, int ldy, float* mean,
                               float* rstd, int rows, int C, int N, float eps, int x_f32, sdmi_stream_t stream) {
  if (rows <= 0 || C <= 0 || C % 8 || C > 512 || N <= 0 || rows % N) return -1;
  if (!x || !y || !mean || !rstd || (v && !xo) || ((shift == nullptr) != (scale == nullptr))) return -2;
  if (!vec_ok(x, ldx) || !vec_ok(v, ldv) || !vec_ok(xo, ldxo) || !vec_ok(y, ldy) || !vec_ok(gate, ld_mod) ||
      !vec_ok(shift, ld_mod) || !vec_ok(scale, ld_mod))
    return -3;
  LnFwdArgs a;
  a.x = x; a.ldx = ldx; a.v = (const bf16_t*)v; a.ldv = ldv; a.gate = (const bf16_t*)gate;
  a.xo = xo; a.ldxo = ldxo; a.shift = (const bf16_t*)shift; a.scale = (const bf16_t*)scale;
  a.ld_mod = ld_mod; a.y = (bf16_t*)y; a.ldy = ldy; a.mean = mean; a.rstd = rstd;
  a.rows = rows; a.C = C; a.N = N; a.eps = eps;
  a.rpw = RPW;
  const int per = WAVES * RPW;
  if (x_f32)
    sdmi_rt::launch(ln_mod_fwd_kernel<true>, dim3((rows + per - 1) / per), dim3(NT), 0, (hipStream_t)stream, a);
  else
    sdmi_rt::launch(ln_mod_fwd_kernel<false>, dim3((rows + per - 1) / per), dim3(NT), 0, (hipStream_t)stream, a);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_ln_mod_bwd(const void* x, int ldx, const float* mean, const float* rstd, const void* dy, int lddy,
                               const void* scale, int ld_mod, const void* dres, int lddres, void* dx, int lddx,
                               float* psh, float* psc, int ws_ld, const void* gate, const void* v, int ldv, void* dv,
                               int lddv, float* pg, int rows, int C, int N, int x_f32, void* dx16, int ld16,
                               sdmi_stream_t stream) {
  if (rows <= 0 || C <= 0 || C % 8 || C > 512 || N <= 0 || rows % N) return -1;
  if (!x || !mean || !rstd || !dy || !dx) return -2;
  if ((psh || psc) && !scale) return -2;
  if (gate && (!v || !dv || !pg)) return -2;
  if (!vec_ok(x, ldx) || !vec_ok(dy, lddy) || !vec_ok(dres, lddres) || !vec_ok(dx, lddx) || !vec_ok(v, ldv) ||
      !vec_ok(dv, lddv) || !vec_ok(scale, ld_mod) || !vec_ok(gate, ld_mod) || !vec_ok(dx16, ld16))
    return -3;
  LnBwdArgs a;
  a.x = x; a.ldx = ldx; a.mean = mean; a.rstd = rstd; a.dy = (const bf16_t*)dy; a.lddy = lddy;
  a.scale = (const bf16_t*)scale; a.ld_mod = ld_mod; a.dres = dres; a.lddres = lddres;
  a.dx = dx; a.lddx = lddx; a.dx16 = (bf16_t*)dx16; a.ld16 = ld16; a.psh = psh; a.psc = psc; a.ws_ld = ws_ld;
  a.gate = (const bf16_t*)gate; a.v = (const bf16_t*)v; a.ldv = ldv; a.dv = (bf16_t*)dv; a.lddv = lddv;
  a.pg = gate ? pg : nullptr;
  a.rows = rows; a.C = C; a.N = N; a.R = sdmi_ln_chunk_rows(N);
  if (x_f32)
    sdmi_rt::launch(ln_mod_bwd_kernel<true>, dim3(rows / a.R), dim3(NT), 0, (hipStream_t)stream, a);
  else
    sdmi_rt::launch(ln_mod_bwd_kernel<false>, dim3(rows / a.R), dim3(NT), 0, (hipStream_t)stream, a);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_mod_finalize(const float* ws, int B, int chunks, int ws_ld, int W, void* out, int ldo,
                                 sdmi_stream_t stream) {
  if (B <= 0 || chunks <= 0 || W <= 0 || ws_ld < W || ldo < W) return -1;
  sdmi_rt::launch(mod_finalize_kernel, dim3(grid_for((long long)B * W)), dim3(256), 0, (hipStream_t)stream, ws, B,
                     chunks, ws_ld, W, (bf16_t*)out, ldo);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_tokens_to_nchw(const void* src, int src_f32, int ld, int B, int C, int H, int W, int p, float* dst,
                                   sdmi_stream_t stream) {
  if (B <= 0 || C <= 0 || p <= 0 || H % p || W % p || ld < p * p * C) return -1;
  const long long total = (long long)B * H * W * C;
  sdmi_rt::launch(tokens_to_nchw_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, src, src_f32, ld,
                     B, C, H, W, p, dst);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_nchw_to_tokens_bf16(const float* src, int B, int C, int H, int W, int p, void* dst, int ld,
                                        sdmi_stream_t stream) {
  if (B <= 0 || C <= 0 || p <= 0 || H % p || W % p || ld < p * p * C) return -1;
  const long long total = (long long)B * (H / p) * (W / p) * ld;
  sdmi_rt::launch(nchw_to_tokens_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, src, B, C, H, W,
                     p, (bf16_t*)dst, ld);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_mse_patch(const float* pred, int ld, const float* target, int B, int C, int H, int W, int p,
                              float gscale, const float* gscale_dev, void* grad, float* ws, float* loss,
                              sdmi_stream_t stream) {
  if (B <= 0 || C <= 0 || p <= 0 || H % p || W % p || ld < p * p * C) return -1;
  const long long total = (long long)B * (H / p) * (W / p) * ld;
  const int blocks = (int)std::min<long long>((total + NT - 1) / NT, 1024);  // ws: sdmi_mse_workspace() floats
  sdmi_rt::launch(mse_patch_kernel, dim3(blocks), dim3(NT), 0, (hipStream_t)stream, pred, ld, target, B, C, H, W, p,
                     gscale, gscale_dev, (bf16_t*)grad, ws);
  SDMI_CHECK_LAUNCH();
  sdmi_rt::launch(sum_rows_kernel, dim3(1), dim3(NT), 0, (hipStream_t)stream, ws, blocks,
                     1.0f / (float)((long long)B * C * H * W), loss);
  SDMI_CHECK_LAUNCH();
  return 0;
}
