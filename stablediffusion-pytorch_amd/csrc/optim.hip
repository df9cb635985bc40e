// Fused optimizer step over the flat fp32 parameter/gradient buffers:
//   GradScaler.unscale_ -> clip_grad_norm_(max_norm) -> skip-if-non-finite -> Adam -> EMA
// (train_ddpm_cond_celebhq_multi_gpu.py:362-378; torch.optim.Adam defaults, EMA decay 0.9999).
// All control state (step, loss scale, growth tracker, found-inf) lives on the device so a whole
// training step can be replayed as one hipGraph without host synchronisation.
#include <cstdint>
#include <cstdlib>

#include "common.h"
#include "../../include/sdmi.h"

namespace {
constexpr int NT = 256;
constexpr int NORM_BLOCKS = 2048;

// Gradient sum of squares in FIXED blocks of NORM_BLK elements at absolute flat offsets: block b of a range that starts
// on a block boundary is summed by workgroup b alone, in a fixed order (per-thread float4 strides, then the wave tree,
// then the four waves in order), into partial[b]. The partial of a block depends only on that block's data, so the
// whole-buffer norm (sdmi_clip_unscale), the pieces overlapped with the backward (sdmi_sumsq_blocks on watermark
// ranges rounded down to block boundaries) and the per-bucket pieces after each data-parallel all-reduce all produce
// the same partial array -- and norm_finalize_kernel sums it in index order: bitwise the same norm for any split.
constexpr long long NORM_BLK = 1 << 17;

// one 1024-thread workgroup per block: each thread sums its float4s (index t, t + 1024, ...) eight loads at a time in a
// fixed order, then the wave trees and the 16 waves in order (the same order for a block wherever it is summed)
constexpr int NTN = 1024;

__device__ __forceinline__ float sq4(const float4 v) { return v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w; }

__device__ __forceinline__ void block_partial(float acc, float* partial) {
  __shared__ float red[NTN / 64];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NTN / 64; ++w) s += red[w];
    *partial = s;
  }
}

__global__ __launch_bounds__(NTN) void sumsq_block_kernel(const float* g, long long n, float* partial) {
  const long long b0 = (long long)blockIdx.x * NORM_BLK;
  const int e = (int)(n - b0 < NORM_BLK ? n - b0 : NORM_BLK);
  const float4* gb = (const float4*)(g + b0);
  const int e4 = e / 4;
  float acc = 0.f;
  int i = threadIdx.x;
  for (; i + 7 * NTN < e4; i += 8 * NTN) {
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = gb[i + k * NTN];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += sq4(v[k]);
  }
  for (; i < e4; i += NTN) acc += sq4(gb[i]);
  for (int j = e4 * 4 + threadIdx.x; j < e; j += NTN) acc += g[b0 + j] * g[b0 + j];
  block_partial(acc, partial + blockIdx.x);
}

// the bf16 gradient wire: dst[i] = float(src[i]) (exact) and, when partial != null, the block sums of squares of dst
// (sumsq_block_kernel's order)
__device__ __forceinline__ float4 widen4(const uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

__global__ __launch_bounds__(NTN) void widen_sumsq_kernel(const bf16_t* src, float* dst, long long n, float* partial) {
  const long long b0 = (long long)blockIdx.x * NORM_BLK;
  const int e = (int)(n - b0 < NORM_BLK ? n - b0 : NORM_BLK);
  const uint2* sb = (const uint2*)(src + b0);
  float4* db = (float4*)(dst + b0);
  const int e4 = e / 4;
  float acc = 0.f;
  int i = threadIdx.x;
  for (; i + 7 * NTN < e4; i += 8 * NTN) {
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = widen4(sb[i + k * NTN]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      db[i + k * NTN] = v[k];
      acc += sq4(v[k]);
    }
  }
  for (; i < e4; i += NTN) {
    const float4 v = widen4(sb[i]);
    db[i] = v;
    acc += sq4(v);
  }
  for (int j = e4 * 4 + threadIdx.x; j < e; j += NTN) {
    const float v = bf2f(src[b0 + j]);
    dst[b0 + j] = v;
    acc += v * v;
  }
  if (partial) block_partial(acc, partial + blockIdx.x);
}

// state layout (fp32 unless noted): [0] grad norm (unscaled)  [1] clip coefficient * inv_scale
// [2] loss scale  [3] growth tracker  [4] step (as float)  [5] found_inf/skip flag  [6] last loss
// [7] data-parallel non-finite-loss flag (sum over ranks of each rank's flag; skip_if_loss_nonfinite == 2)
__global__ void norm_finalize_kernel(const float* partial, int n, float max_norm, float* state, int growth_interval,
                                     int skip_if_loss_nonfinite, float grad_div) {
  __shared__ double red[NT];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += NT) acc += (double)partial[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float scale = state[2];
    float inv = 1.0f / (scale * grad_div);  // unscale and average over data-parallel ranks
    float norm = (float)sqrt(red[0]) * inv;  // ||g/scale|| = ||g|| / scale (power-of-two scale: exact)
    state[0] = norm;
    bool loss_bad = skip_if_loss_nonfinite == 1 ? !isfinite(state[6])
                    : skip_if_loss_nonfinite == 2 ? state[7] != 0.f : false;
    bool bad = !isfinite(norm) || loss_bad;
    state[5] = bad ? 1.f : 0.f;
    float coef = max_norm / (norm + 1e-6f);
    coef = coef < 1.f ? coef : 1.f;
    state[1] = coef * inv;
    if (growth_interval <= 0) {  // no loss scaler (plain fp32 trainer): the scale stays 1, finite steps count
      if (!bad) state[4] = state[4] + 1.f;
    } else if (!loss_bad) {  // reference: non-finite loss skips before scaler.update() (:348-352)
      if (bad) {
        state[2] = scale * 0.5f;
        state[3] = 0.f;
      } else {
        float tr = state[3] + 1.f;
        if ((int)tr >= growth_interval) {
          state[2] = scale * 2.f;
          tr = 0.f;
        }
        state[3] = tr;
        state[4] = state[4] + 1.f;
      }
    }
  }
}

// mode 0: *dst = isfinite(*src) ? 0 : 1 (a rank's non-finite-loss flag); mode 1: *dst = (*src != 0) (the summed flag)
__global__ void loss_flag_kernel(const float* src, float* dst, int mode) {
  if (threadIdx.x == 0) {
    const float v = *src;
    *dst = mode == 0 ? (isfinite(v) ? 0.f : 1.f) : (v != 0.f ? 1.f : 0.f);
  }
}

// one element of Adam + EMA (torch.optim.Adam, non-fused, non-amsgrad; ema as below)
__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float& e, bool ema, float gs, float b1,
                                         float b2, float eps, float step_size, float bc2s, float ema_decay,
                                         float ema_alpha) {
  const float gi = g * gs;
  const float mi = m + (1.f - b1) * (gi - m);  // lerp(m, g, 1 - b1)
  const float vi = v * b2 + (1.f - b2) * gi * gi;
  m = mi;
  v = vi;
  const float denom = sqrtf(vi) / bc2s + eps;
  p = p - step_size * (mi / denom);
  // ema.mul_(decay).add_(p, alpha=1 - decay) (:376-378): a rounded product, then add_'s fused alpha * p + self;
  // alpha is the reference's own fp32 value of (1 - decay) computed in double (1e-4f, not 1 - 0.9999f)
  if (ema) e = __builtin_fmaf(ema_alpha, p, mul_ieee(e, ema_decay));
}

// VEC = 4: 16-B loads / stores of all five streams (host checks the alignment), scalar tail in block 0.
// pb (optional): bf16 image of the updated parameters at the same flat offsets -- the GEMM-ready copy of every weight
// whose packed layout is its flat layout (linears, GEMM-natural conv weights), so no separate cast pass re-reads them
template <int VEC>
__global__ void adam_ema_kernel(float* p, const float* g, float* m, float* v, float* ema, long long n, const float* state,
                                float lr, float b1, float b2, float eps, float ema_decay, float ema_alpha, bf16_t* pb) {
  if (state[5] != 0.f) return;  // skipped step
  const float gs = state[1];
  const int step = (int)state[4];
  const double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  const float step_size = (float)(lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  const long long nv = n / VEC;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < nv; i += (long long)gridDim.x * NT) {
    if constexpr (VEC == 4) {
      float4 pi = ((const float4*)p)[i], mi = ((const float4*)m)[i], vi = ((const float4*)v)[i];
      const float4 gi = ((const float4*)g)[i];
      float4 ei = ema ? ((const float4*)ema)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      const bool he = ema != nullptr;
      adam_one(pi.x, gi.x, mi.x, vi.x, ei.x, he, gs, b1, b2, eps, step_size, bc2s, ema_decay, ema_alpha);
      adam_one(pi.y, gi.y, mi.y, vi.y, ei.y, he, gs, b1, b2, eps, step_size, bc2s, ema_decay, ema_alpha);
      adam_one(pi.z, gi.z, mi.z, vi.z, ei.z, he, gs, b1, b2, eps, step_size, bc2s, ema_decay, ema_alpha);
      adam_one(pi.w, gi.w, mi.w, vi.w, ei.w, he, gs, b1, b2, eps, step_size, bc2s, ema_decay, ema_alpha);
      ((float4*)p)[i] = pi;
      ((float4*)m)[i] = mi;
      ((float4*)v)[i] = vi;
      if (ema) ((float4*)ema)[i] = ei;
      if (pb) *(uint2*)(pb + 4 * i) = make_uint2(pack2bf(pi.x, pi.y), pack2bf(pi.z, pi.w));
    } else {
      float e = ema ? ema[i] : 0.f;
      adam_one(p[i], g[i], m[i], v[i], e, ema != nullptr, gs, b1, b2, eps, step_size, bc2s, ema_decay, ema_alpha);
      if (ema) ema[i] = e;
      if (pb) pb[i] = f2bf(p[i]);
    }
  }
  if (VEC > 1 && blockIdx.x == 0)
    for (long long i = nv * VEC + threadIdx.x; i < n; i += NT) {
      float e = ema ? ema[i] : 0.f;
      adam_one(p[i], g[i], m[i], v[i], e, ema != nullptr, gs, b1, b2, eps, step_size, bc2s, ema_decay, ema_alpha);
      if (ema) ema[i] = e;
      if (pb) pb[i] = f2bf(p[i]);
    }
}

// pb[i] = bf16(p[i]) (round to nearest even): the initial image of the parameters (and after any host-side update)
__global__ void cast_bf16_kernel(const float* p, bf16_t* pb, long long n) {
  const long long n4 = n / 4;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n4; i += (long long)gridDim.x * NT) {
    const float4 x = ((const float4*)p)[i];
    *(uint2*)(pb + 4 * i) = make_uint2(pack2bf(x.x, x.y), pack2bf(x.z, x.w));
  }
  if (blockIdx.x == 0)
    for (long long i = n4 * 4 + threadIdx.x; i < n; i += NT) pb[i] = f2bf(p[i]);
}
}  // namespace

extern "C" size_t sdmi_optim_workspace(void) { return NORM_BLOCKS * sizeof(float); }

// workspace of sdmi_clip_unscale_ws over n gradients: one partial per NORM_BLK block (at least the fixed size above)
extern "C" size_t sdmi_optim_workspace_for(long long n) {
  const long long nb = n > 0 ? (n + NORM_BLK - 1) / NORM_BLK : 0;
  return (size_t)(nb > NORM_BLOCKS ? nb : NORM_BLOCKS) * sizeof(float);
}

extern "C" long long sdmi_norm_block(void) { return NORM_BLK; }

// state: device float[8], initialise to {0, 0, init_scale, 0, 0, 0, 0, 0}
extern "C" int sdmi_clip_unscale_ws(const float* grads, long long n, float max_norm, float* state, float* ws,
                                    size_t ws_bytes, int growth_interval, int skip_if_loss_nonfinite, float grad_div,
                                    sdmi_stream_t stream) {
  if (!grads || !state || !ws || n <= 0 || ((uintptr_t)grads & 15)) return -1;
  const long long nb = (n + NORM_BLK - 1) / NORM_BLK;
  if ((size_t)nb * sizeof(float) > ws_bytes) return -3;  // workspace smaller than sdmi_optim_workspace_for(n)
  hipStream_t s = (hipStream_t)stream;
  sdmi_rt::launch(sumsq_block_kernel, dim3((unsigned)nb), dim3(NTN), 0, s, grads, n, ws);
  SDMI_CHECK_LAUNCH();
  sdmi_rt::launch(norm_finalize_kernel, dim3(1), dim3(NT), 0, s, ws, (int)nb, max_norm, state, growth_interval,
                     skip_if_loss_nonfinite, grad_div);
  SDMI_CHECK_LAUNCH();
  return 0;
}

// the fixed-workspace form (ws of sdmi_optim_workspace() bytes: up to NORM_BLOCKS * NORM_BLK ~ 268 M gradients)
extern "C" int sdmi_clip_unscale(const float* grads, long long n, float max_norm, float* state, float* ws,
                                 int growth_interval, int skip_if_loss_nonfinite, float grad_div, sdmi_stream_t stream) {
  return sdmi_clip_unscale_ws(grads, n, max_norm, state, ws, sdmi_optim_workspace(), growth_interval,
                              skip_if_loss_nonfinite, grad_div, stream);
}

extern "C" int sdmi_sumsq_blocks(const float* grads, long long n, float* partial, sdmi_stream_t stream) {
  if (!grads || !partial || n < 0 || ((uintptr_t)grads & 15)) return -1;
  if (n == 0) return 0;
  sdmi_rt::launch(sumsq_block_kernel, dim3((unsigned)((n + NORM_BLK - 1) / NORM_BLK)), dim3(NTN), 0,
                  (hipStream_t)stream, grads, n, partial);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_widen_bf16_sumsq(const void* src, float* dst, long long n, float* partial, sdmi_stream_t stream) {
  if (!src || !dst || n < 0 || ((uintptr_t)src & 7) || ((uintptr_t)dst & 15)) return -1;
  if (n == 0) return 0;
  sdmi_rt::launch(widen_sumsq_kernel, dim3((unsigned)((n + NORM_BLK - 1) / NORM_BLK)), dim3(NTN), 0,
                  (hipStream_t)stream, (const bf16_t*)src, dst, n, partial);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_clip_finalize(const float* partial, int n, float max_norm, float* state, int growth_interval,
                                  int skip_if_loss_nonfinite, float grad_div, sdmi_stream_t stream) {
  if (!partial || !state || n <= 0) return -1;
  sdmi_rt::launch(norm_finalize_kernel, dim3(1), dim3(NT), 0, (hipStream_t)stream, partial, n, max_norm, state,
                  growth_interval, skip_if_loss_nonfinite, grad_div);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_loss_flag(const float* src, float* dst, int mode, sdmi_stream_t stream) {
  if (!src || !dst || mode < 0 || mode > 1) return -1;
  sdmi_rt::launch(loss_flag_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, src, dst, mode);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_adam_ema(float* params, const float* grads, float* m, float* v, float* ema, long long n,
                             const float* state, float lr, float b1, float b2, float eps, float ema_decay,
                             float ema_alpha, sdmi_stream_t stream) {
  return sdmi_adam_ema_bf16(params, grads, m, v, ema, n, state, lr, b1, b2, eps, ema_decay, ema_alpha, nullptr, stream);
}

extern "C" int sdmi_cast_bf16(const float* src, void* dst, long long n, sdmi_stream_t stream) {
  if (!src || !dst || n < 0 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 7)) return -1;
  if (n == 0) return 0;
  long long blocks = (n / 4 + NT - 1) / NT;
  blocks = blocks < 1 ? 1 : blocks > 8192 ? 8192 : blocks;
  sdmi_rt::launch(cast_bf16_kernel, dim3((unsigned)blocks), dim3(NT), 0, (hipStream_t)stream, src, (bf16_t*)dst, n);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_adam_ema_bf16(float* params, const float* grads, float* m, float* v, float* ema, long long n,
                                  const float* state, float lr, float b1, float b2, float eps, float ema_decay,
                                  float ema_alpha, void* params_bf16, sdmi_stream_t stream) {
  const bool vec = ((((uintptr_t)params | (uintptr_t)grads | (uintptr_t)m | (uintptr_t)v | (uintptr_t)ema) & 15) == 0) &&
                   ((uintptr_t)params_bf16 & 7) == 0;
  long long blocks = (n / (vec ? 4 : 1) + NT - 1) / NT;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  if (vec)
    sdmi_rt::launch(adam_ema_kernel<4>, dim3((unsigned)blocks), dim3(NT), 0, (hipStream_t)stream, params, grads, m, v,
                    ema, n, state, lr, b1, b2, eps, ema_decay, ema_alpha, (bf16_t*)params_bf16);
  else
    sdmi_rt::launch(adam_ema_kernel<1>, dim3((unsigned)blocks), dim3(NT), 0, (hipStream_t)stream, params, grads, m, v,
                    ema, n, state, lr, b1, b2, eps, ema_decay, ema_alpha, (bf16_t*)params_bf16);
  SDMI_CHECK_LAUNCH();
  return 0;
}
