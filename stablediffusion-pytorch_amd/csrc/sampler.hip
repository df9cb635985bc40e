// Reverse-diffusion (sampling) steps for gfx950, one fused elementwise pass each
// (reference scheduler/linear_noise_scheduler.py).
//
//  ddpm_prev : LinearNoiseScheduler.sample_prev_timestep (:50-78). The timestep is read from DEVICE memory and
//              the per-step scalars (sqrt(abar_t), sqrt(alpha_t), the posterior sigma) are derived in-kernel
//              from the reference's fp32 tables with correctly rounded fp32 division / sqrt and no FMA
//              contraction, so x_{t-1} and x0 are bit-identical to the reference for the same z -- and a
//              whole sampling step (model forward + this kernel) can be captured once and replayed with a
//              device-side timestep counter (no host sync per step; the reference syncs on `t == 0`).
//  ddim_prev : DDIMSampler.sample_one_step (:164-182): x_{t-1} = sqrt(a_prev/a_t) x_t + (sqrt(1 - a_prev -
//              sigma^2) - sqrt(a_prev (1 - a_t) / a_t)) eps + sigma noise, sigma = eta sqrt(...).
//  ddim_prev_dev : the same step with (t, t_prev) read from device tables through a device step index, which a
//              follow-up launch decrements (and the model's timestep scalar with it): a captured DDIM loop.
//  affine    : DDPMSampler.sample_one_step (:111-124): (c1 x - c2 eps) + sqrt(var) z with host table scalars.
#include "common.h"
#include "../../include/sdmi.h"
#include <algorithm>

namespace {

constexpr int NT = 256;

// IEEE fp32 division / square root, correctly rounded: evaluated in fp64 and rounded once to fp32 (a double
// result of two floats' quotient or a float's root rounds to the correctly rounded float: p = 53 >= 2*24 + 2).
// The gfx950 fp32 fast paths (v_rcp / v_sqrt based) are ~1 ulp and would break bit parity with the reference.
__device__ __forceinline__ float div_ieee(float a, float b) { return (float)((double)a / (double)b); }
__device__ __forceinline__ float sqrt_ieee(float a) { return (float)__dsqrt_rn((double)a); }

__global__ void ddpm_prev_kernel(const float* xt, const float* eps, const float* z, long long n, const long long* tp,
                                 const float* betas, const float* alphas, const float* abar, const float* s1m,
                                 float* prev, float* x0out) {
#pragma clang fp contract(off)
  const long long t = *tp;
  const float sq_abar = sqrt_ieee(abar[t]);
  const float s1 = s1m[t], beta = betas[t], sq_alpha = sqrt_ieee(alphas[t]);
  float sigma = 0.f;
  if (t > 0) {
    const float var = mul_ieee(div_ieee(sub_ieee(1.0f, abar[t - 1]), sub_ieee(1.0f, abar[t])), beta);
    sigma = sqrt_ieee(var);  // variance ** 0.5 (torch pow(x, 0.5) is sqrt)
  }
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const float x = xt[i], e = eps[i];
    float x0 = div_ieee(sub_ieee(x, mul_ieee(s1, e)), sq_abar);
    x0 = fminf(fmaxf(x0, -1.0f), 1.0f);
    float mean = sub_ieee(x, div_ieee(mul_ieee(beta, e), s1));
    mean = div_ieee(mean, sq_alpha);
    if (x0out) x0out[i] = x0;
    prev[i] = t > 0 ? add_ieee(mean, mul_ieee(sigma, z[i])) : mean;
  }
}

// the device timestep counter moves to t - 1 once every block of the step kernel has read it: a separate
// single-thread launch ordered after the step on the same stream
__global__ void dec_t_kernel(long long* tp) {
  if (threadIdx.x == 0 && *tp > 0) *tp = *tp - 1;
}

__global__ void ddim_prev_kernel(const float* xt, const float* eps, const float* noise, long long n, float at,
                                 float ap, float eta, float* out) {
#pragma clang fp contract(off)
  // sigma_t = eta * sqrt((1 - a_prev) / (1 - a_t) * (1 - a_t / a_prev))
  const float sigma = mul_ieee(eta, sqrt_ieee(mul_ieee(div_ieee(sub_ieee(1.0f, ap), sub_ieee(1.0f, at)),
                                                     sub_ieee(1.0f, div_ieee(at, ap)))));
  const float c1 = sqrt_ieee(div_ieee(ap, at));
  const float c2 = sub_ieee(sqrt_ieee(sub_ieee(sub_ieee(1.0f, ap), mul_ieee(sigma, sigma))),
                             sqrt_ieee(div_ieee(mul_ieee(ap, sub_ieee(1.0f, at)), at)));
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float v = add_ieee(mul_ieee(c1, xt[i]), mul_ieee(c2, eps[i]));
    out[i] = add_ieee(v, mul_ieee(sigma, noise ? noise[i] : 0.0f));
  }
}

// DDIM step with its timestep pair read from DEVICE tables (a captured DDIMSampler.forward loop, reference :209-256):
// step index i = *idx, a_t = abar[ts[i]], a_prev = abar[tp[i]]; the same arithmetic as ddim_prev_kernel, so a replayed
// step is bit-identical to the eager one given the same noise
__global__ void ddim_prev_dev_kernel(const float* xt, const float* eps, const float* noise, long long n,
                                     const long long* ts, const long long* tp, const long long* idx, const float* abar,
                                     float eta, float* out) {
#pragma clang fp contract(off)
  const long long i = *idx;
  const float at = abar[ts[i]], ap = abar[tp[i]];
  const float sigma = mul_ieee(eta, sqrt_ieee(mul_ieee(div_ieee(sub_ieee(1.0f, ap), sub_ieee(1.0f, at)),
                                                     sub_ieee(1.0f, div_ieee(at, ap)))));
  const float c1 = sqrt_ieee(div_ieee(ap, at));
  const float c2 = sub_ieee(sqrt_ieee(sub_ieee(sub_ieee(1.0f, ap), mul_ieee(sigma, sigma))),
                             sqrt_ieee(div_ieee(mul_ieee(ap, sub_ieee(1.0f, at)), at)));
  for (long long j = (long long)blockIdx.x * NT + threadIdx.x; j < n; j += (long long)gridDim.x * NT) {
    float v = add_ieee(mul_ieee(c1, xt[j]), mul_ieee(c2, eps[j]));
    out[j] = add_ieee(v, mul_ieee(sigma, noise ? noise[j] : 0.0f));
  }
}

// after a DDIM step: the step index moves down and the model's timestep scalar follows it (ts[i - 1]); a separate
// single-thread launch ordered after the step on the same stream (every block of the step has read the index)
__global__ void ddim_advance_kernel(const long long* ts, long long* idx, long long* t_dev) {
  if (threadIdx.x == 0 && *idx > 0) {
    const long long i = *idx - 1;
    *idx = i;
    if (t_dev) *t_dev = ts[i];
  }
}

__global__ void affine_kernel(const float* x, const float* eps, const float* z, long long n, float c1, float c2,
                              float var, float* out) {
#pragma clang fp contract(off)
  const float s = sqrt_ieee(var);  // torch.sqrt(var), correctly rounded (host-CPU vector sqrt is not always)
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const float mean = sub_ieee(mul_ieee(c1, x[i]), mul_ieee(c2, eps[i]));
    out[i] = z ? add_ieee(mean, mul_ieee(s, z[i])) : add_ieee(mean, 0.0f);
  }
}

int grid_for(long long n) { return (int)std::max<long long>(1, std::min<long long>((n + NT - 1) / NT, 4096)); }

}  // namespace

extern "C" int sdmi_ddpm_prev(const float* xt, const float* eps, const float* z, long long n, long long* t_dev,
                              const float* betas, const float* alphas, const float* abar, const float* s1m,
                              float* prev, float* x0, int decrement_t, sdmi_stream_t stream) {
  if (!xt || !eps || !t_dev || !betas || !alphas || !abar || !s1m || !prev || n <= 0) return -1;
  sdmi_rt::launch(ddpm_prev_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, xt, eps, z, n, t_dev,
                     betas, alphas, abar, s1m, prev, x0);
  SDMI_CHECK_LAUNCH();
  if (decrement_t) {
    sdmi_rt::launch(dec_t_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, t_dev);
    SDMI_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int sdmi_ddim_prev(const float* xt, const float* eps, const float* noise, long long n, float alpha_t,
                              float alpha_prev, float eta, float* out, sdmi_stream_t stream) {
  if (!xt || !eps || !out || n <= 0) return -1;
  sdmi_rt::launch(ddim_prev_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, xt, eps, noise, n, alpha_t,
                     alpha_prev, eta, out);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_ddim_prev_dev(const float* xt, const float* eps, const float* noise, long long n,
                                  const long long* ts, const long long* tp, long long* idx, long long* t_dev,
                                  const float* abar, float eta, float* out, int advance, sdmi_stream_t stream) {
  if (!xt || !eps || !out || !ts || !tp || !idx || !abar || n <= 0) return -1;
  sdmi_rt::launch(ddim_prev_dev_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, xt, eps, noise, n, ts, tp,
                  (const long long*)idx, abar, eta, out);
  SDMI_CHECK_LAUNCH();
  if (advance) {
    sdmi_rt::launch(ddim_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ts, idx, t_dev);
    SDMI_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int sdmi_affine_step(const float* x, const float* eps, const float* z, long long n, float c1, float c2,
                                float var, float* out, sdmi_stream_t stream) {
  if (!x || !eps || !out || n <= 0) return -1;
  sdmi_rt::launch(affine_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, x, eps, z, n, c1, c2, var,
                     out);
  SDMI_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Device Gaussian noise for captured sampling loops: Philox4x32-10 (Salmon et al., SC'11) keyed by a 64-bit seed,
// counter = (element quad index, 64-bit draw offset read from DEVICE memory), Box-Muller on pairs of 24-bit
// uniforms in (0, 1]. The reference draws z with the host generator every step (scheduler :72); a replayed step
// instead reads its draw offset on the device and (advance != 0) bumps it afterwards, so every replay of the same
// recorded launches gets fresh, reproducible noise with no host round trip.
// ---------------------------------------------------------------------------------------------
namespace {

__device__ __forceinline__ void philox_round(uint32_t (&c)[4], const uint32_t (&k)[2]) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
  const uint32_t hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
  c[0] = hi1 ^ c[1] ^ k[0];
  c[1] = lo1;
  c[2] = hi0 ^ c[3] ^ k[1];
  c[3] = lo0;
}

__global__ void randn_kernel(float* out, long long n, unsigned long long seed, const unsigned long long* offset) {
  const unsigned long long off = *offset;
  const long long quads = (n + 3) / 4;
  for (long long q = (long long)blockIdx.x * NT + threadIdx.x; q < quads; q += (long long)gridDim.x * NT) {
    uint32_t c[4] = {(uint32_t)q, (uint32_t)((unsigned long long)q >> 32), (uint32_t)off, (uint32_t)(off >> 32)};
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      philox_round(c, k);
      k[0] += 0x9E3779B9u;
      k[1] += 0xBB67AE85u;
    }
    float z[4];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float u1 = ((c[2 * p] >> 8) + 1) * (1.0f / 16777216.0f);  // (0, 1]
      const float u2 = (c[2 * p + 1] >> 8) * (1.0f / 16777216.0f);    // [0, 1)
      const float rad = sqrtf(-2.0f * logf(u1));
      float s, co;
      sincosf(6.28318530717958647692f * u2, &s, &co);
      z[2 * p] = rad * co;
      z[2 * p + 1] = rad * s;
    }
    const long long i0 = q * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (i0 + e < n) out[i0 + e] = z[e];
  }
}

__device__ __forceinline__ void philox10(uint32_t (&c)[4], unsigned long long seed) {
  uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k);
    k[0] += 0x9E3779B9u;
    k[1] += 0xBB67AE85u;
  }
}

// per-sample draws of one training step: Philox block (B-independent quad index 2^40 + b, offset) ->
// c[0]: timestep, c[1]: text-drop uniform, c[2]: image-keep uniform (24-bit uniforms in [0, 1), as torch.rand)
__device__ __forceinline__ void sample_draw(int b, unsigned long long seed, unsigned long long off, uint32_t (&c)[4]) {
  const unsigned long long q = (1ull << 40) + (unsigned long long)b;
  c[0] = (uint32_t)q; c[1] = (uint32_t)(q >> 32); c[2] = (uint32_t)off; c[3] = (uint32_t)(off >> 32);
  philox10(c, seed);
}

// One launch for every random draw of a training step (train_ddpm_cond_celebhq_multi_gpu.py:299-330 draws them with
// five torch calls + a where): grid-stride over [noise quads | text rows (float4) | samples].
//   noise[i] ~ N(0, 1) (Philox quad i / 4, Box-Muller as randn_kernel); t[b] = floor(u * T);
//   txt[b] = (u_text < p_text) ? empty : text[b] (diffusion_utils.py:21-28); keep[b] = (u_keep > p_keep) (:31-37)
__global__ void step_draw_kernel(float* noise, long long n, long long* t, int B, int T, const float4* text,
                                 const float4* empty, float4* txt, long long row4, float p_text, float* keep,
                                 float p_keep, unsigned long long seed, unsigned long long off) {
  const long long nq = (n + 3) / 4, ntx = txt ? (long long)B * row4 : 0;
  const long long total = nq + ntx + B;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    if (i < nq) {
      uint32_t c[4] = {(uint32_t)i, (uint32_t)((unsigned long long)i >> 32), (uint32_t)off, (uint32_t)(off >> 32)};
      philox10(c, seed);
      float z[4];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float u1 = ((c[2 * p] >> 8) + 1) * (1.0f / 16777216.0f);  // (0, 1]
        const float u2 = (c[2 * p + 1] >> 8) * (1.0f / 16777216.0f);    // [0, 1)
        const float rad = sqrtf(-2.0f * logf(u1));
        float sn, co;
        sincosf(6.28318530717958647692f * u2, &sn, &co);
        z[2 * p] = rad * co;
        z[2 * p + 1] = rad * sn;
      }
      const long long i0 = i * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (i0 + e < n) noise[i0 + e] = z[e];
    } else if (i < nq + ntx) {
      const long long j = i - nq;
      const int b = (int)(j / row4);
      const long long r = j - (long long)b * row4;
      uint32_t c[4];
      sample_draw(b, seed, off, c);
      const bool drop = (c[1] >> 8) * (1.0f / 16777216.0f) < p_text;
      txt[j] = drop ? empty[r] : text[j];
    } else {
      const int b = (int)(i - nq - ntx);
      uint32_t c[4];
      sample_draw(b, seed, off, c);
      t[b] = (long long)(((unsigned long long)c[0] * (unsigned long long)T) >> 32);
      if (keep) keep[b] = (c[2] >> 8) * (1.0f / 16777216.0f) > p_keep ? 1.0f : 0.0f;
    }
  }
}

__global__ void advance_kernel(unsigned long long* offset) {
  if (threadIdx.x == 0) *offset = *offset + 1;
}

}  // namespace

extern "C" int sdmi_randn(float* out, long long n, unsigned long long seed, unsigned long long* offset_dev,
                          int advance, sdmi_stream_t stream) {
  if (!out || !offset_dev || n <= 0) return -1;
  sdmi_rt::launch(randn_kernel, dim3(grid_for((n + 3) / 4)), dim3(NT), 0, (hipStream_t)stream, out, n, seed,
                  (const unsigned long long*)offset_dev);
  SDMI_CHECK_LAUNCH();
  if (advance) {
    sdmi_rt::launch(advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, offset_dev);
    SDMI_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int sdmi_step_draw(float* noise, long long n, long long* t, int B, int T, const float* text,
                              const float* empty, float* txt, long long row_elems, float p_text, float* keep,
                              float p_keep, unsigned long long seed, unsigned long long offset, sdmi_stream_t stream) {
  if (!noise || n <= 0 || !t || B <= 0 || T <= 0) return -1;
  if (txt && (!text || !empty || row_elems <= 0 || row_elems % 4 || (uintptr_t)text % 16 || (uintptr_t)empty % 16 ||
              (uintptr_t)txt % 16))
    return -2;
  const long long items = (n + 3) / 4 + (txt ? (long long)B * (row_elems / 4) : 0) + B;
  sdmi_rt::launch(step_draw_kernel, dim3(grid_for(items)), dim3(NT), 0, (hipStream_t)stream, noise, n, t, B, T,
                  (const float4*)text, (const float4*)empty, (float4*)txt, row_elems / 4, p_text, keep, p_keep, seed,
                  offset);
  SDMI_CHECK_LAUNCH();
  return 0;
}
