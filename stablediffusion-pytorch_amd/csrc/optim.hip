// Fused optimizer step over the flat fp32 parameter/gradient buffers:
//   GradScaler.unscale_ -> clip_grad_norm_(max_norm) -> skip-if-non-finite -> Adam -> EMA
// (train_ddpm_cond_celebhq_multi_gpu.py:362-378; torch.optim.Adam defaults, EMA decay 0.9999).
// All control state (step, loss scale, growth tracker, found-inf) lives on the device so a whole
// training step can be replayed as one hipGraph without host synchronisation.
#include <cstdlib>

#include "common.h"
#include "../../include/sdmi.h"

namespace {
constexpr int NT = 256;
constexpr int NORM_BLOCKS = 2048;

__global__ void sumsq_kernel(const float* g, long long n, float* partial) {
  float acc = 0.f;
  const long long n4 = n / 4;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n4; i += (long long)gridDim.x * NT) {
    float4 v = ((const float4*)g)[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0)
    for (long long i = n4 * 4 + threadIdx.x; i < n; i += NT) acc += g[i] * g[i];
  __shared__ float red[NT / 64];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// state layout (fp32 unless noted): [0] grad norm (unscaled)  [1] clip coefficient * inv_scale
// [2] loss scale  [3] growth tracker  [4] step (as float)  [5] found_inf/skip flag  [6] last loss
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
    bool loss_bad = skip_if_loss_nonfinite && !isfinite(state[6]);
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

__global__ void adam_ema_kernel(float* p, const float* g, float* m, float* v, float* ema, long long n, const float* state,
                                float lr, float b1, float b2, float eps, float ema_decay, float ema_alpha) {
  if (state[5] != 0.f) return;  // skipped step
  const float gs = state[1];
  const int step = (int)state[4];
  const double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  const float step_size = (float)(lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float gi = g[i] * gs;
    float mi = m[i] + (1.f - b1) * (gi - m[i]);  // lerp(m, g, 1 - b1)
    float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    float denom = sqrtf(vi) / bc2s + eps;
    float pi = p[i] - step_size * (mi / denom);
    p[i] = pi;
    // ema.mul_(decay).add_(p, alpha=1 - decay) (:376-378): a rounded product, then add_'s fused alpha * p + self;
    // alpha is the reference's own fp32 value of (1 - decay) computed in double (1e-4f, not 1 - 0.9999f)
    if (ema) ema[i] = __builtin_fmaf(ema_alpha, pi, mul_ieee(ema[i], ema_decay));
  }
}
}  // namespace

extern "C" size_t sdmi_optim_workspace(void) { return NORM_BLOCKS * sizeof(float); }

// state: device float[8], initialise to {0, 0, init_scale, 0, 0, 0, 0, 0}
extern "C" int sdmi_clip_unscale(const float* grads, long long n, float max_norm, float* state, float* ws,
                                 int growth_interval, int skip_if_loss_nonfinite, float grad_div, sdmi_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  sdmi_rt::launch(sumsq_kernel, dim3(NORM_BLOCKS), dim3(NT), 0, s, grads, n, ws);
  SDMI_CHECK_LAUNCH();
  sdmi_rt::launch(norm_finalize_kernel, dim3(1), dim3(NT), 0, s, ws, NORM_BLOCKS, max_norm, state, growth_interval,
                     skip_if_loss_nonfinite, grad_div);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_adam_ema(float* params, const float* grads, float* m, float* v, float* ema, long long n,
                             const float* state, float lr, float b1, float b2, float eps, float ema_decay,
                             float ema_alpha, sdmi_stream_t stream) {
  static long long max_blocks = -1;  // grid cap (SDMI_ADAM_BLOCKS): a narrower grid leaves CUs to concurrent work
  if (max_blocks < 0) {
    const char* e = getenv("SDMI_ADAM_BLOCKS");
    max_blocks = e ? atoll(e) : 8192;
    if (max_blocks < 1) max_blocks = 8192;
  }
  long long blocks = (n + NT - 1) / NT;
  if (blocks > max_blocks) blocks = max_blocks;
  sdmi_rt::launch(adam_ema_kernel, dim3((unsigned)blocks), dim3(NT), 0, (hipStream_t)stream, params, grads, m, v, ema,
                     n, state, lr, b1, b2, eps, ema_decay, ema_alpha);
  SDMI_CHECK_LAUNCH();
  return 0;
}
