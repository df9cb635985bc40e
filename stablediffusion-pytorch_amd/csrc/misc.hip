// Small fused kernels around the denoiser: input staging (mask gather + 1x1 mask projection),
// output layout, scheduler add_noise, MSE loss, time embedding, SiLU, channel-slice copies and
// bf16 weight packing.
#include <atomic>
#include <hip/hip_ext.h>

#include "common.h"
#include "../../include/sdmi.h"

namespace {
constexpr int NT = 256;

// input staging: one pixel per thread with up to 18 scattered mask reads each -- latency-bound, so small
// workgroups (4x the workgroups of NT-thread blocks: a 32768-pixel batch covers 512 CUs' worth of slots)
constexpr int PREP_NT = 64;
int prep_grid(long long work) {
  long long g = (work + PREP_NT - 1) / PREP_NT;
  return (int)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

int grid_for(long long work) {
  long long g = (work + NT - 1) / NT;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

// ---------------------------------------------------------------------------------------------
// Input staging (unet_cond_base.py:131-140): x (B,cx,H,W) fp32 NCHW -> NHWC bf16 [B*H*W][cpad];
// channels cx .. cx+cmo-1 = 1x1 conv (no bias) of the nearest-resized mask (B,cmi,MH,MW) fp32
// (F.interpolate default 'nearest': src = min(floor(dst * (in/out)), in-1)), rest zero.
// ---------------------------------------------------------------------------------------------
// CMAP: the mask is a uint8 class map (B,MH,MW) -- the reference's one-hot (celeb_dataset.py:164-175:
// clamp(0, cmi), one_hot(cmi + 1), background channel dropped) is never materialised: class c >= 1 selects
// weight column c-1 (min(c, cmi), the clamp), class 0 gives 0 -- the one-hot sum's exact value.
template <bool CMAP>
__global__ void prep_input_kernel(const float* x, int B, int cx, int H, int W, const void* mask, int cmi, int MH,
                                  int MW, const float* wcond, int cmo, bf16_t* out, int cpad, const float* keep) {
  long long total = (long long)B * H * W;
  float sh = (float)MH / (float)H, sw = (float)MW / (float)W;
  for (long long p = (long long)blockIdx.x * PREP_NT + threadIdx.x; p < total; p += (long long)gridDim.x * PREP_NT) {
    int b = (int)(p / (H * W));
    int yx = (int)(p - (long long)b * H * W);
    int y = yx / W, xx = yx - y * W;
    float v[16];
    for (int c = 0; c < 16; ++c) v[c] = 0.f;
    for (int c = 0; c < cx; ++c) v[c] = x[(((long long)b * cx + c) * H + y) * W + xx];
    if (mask) {
      int sy = min((int)floorf((float)y * sh), MH - 1), sx = min((int)floorf((float)xx * sw), MW - 1);
      int cls = 0;
      if (CMAP) cls = min((int)((const unsigned char*)mask)[((long long)b * MH + sy) * MW + sx], cmi);
      for (int o = 0; o < cmo; ++o) {
        float acc = 0.f;
        if (CMAP) {
          acc = cls > 0 ? wcond[o * cmi + cls - 1] : 0.f;
        } else {
          const float* m = (const float*)mask;
          for (int i = 0; i < cmi; ++i) acc += wcond[o * cmi + i] * m[(((long long)b * cmi + i) * MH + sy) * MW + sx];
        }
        v[cx + o] = keep ? acc * keep[b] : acc;
      }
    }
    bf16_t* dst = out + p * cpad;
    for (int c = 0; c < cpad; c += 8) *(uint4*)(dst + c) = pack8(v + c);
  }
}

// d wcond[o][i] = sum_{b,p} dxin[p][cx + o] * mask_resized[b][i][p]    (one block per (o, i))
// Pixel-split form: block (oi, z) sums pixels [z * chunk, (z + 1) * chunk) into part[z][oi] (one block per (o, i)
// left 54 workgroups looping over every pixel: ~90 us at the end of the backward); cond_wgrad_finish_kernel adds the
// CW_SPLITS partials in a fixed order, so the result is deterministic (and identical between the one-hot and the
// class-map forms, which differ only in how mv is read).
constexpr int CW_SPLITS = 32;
constexpr int CW_SLOTS = 8;                  // partial buffers, one per launch round-robin (concurrent engines)
constexpr int CW_MAX = 16 * 255;             // cmo <= 16 (cpad), cmi <= 255
__device__ float g_cw_part[CW_SLOTS][CW_SPLITS][CW_MAX];

template <bool CMAP>
__global__ void cond_wgrad_kernel(const bf16_t* dxin, int ld, int cx, int B, int H, int W, const void* mask, int cmi,
                                  int MH, int MW, int slot, const float* keep) {
  const int oi = blockIdx.x, o = oi / cmi, i = oi - o * cmi;
  float sh = (float)MH / (float)H, sw = (float)MW / (float)W;
  const long long total = (long long)B * H * W;
  const long long chunk = (total + CW_SPLITS - 1) / CW_SPLITS;
  const long long p0 = blockIdx.y * chunk, p1 = min(total, p0 + chunk);
  float acc = 0.f;
  for (long long p = p0 + threadIdx.x; p < p1; p += NT) {
    int b = (int)(p / (H * W));
    int yx = (int)(p - (long long)b * H * W);
    int y = yx / W, xx = yx - y * W;
    int sy = min((int)floorf((float)y * sh), MH - 1), sx = min((int)floorf((float)xx * sw), MW - 1);
    float mv;
    if (CMAP) mv = min((int)((const unsigned char*)mask)[((long long)b * MH + sy) * MW + sx], cmi) == i + 1 ? 1.f : 0.f;
    else mv = ((const float*)mask)[(((long long)b * cmi + i) * MH + sy) * MW + sx];
    acc += bf2f(dxin[p * ld + cx + o]) * (keep ? mv * keep[b] : mv);
  }
  __shared__ float red[NT / 64];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < NT / 64; ++w) s += red[w];
    g_cw_part[slot][blockIdx.y][oi] = s;
  }
}

__global__ void cond_wgrad_finish_kernel(int n, int slot, float* dw) {
  for (int oi = blockIdx.x * NT + threadIdx.x; oi < n; oi += gridDim.x * NT) {
    float s = 0.f;
    for (int z = 0; z < CW_SPLITS; ++z) s += g_cw_part[slot][z][oi];
    dw[oi] = s;
  }
}

int cw_slot() {
  static std::atomic<unsigned> next{0};
  return (int)(next.fetch_add(1) % CW_SLOTS);
}

template <bool CMAP>
int launch_cond_wgrad(const void* dxin, int ld, int cx, int B, int H, int W, const void* mask, int cmi, int MH, int MW,
                      int cmo, float* dw, const float* keep, hipStream_t s) {
  if (cmo < 1 || cmo > 16 || cmi < 1 || cmi > 255) return -1;
  const int slot = cw_slot();
  sdmi_rt::launch(cond_wgrad_kernel<CMAP>, dim3(cmo * cmi, CW_SPLITS), dim3(NT), 0, s, (const bf16_t*)dxin, ld, cx,
                     B, H, W, mask, cmi, MH, MW, slot, keep);
  SDMI_CHECK_LAUNCH();
  sdmi_rt::launch(cond_wgrad_finish_kernel, dim3((cmo * cmi + NT - 1) / NT), dim3(NT), 0, s, cmo * cmi, slot, dw);
  SDMI_CHECK_LAUNCH();
  return 0;
}

// NHWC (fp32 or bf16, row stride ld) -> NCHW fp32 (first C channels), and the reverse for gradients
__global__ void nhwc_to_nchw_kernel(const void* src, int src_f32, int ld, int B, int C, int HW, float* dst) {
  long long total = (long long)B * C * HW;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    int p = (int)(i % HW);
    long long bc = i / HW;
    int c = (int)(bc % C);
    int b = (int)(bc / C);
    long long s = ((long long)b * HW + p) * ld + c;
    dst[i] = src_f32 ? ((const float*)src)[s] : bf2f(((const bf16_t*)src)[s]);
  }
}

__global__ void nchw_to_nhwc_bf16_kernel(const float* src, int B, int C, int HW, bf16_t* dst, int ld) {
  long long total = (long long)B * HW * ld;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    int c = (int)(i % ld);
    long long bp = i / ld;
    int p = (int)(bp % HW);
    int b = (int)(bp / HW);
    dst[i] = c < C ? f2bf(src[((long long)b * C + c) * HW + p]) : (bf16_t)0;
  }
}

// x_t = sqrt(abar[t]) * x0 + sqrt(1-abar[t]) * eps   (scheduler :26-48; separate mul/mul/add, no FMA,
// so the result is bit-identical to the reference's fp32 CPU arithmetic)
__global__ void add_noise_kernel(const float* x0, const float* eps, const long long* t, const float* sa,
                                 const float* s1a, int B, long long per, float* out) {
#pragma clang fp contract(off)
  long long total = (long long)B * per;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    int b = (int)(i / per);
    long long ti = t[b];
    out[i] = add_ieee(mul_ieee(sa[ti], x0[i]), mul_ieee(s1a[ti], eps[i]));
  }
}

// MSE(pred, target): pred NHWC fp32 (ld), target NCHW fp32. Writes per-block partial sums and
// grad = 2 (pred - target) / n * gscale as NHWC bf16 (ld, pad channels zero).
__global__ void mse_kernel(const float* pred, int ld, const float* target, int B, int C, int HW, float gscale,
                           const float* gscale_dev, bf16_t* grad, float* partial) {
  if (gscale_dev) gscale = *gscale_dev;
  long long total = (long long)B * HW * ld;
  float n = (float)((long long)B * C * HW);
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    int c = (int)(i % ld);
    long long bp = i / ld;
    int p = (int)(bp % HW);
    int b = (int)(bp / HW);
    float g = 0.f;
    if (c < C) {
      float d = pred[i] - target[((long long)b * C + c) * HW + p];
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

__global__ void sum_partials_kernel(const float* partial, int n, float scale, float* out) {
  __shared__ float red[NT / 64];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += NT) acc += partial[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < NT / 64; ++w) s += red[w];
    out[0] = s * scale;
  }
}

// sinusoidal embedding (blocks.py:5-24): [sin(t / 10000^(i/half)), cos(...)] -> bf16 [B][ld]
__global__ void time_embedding_kernel(const long long* t, int tstride, int B, int dim, bf16_t* out, int ld,
                                      float* out_f32) {
  int half = dim / 2;
  int total = B * half;
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    int b = i / half, j = i - b * half;
    float f = powf(10000.f, (float)j / (float)half);
    float a = (float)t[b * tstride] / f;
    float s = sinf(a), c = cosf(a);
    out[(long long)b * ld + j] = f2bf(s);
    out[(long long)b * ld + half + j] = f2bf(c);
    if (out_f32) {
      out_f32[(long long)b * dim + j] = s;
      out_f32[(long long)b * dim + half + j] = c;
    }
  }
}

// y = silu(x) (bf16), or dx = dy * silu'(x) when dy != null
__global__ void silu_kernel(const bf16_t* x, const bf16_t* dy, bf16_t* y, long long n) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float v = bf2f(x[i]);
    y[i] = dy ? f2bf(bf2f(dy[i]) * silu_grad_f(v)) : f2bf(silu_f(v));
  }
}

// ReLU on fp32 (the leaf path's nn.ReLU, transformer.py:72,80): y = max(x, 0); with dy: dx = dy where x > 0
__global__ void relu_kernel(const float* x, const float* dy, float* y, long long n) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const float v = x[i];
    y[i] = dy ? (v > 0.f ? dy[i] : 0.f) : (v > 0.f ? v : 0.f);
  }
}

// dst[p][0:C] (+)= src[p][0:C]  (bf16 NHWC channel slices, C % 8 == 0)
__global__ void copy_slice_kernel(const bf16_t* src, int lds, bf16_t* dst, int ldd, long long P, int C, int accumulate) {
  int C8 = C >> 3;
  long long total = P * C8;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    long long p = i / C8;
    int c = (int)(i - p * C8) * 8;
    uint4 v = *(const uint4*)(src + p * lds + c);
    if (accumulate) {
      float a[8], b[8];
      unpack8(v, a);
      unpack8(*(const uint4*)(dst + p * ldd + c), b);
      for (int e = 0; e < 8; ++e) a[e] += b[e];
      v = pack8(a);
    }
    *(uint4*)(dst + p * ldd + c) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// batched fp32 -> bf16 weight packing:  dst[o][a][b][i] = src[o*so + i*si + kh(a)*skh + kw(b)*skw]
// with kh(a) = kh_off + kh_mul*a (identity, spatial flip, sub-pixel phase taps), zero for i >= I.
// ---------------------------------------------------------------------------------------------
}  // namespace


namespace {
constexpr int PACK_CHUNK = 4096;   // target elements per workgroup; bmap[blk] = (descriptor, first row)
constexpr int PACK_LDS_ELEMS = 16384;  // bf16 staging capacity (32 KiB, 4+ workgroups per CU): taps * (Ipad + 8)

template <int TAPS>
__device__ __forceinline__ void pack_gather(const sdmi_pack_desc& d, const float* src, bf16_t* st, int ld, int taps) {
  const int T = TAPS > 0 ? TAPS : taps;
  // channel-contiguous sources (GEMM-natural (co, kh, kw, ci) weights, linears): channel fastest, coalesced reads
  const bool cfast = d.si == 1;
  for (int idx = threadIdx.x; idx < T * d.I; idx += NT) {
    const int i = cfast ? idx % d.I : idx / T, t = cfast ? idx / d.I : idx - i * T;
    const int a = t / d.KW, b = t - a * d.KW;
    const int kh = d.kh_off + d.kh_mul * a, kw = d.kw_off + d.kw_mul * b;
    st[t * ld + i] = f2bf(src[(long long)i * d.si + (long long)kh * d.skh + (long long)kw * d.skw]);
  }
}

// One workgroup packs whole destination rows o0 .. o0+rows-1 of one descriptor. Phase 1 gathers the
// row's source elements in SOURCE order (tap fastest: contiguous [I][KH][KW] runs for conv weights)
// into LDS as bf16, phase 2 writes the [tap][Ipad] row with 16-byte stores.
__global__ void pack_kernel(const sdmi_pack_desc* descs, const int2* bmap) {
  extern __shared__ __attribute__((aligned(16))) bf16_t st[];
  const int2 bm = bmap[blockIdx.x];
  const sdmi_pack_desc& d = descs[bm.x];
  const int taps = d.KH * d.KW;
  const int ld = d.Ipad + 8;  // staging row stride: 16-B aligned, shifts banks per tap
  const int row = taps * d.Ipad;
  const int rows = max(1, PACK_CHUNK / row);
  const int o_end = min(d.O, bm.y + rows);
  // identity layout (the packed rows are the source rows in the same order: linears, GEMM-natural conv weights, rows
  // into a compact view): one contiguous cast, 8 elements per thread with 16-B loads and stores, no LDS staging
  const bool ident = d.Ipad == d.I && d.si == 1 && d.dst_ld == 0 && d.kh_off == 0 && d.kh_mul == 1 && d.kw_off == 0 &&
                     d.kw_mul == 1 && (d.KW == 1 || d.skw == d.I) && (d.KH == 1 || d.skh == (long long)d.KW * d.I) &&
                     d.so == (long long)row && row % 8 == 0 && ((uintptr_t)d.src & 15) == 0 &&
                     ((uintptr_t)d.dst & 15) == 0;
  if (ident) {
    const float* src = d.src + (long long)bm.y * row;
    bf16_t* dst = (bf16_t*)d.dst + (long long)bm.y * row;
    const int n8 = (o_end - bm.y) * row / 8;
    for (int q = threadIdx.x; q < n8; q += NT) {
      const float4 a = *(const float4*)(src + 8 * q), b = *(const float4*)(src + 8 * q + 4);
      *(uint4*)(dst + 8 * q) = make_uint4(pack2bf(a.x, a.y), pack2bf(a.z, a.w), pack2bf(b.x, b.y), pack2bf(b.z, b.w));
    }
    return;
  }
  const int nrows = o_end - bm.y;
  if (nrows > 1 && nrows * taps * ld <= PACK_LDS_ELEMS) {
    // short rows (conv_in's 4-channel taps, transposed up-sampling convs): every row of the block is gathered in ONE
    // pass -- all loads in flight together -- instead of one dependent load round trip and two barriers per row
    const int per = taps * d.I;
    const bool cfast = d.si == 1;
    for (int idx = threadIdx.x; idx < nrows * per; idx += NT) {
      const int rr = idx / per, rem = idx - rr * per;
      const int i = cfast ? rem % d.I : rem / taps, t = cfast ? rem / d.I : rem - i * taps;
      const int a = t / d.KW, b = t - a * d.KW;
      const int kh = d.kh_off + d.kh_mul * a, kw = d.kw_off + d.kw_mul * b;
      const float* src = d.src + (long long)(bm.y + rr) * d.so;
      st[(rr * taps + t) * ld + i] = f2bf(src[(long long)i * d.si + (long long)kh * d.skh + (long long)kw * d.skw]);
    }
    __syncthreads();
    const int q8 = row / 8;
    for (int q = threadIdx.x; q < nrows * q8; q += NT) {
      const int rr = q / q8, qq = q - rr * q8;
      const int t = (qq * 8) / d.Ipad, i0 = qq * 8 - t * d.Ipad;
      const bf16_t* sr = st + (rr * taps + t) * ld;
      uint4 v;
      if (i0 + 8 <= d.I) {
        v = *(const uint4*)(sr + i0);
      } else {  // zero padding columns I .. Ipad
        bf16_t tmp[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) tmp[e] = i0 + e < d.I ? sr[i0 + e] : (bf16_t)0;
        v = *(const uint4*)tmp;
      }
      const int o = bm.y + rr;
      bf16_t* dst = (bf16_t*)d.dst + (d.dst_ld ? (long long)o * d.dst_ld : (long long)o * row);
      *(uint4*)(dst + qq * 8) = v;
    }
    return;
  }
#pragma unroll 1
  for (int o = bm.y; o < o_end; ++o) {
    const float* src = d.src + (long long)o * d.so;
    switch (taps) {  // constant divisors for the common tap counts
      case 1: pack_gather<1>(d, src, st, ld, taps); break;
      case 4: pack_gather<4>(d, src, st, ld, taps); break;
      case 9: pack_gather<9>(d, src, st, ld, taps); break;
      case 16: pack_gather<16>(d, src, st, ld, taps); break;
      default: pack_gather<0>(d, src, st, ld, taps); break;
    }
    __syncthreads();
    bf16_t* dst = (bf16_t*)d.dst + (d.dst_ld ? (long long)o * d.dst_ld : (long long)o * row);
    for (int q = threadIdx.x; q < row / 8; q += NT) {
      const int t = (q * 8) / d.Ipad, i0 = q * 8 - t * d.Ipad;
      uint4 v;
      if (i0 + 8 <= d.I) {
        v = *(const uint4*)(st + t * ld + i0);
      } else {  // zero padding columns I .. Ipad
        bf16_t tmp[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) tmp[e] = i0 + e < d.I ? st[t * ld + i0 + e] : (bf16_t)0;
        v = *(const uint4*)tmp;
      }
      *(uint4*)(dst + q * 8) = v;
    }
    __syncthreads();
  }
}
// dst[i][t][o] = src[o][smap[t]][i] over 64 x 64 tiles staged in LDS: 16-byte loads of src rows, 16-byte stores of
// dst rows (each gathered from one LDS column).
__global__ __launch_bounds__(NT) void pack_transpose_kernel(const sdmi_tpack_desc* descs, const int4* bmap) {
  __shared__ __attribute__((aligned(16))) bf16_t t[64][72];  // [o][i]
  const int4 bm = bmap[blockIdx.x];
  const sdmi_tpack_desc& d = descs[bm.x];
  const int i0 = bm.y, o0 = bm.z, tap = bm.w;
  const bf16_t* src = (const bf16_t*)d.src + (long long)d.smap[tap] * d.src_tap;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + k * NT;  // 64 rows x 8 chunks
    const int r = q >> 3, c = (q & 7) * 8;
    const int o = o0 + r, i = i0 + c;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (o < d.O && i < d.I) v = *(const uint4*)(src + (long long)o * d.src_ld + i);
    *(uint4*)&t[r][c] = v;
  }
  __syncthreads();
  bf16_t* dst = (bf16_t*)d.dst + (long long)tap * d.dst_tap;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + k * NT;  // 64 dst rows (i) x 8 chunks of o
    const int r = q >> 3, c = (q & 7) * 8;
    const int i = i0 + r, o = o0 + c;
    if (i >= d.I || o >= d.O) continue;
    bf16_t w[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) w[e] = t[c + e][r];
    *(uint4*)(dst + (long long)i * d.dst_ld + o) = *(const uint4*)w;
  }
}
}  // namespace

extern "C" int sdmi_pack_transpose(const sdmi_tpack_desc* descs_dev, const void* bmap_dev, int nblocks,
                                   sdmi_stream_t stream) {
  if (nblocks <= 0) return 0;
  sdmi_rt::launch(pack_transpose_kernel, dim3(nblocks), dim3(NT), 0, (hipStream_t)stream, descs_dev,
                     (const int4*)bmap_dev);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_prep_input(const float* x, int B, int cx, int H, int W, const float* mask, int cmi, int MH, int MW,
                               const float* wcond, int cmo, void* out, int cpad, const float* keep,
                               sdmi_stream_t stream) {
  if (cpad % 8 || cx + (mask ? cmo : 0) > cpad || cpad > 16) return -1;
  sdmi_rt::launch(prep_input_kernel<false>, dim3(prep_grid((long long)B * H * W)), dim3(PREP_NT), 0, (hipStream_t)stream, x,
                     B, cx, H, W, mask, cmi, MH, MW, wcond, cmo, (bf16_t*)out, cpad, keep);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_prep_input_cmap(const float* x, int B, int cx, int H, int W, const unsigned char* cmap, int cmi,
                                    int MH, int MW, const float* wcond, int cmo, void* out, int cpad, const float* keep,
                                    sdmi_stream_t stream) {
  if (cpad % 8 || cx + (cmap ? cmo : 0) > cpad || cpad > 16 || cmi < 1 || cmi > 255) return -1;
  sdmi_rt::launch(prep_input_kernel<true>, dim3(prep_grid((long long)B * H * W)), dim3(PREP_NT), 0, (hipStream_t)stream, x,
                     B, cx, H, W, cmap, cmi, MH, MW, wcond, cmo, (bf16_t*)out, cpad, keep);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_cond_wgrad(const void* dxin, int ld, int cx, int B, int H, int W, const float* mask, int cmi,
                               int MH, int MW, int cmo, float* dw, const float* keep, sdmi_stream_t stream) {
  return launch_cond_wgrad<false>(dxin, ld, cx, B, H, W, mask, cmi, MH, MW, cmo, dw, keep, (hipStream_t)stream);
}

extern "C" int sdmi_cond_wgrad_cmap(const void* dxin, int ld, int cx, int B, int H, int W, const unsigned char* cmap,
                                    int cmi, int MH, int MW, int cmo, float* dw, const float* keep,
                                    sdmi_stream_t stream) {
  return launch_cond_wgrad<true>(dxin, ld, cx, B, H, W, cmap, cmi, MH, MW, cmo, dw, keep, (hipStream_t)stream);
}

extern "C" int sdmi_nhwc_to_nchw(const void* src, int src_f32, int ld, int B, int C, int HW, float* dst,
                                 sdmi_stream_t stream) {
  sdmi_rt::launch(nhwc_to_nchw_kernel, dim3(grid_for((long long)B * C * HW)), dim3(NT), 0, (hipStream_t)stream, src,
                     src_f32, ld, B, C, HW, dst);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_nchw_to_nhwc_bf16(const float* src, int B, int C, int HW, void* dst, int ld, sdmi_stream_t stream) {
  sdmi_rt::launch(nchw_to_nhwc_bf16_kernel, dim3(grid_for((long long)B * HW * ld)), dim3(NT), 0, (hipStream_t)stream,
                     src, B, C, HW, (bf16_t*)dst, ld);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_add_noise(const float* x0, const float* eps, const long long* t, const float* sqrt_abar,
                              const float* sqrt_one_minus_abar, int B, long long per_sample, float* out,
                              sdmi_stream_t stream) {
  sdmi_rt::launch(add_noise_kernel, dim3(grid_for((long long)B * per_sample)), dim3(NT), 0, (hipStream_t)stream, x0,
                     eps, t, sqrt_abar, sqrt_one_minus_abar, B, per_sample, out);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" size_t sdmi_mse_workspace(void) { return 1024 * sizeof(float); }

extern "C" int sdmi_mse(const float* pred, int ld, const float* target, int B, int C, int HW, float gscale,
                        const float* gscale_dev, void* grad, float* ws, float* loss, sdmi_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  int blocks = grid_for((long long)B * HW * ld);
  if (blocks > 1024) blocks = 1024;
  sdmi_rt::launch(mse_kernel, dim3(blocks), dim3(NT), 0, s, pred, ld, target, B, C, HW, gscale, gscale_dev,
                     (bf16_t*)grad, ws);
  SDMI_CHECK_LAUNCH();
  sdmi_rt::launch(sum_partials_kernel, dim3(1), dim3(NT), 0, s, ws, blocks, 1.0f / (float)((long long)B * C * HW),
                     loss);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_time_embedding(const long long* t, int tstride, int B, int dim, void* out, int ld, float* out_f32,
                                   sdmi_stream_t stream) {
  if (dim % 2) return -1;
  sdmi_rt::launch(time_embedding_kernel, dim3(grid_for((long long)B * dim / 2)), dim3(NT), 0, (hipStream_t)stream, t,
                     tstride, B, dim, (bf16_t*)out, ld, out_f32);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_silu(const void* x, const void* dy, void* y, long long n, sdmi_stream_t stream) {
  sdmi_rt::launch(silu_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, (const bf16_t*)x,
                     (const bf16_t*)dy, (bf16_t*)y, n);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_relu(const float* x, const float* dy, float* y, long long n, sdmi_stream_t stream) {
  if (!x || !y || n < 0) return -1;
  if (n == 0) return 0;
  sdmi_rt::launch(relu_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, x, dy, y, n);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_copy_slice(const void* src, int lds, void* dst, int ldd, long long P, int C, int accumulate,
                               sdmi_stream_t stream) {
  if (C % 8 || lds % 8 || ldd % 8) return -1;
  sdmi_rt::launch(copy_slice_kernel, dim3(grid_for(P * C / 8)), dim3(NT), 0, (hipStream_t)stream, (const bf16_t*)src,
                     lds, (bf16_t*)dst, ldd, P, C, accumulate);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_pack_chunk(void) { return PACK_CHUNK; }

// descs_dev: device array of descriptors; bmap_dev: device array of int2 (descriptor, chunk), one per workgroup
extern "C" int sdmi_pack_weights(const sdmi_pack_desc* descs_dev, const void* bmap_dev, int nblocks, sdmi_stream_t stream) {
  if (nblocks <= 0) return 0;
  sdmi_rt::launch(pack_kernel, dim3(nblocks), dim3(NT), PACK_LDS_ELEMS * sizeof(bf16_t), (hipStream_t)stream, descs_dev,
                     (const int2*)bmap_dev);
  SDMI_CHECK_LAUNCH();
  return 0;
}

