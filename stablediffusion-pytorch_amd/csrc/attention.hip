// Fused multi-head attention (flash-style) on MFMA 16x16x32 bf16 for gfx950.
//
// Replaces the core of torch nn.MultiheadAttention as the reference calls it (models/blocks.py:
// 83, 94, 128, 140; self- and cross-attention, need_weights=True path): softmax(q k^T / sqrt(d)) v
// per head, without materialising the (B*H, N, S) probability tensor. Head dims of the cond-UNet
// are 8..48 (16 heads over 128..768 channels); the contraction over d is zero-padded to DP = 32 or
// 64, the output d is covered by ceil(d/16) MFMA row tiles. Softmax statistics are fp32.
//
// Layout: Q/K/V/O are row-major [batch*len][ld] bf16 with head h at columns h*d .. h*d+d-1 (the
// packed in-projection output is used in place: q, k, v are column offsets of one buffer).
//
// Forward  : per (b, h, 64-query tile), 4 waves x 16 queries, keys streamed through LDS in 64-key
//            tiles. "Swapped" product S^T = K Q^T puts the query on the lane, so the softmax
//            row statistics are per lane and P^T feeds the PV MFMA directly from the accumulator
//            registers (keys permuted consistently in both operands; V read with ds_read_b64_tr_b16).
// Backward : two kernels, no atomics:
//            dkv: per (b, h, 64-key tile), keys on the lane (S = Q K^T): dV^T += dO^T P, dK^T += Q^T dS
//            dq : per (b, h, 64-query tile), queries on the lane (S^T = K Q^T): dQ^T += K^T dS^T
//            with P recomputed from the forward's log-sum-exp and delta = rowsum(dO * O).
#include "common.h"
#include "../../include/sdmi.h"

namespace {

constexpr int TQ = 64, TK = 64, NT = 256;
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* o; const bf16_t* dout;
  bf16_t* out; bf16_t* dq; bf16_t* dk; bf16_t* dv;
  float* lse;        // [B*H][N]  base-2 log-sum-exp of (score * scale * log2e)
  const float* delta; // [B*H][N]
  int ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv;
  int B, H, N, S, d;
  float scale;       // 1/sqrt(d)
};

// LDS tile [64 rows][DP + 8] bf16 (row padded by 16 B)
template <int DP> struct Tile {
  static constexpr int LD = DP + 8;
  static constexpr int BYTES = 64 * LD * 2;
};

// load a 64-row x DP-col tile of head columns [col0, col0 + d) (zero outside rows < nrows, cols < d)
template <int DP>
__device__ __forceinline__ void load_tile(bf16_t* t, const bf16_t* src, int ld, int row0, int nrows, int col0, int d) {
  constexpr int CPR = DP / 8;  // 16-B chunks per row
  for (int c = threadIdx.x; c < 64 * CPR; c += NT) {
    int r = c / CPR, ch = c - r * CPR;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row0 + r < nrows && ch * 8 < d) v = *(const uint4*)(src + (long long)(row0 + r) * ld + col0 + ch * 8);
    *(uint4*)(t + r * Tile<DP>::LD + ch * 8) = v;
  }
}

// A/B fragment where the MFMA row index = tile row (16 rows from rbase), k = tile column (32 from kbase)
template <int DP>
__device__ __forceinline__ s16x8 frag_rows(const bf16_t* t, int rbase, int kbase, int lane) {
  return *(const s16x8*)(t + (rbase + (lane & 15)) * Tile<DP>::LD + kbase + (lane >> 4) * 8);
}

// transposed fragment: MFMA row index = tile column (16 cols from cbase), k = tile rows
// permuted as {rbase + 4g + j (j<4), rbase + 16 + 4g + j-4 (j>=4)} for lane group g = lane>>4.
template <int DP>
__device__ __forceinline__ s16x8 frag_tr(const bf16_t* t, int rbase, int cbase, int lane) {
  int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16_t* a1 = t + (rbase + 4 * g + q) * Tile<DP>::LD + cbase + 4 * p;
  const bf16_t* a2 = a1 + 16 * Tile<DP>::LD;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)a1);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)a2);
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// B-operand fragment from two accumulator tiles (rows = k): elements j<4 from a[j], j>=4 from b[j-4]
__device__ __forceinline__ s16x8 pack_acc(const f32x4& a, const f32x4& b) {
  s16x8 r;
  r[0] = (short)f2bf(a[0]); r[1] = (short)f2bf(a[1]); r[2] = (short)f2bf(a[2]); r[3] = (short)f2bf(a[3]);
  r[4] = (short)f2bf(b[0]); r[5] = (short)f2bf(b[1]); r[6] = (short)f2bf(b[2]); r[7] = (short)f2bf(b[3]);
  return r;
}

// per-lane register fragment of one row (16-row block on lanes): row = row0 + (lane&15), d = 8*(lane>>4) + 32*ks
template <int DP>
__device__ __forceinline__ void row_frags(s16x8 (&f)[DP / 32], const bf16_t* src, int ld, int row, int nrows, int col0, int d, int lane) {
#pragma unroll
  for (int ks = 0; ks < DP / 32; ++ks) {
    int dd = ks * 32 + (lane >> 4) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < nrows && dd < d) v = *(const uint4*)(src + (long long)row * ld + col0 + dd);
    f[ks] = __builtin_bit_cast(s16x8, v);
  }
}

// =============================================================================================
// forward
// =============================================================================================
template <int DP>
__global__ __launch_bounds__(NT) void attn_fwd_kernel(AttnArgs a) {
  constexpr int DT = DP / 16;  // max output row tiles (d <= DP)
  __shared__ __attribute__((aligned(16))) bf16_t sK[64 * Tile<DP>::LD];
  __shared__ __attribute__((aligned(16))) bf16_t sV[64 * Tile<DP>::LD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  const int q0 = blockIdx.x * TQ + wave * 16;
  const int myq = q0 + (lane & 15);
  const int dt_n = (a.d + 15) / 16;
  const float c = a.scale * LOG2E;

  const bf16_t* Q = a.q + (long long)b * a.N * a.ldq;
  const bf16_t* K = a.k + (long long)b * a.S * a.ldk;
  const bf16_t* V = a.v + (long long)b * a.S * a.ldv;
  s16x8 qf[DP / 32];
  row_frags<DP>(qf, Q, a.ldq, myq, a.N, h * a.d, a.d, lane);

  float m = -INFINITY, l = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < a.S; k0 += TK) {
    __syncthreads();
    load_tile<DP>(sK, K, a.ldk, k0, a.S, h * a.d, a.d);
    load_tile<DP>(sV, V, a.ldv, k0, a.S, h * a.d, a.d);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < DP / 32; ++ks)
        s[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<DP>(sK, kb * 16, ks * 32, lane), qf[ks], s[kb], 0, 0, 0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int key = k0 + kb * 16 + (lane >> 4) * 4 + i;
        float v = key < a.S ? s[kb][i] * c : -INFINITY;
        s[kb][i] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float mn = fmaxf(m, mx);
    float alpha = exp2f(m - mn);
    m = mn;
    l *= alpha;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] *= alpha;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float p = exp2f(s[kb][i] - mn);
        s[kb][i] = p;
        l += p;
      }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s16x8 pf = pack_acc(s[2 * s2], s[2 * s2 + 1]);
#pragma unroll
      for (int t = 0; t < DT; ++t)
        if (t < dt_n) o[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<DP>(sV, 32 * s2, 16 * t, lane), pf, o[t], 0, 0, 0);
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (myq < a.N) {
    float inv = 1.f / l;
    bf16_t* O = a.out + ((long long)b * a.N + myq) * a.ldo + h * a.d;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      int d0 = 16 * t + (lane >> 4) * 4;
      if (t < dt_n && d0 < a.d) {
        uint2 w;
        w.x = pack2bf(o[t][0] * inv, o[t][1] * inv);
        w.y = pack2bf(o[t][2] * inv, o[t][3] * inv);
        *(uint2*)(O + d0) = w;
      }
    }
    if ((lane >> 4) == 0) a.lse[(long long)bh * a.N + myq] = m + __log2f(l);
  }
}

// delta[bh][q] = sum_d dO[q][h*d + .] * O[q][h*d + .]   (one wave per query row segment)
__global__ void attn_delta_kernel(AttnArgs a) {
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // (b, q, h)
  long long total = (long long)a.B * a.N * a.H;
  if (idx >= total) return;
  int h = idx % a.H;
  long long bq = idx / a.H;
  int q = bq % a.N;
  int b = bq / a.N;
  const bf16_t* O = a.o + bq * a.ldo + h * a.d;
  const bf16_t* dO = a.dout + bq * a.lddo + h * a.d;
  float s = 0.f;
  for (int j = 0; j < a.d; j += 8) {
    float x[8], y[8];
    unpack8(*(const uint4*)(O + j), x);
    unpack8(*(const uint4*)(dO + j), y);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += x[e] * y[e];
  }
  ((float*)a.delta)[((long long)b * a.H + h) * a.N + q] = s;
}

// =============================================================================================
// backward: dK, dV (keys on lanes)
// =============================================================================================
template <int DP>
__global__ __launch_bounds__(NT) void attn_bwd_dkv_kernel(AttnArgs a) {
  constexpr int DT = DP / 16;
  __shared__ __attribute__((aligned(16))) bf16_t sQ[64 * Tile<DP>::LD];
  __shared__ __attribute__((aligned(16))) bf16_t sO[64 * Tile<DP>::LD];  // dO tile
  __shared__ float sL[64], sD[64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  const int kk0 = blockIdx.x * TK + wave * 16;
  const int mykey = kk0 + (lane & 15);
  const int dt_n = (a.d + 15) / 16;
  const float c = a.scale * LOG2E;

  const bf16_t* Q = a.q + (long long)b * a.N * a.ldq;
  const bf16_t* dO = a.dout + (long long)b * a.N * a.lddo;
  s16x8 kf[DP / 32], vf[DP / 32];
  row_frags<DP>(kf, a.k + (long long)b * a.S * a.ldk, a.ldk, mykey, a.S, h * a.d, a.d, lane);
  row_frags<DP>(vf, a.v + (long long)b * a.S * a.ldv, a.ldv, mykey, a.S, h * a.d, a.d, lane);

  f32x4 dk[DT], dv[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) { dk[t] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[t] = dk[t]; }

  for (int q0 = 0; q0 < a.N; q0 += TQ) {
    __syncthreads();
    load_tile<DP>(sQ, Q, a.ldq, q0, a.N, h * a.d, a.d);
    load_tile<DP>(sO, dO, a.lddo, q0, a.N, h * a.d, a.d);
    if (threadIdx.x < 64) {
      int q = q0 + threadIdx.x;
      sL[threadIdx.x] = q < a.N ? a.lse[(long long)bh * a.N + q] : INFINITY;
      sD[threadIdx.x] = q < a.N ? a.delta[(long long)bh * a.N + q] : 0.f;
    }
    __syncthreads();
    f32x4 p[4], ds[4];
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
      f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f}, dp = s;
#pragma unroll
      for (int ks = 0; ks < DP / 32; ++ks) {
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<DP>(sQ, qb * 16, ks * 32, lane), kf[ks], s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<DP>(sO, qb * 16, ks * 32, lane), vf[ks], dp, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int qi = qb * 16 + (lane >> 4) * 4 + i;  // row within tile; invalid rows have lse = +inf -> p = 0
        float pv = exp2f(s[i] * c - sL[qi]);
        p[qb][i] = pv;
        ds[qb][i] = pv * (dp[i] - sD[qi]);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s16x8 pf = pack_acc(p[2 * s2], p[2 * s2 + 1]);
      s16x8 df = pack_acc(ds[2 * s2], ds[2 * s2 + 1]);
#pragma unroll
      for (int t = 0; t < DT; ++t)
        if (t < dt_n) {
          dv[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<DP>(sO, 32 * s2, 16 * t, lane), pf, dv[t], 0, 0, 0);
          dk[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<DP>(sQ, 32 * s2, 16 * t, lane), df, dk[t], 0, 0, 0);
        }
    }
  }
  if (mykey < a.S) {
    bf16_t* DK = a.dk + ((long long)b * a.S + mykey) * a.lddk + h * a.d;
    bf16_t* DV = a.dv + ((long long)b * a.S + mykey) * a.lddv + h * a.d;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      int d0 = 16 * t + (lane >> 4) * 4;
      if (t < dt_n && d0 < a.d) {
        uint2 w;
        w.x = pack2bf(dk[t][0] * a.scale, dk[t][1] * a.scale);
        w.y = pack2bf(dk[t][2] * a.scale, dk[t][3] * a.scale);
        *(uint2*)(DK + d0) = w;
        w.x = pack2bf(dv[t][0], dv[t][1]);
        w.y = pack2bf(dv[t][2], dv[t][3]);
        *(uint2*)(DV + d0) = w;
      }
    }
  }
}

// =============================================================================================
// backward: dQ (queries on lanes)
// =============================================================================================
template <int DP>
__global__ __launch_bounds__(NT) void attn_bwd_dq_kernel(AttnArgs a) {
  constexpr int DT = DP / 16;
  __shared__ __attribute__((aligned(16))) bf16_t sK[64 * Tile<DP>::LD];
  __shared__ __attribute__((aligned(16))) bf16_t sV[64 * Tile<DP>::LD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  const int q0 = blockIdx.x * TQ + wave * 16;
  const int myq = q0 + (lane & 15);
  const int dt_n = (a.d + 15) / 16;
  const float c = a.scale * LOG2E;

  const bf16_t* K = a.k + (long long)b * a.S * a.ldk;
  const bf16_t* V = a.v + (long long)b * a.S * a.ldv;
  s16x8 qf[DP / 32], of[DP / 32];
  row_frags<DP>(qf, a.q + (long long)b * a.N * a.ldq, a.ldq, myq, a.N, h * a.d, a.d, lane);
  row_frags<DP>(of, a.dout + (long long)b * a.N * a.lddo, a.lddo, myq, a.N, h * a.d, a.d, lane);
  const bool qok = myq < a.N;
  const float lse = qok ? a.lse[(long long)bh * a.N + myq] : INFINITY;
  const float dlt = qok ? a.delta[(long long)bh * a.N + myq] : 0.f;

  f32x4 dq[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) dq[t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < a.S; k0 += TK) {
    __syncthreads();
    load_tile<DP>(sK, K, a.ldk, k0, a.S, h * a.d, a.d);
    load_tile<DP>(sV, V, a.ldv, k0, a.S, h * a.d, a.d);
    __syncthreads();
    f32x4 ds[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f}, dp = s;
#pragma unroll
      for (int ks = 0; ks < DP / 32; ++ks) {
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<DP>(sK, kb * 16, ks * 32, lane), qf[ks], s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_rows<DP>(sV, kb * 16, ks * 32, lane), of[ks], dp, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int key = k0 + kb * 16 + (lane >> 4) * 4 + i;
        float pv = key < a.S ? exp2f(s[i] * c - lse) : 0.f;
        ds[kb][i] = pv * (dp[i] - dlt);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s16x8 df = pack_acc(ds[2 * s2], ds[2 * s2 + 1]);
#pragma unroll
      for (int t = 0; t < DT; ++t)
        if (t < dt_n) dq[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<DP>(sK, 32 * s2, 16 * t, lane), df, dq[t], 0, 0, 0);
    }
  }
  if (qok) {
    bf16_t* DQ = a.dq + ((long long)b * a.N + myq) * a.lddq + h * a.d;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      int d0 = 16 * t + (lane >> 4) * 4;
      if (t < dt_n && d0 < a.d) {
        uint2 w;
        w.x = pack2bf(dq[t][0] * a.scale, dq[t][1] * a.scale);
        w.y = pack2bf(dq[t][2] * a.scale, dq[t][3] * a.scale);
        *(uint2*)(DQ + d0) = w;
      }
    }
  }
}

int check_args(const AttnArgs& a) {
  if (a.B <= 0 || a.H <= 0 || a.N <= 0 || a.S <= 0 || a.d <= 0) return -1;
  if (a.d % 8 || a.d > 64) return -2;
  return 0;
}

}  // namespace

extern "C" int sdmi_attn_fwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                             void* out, int ldo, float* lse, int B, int H, int N, int S, int d,
                             sdmi_stream_t stream) {
  AttnArgs a = {};
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.out = (bf16_t*)out; a.lse = lse;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
  a.B = B; a.H = H; a.N = N; a.S = S; a.d = d; a.scale = 1.0f / sqrtf((float)d);
  int rc = check_args(a);
  if (rc) return rc;
  dim3 grid((N + TQ - 1) / TQ, B * H);
  hipStream_t s = (hipStream_t)stream;
  if (d <= 32) hipLaunchKernelGGL(attn_fwd_kernel<32>, grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(NT), 0, s, a);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_attn_bwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                             const void* o, int ldo, const void* dout, int lddo, const float* lse,
                             float* delta_ws, void* dq, int lddq, void* dk, int lddk, void* dv, int lddv,
                             int B, int H, int N, int S, int d, sdmi_stream_t stream) {
  AttnArgs a = {};
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (const bf16_t*)o;
  a.dout = (const bf16_t*)dout; a.lse = (float*)lse; a.delta = delta_ws;
  a.dq = (bf16_t*)dq; a.dk = (bf16_t*)dk; a.dv = (bf16_t*)dv;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo; a.lddo = lddo; a.lddq = lddq; a.lddk = lddk; a.lddv = lddv;
  a.B = B; a.H = H; a.N = N; a.S = S; a.d = d; a.scale = 1.0f / sqrtf((float)d);
  int rc = check_args(a);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  long long rows = (long long)B * N * H;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, a);
  SDMI_CHECK_LAUNCH();
  dim3 gk((S + TK - 1) / TK, B * H), gq((N + TQ - 1) / TQ, B * H);
  if (d <= 32) {
    hipLaunchKernelGGL(attn_bwd_dkv_kernel<32>, gk, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<32>, gq, dim3(NT), 0, s, a);
  } else {
    hipLaunchKernelGGL(attn_bwd_dkv_kernel<64>, gk, dim3(NT), 0, s, a);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<64>, gq, dim3(NT), 0, s, a);
  }
  SDMI_CHECK_LAUNCH();
  return 0;
}
