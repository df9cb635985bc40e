// GroupNorm (+ fused SiLU) forward/backward and per-(batch, channel) pixel reductions on NHWC bf16.
//
// Replaces nn.GroupNorm(32, C) -> nn.SiLU() (models/blocks.py:45-47, 64-66 and the Mid/Up copies),
// the attention pre-norms on the (B, C, HW) view (blocks.py:124-126, 137-139: same statistics as
// 4-D) and unet_cond_base.py:179-180. Statistics: fp32 per-thread / per-channel sums, fp64 group merge,
// eps 1e-5.
//
// All kernels see an activation as x[b][p][c] = x[(b*P + p)*ld + c], P = H*W pixels.
// Reductions run as ONE launch each: a workgroup owns a channel strip of one batch row (for GroupNorm a
// strip of whole groups) and reduces all of its pixels, so per-(b, c) and per-(b, g) results come out
// of the workgroup directly. Sums over the batch (dgamma/dbeta, bias gradients) are finished by the
// last-arriving workgroup of each strip: rows are published with device-coherent (sc1) stores and a
// relaxed device-scope arrival counter, so no L2 write-back fence is needed.
//   sdmi_gn_stats     : table {a = rstd*gamma, s = beta - mean*a, mean, rstd} per (b, c)
//   sdmi_gn_bwd       : (sum dz, sum dz*xhat) -> table2 {a, s, q, o} + dgamma/dbeta, then the apply pass
//   sdmi_chan_sum     : per-(b, c) and per-c sums of dy (bias / time-embedding gradients)
//   sdmi_gn_apply / gn_bwd_apply : vectorised elementwise passes (8 channels per lane).
#include <atomic>
#include <cstdlib>

#include "common.h"
#include "../../include/sdmi.h"

namespace {

constexpr int NT = 256;
constexpr int NSLOTS = 2048;      // counter slots, one per launch, round-robin
constexpr int SLOT_CTRS = 2048;   // [0, 1024): per (strip, b) pixel-split counters, [1024, 2048): per strip
constexpr int BATCH_CTR = 1024;
constexpr int PS_MAX = 32;        // pixel splits per (strip, b) (small batches of large images: VQVAE B = 8 at 256^2)
__device__ unsigned g_norm_counters[NSLOTS * SLOT_CTRS];  // zero at load; the last arriver re-arms

struct StripArgs {
  const bf16_t* x; int ldx;   // GN input (modes 0, 1)
  const bf16_t* dy; int ldy;  // upstream gradient (modes 1, 2)
  const float4* tab;          // mode 1: forward table
  int B, P, C, G, CW, silu;
  float eps;
  const float* gamma; const float* beta;
  float4* out_tab;            // mode 0: table, mode 1: table2
  float* rows;                // [nb][C][2] per-row sums for the batch tail (sc1 stores)
  float* part;                // [nb][psplit][C][2] pixel-split partials (sc1 stores)
  unsigned* ctr;              // [nchunks] arrival counters
  float* sum1; float* sum2;   // batch tail outputs: mode 1 dbeta/dgamma, mode 2 per_c/per_c2
  bf16_t* per_bc; int ld_bc;  // mode 2
  int c_store;
  long long seg;              // mode 2: rows per (virtual) batch row; 0 = P
  int nb;                     // batch rows (virtual for mode 2)
  int rows_only;              // GroupNorm backward: publish the per-(b, c) sums to rows, no batch tail
};

__device__ __forceinline__ void st_coherent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_coherent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// true in every thread of the workgroup that arrives last among n at *ctr (which it re-arms)
__device__ __forceinline__ bool arrive_last(unsigned* ctr, int n) {
  __shared__ int flag;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's coherent row stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (unsigned)(n - 1);
    if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = last;
  }
  __syncthreads();
  if (flag) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // acquire before reading the other arrivals' rows
  return flag != 0;
}

// Per-channel sums over rows [row0, row0 + nrows) of the strip [c0, c0 + cw) -> s1[cw], s2[cw] in LDS.
// mode 0: (x, x^2); mode 1: (dz, dz*xhat) with dz = dy [* silu'(x*a + s)]; mode 2: (dy, -).
template <int MODE>
__device__ __forceinline__ void strip_reduce(const StripArgs& a, int b, long long row0, long long nrows, int c0, int cw,
                                             float* s1, float* s2) {
  __shared__ float red[NT][17];
  const int L = cw >> 3;            // lanes per pixel row
  const int R = NT / L;             // pixel rows per iteration
  const int t = threadIdx.x;
  const int lane = t % L, r = t / L;
  const int cc = c0 + lane * 8;
  float u[8], v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { u[e] = 0.f; v[e] = 0.f; }
  float4 tb[8];
  if (MODE == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) tb[e] = r < R ? a.tab[(long long)b * a.C + cc + e] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (r < R && nrows > 0) {
    // rows in batches of RB: the batch's loads are issued together from clamped (valid) rows and masked after, so
    // each thread keeps RB (x2 in mode 1) 16-byte loads in flight instead of one row per round trip
    constexpr int RB = MODE == 1 ? 4 : 8;
    for (long long p0 = r; p0 < nrows; p0 += (long long)RB * R) {
      uint4 rx[RB], rg[RB];
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        const long long row = row0 + min(p0 + (long long)q * R, nrows - 1);
        if (MODE != 2) rx[q] = *(const uint4*)(a.x + row * a.ldx + cc);
        if (MODE != 0) rg[q] = *(const uint4*)(a.dy + row * a.ldy + cc);
      }
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        if (p0 + (long long)q * R >= nrows) break;
        float xv[8], gv[8];
        if (MODE == 0) {
          unpack8(rx[q], xv);
#pragma unroll
          for (int e = 0; e < 8; ++e) { u[e] += xv[e]; v[e] = fmaf(xv[e], xv[e], v[e]); }
        } else if (MODE == 1) {
          unpack8(rx[q], xv);
          unpack8(rg[q], gv);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float dz = gv[e];
            if (a.silu) dz *= silu_grad_f(fmaf(xv[e], tb[e].x, tb[e].y));
            u[e] += dz;
            v[e] = fmaf(dz, (xv[e] - tb[e].z) * tb[e].w, v[e]);
          }
        } else {
          unpack8(rg[q], gv);
#pragma unroll
          for (int e = 0; e < 8; ++e) u[e] += gv[e];
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[t][e] = u[e]; red[t][8 + e] = v[e]; }
  __syncthreads();
  for (int ch = t; ch < cw; ch += NT) {
    const int l = ch >> 3, e = ch & 7;
    float x1 = 0.f, x2 = 0.f;
    for (int rr = 0; rr < R; ++rr) {
      x1 += red[rr * L + l][e];
      x2 += red[rr * L + l][8 + e];
    }
    s1[ch] = x1;
    s2[ch] = x2;
  }
  __syncthreads();
}

// Last strip of a batch column: out1[c] = sum_b rows[b][c][0], out2[c] = sum_b rows[b][c][1] for the strip.
__device__ __forceinline__ void batch_tail(const StripArgs& a, int c0, int cw, float* o1, float* o2, int c_store,
                                           bool dup = false) {
  __shared__ float acc[NT][2];
  const int t = threadIdx.x;
  const int nthr = min((int)blockDim.x, NT);  // the single-pass kernels run 64 .. 1024 threads
  if (cw > nthr) {  // narrow workgroup, wide strip: one thread per channel, all batch rows in order
    for (int ch = t; ch < cw; ch += blockDim.x) {
      float x1 = 0.f, x2 = 0.f;
      // 16 rows' coherent loads in flight before they are summed (in row order): one cross-XCD round trip per 16
      // rows instead of one per row
      for (int b0 = 0; b0 < a.nb; b0 += 16) {
        float r1[16], r2[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int b = min(b0 + u, a.nb - 1);
          const float* rp = a.rows + ((long long)b * a.C + c0 + ch) * 2;
          r1[u] = ld_coherent(rp);
          r2[u] = ld_coherent(rp + 1);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          if (b0 + u < a.nb) {
            x1 += r1[u];
            x2 += r2[u];
          }
        }
      }
      const int c = c0 + ch;
      if (c < c_store) {
        if (o1) o1[c] = x1;
        if (o2) o2[c] = dup ? x1 : x2;
      }
    }
    return;
  }
  const int nbg = max(1, nthr / cw);
  const int ch = t % cw, bg = t / cw;
  float x1 = 0.f, x2 = 0.f;
  if (t < nthr && bg < nbg && t < nbg * cw) {
    // issue 16 rows' coherent loads before summing them: the sum then waits once per batch of loads instead of
    // once per load (a dependent chain of cross-XCD round trips otherwise)
    for (int b0 = bg; b0 < a.nb; b0 += 16 * nbg) {
      float r1[16], r2[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int b = min(b0 + u * nbg, a.nb - 1);
        const float* rp = a.rows + ((long long)b * a.C + c0 + ch) * 2;
        r1[u] = ld_coherent(rp);
        r2[u] = ld_coherent(rp + 1);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if (b0 + u * nbg < a.nb) {
          x1 += r1[u];
          x2 += r2[u];
        }
      }
    }
  }
  if (t < nthr) {
    acc[t][0] = x1;
    acc[t][1] = x2;
  }
  __syncthreads();
  if (t < cw) {
    float y1 = 0.f, y2 = 0.f;
    for (int g = 0; g < nbg; ++g) {
      y1 += acc[g * cw + t][0];
      y2 += acc[g * cw + t][1];
    }
    const int c = c0 + t;
    if (c < c_store) {
      if (o1) o1[c] = y1;
      if (o2) o2[c] = dup ? y1 : y2;
    }
  }
}

// Pixel-split combine: with gridDim.z > 1 every workgroup publishes its strip sums and the last of the
// (strip, b) group continues with the complete sums in s1/s2; the others return false.
__device__ __forceinline__ bool combine_psplits(const StripArgs& a, int b, int c0, int cw, float* s1, float* s2) {
  const int nz = gridDim.z;
  if (nz == 1) return true;
  float* mine = a.part + (((long long)b * nz + blockIdx.z) * a.C + c0) * 2;
  for (int ch = threadIdx.x; ch < cw; ch += NT) {
    st_coherent(mine + 2 * ch, s1[ch]);
    st_coherent(mine + 2 * ch + 1, s2[ch]);
  }
  if (!arrive_last(a.ctr + blockIdx.x * gridDim.y + b, nz)) return false;
  for (int ch = threadIdx.x; ch < cw; ch += NT) {
    float x1 = 0.f, x2 = 0.f;
    const float* pp = a.part + ((long long)b * nz * a.C + c0 + ch) * 2;
    // splits in batches of 8: a batch's loads are in flight together, the sum stays in split order (deterministic)
    for (int z0 = 0; z0 < nz; z0 += 8) {
      float r1[8], r2[8];
#pragma unroll
      for (int z = 0; z < 8; ++z) {
        const int zz = min(z0 + z, nz - 1);
        r1[z] = ld_coherent(pp + (long long)zz * a.C * 2);
        r2[z] = ld_coherent(pp + (long long)zz * a.C * 2 + 1);
      }
#pragma unroll
      for (int z = 0; z < 8; ++z) {
        if (z0 + z < nz) {
          x1 += r1[z];
          x2 += r2[z];
        }
      }
    }
    s1[ch] = x1;
    s2[ch] = x2;
  }
  __syncthreads();
  return true;
}

__device__ __forceinline__ void pixel_range(long long n, long long& p0, long long& p1) {
  const long long per = (n + gridDim.z - 1) / gridDim.z;
  p0 = blockIdx.z * per;
  p1 = min(n, p0 + per);
  if (p1 < p0) p1 = p0;
}

// grid (nchunks, B): GroupNorm statistics of whole groups -> forward table
__global__ __launch_bounds__(NT) void gn_stats_kernel(StripArgs a) {
  __shared__ float s1[NT], s2[NT];
  __shared__ float2 grp[NT];
  const int b = blockIdx.y;
  const int c0 = blockIdx.x * a.CW;
  const int cw = min(a.CW, a.C - c0);
  const int Cg = a.C / a.G;
  long long p0, p1;
  pixel_range(a.P, p0, p1);
  strip_reduce<0>(a, b, (long long)b * a.P + p0, p1 - p0, c0, cw, s1, s2);
  if (!combine_psplits(a, b, c0, cw, s1, s2)) return;
  const int ng = cw / Cg;
  if ((int)threadIdx.x < ng) {
    double m1 = 0, m2 = 0;
    for (int c = threadIdx.x * Cg; c < (int)(threadIdx.x + 1) * Cg; ++c) {
      m1 += s1[c];
      m2 += s2[c];
    }
    const double n = (double)a.P * Cg;
    const double mu = m1 / n;
    double var = m2 / n - mu * mu;
    if (var < 0) var = 0;
    grp[threadIdx.x] = make_float2((float)mu, (float)(1.0 / sqrt(var + (double)a.eps)));
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < cw; ch += NT) {
    const int c = c0 + ch;
    const float2 mr = grp[ch / Cg];
    const float sc = mr.y * a.gamma[c];
    a.out_tab[(long long)b * a.C + c] = make_float4(sc, a.beta[c] - mr.x * sc, mr.x, mr.y);
  }
}

// grid (nchunks, B): GroupNorm backward coefficients -> table2 {a, s, q, o}; dgamma/dbeta by the batch tail.
// dx = rstd*(dz*gamma - A/n - xhat*Bc/n) = a*dz + q*x + o with q = -rstd^2 Bc/n, o = rstd^2 mean Bc/n - rstd A/n
__global__ __launch_bounds__(NT) void gn_bwd_reduce_kernel(StripArgs a) {
  __shared__ float s1[NT], s2[NT];
  __shared__ float2 grp[NT];
  const int b = blockIdx.y;
  const int c0 = blockIdx.x * a.CW;
  const int cw = min(a.CW, a.C - c0);
  const int Cg = a.C / a.G;
  long long p0, p1;
  pixel_range(a.P, p0, p1);
  strip_reduce<1>(a, b, (long long)b * a.P + p0, p1 - p0, c0, cw, s1, s2);
  if (!combine_psplits(a, b, c0, cw, s1, s2)) return;
  const int ng = cw / Cg;
  const float inv_n = 1.0f / ((float)a.P * Cg);
  if ((int)threadIdx.x < ng) {
    float A = 0.f, Bc = 0.f;
    for (int ch = threadIdx.x * Cg; ch < (int)(threadIdx.x + 1) * Cg; ++ch) {
      A += a.gamma[c0 + ch] * s1[ch];
      Bc += a.gamma[c0 + ch] * s2[ch];
    }
    const float4 t = a.tab[(long long)b * a.C + c0 + threadIdx.x * Cg];
    const float r = t.w, mu = t.z;
    grp[threadIdx.x] = make_float2(-r * r * Bc * inv_n, r * r * mu * Bc * inv_n - r * A * inv_n);
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < cw; ch += NT) {
    const int c = c0 + ch;
    const float4 t = a.tab[(long long)b * a.C + c];
    const float2 qo = grp[ch / Cg];
    a.out_tab[(long long)b * a.C + c] = make_float4(t.x, t.y, qo.x, qo.y);
    if (a.sum1 || a.rows_only) {
      float* rp = a.rows + ((long long)b * a.C + c) * 2;
      st_coherent(rp, s1[ch]);
      st_coherent(rp + 1, s2[ch]);
    }
  }
  if (!a.sum1) return;
  if (!arrive_last(a.ctr + BATCH_CTR + blockIdx.x, a.nb)) return;
  batch_tail(a, c0, cw, a.sum1, a.sum2, a.C);
}

// grid (nchunks, nb): per-(row, c) sums of dy -> per_bc (bf16), per-c sums by the batch tail
__global__ __launch_bounds__(NT) void chan_sum_kernel(StripArgs a) {
  __shared__ float s1[NT], s2[NT];
  const int b = blockIdx.y;
  const int c0 = blockIdx.x * a.CW;
  const int cw = min(a.CW, a.C - c0);
  const long long total = (long long)a.B * a.P;
  const long long row0 = (long long)b * a.seg;
  const long long nrows = max(0LL, min(a.seg, total - row0));
  long long p0, p1;
  pixel_range(nrows, p0, p1);
  strip_reduce<2>(a, b, row0 + p0, p1 - p0, c0, cw, s1, s2);
  if (!combine_psplits(a, b, c0, cw, s1, s2)) return;
  const bool tail = a.sum1 || a.sum2;
  for (int ch = threadIdx.x; ch < cw; ch += NT) {
    const int c = c0 + ch;
    if (a.per_bc) a.per_bc[(long long)b * a.ld_bc + c] = f2bf(s1[ch]);
    if (tail) {
      float* rp = a.rows + ((long long)b * a.C + c) * 2;
      st_coherent(rp, s1[ch]);
      st_coherent(rp + 1, 0.f);
    }
  }
  if (!tail) return;
  if (!arrive_last(a.ctr + BATCH_CTR + blockIdx.x, a.nb)) return;
  batch_tail(a, c0, cw, a.sum1, a.sum2, a.c_store, /*dup=*/true);  // per_c2: a second bias with the same gradient
}

// ---------------------------------------------------------------------------------------------
// Single-pass GroupNorm: one workgroup (NTH = 256 or 1024 threads) owns a (batch row, channel strip of whole
// groups), keeps its P x strip slab in registers as packed bf16 (small_it(NTH) rows per thread), reduces, and applies
// -- one launch and one read of x (and dy) instead of a statistics pass, a cross-workgroup combine and a second
// elementwise pass. 256 threads cover P <= 256 (16x16 and smaller levels), 1024 threads P <= 1024 (32x32).
// ---------------------------------------------------------------------------------------------
// pixel rows per thread: P <= small_it(NTH) * (NTH / (strip/8)); 8 for the 1024-thread form keeps its x and dy
// slabs (64 VGPRs) within the 128 VGPRs a 16-wave workgroup allows (32x32 levels with 64-channel strips)
__host__ __device__ constexpr int small_it(int nth) { return nth == 1024 ? 8 : 10; }

__host__ __device__ __forceinline__ int small_rows(int cw, int nth = NT) { return nth / (cw >> 3); }

// per-channel sums of u (and v) over the workgroup's rows -> s1/s2[cw] in LDS (red: [NTH][17] scratch), in two
// fixed-order stages so no thread sums more than ~8 + NTH / cw partials: (1) thread j sums a contiguous segment of
// ~8 rows of channel j % cw (segment j / cw), (2) one thread per channel sums the segments
template <int NTH>
__device__ __forceinline__ void small_reduce(const float* u, const float* v, int cw, float (*red)[17], float* s1,
                                             float* s2) {
  __shared__ float seg[NTH][2];
  const int t = threadIdx.x, L = cw >> 3, R = NTH / L;
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[t][e] = u[e]; red[t][8 + e] = v[e]; }
  __syncthreads();
  const int S = max(1, min(R, NTH / cw));  // segments per channel
  const int RS = (R + S - 1) / S;          // rows per segment
  for (int j = t; j < S * cw; j += NTH) {  // S * cw <= NTH unless the strip is wider than the workgroup (S = 1)
    const int ch = j % cw, sg = j / cw, l = ch >> 3, e = ch & 7;
    const int r1 = min(R, (sg + 1) * RS);
    float x1 = 0.f, x2 = 0.f;
    for (int rr = sg * RS; rr < r1; ++rr) {
      x1 += red[rr * L + l][e];
      x2 += red[rr * L + l][8 + e];
    }
    if (S > 1) {
      seg[j][0] = x1;
      seg[j][1] = x2;
    } else {
      s1[ch] = x1;
      s2[ch] = x2;
    }
  }
  __syncthreads();
  if (S == 1) return;
  for (int ch = t; ch < cw; ch += NTH) {
    float x1 = 0.f, x2 = 0.f;
    for (int sg = 0; sg < S; ++sg) {
      x1 += seg[sg * cw + ch][0];
      x2 += seg[sg * cw + ch][1];
    }
    s1[ch] = x1;
    s2[ch] = x2;
  }
  __syncthreads();
}

// (strip, batch row) of a single-pass workgroup on an (nchunks, B) grid, XCD-aware: workgroups are dispatched
// round-robin over the 8 XCDs (dispatch id d on XCD d % 8, one 4 MiB L2 each); the logical ids are re-numbered so
// every XCD owns a contiguous band, strips fastest -- the narrow strips that share the 128-B lines of one batch row's
// pixel rows then read them through ONE L2 instead of up to eight (bijective for any grid size)
__device__ __forceinline__ void strip_block(int& strip, int& b) {
  const int total = gridDim.x * gridDim.y;
  const int d = blockIdx.y * gridDim.x + blockIdx.x;
  const int xcd = d & 7, q = total >> 3, r = total & 7;
  const int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (d >> 3);
  b = l / gridDim.x;
  strip = l - b * gridDim.x;
}

// grid (nchunks, B): y = act(GroupNorm(x)), and the forward table for the backward pass. NTH threads, IT pixel rows
// per thread (P <= IT * (NTH / (strip / 8)))
template <int NTH, int IT>
__global__ __launch_bounds__(NTH) void gn_fwd_pass_kernel(StripArgs a, bf16_t* y, int ldy) {
  __shared__ float red[NTH][17];
  __shared__ float s1[NT], s2[NT];
  __shared__ float2 grp[NT];
  int strip, b;
  strip_block(strip, b);
  const int c0 = strip * a.CW, cw = min(a.CW, a.C - c0);
  const int L = cw >> 3, R = NTH / L, t = threadIdx.x, lane = t % L, r = t / L;
  const int cc = c0 + lane * 8, Cg = a.C / a.G;
  const bool act = r < R;
  float u[8], v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { u[e] = 0.f; v[e] = 0.f; }
  const bf16_t* X = a.x + (long long)b * a.P * a.ldx + cc;
  // every row load issued first from a clamped (valid) row, masked afterwards: a guarded load per row would make
  // the compiler wait for each one before the next
  constexpr int SMALL_IT = IT;
  uint4 rx[SMALL_IT];
#pragma unroll
  for (int it = 0; it < SMALL_IT; ++it) {
    const int p = min(min(r, R - 1) + it * R, a.P - 1);
    rx[it] = *(const uint4*)(X + (long long)p * a.ldx);
  }
#pragma unroll
  for (int it = 0; it < SMALL_IT; ++it) {
    float xv[8];
    unpack8(rx[it], xv);
    if (act && r + it * R < a.P) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { u[e] += xv[e]; v[e] = fmaf(xv[e], xv[e], v[e]); }
    }
  }
  small_reduce<NTH>(u, v, cw, red, s1, s2);
  const int ng = cw / Cg;
  for (int gi = t; gi < ng; gi += NTH) {
    double m1 = 0, m2 = 0;
    for (int c = gi * Cg; c < (gi + 1) * Cg; ++c) { m1 += s1[c]; m2 += s2[c]; }
    const double n = (double)a.P * Cg, mu = m1 / n;
    double var = m2 / n - mu * mu;
    if (var < 0) var = 0;
    grp[gi] = make_float2((float)mu, (float)(1.0 / sqrt(var + (double)a.eps)));
  }
  __syncthreads();
  for (int ch = t; ch < cw; ch += NTH) {
    const int c = c0 + ch;
    const float2 mr = grp[ch / Cg];
    const float sc = mr.y * a.gamma[c];
    a.out_tab[(long long)b * a.C + c] = make_float4(sc, a.beta[c] - mr.x * sc, mr.x, mr.y);
  }
  if (!act) return;
  float ta[8], ts[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float2 mr = grp[(lane * 8 + e) / Cg];
    ta[e] = mr.y * a.gamma[cc + e];
    ts[e] = a.beta[cc + e] - mr.x * ta[e];
  }
  bf16_t* Y = y + (long long)b * a.P * ldy + cc;
#pragma unroll
  for (int it = 0; it < SMALL_IT; ++it) {
    const int p = r + it * R;
    if (p < a.P) {
      float xv[8], o[8];
      unpack8(rx[it], xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float z = fmaf(xv[e], ta[e], ts[e]);
        o[e] = a.silu ? silu_f(z) : z;
      }
      *(uint4*)(Y + (long long)p * ldy) = pack8(o);
    }
  }
}

// grid (nchunks, B): GroupNorm (+SiLU) backward in one pass; dgamma/dbeta by the batch tail. x (and, for the
// 256-thread form, dy) stay packed in registers; the 1024-thread form re-reads dy in the apply pass (an L2 hit:
// the workgroup read it moments before) to stay within 128 VGPRs; dz = dy * SiLU'(...) is recomputed there.
template <int NTH, int IT>
__global__ __launch_bounds__(NTH) void gn_bwd_pass_kernel(StripArgs a, bf16_t* dx, int lddx, const bf16_t* add,
                                                          int ldadd) {
  __shared__ float red[NTH][17];
  __shared__ float s1[NT], s2[NT];
  __shared__ float2 grp[NT];
  __shared__ float4 stb[NT];  // forward table of the strip
  int strip, b;
  strip_block(strip, b);
  const int c0 = strip * a.CW, cw = min(a.CW, a.C - c0);
  const int L = cw >> 3, R = NTH / L, t = threadIdx.x, lane = t % L, r = t / L;
  const int cc = c0 + lane * 8, Cg = a.C / a.G;
  const bool act = r < R;
  const long long rb = (long long)b * a.P;
  constexpr int SMALL_IT = IT;
  constexpr bool KEEP_DY = IT <= 4 || NTH <= 256;  // else dy is re-read in the apply pass (VGPR budget)
  // IT <= 4: dz = dy * SiLU'(x a + s) of the reduction pass is kept (fp32) for the apply pass instead of being
  // recomputed there (the SiLU derivative is an exp + a reciprocal per element: ~1/3 of the kernel's VALU work)
  constexpr bool KEEP_DZ = KEEP_DY && IT <= 4;
  float dzk[KEEP_DZ ? SMALL_IT * 8 : 1];
  uint4 rx[SMALL_IT], rg[SMALL_IT];  // all row loads in flight first
#pragma unroll
  for (int it = 0; it < SMALL_IT; ++it) {
    const int p = min(min(r, R - 1) + it * R, a.P - 1);
    rx[it] = *(const uint4*)(a.x + (rb + p) * a.ldx + cc);
    rg[it] = *(const uint4*)(a.dy + (rb + p) * a.ldy + cc);
  }
  for (int ch = t; ch < cw; ch += NTH) stb[ch] = a.tab[(long long)b * a.C + c0 + ch];
  __syncthreads();
  float u[8], v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { u[e] = 0.f; v[e] = 0.f; }
#pragma unroll
  for (int it = 0; it < SMALL_IT; ++it) {
    float xv[8], gv[8];
    unpack8(rx[it], xv);
    unpack8(rg[it], gv);
    if (act && r + it * R < a.P) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float4 tb = stb[lane * 8 + e];
        float dz = gv[e];
        if (a.silu) dz *= silu_grad_f(fmaf(xv[e], tb.x, tb.y));
        if constexpr (KEEP_DZ) dzk[it * 8 + e] = dz;
        u[e] += dz;
        v[e] = fmaf(dz, (xv[e] - tb.z) * tb.w, v[e]);
      }
    }
  }
  small_reduce<NTH>(u, v, cw, red, s1, s2);
  const int ng = cw / Cg;
  const float inv_n = 1.0f / ((float)a.P * Cg);
  for (int gi = t; gi < ng; gi += NTH) {
    float A = 0.f, Bc = 0.f;
    for (int ch = gi * Cg; ch < (gi + 1) * Cg; ++ch) {
      A += a.gamma[c0 + ch] * s1[ch];
      Bc += a.gamma[c0 + ch] * s2[ch];
    }
    const float4 tt = stb[gi * Cg];
    const float rs = tt.w, mu = tt.z;
    grp[gi] = make_float2(-rs * rs * Bc * inv_n, rs * rs * mu * Bc * inv_n - rs * A * inv_n);
  }
  if (a.sum1 || a.rows_only) {
    for (int ch = t; ch < cw; ch += NTH) {
      float* rp = a.rows + ((long long)b * a.C + c0 + ch) * 2;
      st_coherent(rp, s1[ch]);
      st_coherent(rp + 1, s2[ch]);
    }
  }
  __syncthreads();
  if (act) {
#pragma unroll
    for (int it = 0; it < SMALL_IT; ++it) {
      const int p = r + it * R;
      if (p < a.P) {
        float xv[8], gv[8], av[8], ov[8];
        unpack8(rx[it], xv);
        if constexpr (KEEP_DZ) {
#pragma unroll
          for (int e = 0; e < 8; ++e) gv[e] = dzk[it * 8 + e];
        } else if (KEEP_DY) {
          unpack8(rg[it], gv);
        } else {
          unpack8(*(const uint4*)(a.dy + (rb + p) * a.ldy + cc), gv);
        }
        if (add) {
          unpack8(*(const uint4*)(add + (rb + p) * ldadd + cc), av);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) av[e] = 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float4 tb = stb[lane * 8 + e];
          const float2 qo = grp[(lane * 8 + e) / Cg];
          float dz = gv[e];
          if (!KEEP_DZ && a.silu) dz *= silu_grad_f(fmaf(xv[e], tb.x, tb.y));
          ov[e] = av[e] + fmaf(tb.x, dz, fmaf(qo.x, xv[e], qo.y));
        }
        *(uint4*)(dx + (rb + p) * lddx + cc) = pack8(ov);
      }
    }
  }
  if (!a.sum1) return;
  if (!arrive_last(a.ctr + BATCH_CTR + strip, a.nb)) return;
  batch_tail(a, c0, cw, a.sum1, a.sum2, a.C);
}

int strip_width(int C, int unit);

// Single-pass launch shape: strip width (whole groups, 8-channel lanes), threads per workgroup, pixel rows per thread.
struct PassCfg {
  int cw, nth, it;
};

// Occupancy-first choice: the widest strip that still gives >= 512 workgroups (2 per CU, measured best of 512 / 1024 /
// 2048; narrow strips share 128-B lines with their neighbours, which strip_block() keeps on one XCD), else the
// narrowest strip; per strip the fewest threads with <= 4 pixel rows each (loads in flight per thread), else <= 8.
bool pick_pass(int B, int P, int C, int G, PassCfg& pc) {
  const int Cg = C / G;
  // 32x32 and larger images (P >= 1024): 256 workgroups of wider strips measured better in isolation (32^2 C=384
  // fwd 19.7 -> 15.2 us, bwd 35.1 -> 33.7 us; C=128 bwd 18.2 -> 16.6 us; others equal), smaller images keep 512
  const int target = P >= 1024 ? 256 : 512;
  int u = Cg;
  while (u % 8) u += Cg;
  static const int NTHS[] = {64, 256, 512, 1024};
  PassCfg good = {0, 0, 0}, any = {0, 0, 0};
  long long any_wg = 0;
  for (int cw = u; cw <= NT && cw - u < C; cw += u) {
    const int L = cw / 8;
    PassCfg c = {0, 0, 0};
    for (int lim : {4, 8}) {
      for (int nth : NTHS) {
        const int R = nth / L;
        if (R == 0) continue;
        const int it = (P + R - 1) / R;
        if (it <= lim) {
          c = {cw, nth, it <= 1 ? 1 : it <= 2 ? 2 : it <= 4 ? 4 : 8};
          break;
        }
      }
      if (c.nth) break;
    }
    if (!c.nth) continue;
    const long long wg = (long long)((C + cw - 1) / cw) * B;
    if (wg >= target) good = c;  // widest so far with enough workgroups (cw ascends)
    if (wg > any_wg) {
      any = c;
      any_wg = wg;
    }
  }
  const PassCfg best = good.nth ? good : any;
  if (!best.nth || (C + best.cw - 1) / best.cw > BATCH_CTR) return false;
  pc = best;
  return true;
}

template <int NTH>
void launch_pass_it(bool bwd, int it, dim3 grid, hipStream_t s, const StripArgs& a, bf16_t* out, int ldo,
                    const bf16_t* add, int ldadd) {
#define SDMI_GN_PASS(IT)                                                                                  \
  if (bwd) sdmi_rt::launch(gn_bwd_pass_kernel<NTH, IT>, grid, dim3(NTH), 0, s, a, out, ldo, add, ldadd); \
  else sdmi_rt::launch(gn_fwd_pass_kernel<NTH, IT>, grid, dim3(NTH), 0, s, a, out, ldo);                 \
  return;
  switch (it) {
    case 1: SDMI_GN_PASS(1)
    case 2: SDMI_GN_PASS(2)
    case 4: SDMI_GN_PASS(4)
    case 8: SDMI_GN_PASS(8)
    default:
      if constexpr (NTH == 256) { SDMI_GN_PASS(10) }
  }
#undef SDMI_GN_PASS
}

void launch_pass(bool bwd, const PassCfg& pc, dim3 grid, hipStream_t s, const StripArgs& a, bf16_t* out, int ldo,
                 const bf16_t* add = nullptr, int ldadd = 0) {
  switch (pc.nth) {
    case 64: launch_pass_it<64>(bwd, pc.it, grid, s, a, out, ldo, add, ldadd); break;
    case 256: launch_pass_it<256>(bwd, pc.it, grid, s, a, out, ldo, add, ldadd); break;
    case 512: launch_pass_it<512>(bwd, pc.it, grid, s, a, out, ldo, add, ldadd); break;
    default: launch_pass_it<1024>(bwd, pc.it, grid, s, a, out, ldo, add, ldadd); break;
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

// Elementwise passes: grid (C/64 strips, B, pixel splits); a thread owns 8 channels of one strip for
// all of its pixels, so its table entries are loaded once and stay in registers.
constexpr int APPLY_CW = 64;

__device__ __forceinline__ void apply_coords(const ApplyArgs& a, int& cc, int& r, int& p0, int& p1, bool& on) {
  const int lane = threadIdx.x & 7;
  r = threadIdx.x >> 3;  // 32 pixel rows per iteration
  cc = blockIdx.x * APPLY_CW + lane * 8;
  const int per = (a.P + gridDim.z - 1) / gridDim.z;
  p0 = blockIdx.z * per;
  p1 = min(a.P, p0 + per);
  on = cc < a.C;
}

// y = act(x*a + s)
__global__ __launch_bounds__(NT) void gn_apply_kernel(ApplyArgs a) {
  int cc, r, p0, p1;
  bool on;
  apply_coords(a, cc, r, p0, p1, on);
  if (!on) return;
  const int b = blockIdx.y;
  float ta[8], ts[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float4 t = a.tab[(long long)b * a.C + cc + e];
    ta[e] = t.x;
    ts[e] = t.y;
  }
  const bf16_t* X = a.x + (long long)b * a.P * a.ldx + cc;
  bf16_t* Y = a.y + (long long)b * a.P * a.ldy + cc;
#pragma unroll 4
  for (int p = p0 + r; p < p1; p += NT / 8) {
    float xv[8], yv[8];
    unpack8(*(const uint4*)(X + (long long)p * a.ldx), xv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float z = fmaf(xv[e], ta[e], ts[e]);
      yv[e] = a.silu ? silu_f(z) : z;
    }
    *(uint4*)(Y + (long long)p * a.ldy) = pack8(yv);
  }
}

// dx = a*dz + q*x + o (+ addend), dz = dy [* silu'(x*a + s)]
__global__ __launch_bounds__(NT) void gn_bwd_apply_kernel(ApplyArgs a) {
  int cc, r, p0, p1;
  bool on;
  apply_coords(a, cc, r, p0, p1, on);
  if (!on) return;
  const int b = blockIdx.y;
  float4 tb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) tb[e] = a.tab[(long long)b * a.C + cc + e];
  const long long rb = (long long)b * a.P;
#pragma unroll 2
  for (int p = p0 + r; p < p1; p += NT / 8) {
    const long long row = rb + p;
    float xv[8], gv[8], ov[8], av[8];
    unpack8(*(const uint4*)(a.x + row * a.ldx + cc), xv);
    unpack8(*(const uint4*)(a.dy + row * a.lddy + cc), gv);
    if (a.add) {
      unpack8(*(const uint4*)(a.add + row * a.ldadd + cc), av);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float dz = gv[e];
      if (a.silu) dz *= silu_grad_f(fmaf(xv[e], tb[e].x, tb[e].y));
      ov[e] = av[e] + fmaf(tb[e].x, dz, fmaf(tb[e].z, xv[e], tb[e].w));
    }
    *(uint4*)(a.dx + row * a.lddx + cc) = pack8(ov);
  }
}

// s1[ch], s2[ch] (ch < cw <= NT) = the sums over the nseg segment partials {sum, sum2} of (batch row b, channel
// c0 + ch) for gn_bwd_part_kernel. Each thread loads two channels (16 B) of every SLN-th segment -- SLN = NT / (cw / 2)
// segment lanes (<= 4), all loads of a lane independent -- and the lanes are merged in lane order: a fixed summation
// order (deterministic) with nseg / SLN loads per thread instead of nseg.
__device__ __forceinline__ void part_sums(const float2* part, int b, int nseg, int C, int c0, int cw, float* s1,
                                          float* s2, float* p1, float* p2) {
  const int t = threadIdx.x, hc = cw >> 1, sln = min(NT / hc, 4), c2 = t % hc, sl = t / hc;
  if (sl < sln) {
    const float4* pp = (const float4*)(part + (long long)b * nseg * C + c0) + c2;
    const long long ld4 = C >> 1;
    float x1 = 0.f, x2 = 0.f, y1 = 0.f, y2 = 0.f;
#pragma unroll 8
    for (int j = sl; j < nseg; j += sln) {
      const float4 v = pp[(long long)j * ld4];
      x1 += v.x;
      x2 += v.y;
      y1 += v.z;
      y2 += v.w;
    }
    p1[sl * cw + 2 * c2] = x1;
    p2[sl * cw + 2 * c2] = x2;
    p1[sl * cw + 2 * c2 + 1] = y1;
    p2[sl * cw + 2 * c2 + 1] = y2;
  }
  __syncthreads();
  for (int c = t; c < cw; c += NT) {
    float a1 = 0.f, a2 = 0.f;
    for (int l = 0; l < sln; ++l) {
      a1 += p1[l * cw + c];
      a2 += p2[l * cw + c];
    }
    s1[c] = a1;
    s2[c] = a2;
  }
  __syncthreads();
}

// GroupNorm (+SiLU) backward from the producing GEMM's statistics (sdmi_gemm_desc::gn_part): grid (strips of whole
// groups, B, pixel splits). Every workgroup sums the P / rb segment partials of its (batch row, strip) in segment order
// (fp32, fixed order: deterministic), forms the group coefficients exactly as gn_bwd_pass_kernel does, and streams
// dx = a*dz + q*x + o (+ addend) over its pixel range -- one read of x, dy and the addend, one write of dx, no
// reduction phase. dgamma / dbeta: the pixel-split-0 workgroups publish their (b, c) sums and the last of the B
// arrivals per strip sums them (batch_tail).
__global__ __launch_bounds__(NT) void gn_bwd_part_kernel(StripArgs a, const float2* part, int rb, bf16_t* dx, int lddx,
                                                         const bf16_t* add, int ldadd) {
  __shared__ float s1[NT], s2[NT], q1[2 * NT], q2[2 * NT];
  __shared__ float2 grp[NT];
  __shared__ float4 stb[NT];
  const int strip = blockIdx.x, b = blockIdx.y;
  const int c0 = strip * a.CW, cw = min(a.CW, a.C - c0);
  const int t = threadIdx.x, Cg = a.C / a.G;
  for (int ch = t; ch < cw; ch += NT) stb[ch] = a.tab[(long long)b * a.C + c0 + ch];
  part_sums(part, b, a.P / rb, a.C, c0, cw, s1, s2, q1, q2);
  const int ng = cw / Cg;
  const float inv_n = 1.0f / ((float)a.P * Cg);
  for (int gi = t; gi < ng; gi += NT) {
    float A = 0.f, Bc = 0.f;
    for (int ch = gi * Cg; ch < (gi + 1) * Cg; ++ch) {
      A += a.gamma[c0 + ch] * s1[ch];
      Bc += a.gamma[c0 + ch] * s2[ch];
    }
    const float4 tt = stb[gi * Cg];
    const float rs = tt.w, mu = tt.z;
    grp[gi] = make_float2(-rs * rs * Bc * inv_n, rs * rs * mu * Bc * inv_n - rs * A * inv_n);
  }
  const bool publish = (a.sum1 || a.rows_only) && blockIdx.z == 0;
  if (publish) {
    for (int ch = t; ch < cw; ch += NT) {
      float* rp = a.rows + ((long long)b * a.C + c0 + ch) * 2;
      st_coherent(rp, s1[ch]);
      st_coherent(rp + 1, s2[ch]);
    }
  }
  __syncthreads();
  const int L = cw >> 3, R = NT / L, lane = t % L, r = t / L;
  if (r < R) {
    const int cc = c0 + lane * 8;
    float ta[8], tsv[8], tq[8], to[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float4 tb = stb[lane * 8 + e];
      const float2 qo = grp[(lane * 8 + e) / Cg];
      ta[e] = tb.x;
      tsv[e] = tb.y;
      tq[e] = qo.x;
      to[e] = qo.y;
    }
    const int per = (a.P + gridDim.z - 1) / gridDim.z;
    const int p0 = blockIdx.z * per, p1 = min(a.P, p0 + per);
    const long long rbase = (long long)b * a.P;
#pragma unroll 4
    for (int p = p0 + r; p < p1; p += R) {
      const long long row = rbase + p;
      float xv[8], gv[8], av[8], ov[8];
      unpack8(*(const uint4*)(a.x + row * a.ldx + cc), xv);
      unpack8(*(const uint4*)(a.dy + row * a.ldy + cc), gv);
      if (add) {
        unpack8(*(const uint4*)(add + row * ldadd + cc), av);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float dz = gv[e];
        if (a.silu) dz *= silu_grad_f(fmaf(xv[e], ta[e], tsv[e]));
        ov[e] = av[e] + fmaf(ta[e], dz, fmaf(tq[e], xv[e], to[e]));
      }
      *(uint4*)(dx + row * lddx + cc) = pack8(ov);
    }
  }
  if (!publish || !a.sum1) return;
  if (!arrive_last(a.ctr + BATCH_CTR + strip, a.nb)) return;
  batch_tail(a, c0, cw, a.sum1, a.sum2, a.C);
}

// grid of an elementwise pass: C/64 strips x B x pixel splits, >= ~2048 workgroups, >= 64 pixels each
dim3 apply_grid(int B, int P, int C) {
  const int strips = (C + APPLY_CW - 1) / APPLY_CW;
  int ps = 1;
  while ((long long)strips * B * ps < 2048 && P / (ps * 2) >= 64) ps *= 2;
  return dim3(strips, B, ps);
}


// Strip width: a multiple of `unit` (whole groups) and of 8 channels, at least 64 channels when C allows
// (narrower strips measured slower: 16-byte row segments coalesce poorly).
int strip_width(int C, int unit) {
  int cw = unit;
  while (cw % 8 || (cw < 64 && cw * 2 <= C)) cw += unit;
  while ((C + cw - 1) / cw > SLOT_CTRS) cw += unit;
  return cw;
}

// Strip width of the streaming gn_bwd_part_kernel: whole groups AND a multiple of 64 channels (128-B row segments, so no
// cache line is shared by two strips' workgroups), else the whole row -- e.g. C = 384 in 32 groups: 192, not 72
int part_strip_width(int C, int unit) {
  int cw = unit;
  while (cw % 64 && cw < C) cw += unit;
  if (cw > C || cw > NT) cw = strip_width(C, unit);
  return cw;
}

unsigned* counter_slot() {
  static std::atomic<unsigned> next{0};
  static unsigned* base[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!base[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_norm_counters)) != hipSuccess) return nullptr;
    base[dev] = (unsigned*)p;
  }
  return base[dev] + (size_t)(next.fetch_add(1) % NSLOTS) * SLOT_CTRS;
}

// pixel splits per (strip, batch row): aim for >= 512 workgroups with >= 128 pixels each
int pick_psplit(int nch, int nb, long long rows_per_b) {
  int ps = 1;
  if ((long long)nch * nb > BATCH_CTR) return 1;
  while ((long long)nch * nb * ps < 512 && rows_per_b / (ps * 2) >= 128 && ps < PS_MAX) ps *= 2;
  return ps;
}

float* part_base(float* ws, int nb, int C) { return ws + (size_t)(nb > 32 ? nb : 32) * C * 2; }

}  // namespace

extern "C" size_t sdmi_chan_reduce_workspace(int B, int P, int C) {
  (void)P;
  const size_t nb = B > 32 ? B : 32;
  return (nb + nb * PS_MAX) * C * 2 * sizeof(float);
}

// stats -> per-(b,c) table {a = rstd*gamma, s = beta - mean*a, mean, rstd} (fp32 float4 [B][C])
extern "C" int sdmi_gn_stats(const void* x, int ldx, int B, int P, int C, int G, float eps, const float* gamma,
                             const float* beta, float* ws, float* table, sdmi_stream_t stream) {
  if (C % 8 || G <= 0 || C % G) return -1;
  StripArgs a = {};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.B = B; a.P = P; a.C = C; a.G = G; a.eps = eps;
  a.gamma = gamma; a.beta = beta; a.out_tab = (float4*)table;
  a.CW = strip_width(C, C / G);
  const int nch = (C + a.CW - 1) / a.CW;
  if (a.CW > NT || nch > BATCH_CTR) return -2;
  const int ps = pick_psplit(nch, B, P);
  if (ps > 1) {
    a.part = part_base(ws, B, C);
    if (!(a.ctr = counter_slot())) return -4;
  }
  sdmi_rt::launch(gn_stats_kernel, dim3(nch, B, ps), dim3(NT), 0, (hipStream_t)stream, a);
  SDMI_CHECK_LAUNCH();
  return 0;
}

// stats + apply in one call: the single-pass kernel when the image is small, else gn_stats then gn_apply
extern "C" int sdmi_gn_fwd(const void* x, int ldx, void* y, int ldy, int B, int P, int C, int G, float eps,
                           const float* gamma, const float* beta, int silu, float* ws, float* table, sdmi_stream_t stream) {
  if (C % 8 || G <= 0 || C % G) return -1;
  PassCfg pc;
  if (pick_pass(B, P, C, G, pc)) {
    StripArgs a = {};
    a.x = (const bf16_t*)x; a.ldx = ldx; a.B = B; a.P = P; a.C = C; a.G = G; a.eps = eps; a.silu = silu;
    a.gamma = gamma; a.beta = beta; a.out_tab = (float4*)table; a.CW = pc.cw;
    launch_pass(false, pc, dim3((C + pc.cw - 1) / pc.cw, B), (hipStream_t)stream, a, (bf16_t*)y, ldy);
    SDMI_CHECK_LAUNCH();
    return 0;
  }
  int rc = sdmi_gn_stats(x, ldx, B, P, C, G, eps, gamma, beta, ws, table, stream);
  if (rc) return rc;
  return sdmi_gn_apply(x, ldx, y, ldy, table, B, P, C, silu, stream);
}

extern "C" int sdmi_gn_apply(const void* x, int ldx, void* y, int ldy, const float* table, int B, int P, int C,
                             int silu, sdmi_stream_t stream) {
  if (C % 8) return -1;
  ApplyArgs a = {};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.y = (bf16_t*)y; a.ldy = ldy;
  a.tab = (const float4*)table; a.B = B; a.P = P; a.C = C; a.silu = silu;
  sdmi_rt::launch(gn_apply_kernel, apply_grid(B, P, C), dim3(NT), 0, (hipStream_t)stream, a);
  SDMI_CHECK_LAUNCH();
  return 0;
}

// table: forward table from sdmi_gn_stats; table2_ws: float4 [B][C] scratch; ws: sdmi_chan_reduce_workspace
namespace {
// rows_out != null: the per-(batch row, channel) sums {sum dz, sum dz*xhat} go to rows_out [B][C][2] and dgamma / dbeta
// (which must be null) are left to sdmi_gn_rows_sum -- no batch tail on the launching stream
int gn_bwd_impl(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                const float* gamma, int B, int P, int C, int G, int silu, float* ws, float* table2_ws, float* dgamma,
                float* dbeta, float* rows_out, const void* addend, int ldadd, sdmi_stream_t stream) {
  if (C % 8 || G <= 0 || C % G) return -1;
  if ((dgamma == nullptr) != (dbeta == nullptr) || (rows_out && dgamma)) return -3;
  hipStream_t s = (hipStream_t)stream;
  StripArgs r = {};
  r.x = (const bf16_t*)x; r.ldx = ldx; r.dy = (const bf16_t*)dy; r.ldy = lddy; r.tab = (const float4*)table;
  r.B = B; r.P = P; r.C = C; r.G = G; r.silu = silu; r.gamma = gamma; r.out_tab = (float4*)table2_ws;
  r.rows = rows_out ? rows_out : ws; r.rows_only = rows_out != nullptr; r.nb = B; r.sum1 = dbeta; r.sum2 = dgamma;
  PassCfg pc;
  if (pick_pass(B, P, C, G, pc)) {  // single pass
    r.CW = pc.cw;
    if (dgamma && !(r.ctr = counter_slot())) return -4;
    launch_pass(true, pc, dim3((C + pc.cw - 1) / pc.cw, B), s, r, (bf16_t*)dx, lddx, (const bf16_t*)addend, ldadd);
    SDMI_CHECK_LAUNCH();
    return 0;
  }
  r.CW = strip_width(C, C / G);
  const int nch = (C + r.CW - 1) / r.CW;
  if (r.CW > NT || nch > BATCH_CTR) return -2;
  const int ps = pick_psplit(nch, B, P);
  r.part = part_base(ws, B, C);
  if ((dgamma || ps > 1) && !(r.ctr = counter_slot())) return -4;
  sdmi_rt::launch(gn_bwd_reduce_kernel, dim3(nch, B, ps), dim3(NT), 0, s, r);
  SDMI_CHECK_LAUNCH();
  ApplyArgs a = {};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.dy = (const bf16_t*)dy; a.lddy = lddy; a.dx = (bf16_t*)dx; a.lddx = lddx;
  a.tab = (const float4*)table2_ws; a.add = (const bf16_t*)addend; a.ldadd = ldadd;
  a.B = B; a.P = P; a.C = C; a.silu = silu;
  sdmi_rt::launch(gn_bwd_apply_kernel, apply_grid(B, P, C), dim3(NT), 0, s, a);
  SDMI_CHECK_LAUNCH();
  return 0;
}
}  // namespace

extern "C" int sdmi_gn_bwd(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                           const float* gamma, int B, int P, int C, int G, int silu, float* ws, float* table2_ws,
                           float* dgamma, float* dbeta, const void* addend, int ldadd, sdmi_stream_t stream) {
  return gn_bwd_impl(x, ldx, dy, lddy, dx, lddx, table, gamma, B, P, C, G, silu, ws, table2_ws, dgamma, dbeta, nullptr,
                     addend, ldadd, stream);
}

extern "C" int sdmi_gn_bwd_rows(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                                const float* gamma, int B, int P, int C, int G, int silu, float* ws, float* table2_ws,
                                float* rows, const void* addend, int ldadd, sdmi_stream_t stream) {
  if (!rows) return -1;
  return gn_bwd_impl(x, ldx, dy, lddy, dx, lddx, table, gamma, B, P, C, G, silu, ws, table2_ws, nullptr, nullptr, rows,
                     addend, ldadd, stream);
}

// GroupNorm backward from the dgrad GEMM's segment partials (sdmi_gemm_desc::gn_part, rb rows per segment)
namespace {
int gn_bwd_part_impl(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                     const float* gamma, int B, int P, int C, int G, int silu, const float* part, int rb, float* ws,
                     float* dgamma, float* dbeta, float* rows_out, const void* addend, int ldadd, sdmi_stream_t stream) {
  if (C % 8 || G <= 0 || C % G || B <= 0 || P <= 0 || rb <= 0 || P % rb || !part) return -1;
  if ((dgamma == nullptr) != (dbeta == nullptr) || (rows_out && dgamma)) return -3;
  if (ldx % 8 || lddy % 8 || lddx % 8 || (addend && ldadd % 8)) return -5;
  StripArgs r = {};
  r.x = (const bf16_t*)x; r.ldx = ldx; r.dy = (const bf16_t*)dy; r.ldy = lddy; r.tab = (const float4*)table;
  r.B = B; r.P = P; r.C = C; r.G = G; r.silu = silu; r.gamma = gamma;
  r.rows = rows_out ? rows_out : ws; r.rows_only = rows_out != nullptr; r.nb = B; r.sum1 = dbeta; r.sum2 = dgamma;
  r.CW = part_strip_width(C, C / G);
  const int nch = (C + r.CW - 1) / r.CW;
  if (r.CW > NT || nch > BATCH_CTR) return -2;
  if (dgamma && !(r.ctr = counter_slot())) return -4;
  // pixel splits: >= 1024 workgroups while every split keeps >= 64 pixels
  int ps = 1;
  while ((long long)nch * B * ps < 1024 && P / (ps * 2) >= 64) ps *= 2;
  sdmi_rt::launch(gn_bwd_part_kernel, dim3(nch, B, ps), dim3(NT), 0, (hipStream_t)stream, r, (const float2*)part, rb,
                  (bf16_t*)dx, lddx, (const bf16_t*)addend, ldadd);
  SDMI_CHECK_LAUNCH();
  return 0;
}

// dgamma[c] = sum_b rows[b][c][1], dbeta[c] = sum_b rows[b][c][0], batch rows in order (deterministic)
__global__ __launch_bounds__(NT) void gn_rows_sum_kernel(const float2* rows, int B, int C, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 8
  for (int b = 0; b < B; ++b) {
    const float2 v = rows[(long long)b * C + c];
    s1 += v.x;
    s2 += v.y;
  }
  dbeta[c] = s1;
  dgamma[c] = s2;
}

struct RowsGroup {
  sdmi_gn_rows_job j[SDMI_GN_ROWS_GROUP_MAX];
};

// blockIdx.y = job; the same per-channel batch-ordered sum as gn_rows_sum_kernel
__global__ __launch_bounds__(NT) void gn_rows_sum_grouped_kernel(const RowsGroup g) {
  const sdmi_gn_rows_job& J = g.j[blockIdx.y];
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= J.C) return;
  const float2* rows = (const float2*)J.rows;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 8
  for (int b = 0; b < J.B; ++b) {
    const float2 v = rows[(long long)b * J.C + c];
    s1 += v.x;
    s2 += v.y;
  }
  J.dbeta[c] = s1;
  J.dgamma[c] = s2;
}
}  // namespace

extern "C" int sdmi_gn_bwd_part(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, const float* table,
                                const float* gamma, int B, int P, int C, int G, int silu, const float* part, int rb,
                                float* ws, float* dgamma, float* dbeta, const void* addend, int ldadd,
                                sdmi_stream_t stream) {
  return gn_bwd_part_impl(x, ldx, dy, lddy, dx, lddx, table, gamma, B, P, C, G, silu, part, rb, ws, dgamma, dbeta,
                          nullptr, addend, ldadd, stream);
}

extern "C" int sdmi_gn_bwd_part_rows(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx,
                                     const float* table, const float* gamma, int B, int P, int C, int G, int silu,
                                     const float* part, int rb, float* ws, float* rows, const void* addend, int ldadd,
                                     sdmi_stream_t stream) {
  if (!rows) return -1;
  return gn_bwd_part_impl(x, ldx, dy, lddy, dx, lddx, table, gamma, B, P, C, G, silu, part, rb, ws, nullptr, nullptr,
                          rows, addend, ldadd, stream);
}

extern "C" int sdmi_gn_rows_sum(const float* rows, int B, int C, float* dgamma, float* dbeta, sdmi_stream_t stream) {
  if (!rows || !dgamma || !dbeta || B <= 0 || C <= 0 || ((uintptr_t)rows & 7)) return -1;
  sdmi_rt::launch(gn_rows_sum_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, (hipStream_t)stream, (const float2*)rows, B,
                  C, dgamma, dbeta);
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_gn_rows_sum_grouped(const sdmi_gn_rows_job* jobs, int njobs, sdmi_stream_t stream) {
  if (!jobs || njobs <= 0 || njobs > SDMI_GN_ROWS_GROUP_MAX) return -1;
  RowsGroup g = {};
  int cmax = 0;
  for (int i = 0; i < njobs; ++i) {
    const sdmi_gn_rows_job& J = jobs[i];
    if (!J.rows || !J.dgamma || !J.dbeta || J.B <= 0 || J.C <= 0 || ((uintptr_t)J.rows & 7)) return -1;
    g.j[i] = J;
    cmax = J.C > cmax ? J.C : cmax;
  }
  sdmi_rt::launch(gn_rows_sum_grouped_kernel, dim3((cmax + NT - 1) / NT, njobs), dim3(NT), 0, (hipStream_t)stream, g);
  SDMI_CHECK_LAUNCH();
  return 0;
}

// per-(b, c) and per-c sums of dy over pixels (bias and time-embedding-bias gradients)
extern "C" int sdmi_chan_sum(const void* dy, int lddy, int B, int P, int C, float* ws, void* per_bc, int ld_bc,
                             float* per_c, float* per_c2, int c_store, sdmi_stream_t stream) {
  if (c_store <= 0 || c_store > C) c_store = C;
  if (C % 8 || B <= 0 || P <= 0) return -1;
  StripArgs r = {};
  r.dy = (const bf16_t*)dy; r.ldy = lddy; r.B = B; r.P = P; r.C = C;
  r.per_bc = (bf16_t*)per_bc; r.ld_bc = ld_bc; r.c_store = c_store;
  r.sum1 = per_c; r.sum2 = per_c2; r.rows = ws;
  if (per_bc) {
    r.nb = B;
    r.seg = P;
  } else {  // only batch totals: cut the B*P rows into <= 32 contiguous segments of >= 64 rows
    const long long total = (long long)B * P;
    long long nb = total / 64;
    nb = nb < 1 ? 1 : (nb > 32 ? 32 : nb);
    r.seg = (total + nb - 1) / nb;
    r.nb = (int)((total + r.seg - 1) / r.seg);
  }
  r.CW = strip_width(C, 8);
  const int nch = (C + r.CW - 1) / r.CW;
  if (nch > BATCH_CTR || r.CW > NT) return -2;
  const int ps = pick_psplit(nch, r.nb, r.seg);
  r.part = part_base(ws, r.nb, C);
  if ((per_c || per_c2 || ps > 1) && !(r.ctr = counter_slot())) return -4;
  sdmi_rt::launch(chan_sum_kernel, dim3(nch, r.nb, ps), dim3(NT), 0, (hipStream_t)stream, r);
  SDMI_CHECK_LAUNCH();
  return 0;
}
