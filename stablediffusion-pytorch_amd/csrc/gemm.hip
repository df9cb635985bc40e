// MFMA bf16 GEMM family for gfx950 with implicit-GEMM convolution gathers.
//
// One kernel template covers every contraction of the denoiser step (reference aten calls:
// nn.Conv2d models/blocks.py:48-53,67-72,102-109; nn.ConvTranspose2d blocks.py:457-459;
// nn.Linear blocks.py:58-61,97 and MHA in/out projections blocks.py:83,94) in forward and
// backward:
//   conv fwd / dgrad : A = im2col(NHWC activation) [m=pixel][k=(tap,cin)],  B = packed weight [n][k]
//   conv wgrad       : A = dY^T (col-major),                               B = im2col(X) [k=pixel][n=(tap,cin)]
//   linear fwd/dgrad/wgrad : plain row/col-major operands.
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 MFMA 16x16x32 bf16 tiles.
// Operands are register-staged (so the conv gathers can zero-pad) into two LDS buffers:
//   "K-contiguous" tiles [128 rows][64 k] (A row-major / conv, B [n][k]) read with ds_read_b128,
//      16-B chunk c of row r stored at chunk (c ^ (r & 7))  -> conflict-free b128 fragment reads;
//   "MN-contiguous" tiles [64 k][128 cols] (A col-major, B [k][n]) read with ds_read_b64_tr_b16
//      (hardware transpose), chunk c of row r stored at c ^ (((r&3) | ((r>>1)&4)) << 1)
//      -> conflict-free transposed reads.
// Split-K (for the small-grid weight-gradient and deep low-resolution GEMMs) writes fp32 slabs that
// a second kernel reduces while applying the same epilogue.
#include <atomic>

#include "common.h"
#include "../../include/sdmi.h"
#include <string.h>
#include <algorithm>
#include <stdlib.h>
#include <type_traits>

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;  // 16 KiB per operand tile (both layouts)

struct Args {
  int M, N, K;
  const bf16_t* A; int lda;
  const bf16_t* B; int ldb;
  // gather geometry
  int ih, iw, cin, ldx, kw, sy, sx, oy0, ox0;
  FastDiv ohw_d, ow_d;  // GEMM pixel grid: pixel m -> (b, oy, ox) = (m / (oh*ow), (m % (oh*ow)) / ow, m % ow)
  int ktiles_per_split, nsplit;
  const bf16_t* A2; int lda2; int k_split;
  // reduction columns (col-major A only): B columns n >= n_x0 are synthesised instead of loaded -- column n_x0 is
  // all ones (C gets the row sums of A over k: a bias gradient), columns n_x0 + 8 + j are the indicator of
  // k / grp == j (C gets per-group row sums: the per-sample time-embedding gradient). 0 = none.
  int n_x0;
  FastDiv grp_d;
  // 1: row sums of A over k accumulated from the staged A chunks in VALU (bias gradient without the extra tile
  // column the synthesised-column path costs; used when no per-group sums are wanted)
  int rowsum;
  // implicit-im2col B (weight gradients, k = pixel): how a full k-tile of KBK consecutive pixels maps onto the output
  // grid, bit flags per staged depth (bits 0-1: KBK 64, bits 2-3: KBK 32). Form 1: the tile is KBK / ow whole rows of
  // one image (oh * ow % KBK == 0, KBK % ow == 0) -> image and first row are tile-uniform, each lane's row offset and
  // column are fixed; form 2: the tile is KBK / (oh * ow) whole images (KBK % (oh * ow) == 0) -> only the first image
  // is tile-uniform. Either way the per-piece gather needs no division (DMA kernel, issue_fast_b).
  int bfast;
  // grouped launch (sdmi_gemm_grouped): ngroups > 1 independent problems of one shape; the grid's z runs over
  // (problem, split) and problem p reads its operands from Ag[p] / Bg[p] (Ag[0] = A, Bg[0] = B)
  int ngroups;
  const bf16_t* Ag[SDMI_GEMM_GROUP_MAX];
  const bf16_t* Bg[SDMI_GEMM_GROUP_MAX];
  // the outputs of problem p (copies of EpiArgs::Cg / sum_g: indexed here, in the kernel-argument segment, so the
  // epilogue's local EpiArgs copy is never indexed dynamically -- that would put it in scratch)
  void* Cg[SDMI_GEMM_GROUP_MAX];
  float* sum_g[SDMI_GEMM_GROUP_MAX];
};

__device__ __forceinline__ void pixel_coords(const Args& g, int m, int& b, int& oy, int& ox) {
  b = (int)g.ohw_d.div((unsigned)m);
  const int r = m - b * g.ohw_d.d();
  oy = (int)g.ow_d.div((unsigned)r);
  ox = r - oy * g.ow_d.d();
}

// 8 synthesised B values (one 16-B chunk, columns [n, n + 8)) of the reduction columns at k (see Args::n_x0):
// bf16 1.0 where the column's indicator holds, 0 elsewhere and for k >= K
__device__ __forceinline__ uint4 reduction_cols(const Args& g, int n, int k) {
  uint4 r = make_uint4(0u, 0u, 0u, 0u);
  if (k >= g.K) return r;
  const int j = n - g.n_x0;
  const int d = j == 0 ? 0 : (int)g.grp_d.div((unsigned)k) - (j - 8);
  if (d < 0 || d >= 8) return r;
  const unsigned one = 0x3F80u << ((d & 1) * 16);  // bf16 1.0 in the low / high half of the 32-bit lane
  if ((d >> 1) == 0) r.x = one;
  else if ((d >> 1) == 1) r.y = one;
  else if ((d >> 1) == 2) r.z = one;
  else r.w = one;
  return r;
}

// epilogue parameters (a separate kernel argument keeps both structs small enough to stay in SGPRs)
struct EpiArgs {
  int M, N;
  void* C; int ldc; int c_f32; long long split_stride;
  const float* bias; const float* bias2; const bf16_t* rowbias; int rb_ld;
  const bf16_t* resid; int ldr;
  float alpha; int act;
  int remap, r_oh, r_ow, r_sy, r_sx, r_oy, r_ox;
  // output-row grid of the GEMM: rows per sample (the rowbias row divisor, and gh * gw of a remap) and the remap's
  // grid width gw (fill_args rejects a remap whose rowbias divisor differs)
  FastDiv pix_d, gw_d;
  int perm, p_cin, p_taps, p_cvalid;
  unsigned p_magic;   // ceil(2^32 / p_cin): tap = umulhi(col, p_magic), exact for col < 2^32 / p_cin
  unsigned n8_magic;  // ceil(2^32 / (N / 8)) for the reducer's row split (0: N / 8 == 1)
  int m_store, n_store;
  int raw;  // 1: write raw fp32 partials (split-K) to ws, epilogue applied by the reducer
  int nsplit;
  const float* ws;  // split-K slabs [nsplit][M][N]
  int vec;          // LDS-staged 16-B row stores (no column permute, 8-aligned columns/strides)
  int n8;           // N % 8 == 0: split-K slabs are written / read as 16-B rows even when !vec
  int rb_mod;       // rowbias row = (row / rb_div) % rb_mod when > 0 (per-token tables, e.g. position embedding)
  const bf16_t* aux; int ld_aux;  // act 3: ReLU-gradient mask source (aux[orow*ld_aux + col] > 0)
  // reduction columns (Args::n_x0): column n_x0 -> sum_out[row] (and sum_out2), column n_x0 + 8 + j (j < ngrp)
  // -> gsum[j * gsum_ld + row] (bf16); rows < m_store only
  int n_x0, ngrp, gsum_ld;
  float* sum_out;
  float* sum_out2;
  bf16_t* gsum;
  int n_gemm;  // columns the MFMA tiles produce (N, or N plus the synthesised reduction columns); with split-K the
               // slab row width N is n_gemm + 8 when the VALU row sums ride along in slab column n_x0 = n_gemm
  // grouped launch: problem p stores to Cg[p] / sum_g[p], its split-K slabs start p * ws_gstride floats into ws
  void* Cg[SDMI_GEMM_GROUP_MAX];
  float* sum_g[SDMI_GEMM_GROUP_MAX];
  long long ws_gstride;
  // GroupNorm-backward statistics (sdmi_gemm_desc::gn_part): per gn_rb-row segment and column, sum dz and dz*xhat
  const bf16_t* gn_x; int gn_ldx;
  const float4* gn_tab;
  float* gn_part;
  int gn_rb, gn_silu;
  FastDiv gn_pd;  // rows per sample
  int gn_sl;      // split-K reducer: slab lanes of splitk_reduce_n8_kernel for the same launch (same summation order)
};

// the epilogue arguments of problem p of a grouped launch (C / sum read from the kernel-argument segment)
__device__ __forceinline__ void group_epi(EpiArgs& e, void* C, float* sum, int p) {
  e.C = C;
  e.sum_out = sum;
  e.ws += (long long)p * e.ws_gstride;
}

__device__ __forceinline__ long long rb_row(const EpiArgs& g, int row) {
  long long r = g.pix_d.div((unsigned)row);
  return g.rb_mod > 0 ? r % g.rb_mod : r;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int CPOL_SC1 = 16;  // buffer cache policy: device (agent) scope coherence

__device__ __forceinline__ int kc_off(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }
__device__ __forceinline__ int tr_swz(int r) { return ((r & 3) | ((r >> 1) & 4)) << 1; }
__device__ __forceinline__ int tr_off(int r, int c) { return r * 256 + ((c ^ tr_swz(r)) << 4); }

// activation of the epilogue: 1 SiLU, 2 ReLU, 3 ReLU gradient (keep v where aux > 0)
__device__ __forceinline__ float act1(const EpiArgs& g, float v, long long orow, int col) {
  if (g.act == 1) return silu_f(v);
  if (g.act == 2) return fmaxf(v, 0.f);
  if (g.act == 3) return bf2f(g.aux[orow * g.ld_aux + col]) > 0.f ? v : 0.f;
  return v;
}

struct Epi {
  // reduction columns [col, col + nv) of one row (raw sums: no alpha / bias / activation)
  __device__ __forceinline__ static void extra(const EpiArgs& g, int row, int col, const float* v, int nv) {
    if (row >= g.m_store) return;
    for (int q = 0; q < nv; ++q) {
      const int j = col + q - g.n_x0;
      if (j == 0) {
        if (g.sum_out) g.sum_out[row] = v[q];
        if (g.sum_out2) g.sum_out2[row] = v[q];
      } else if (j >= 8 && j - 8 < g.ngrp && g.gsum) {
        g.gsum[(long long)(j - 8) * g.gsum_ld + row] = f2bf(v[q]);
      }
    }
  }

  // v already holds alpha*acc + bias + bias2
  __device__ __forceinline__ static void finish(const EpiArgs& g, int row, int col, float v) {
    if (g.rowbias) v += bf2f(g.rowbias[rb_row(g, row) * g.rb_ld + col]);
    long long orow = row;
    if (g.remap) {
      const int b = (int)g.pix_d.div((unsigned)row);
      const int rr = row - b * g.pix_d.d();
      const int oy = (int)g.gw_d.div((unsigned)rr);
      const int ox = rr - oy * g.gw_d.d();
      orow = ((long long)b * g.r_oh + oy * g.r_sy + g.r_oy) * g.r_ow + ox * g.r_sx + g.r_ox;
    }
    if (g.resid) v += bf2f(g.resid[orow * g.ldr + col]);
    v = act1(g, v, orow, col);
    long long ocol = col;
    if (g.perm) {
      int tap = (int)__umulhi((unsigned)col, g.p_magic);
      int c = col - tap * g.p_cin;
      if (c >= g.p_cvalid) return;
      ocol = g.perm == 2 ? (long long)tap * g.p_cvalid + c : (long long)c * g.p_taps + tap;
    }
    if (g.c_f32) ((float*)g.C)[orow * g.ldc + ocol] = v;
    else ((bf16_t*)g.C)[orow * g.ldc + ocol] = f2bf(v);
  }

  // 8 consecutive columns [col, col+8) of one row, acc values in v (alpha/bias not yet applied)
  __device__ __forceinline__ static void finish8(const EpiArgs& g, int row, int col, float* v) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= g.alpha;
    if (g.bias) {
      const float4 b0 = *(const float4*)(g.bias + col), b1 = *(const float4*)(g.bias + col + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
    if (g.bias2) {
      const float4 b0 = *(const float4*)(g.bias2 + col), b1 = *(const float4*)(g.bias2 + col + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
    if (g.rowbias) {
      float t[8];
      unpack8(*(const uint4*)(g.rowbias + rb_row(g, row) * g.rb_ld + col), t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    long long orow = row;
    if (g.remap) {
      const int b = (int)g.pix_d.div((unsigned)row);
      const int rr = row - b * g.pix_d.d();
      const int oy = (int)g.gw_d.div((unsigned)rr);
      const int ox = rr - oy * g.gw_d.d();
      orow = ((long long)b * g.r_oh + oy * g.r_sy + g.r_oy) * g.r_ow + ox * g.r_sx + g.r_ox;
    }
    if (g.resid) {
      float t[8];
      unpack8(*(const uint4*)(g.resid + orow * g.ldr + col), t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    if (g.act == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = silu_f(v[e]);
    } else if (g.act == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    } else if (g.act == 3) {
      float t[8];
      unpack8(*(const uint4*)(g.aux + orow * g.ld_aux + col), t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = t[e] > 0.f ? v[e] : 0.f;
    }
    if (g.c_f32) {
      float* d = (float*)g.C + orow * g.ldc + col;
      *(float4*)d = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      *(uint4*)((bf16_t*)g.C + orow * g.ldc + col) = pack8(v);
    }
  }

  __device__ __forceinline__ static void store(const EpiArgs& g, int row, int col, float acc, int z) {
    if (row >= g.M || col >= g.N) return;
    if (g.raw) {
      ((float*)g.ws)[(long long)z * g.split_stride + (long long)row * g.N + col] = acc;
      return;
    }
    store_final(g, row, col, acc);
  }

  __device__ __forceinline__ static void store_final(const EpiArgs& g, int row, int col, float acc) {
    if (g.n_x0 && col >= g.n_x0) {
      extra(g, row, col, &acc, 1);
      return;
    }
    if (row >= g.m_store || col >= g.n_store) return;
    float v = g.alpha * acc;
    if (g.bias) v += g.bias[col];
    if (g.bias2) v += g.bias2[col];
    if (g.rowbias) v += bf2f(g.rowbias[rb_row(g, row) * g.rb_ld + col]);
    long long orow = row;
    if (g.remap) {
      const int b = (int)g.pix_d.div((unsigned)row);
      const int rr = row - b * g.pix_d.d();
      const int oy = (int)g.gw_d.div((unsigned)rr);
      const int ox = rr - oy * g.gw_d.d();
      orow = ((long long)b * g.r_oh + oy * g.r_sy + g.r_oy) * g.r_ow + ox * g.r_sx + g.r_ox;
    }
    if (g.resid) v += bf2f(g.resid[orow * g.ldr + col]);
    v = act1(g, v, orow, col);
    long long ocol = col;
    if (g.perm) {
      int tap = (int)__umulhi((unsigned)col, g.p_magic);
      int c = col - tap * g.p_cin;
      if (c >= g.p_cvalid) return;
      ocol = g.perm == 2 ? (long long)tap * g.p_cvalid + c : (long long)c * g.p_taps + tap;
    }
    if (g.c_f32) ((float*)g.C)[orow * g.ldc + ocol] = v;
    else ((bf16_t*)g.C)[orow * g.ldc + ocol] = f2bf(v);
  }
};

// dz and dz * xhat of one 8-column chunk of one output row (GroupNorm backward, EpiArgs::gn_part): v = the stored bf16
// dy values, x the GroupNorm input there, tb the forward table {a, s, mean, rstd} of the chunk's columns
__device__ __forceinline__ void gn_accum(const EpiArgs& e, const float* v, const uint4 xr, const float4* tb, float* u,
                                         float* w) {
  float xv[8];
  unpack8(xr, xv);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float dz = v[q];
    if (e.gn_silu) dz *= silu_grad_f(fmaf(xv[q], tb[q].x, tb[q].y));
    u[q] += dz;
    w[q] = fmaf(dz, (xv[q] - tb[q].z) * tb[q].w, w[q]);
  }
}

// The GroupNorm-backward statistics epilogue of one staged 64-row half (m0h = its first row): thread t owns column
// chunk t % CH of rows t / CH + R k (R = NTH / CH row lanes); per gn_rb-row segment it stores bf16(alpha acc) with
// 16-B stores, accumulates dz / dz * xhat over its rows, and the R row lanes are summed in a fixed order through LDS
// (red: R x TBN x 2 floats) into the segment's column partials -- deterministic, no atomics.
template <int TBN, int NTH>
__device__ __forceinline__ void epi_gn_half(const EpiArgs& e, const float* st, float* red, int m0h, int n0) {
  constexpr int SROW = TBN + 4, CH = TBN / 8, R = NTH / CH;
  const int t = threadIdx.x, c8 = t % CH, rl0 = t / CH;
  const int col = n0 + c8 * 8;
  const bool on = rl0 < R && col < e.N;
#pragma unroll 1
  for (int s0 = 0; s0 < 64 && m0h + s0 < e.M; s0 += e.gn_rb) {
    float u[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, w[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (on) {
      const int b = (int)e.gn_pd.div((unsigned)(m0h + s0));  // a segment lies inside one sample (gn_rb | gn_P)
      float4 tb[8];
      const float4* tp = e.gn_tab + (long long)b * e.N + col;
#pragma unroll
      for (int q = 0; q < 8; ++q) tb[q] = tp[q];
      // every x row of this thread's share of the segment is loaded up front (one memory round trip per segment
      // instead of one per row); the rows are then consumed in the same order as before
      constexpr int MR = (64 + R - 1) / R;
      uint4 xr[MR];
#pragma unroll
      for (int k = 0; k < MR; ++k) {
        const int rl = s0 + rl0 + k * R, row = m0h + rl;
        if (rl < s0 + e.gn_rb && row < e.M) xr[k] = *(const uint4*)(e.gn_x + (long long)row * e.gn_ldx + col);
      }
#pragma unroll
      for (int k = 0; k < MR; ++k) {
        const int rl = s0 + rl0 + k * R, row = m0h + rl;
        if (rl >= s0 + e.gn_rb || row >= e.M) break;
        const float4 lo = *(const float4*)(st + rl * SROW + c8 * 8), hi = *(const float4*)(st + rl * SROW + c8 * 8 + 4);
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] *= e.alpha;
        const uint4 pk = pack8(v);
        *(uint4*)((bf16_t*)e.C + (long long)row * e.ldc + col) = pk;
        unpack8(pk, v);  // the statistics are of the stored bf16 dy, as the apply pass reads it
        gn_accum(e, v, xr[k], tb, u, w);
      }
    }
    if (rl0 < R) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[(rl0 * TBN + c8 * 8 + q) * 2] = u[q];
        red[(rl0 * TBN + c8 * 8 + q) * 2 + 1] = w[q];
      }
    }
    __syncthreads();
    const long long seg = (m0h + s0) / e.gn_rb;
#pragma unroll 1
    for (int j = t; j < TBN; j += NTH) {
      if (n0 + j >= e.N) continue;
      float a1 = 0.f, a2 = 0.f;
#pragma unroll 1
      for (int r = 0; r < R; ++r) {
        a1 += red[(r * TBN + j) * 2];
        a2 += red[(r * TBN + j) * 2 + 1];
      }
      *(float2*)(e.gn_part + (seg * e.N + n0 + j) * 2) = make_float2(a1, a2);
    }
    __syncthreads();
  }
}

// Shared epilogue of the GEMM kernels: acc = this wave's 64 x (NJ*16) sub-tile (4 x NJ MFMA tiles) at (wm, wn) of a
// TBM x TBN workgroup tile computed by NT threads; smem >= 64 x (TBN + 4) fp32 of LDS that no wave reads any more (the
// caller synchronises before). GNE: the GroupNorm-statistics form (EpiArgs::gn_part, unsplit launches only) -- a
// separate instantiation, so the plain epilogue's code and registers stay those of a kernel without it (measured: the
// runtime-branch form slowed every GEMM of the step, 14.15-14.24 vs 13.90-13.94 ms/step with no statistics in use).
template <int TBN = BN, bool XCOL = false, int TBM = BM, int NJ = TBN / 32, int NTH = NT, bool GNE = false>
__device__ __forceinline__ void gemm_epilogue(const EpiArgs& e, f32x4 (&acc)[4][NJ], char* smem, int m0, int n0,
                                              int wm, int wn, int lane, int z) {
  // Stage the fp32 tile through LDS in 64-row parts; each thread then owns runs of 8 consecutive columns of one
  // row: 16-B stores (8 bf16 or 2 x 4 fp32) on the aligned paths, and a ROLLED per-element loop on the rare general
  // path (column permutes of weight gradients, unaligned outputs) instead of 4 x NJ x 4 unrolled scattered stores,
  // whose code and register footprint pushed the 192-column tile's accumulators to scratch.
  float* st = (float*)smem;      // [64][SROW] fp32, 33 KB (TBN 128) / 49 KB (TBN 192) / 97 KB (TBN 384)
  constexpr int SROW = TBN + 4;  // +4 floats: lanes of one ds_write hit distinct banks
  static_assert((64 * TBN / 8) % NTH == 0, "epilogue chunks per thread");
#pragma unroll
  for (int half = 0; half < TBM / 64; ++half) {
    if (wm == half * 64) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int cl = wn + 16 * j + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) st[(16 * i + 4 * (lane >> 4) + r) * SROW + cl] = acc[i][j][r];
      }
    }
    __syncthreads();
    if constexpr (GNE) {  // GroupNorm statistics (plain bf16 epilogue, checked on the host)
      epi_gn_half<TBN, NTH>(e, st, st + 64 * SROW, m0 + half * 64, n0);
      continue;
    }
#pragma unroll 1
    for (int it = 0; it < 64 * TBN / 8 / NTH; ++it) {  // 64 rows x TBN/8 chunks of 8 columns
      const int ch = threadIdx.x + it * NTH;
      const int rl = ch / (TBN / 8), c8 = (ch - rl * (TBN / 8)) * 8;
      const int row = m0 + half * 64 + rl, col = n0 + c8;
      float v[8];
      const float4 lo = *(const float4*)(st + rl * SROW + c8), hi = *(const float4*)(st + rl * SROW + c8 + 4);
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      if (XCOL && col >= e.n_gemm) continue;  // beyond the produced columns (tile padding)
      if (e.raw) {
        // only produced columns: with VALU row sums the slab column n_x0 = n_gemm belongs to those sums
        if (row >= e.M || col >= e.n_gemm) continue;
        // split-K slab, device-coherent (sc1) stores: the tile's last split may run on another XCD
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)e.ws, (short)0, 0x7fffffff, 0x00020000);
        const int off = (int)(((long long)z * e.split_stride + (long long)row * e.N + col) * 4);
        if (e.n8) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo), rw, off, 0, CPOL_SC1);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi), rw, off + 16, 0, CPOL_SC1);
        } else {
#pragma unroll 1
          for (int q = 0; q < 8 && col + q < e.N; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[q]), rw, off + 4 * q, 0, CPOL_SC1);
        }
      } else if (XCOL && e.n_x0 && col >= e.n_x0) {
        if (row < e.M) Epi::extra(e, row, col, v, 8);
      } else if (e.vec) {
        if (row < e.m_store && col < e.n_store) Epi::finish8(e, row, col, v);
      } else if (row < e.m_store) {
#pragma unroll 1
        for (int q = 0; q < 8 && col + q < e.n_store; ++q) {
          float b = 0.f;
          if (e.bias) b += e.bias[col + q];
          if (e.bias2) b += e.bias2[col + q];
          Epi::finish(e, row, col + q, e.alpha * v[q] + b);
        }
      }
    }
    __syncthreads();
  }
}

// The kernels take (const Args g, const EpiArgs e): e sits in the kernel-argument segment right after g. Reading it
// through a laundered segment pointer AFTER the main loop keeps the compiler from hoisting ~50 scalar loads of
// epilogue fields to the kernel entry, where they stayed live (and spilled) in SGPRs across the whole main loop.
__device__ __forceinline__ EpiArgs epi_args_late() {
  EpiArgs r;
#if defined(__HIP_DEVICE_COMPILE__)  // the host compilation pass never runs device code
  typedef __attribute__((address_space(4))) const char* kptr_t;
  kptr_t ka = (kptr_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ka));
  constexpr size_t off = (sizeof(Args) + alignof(EpiArgs) - 1) / alignof(EpiArgs) * alignof(EpiArgs);
  __builtin_memcpy(&r, ka + off, sizeof(EpiArgs));
#endif
  return r;
}

// XCD-aware tile order. Workgroups are dispatched round-robin over the 8 XCDs (dispatch id d runs on XCD d % 8,
// each XCD has its own 4 MiB L2). The grid is (N tiles, M tiles, splits); re-number it so every XCD owns a
// CONTIGUOUS band of logical tiles (bijective for any grid size), with N tiles fastest: the N tiles of one
// 128-row A band -- and, for implicit-GEMM convs, the neighbouring bands whose halo rows it re-reads -- are
// then fetched into ONE L2 instead of up to eight.
struct TileId {
  int m0, n0, z, tile;  // tile = logical (m, n) index within the split slice
};

template <int TBN = BN, int TBM = BM>
__device__ __forceinline__ TileId tile_id() {
  const int gx = gridDim.x, per = gridDim.x * gridDim.y;
  const int total = per * gridDim.z;
  const int d = (blockIdx.z * gridDim.y + blockIdx.y) * gx + blockIdx.x;
  const int xcd = d & 7, q = total >> 3, r = total & 7;
  const int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (d >> 3);
  TileId t;
  t.z = l / per;
  t.tile = l - t.z * per;
  const int mt = t.tile / gx;
  t.m0 = mt * TBM;
  t.n0 = (t.tile - mt * gx) * TBN;
  return t;
}

// RED (col-major A only): 0 plain GEMM, 1 + VALU row sums of A (bias gradient), 2 + synthesised reduction columns
// (bias and per-group sums) -- compile-time so the plain instantiations carry none of it
template <int AM, int BMODE, int RED = 0, bool GNE = false>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(const Args g, const EpiArgs e) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];
  // buffer b: A tile at smem + 2*b*TILE_BYTES, B tile right after it
#define SA(b) (smem + (b) * 2 * TILE_BYTES)
#define SB(b) (smem + (b) * 2 * TILE_BYTES + TILE_BYTES)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const TileId tl = tile_id();
  const int m0 = tl.m0, n0 = tl.n0;
  const int grp = g.ngroups > 1 ? tl.z / g.nsplit : 0;  // grouped launch: problem index, then the split within it
  const int z = tl.z - grp * g.nsplit;
  const bf16_t* const opA = grp ? g.Ag[grp] : g.A;
  const bf16_t* const opB = grp ? g.Bg[grp] : g.B;
  const int nkt_total = (g.K + BK - 1) / BK;
  const int kt0 = z * g.ktiles_per_split;
  const int kt1 = min(nkt_total, kt0 + g.ktiles_per_split);

  // ---------------- per-thread staging coordinates ----------------
  // K-contiguous staging: rows (tid>>3)+32i, chunk tid&7.   MN-contiguous: k-rows (tid>>4)+16i, chunk tid&15.
  int a_pb[4], a_iy[4], a_ix[4];
  bool a_ok[4];
  if (AM == SDMI_A_CONV) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int m = m0 + (tid >> 3) + 32 * i;
      a_ok[i] = m < g.M;
      int b, oy, ox;
      pixel_coords(g, m, b, oy, ox);
      a_pb[i] = b * g.ih;
      a_iy[i] = oy * g.sy + g.oy0;
      a_ix[i] = ox * g.sx + g.ox0;
    }
  }
  int b_ty = 0, b_tx = 0, b_ci = 0;
  bool b_nok = true;
  if (BMODE == SDMI_B_KN_CONV) {
    int n = n0 + (tid & 15) * 8;
    b_nok = n < g.N;
    int tap = n / g.cin;
    b_ci = n - tap * g.cin;
    b_ty = tap / g.kw;
    b_tx = tap - b_ty * g.kw;
  }

  uint4 ra[4], rb[4];
  // Buffer descriptors: out-of-range offsets return zeros in hardware, which is how padding taps,
  // ragged tiles and k >= K are zero-filled without a select on a pointer.
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)opA, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)opB, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsA2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.A2 ? g.A2 : opA), (short)0, 0x7fffffff, 0x00020000);
  constexpr int OOB = (int)0x80000000;
#define BUF_LD(rs, off) __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128((rs), (off), 0, 0))

  auto load_tiles = [&](int kt) __attribute__((always_inline)) {
    const int k0 = kt * BK;
    // ---- A ----
    if (AM == SDMI_A_ROWMAJOR) {
      int k = k0 + (tid & 7) * 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int m = m0 + (tid >> 3) + 32 * i;
        int off = (m < g.M && k < g.K) ? (m * g.lda + k) * 2 : OOB;
        ra[i] = BUF_LD(rsA, off);
      }
    } else if (AM == SDMI_A_CONV) {
      int k = k0 + (tid & 7) * 8;
      if (k >= g.k_split) {  // K-concatenated second source: plain row-major rows (fused 1x1 conv)
        int kk = k - g.k_split;
        bool kok = k < g.K;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int m = m0 + (tid >> 3) + 32 * i;
          int off = (kok && a_ok[i]) ? (m * g.lda2 + kk) * 2 : OOB;
          ra[i] = BUF_LD(rsA2, off);
        }
      } else {
        int tap = k / g.cin;
        int ci = k - tap * g.cin;
        int ty = tap / g.kw;
        int tx = tap - ty * g.kw;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int iy = a_iy[i] + ty, ix = a_ix[i] + tx;
          bool ok = a_ok[i] && (unsigned)iy < (unsigned)g.ih && (unsigned)ix < (unsigned)g.iw;
          int off = ok ? (((a_pb[i] + iy) * g.iw + ix) * g.ldx + ci) * 2 : OOB;
          ra[i] = BUF_LD(rsA, off);
        }
      }
    } else {  // col-major A: A[k*lda + m]
      int m = m0 + (tid & 15) * 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int k = k0 + (tid >> 4) + 16 * i;
        int off = (m < g.M && k < g.K) ? (k * g.lda + m) * 2 : OOB;
        ra[i] = BUF_LD(rsA, off);
      }
    }
    // ---- B ----
    if (BMODE == SDMI_B_NK) {
      int k = k0 + (tid & 7) * 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int n = n0 + (tid >> 3) + 32 * i;
        int off = (n < g.N && k < g.K) ? (n * g.ldb + k) * 2 : OOB;
        rb[i] = BUF_LD(rsB, off);
      }
    } else if (RED == 2 && n0 + (tid & 15) * 8 >= g.n_x0) {  // reduction columns (both MN-contiguous B modes)
      const int n = n0 + (tid & 15) * 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) rb[i] = reduction_cols(g, n, k0 + (tid >> 4) + 16 * i);
    } else if (BMODE == SDMI_B_KN) {
      int n = n0 + (tid & 15) * 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int k = k0 + (tid >> 4) + 16 * i;
        int off = (n < g.N && k < g.K) ? (k * g.ldb + n) * 2 : OOB;
        rb[i] = BUF_LD(rsB, off);
      }
    } else {  // conv gather, k = pixel of the (oh x ow) grid
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int p = k0 + (tid >> 4) + 16 * i;
        int b, oy, ox;
        pixel_coords(g, p, b, oy, ox);
        int iy = oy * g.sy + g.oy0 + b_ty, ix = ox * g.sx + g.ox0 + b_tx;
        bool ok = b_nok && p < g.K && (unsigned)iy < (unsigned)g.ih && (unsigned)ix < (unsigned)g.iw;
        int off = ok ? (((b * g.ih + iy) * g.iw + ix) * g.ldx + b_ci) * 2 : OOB;
        rb[i] = BUF_LD(rsB, off);
      }
    }
  };

  auto store_tiles = [&](int buf) __attribute__((always_inline)) {
    if (AM == SDMI_A_COLMAJOR) {
#pragma unroll
      for (int i = 0; i < 4; ++i) *(uint4*)(SA(buf) + tr_off((tid >> 4) + 16 * i, tid & 15)) = ra[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) *(uint4*)(SA(buf) + kc_off((tid >> 3) + 32 * i, tid & 7)) = ra[i];
    }
    if (BMODE == SDMI_B_NK) {
#pragma unroll
      for (int i = 0; i < 4; ++i) *(uint4*)(SB(buf) + kc_off((tid >> 3) + 32 * i, tid & 7)) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) *(uint4*)(SB(buf) + tr_off((tid >> 4) + 16 * i, tid & 15)) = rb[i];
    }
  };

  // fragment readers
  auto read_kc = [&](const char* tile, int rbase, int ks) __attribute__((always_inline)) -> s16x8 {
    int r = rbase + (lane & 15);
    int c = ks * 4 + (lane >> 4);
    return *(const s16x8*)(tile + kc_off(r, c));
  };
  auto read_tr = [&](const char* tile, int cbase, int ks) __attribute__((always_inline)) -> s16x8 {
    int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    int r1 = ks * 32 + gq * 8 + q;
    int c = (cbase >> 3) + (p >> 1);
    int o1 = tr_off(r1, c) + (p & 1) * 8;
    int o2 = tr_off(r1 + 4, c) + (p & 1) * 8;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)(tile + o1));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)(tile + o2));
    s16x8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // VALU row sums of col-major A (Args::rowsum) by the workgroups of n-tile 0: m = m0 + (tid & 15) * 8 + e
  const bool rowsum = RED == 1 && n0 == 0;
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto sum_rows = [&]() __attribute__((always_inline)) {
    if (rowsum) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float t[8];
        unpack8(ra[i], t);
#pragma unroll
        for (int q = 0; q < 8; ++q) rs[q] += t[q];
      }
    }
  };

  if (kt0 < kt1) {
    load_tiles(kt0);
    sum_rows();
    store_tiles(0);
    __syncthreads();
    int cur = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load_tiles(kt + 1);
      const char* ta = SA(cur);
      const char* tb = SB(cur);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s16x8 fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fa[i] = (AM == SDMI_A_COLMAJOR) ? read_tr(ta, wm + 16 * i, ks) : read_kc(ta, wm + 16 * i, ks);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          fb[j] = (BMODE == SDMI_B_NK) ? read_kc(tb, wn + 16 * j, ks) : read_tr(tb, wn + 16 * j, ks);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
      if (more) {
        sum_rows();
        store_tiles(cur ^ 1);
      }
      __syncthreads();
      cur ^= 1;
    }
  }
  // The epilogue arguments are read through a laundered pointer into the kernel-argument segment: the compiler
  // cannot hoist those scalar loads above this point, so ~50 EpiArgs fields are not held (and spilled) in SGPRs
  // across the main loop.
  EpiArgs ev = epi_args_late();
  if (grp) group_epi(ev, g.Cg[grp], g.sum_g[grp], grp);
  const EpiArgs* ep = &ev;
  if (rowsum) {  // combine the 16 k-row lanes of each 8-column chunk in LDS (workgroup-uniform branch)
    float* red = (float*)smem;  // [16][128]
#pragma unroll
    for (int q = 0; q < 8; ++q) red[(tid >> 4) * 128 + (tid & 15) * 8 + q] = rs[q];
    __syncthreads();
    if (tid < BM) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) t += red[r * 128 + tid];
      const int m = m0 + tid;
      if (m < ep->M) {
        if (ep->raw) {  // slab column n_x0 of this split (the reducer routes it to sum_out / sum_out2)
          ((float*)ep->ws)[(long long)z * ep->split_stride + (long long)m * ep->N + ep->n_x0] = t;
        } else if (m < ep->m_store) {
          if (ep->sum_out) ep->sum_out[m] = t;
          if (ep->sum_out2) ep->sum_out2[m] = t;
        }
      }
    }
    __syncthreads();
  }

  gemm_epilogue<BN, RED == 2, BM, BN / 32, NT, GNE>(*ep, acc, smem, m0, n0, wm, wn, lane, z);
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA pipelined variant: operands go global -> LDS with buffer_load ... lds (no VGPR staging, no
// ds_write), STAGES-deep ring, one barrier per 64-deep K tile. The LDS destination of a DMA
// wave-instruction is lane-linear (1 KiB per instruction), so the XOR swizzles of the LDS images are
// applied to the per-lane SOURCE addresses (logical chunk = physical slot ^ swizzle(row)); the
// fragment reads are unchanged. Out-of-range lanes (conv padding, ragged tiles) use an offset beyond
// the buffer record and the hardware writes zeros.
// ---------------------------------------------------------------------------------------------
// K-contiguous LDS image with KBK-deep rows: 128-B rows (KBK 64), chunk c of row r at slot c ^ (r & 7); 64-B rows
// (KBK 32), chunk c at slot c ^ f((r >> 2) & 3) with f = {0, 2, 3, 1}: the four ds_read_b128 lane groups of a
// fragment read (rows 0-15 x chunks 0-3) then each hit 16 distinct 16-B slots of the 256-B bank row
template <int KBK>
__device__ __forceinline__ int kc_off_k(int r, int c) {
  if constexpr (KBK == 64) return r * 128 + ((c ^ (r & 7)) << 4);
  return r * 64 + ((c ^ ((0x1320 >> (((r >> 2) & 3) * 4)) & 3)) << 4);
}

template <int KBK>
__device__ __forceinline__ s16x8 frag_kc_k(const char* tile, int rbase, int ks, int lane) {
  int r = rbase + (lane & 15);
  int c = ks * 4 + (lane >> 4);
  return *(const s16x8*)(tile + kc_off_k<KBK>(r, c));
}

__device__ __forceinline__ s16x8 frag_kc(const char* tile, int rbase, int ks, int lane) {
  int r = rbase + (lane & 15);
  int c = ks * 4 + (lane >> 4);
  return *(const s16x8*)(tile + kc_off(r, c));
}

__device__ __forceinline__ s16x8 frag_tr(const char* tile, int cbase, int ks, int lane) {
  int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  int r1 = ks * 32 + gq * 8 + q;
  int c = (cbase >> 3) + (p >> 1);
  int o1 = tr_off(r1, c) + (p & 1) * 8;
  int o2 = tr_off(r1 + 4, c) + (p & 1) * 8;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)(tile + o1));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)(tile + o2));
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// Transposed fragment read for the LDS-DMA kernels, as inline asm. hipcc (ROCm 7.2) cannot prove a
// ds_read_b64_tr_b16 builtin disjoint from the LDS-DMA writes in flight and emits s_waitcnt vmcnt(0) before it --
// which drains the prefetch of the NEXT k-tile issued just before (measured: every DMA kernel with an MN-contiguous
// operand ran fully serialised). The asm reads are invisible to hipcc's lgkmcnt bookkeeping, so the caller waits
// for them explicitly (lds_wait_frags) before the MFMAs that consume them.
__device__ __forceinline__ s16x4 ds_tr_asm(const char* p) {
  s16x4 r;
  const unsigned a = (unsigned)(uintptr_t)(SDMI_LDS const char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}

__device__ __forceinline__ s16x8 frag_tr_asm(const char* tile, int cbase, int ks, int lane) {
  int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  int r1 = ks * 32 + gq * 8 + q;
  int c = (cbase >> 3) + (p >> 1);
  s16x4 lo = ds_tr_asm(tile + tr_off(r1, c) + (p & 1) * 8);
  s16x4 hi = ds_tr_asm(tile + tr_off(r1 + 4, c) + (p & 1) * 8);
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// the same read at LDS byte address a + OFF (OFF < 65536: the instruction's offset field), so the loop-invariant part of
// an address stays in one VGPR and the stage / k-step / row part is an immediate (no per-iteration VALU address adds)
template <int OFF>
__device__ __forceinline__ s16x4 ds_tr_off(unsigned a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}

template <int OFF>
__device__ __forceinline__ s16x8 frag_tr_off(unsigned a) {
  const s16x4 lo = ds_tr_off<OFF>(a), hi = ds_tr_off<OFF + 1024>(a);  // k-rows +4: same swizzle (tr_swz ignores bit 2)
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// lane part of frag_tr_asm's address for column base cbase (% 128) at k-step 0 (k-step ks adds 32 rows = 8192 B: the
// swizzle ignores bit 5 of the row)
__device__ __forceinline__ int frag_tr_lane(int cbase, int lane) {
  const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  return tr_off(gq * 8 + q, (cbase >> 3) + (p >> 1)) + (p & 1) * 8;
}

template <int N>
struct IC { static constexpr int value = N; };
struct RT { int value; };  // a runtime ring stage (K-contiguous-only kernels keep their plain loop)

// all LDS reads issued so far have landed; the fragments are re-defined after the wait so no consumer (an MFMA is
// register-only and would otherwise be hoisted above an asm wait) reads them earlier
template <int N>
__device__ __forceinline__ void lds_wait_frags(s16x8 (&f)[N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_wave_base, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (SDMI_LDS void*)lds_wave_base, 16, off, 0, 0, 0);
}

// Tile shapes (TBM x TBN, NWN waves along N, TBM / 64 along M; every wave owns 64 x TBN/NWN):
//   128 x {64, 128, 192}, 4 waves (2 x 2): the default family -- 2 x <= 80 KiB of LDS fits two workgroups per CU;
//     N = 384 outputs split into 2 (not 3) 192-column tiles, so a 32768 x 384 conv is exactly 512 tiles = one round
//   256 x {128, 192}, 8 waves (4 x 2), B_NK: the large-M convolutions / linears -- 1.5x the MFMA work per byte staged
//   128 x {256, 384}, 8 waves (2 x 4), MN-contiguous B: weight gradients, whose N = 9 * cin is a multiple of 384
//   64 x {64, 128}, 4 waves (1 x 4), K-contiguous A and B: the latency-bound low-resolution GEMMs (M <= 8192, a grid
//     of <= 256 tiles, K of 8-40 k-tiles) with a 6-stage ring -- five 64-deep k-tiles in flight per workgroup, so the
//     DMA latency is paid about once per launch instead of once per k-tile
// The MN-contiguous (ds_read_b64_tr_b16) LDS images are kept as 128-column sub-tiles [64 k][128] (256-B rows).
// RED (col-major A only): reduction columns as extra MFMA tiles against synthesised B fragments (see reduce_frag).
template <int TBM, int NWN>
constexpr int dma_threads() { return 64 * (TBM / 64) * NWN; }

// B fragment (8 k-values of one column, lane layout of mfma_f32_16x16x32_bf16: k = kb .. kb+7, column = lane & 15)
// of reduction tile r: column 0 all ones (row sums: bias gradient), column 8 + j the indicator of group j = k / grp
// (per-sample sums: time-embedding gradient; needs grp % 8 == 0 so 8 consecutive k share one group)
template <int RED>
__device__ __forceinline__ s16x8 reduce_frag(const Args& g, int r, int kb, int lane) {
  const int col = r * 16 + (lane & 15);
  bool one = col == 0;
  if (RED == 2 && col >= 8) one = (int)g.grp_d.div((unsigned)kb) == col - 8;
  const short v = one ? (short)0x3F80 : (short)0;
  return (s16x8){v, v, v, v, v, v, v, v};
}

// KBK: k depth of one staged tile (64, or 32 for deeper rings in the same LDS: more bytes in flight per CU). Split-K
// slices stay in units of 64 (host k-tiles).
// KG (col-major A, the weight gradients): k-groups per workgroup. KG wave groups, each with its own LDS ring, compute
// the same output tile over interleaved k-tiles of the split's range (group g: tiles g, g + KG, ...); their fp32
// accumulators are summed through LDS in group order (deterministic) before the epilogue. A tile's k range then
// needs KG x fewer split-K slices for the same number of waves on the chip: fewer fp32 slabs written, read and reduced.
template <int TBM, int NWN, int KG>
constexpr int dma_min_waves(int ring_bytes) {
  return KG > 1 ? 2 : ((dma_threads<TBM, NWN>() == 256 && ring_bytes <= 80 * 1024) ? 2 : 1);
}

#ifdef SDMI_GEMM_TRACE
// Probe build only (scripts/gemm_phase_probe.py): per-workgroup phase timestamps of the LDS-DMA kernel, 100 MHz
// s_memrealtime -- entry, first k-tile landed, main loop done, epilogue done -- by thread 0, vector stores.
__device__ unsigned long long g_gemm_trace[1 << 20];
#define SDMI_TRACE_T(i) \
  do {                  \
    if (threadIdx.x == 0) tr_t[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define SDMI_TRACE_T(i) \
  do {                  \
  } while (0)
#endif

template <int AM, int BMODE, int STAGES, int TBN = BN, int TBM = BM, int NWN = 2, int RED = 0, int KBK = BK,
          bool GNE = false, int KG = 1>
__global__ __launch_bounds__((dma_threads<TBM, NWN>() * KG),
                             (dma_min_waves<TBM, NWN, KG>(STAGES * (TBM + TBN) * KBK * 2)))
void gemm_dma_kernel(const Args g, const EpiArgs e) {
  constexpr int NTH = dma_threads<TBM, NWN>() * KG;  // all threads; the DMA pieces are shared out per k-group
  constexpr int NW = NTH / 64 / KG;                    // waves per k-group
  constexpr int WTN = TBN / NWN;                     // columns per wave
  constexpr int NJ = WTN / 16;                       // 16-column MFMA tiles per wave
  constexpr bool A_MN = AM == SDMI_A_COLMAJOR, B_MN = BMODE != SDMI_B_NK;
  static_assert(KBK == 64 || KBK == 32, "staged k depth");
  constexpr int KS = KBK / 32;                        // MFMA k-steps per staged tile
  constexpr int RB = KBK * 2;                         // K-contiguous image row bytes
  constexpr int RPI = 1024 / RB, CPR = KBK / 8;       // rows per DMA wave-instruction, 16-B chunks per row
  constexpr int SUB = KBK * 256, IPS = KBK / 4;       // MN image: 128-column sub-tile bytes, DMA pieces per sub-tile
  constexpr int A_BYTES = TBM * KBK * 2, B_BYTES = TBN * KBK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;     // A | B
  constexpr int A_PW = A_BYTES / 1024 / NW, B_PW = B_BYTES / 1024 / NW;  // DMA wave-instructions per tile
  static_assert(A_PW * NW * 1024 == A_BYTES && B_PW * NW * 1024 == B_BYTES, "DMA pieces per wave");
  static_assert(!A_MN || TBM % 128 == 0, "MN-contiguous A: 128-column sub-tiles");
  static_assert(!B_MN || TBN % 128 == 0, "MN-contiguous B: 128-column sub-tiles");
  static_assert(WTN % 16 == 0 && TBM % 64 == 0, "wave tile");
  static_assert(RED == 0 || A_MN, "reductions: col-major A only");
  static_assert(KG == 1 || TBM == 128, "k-groups: 128-row tiles");
  constexpr int RPW = RED == 0 ? 0 : (RED == 1 ? 1 : (3 + NWN - 1) / NWN);  // reduction tiles per wave (<= 3 total)
  extern __shared__ __attribute__((aligned(16))) char smem[];  // STAGES x (A | B)
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform: scalar LDS bases / M0
  const int kg = wave_all / NW, wave = wave_all - kg * NW;            // k-group, wave within it
  char* const ring = smem + kg * STAGES * (TBM + TBN) * KBK * 2;       // this k-group's LDS ring
  const int wm = (wave / NWN) * 64, wn = (wave % NWN) * WTN;
#ifdef SDMI_GEMM_TRACE
  unsigned long long tr_t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  SDMI_TRACE_T(0);
  const TileId tl = tile_id<TBN, TBM>();
  const int m0 = tl.m0, n0 = tl.n0;
  const int grp = g.ngroups > 1 ? tl.z / g.nsplit : 0;  // grouped launch: problem index, then the split within it
  const int z = tl.z - grp * g.nsplit;
  const bf16_t* const opA = grp ? g.Ag[grp] : g.A;
  const bf16_t* const opB = grp ? g.Bg[grp] : g.B;
  const int nkt_total = (g.K + KBK - 1) / KBK;
  const int kt0 = z * g.ktiles_per_split * (BK / KBK);
  const int kt1 = min(nkt_total, kt0 + g.ktiles_per_split * (BK / KBK));
  constexpr int OOB = (int)0x80000000;

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)opA, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)opB, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsA2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.A2 ? g.A2 : opA), (short)0, 0x7fffffff, 0x00020000);

  // ---- per-lane, per-instruction coordinates, fixed over the K loop ----
  // instruction q = wave * PW + j writes 1 KiB at tile + q * 1024 (lane-linear):
  //   K-contiguous image: rows q*8 .. +8, lane -> row + lane>>3, physical slot lane&7
  //   MN-contiguous image: 128-column sub-tile q >> 4, k-rows (q & 15)*4 .. +4, lane -> k-row + lane>>4, slot lane&15
  int a_base[A_PW], b_base[B_PW];  // element offsets (without the k / pixel part)
  int a_kk[A_PW], b_kk[B_PW];      // k offset inside the tile (KC: chunk*8) or k-row (MN)
  bool a_ok[A_PW], b_ok[B_PW];
  int a_iy[A_PW], a_ix[A_PW], a_pb[A_PW], a_pix[A_PW];
  int b_ty[B_PW], b_tx[B_PW];
  const bool cin64 = AM == SDMI_A_CONV && g.cin % KBK == 0;  // k tile lies inside one tap
#pragma unroll
  for (int j = 0; j < A_PW; ++j) {
    const int q = wave * A_PW + j;
    if (A_MN) {
      int kr = (q % IPS) * 4 + (lane >> 4);
      int c = (lane & 15) ^ tr_swz(kr);
      int m = m0 + (q / IPS) * 128 + c * 8;
      a_ok[j] = m < g.M;
      a_base[j] = m;
      a_kk[j] = kr;
    } else {
      int r = q * RPI + lane / CPR;
      int c = (kc_off_k<KBK>(r, lane % CPR) - r * RB) >> 4;  // logical chunk of the lane's physical slot (involution)
      int m = m0 + r;
      a_ok[j] = m < g.M;
      a_kk[j] = c * 8;
      if (AM == SDMI_A_ROWMAJOR) {
        a_base[j] = m * g.lda;
      } else {
        int b, oy, ox;
        pixel_coords(g, m, b, oy, ox);
        a_pb[j] = b * g.ih;
        a_iy[j] = oy * g.sy + g.oy0;
        a_ix[j] = ox * g.sx + g.ox0;
        a_base[j] = m * g.lda2;  // second (K-concatenated) source row
        a_pix[j] = ((a_pb[j] + a_iy[j]) * g.iw + a_ix[j]) * g.ldx;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < B_PW; ++j) {
    const int q = wave * B_PW + j;
    if (!B_MN) {
      int r = q * RPI + lane / CPR;
      int c = (kc_off_k<KBK>(r, lane % CPR) - r * RB) >> 4;
      int n = n0 + r;
      b_ok[j] = n < g.N;
      b_base[j] = n * g.ldb;
      b_kk[j] = c * 8;
    } else {
      int kr = (q % IPS) * 4 + (lane >> 4);
      int c = (lane & 15) ^ tr_swz(kr);
      int n = n0 + (q / IPS) * 128 + c * 8;
      b_ok[j] = n < g.N;
      b_kk[j] = kr;
      b_base[j] = n;
      if (BMODE == SDMI_B_KN_CONV) {
        int tap = n / g.cin;
        int ci = n - tap * g.cin;
        b_ty[j] = tap / g.kw;
        b_tx[j] = tap - b_ty[j] * g.kw;
        b_base[j] = ci;
      }
    }
  }
  // implicit-im2col B, full k-tiles of a regular pixel grid (Args::bfast): the tile-invariant part of every lane's
  // gather offset, so issue_fast_b needs an add, a range check and a select per piece (no per-piece divisions)
  const int bform = BMODE == SDMI_B_KN_CONV ? ((g.bfast >> (KBK == 64 ? 0 : 2)) & 3) : 0;
  int bf_c[B_PW], bf_y[B_PW];
#pragma unroll
  for (int j = 0; j < B_PW; ++j) {
    bf_c[j] = OOB;
    bf_y[j] = -(1 << 29);
    if (BMODE == SDMI_B_KN_CONV && bform) {
      const int kr = b_kk[j];
      if (bform == 1) {  // lane row kr of the tile: row dy below the tile's first output row, column ox
        const int dy = (int)g.ow_d.div((unsigned)kr), ox = kr - dy * g.ow_d.d();
        const int ix = ox * g.sx + g.ox0 + b_tx[j];
        if (b_ok[j] && (unsigned)ix < (unsigned)g.iw) {
          bf_y[j] = dy * g.sy + g.oy0 + b_ty[j];
          bf_c[j] = (ix * g.ldx + b_base[j]) * 2;
        }
      } else {  // image db after the tile's first image, at (oy, ox)
        const int db = (int)g.ohw_d.div((unsigned)kr), r = kr - db * g.ohw_d.d();
        const int oy = (int)g.ow_d.div((unsigned)r), ox = r - oy * g.ow_d.d();
        const int iy = oy * g.sy + g.oy0 + b_ty[j], ix = ox * g.sx + g.ox0 + b_tx[j];
        if (b_ok[j] && (unsigned)iy < (unsigned)g.ih && (unsigned)ix < (unsigned)g.iw)
          bf_c[j] = (((db * g.ih + iy) * g.iw + ix) * g.ldx + b_base[j]) * 2;
      }
    }
  }

  // implicit-conv tap state (cin % 64 == 0): the (ty, tx, channel offset) of the next k-tile to issue, advanced
  // incrementally -- issue() is called for consecutive k-tiles -- instead of two runtime divisions per tile
  int c_ty = 0, c_tx = 0, c_ci = 0;
  // (k-groups: this group's first tile is kt0 + kg, and each issue advances KG tiles)
  if (AM == SDMI_A_CONV && cin64 && (kt0 + kg) * KBK < g.k_split) {
    const int tap = ((kt0 + kg) * KBK) / g.cin;
    c_ci = (kt0 + kg) * KBK - tap * g.cin;
    c_ty = tap / g.kw;
    c_tx = tap - c_ty * g.kw;
  }
  auto advance_tap = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < KG; ++q) {
      c_ci += KBK;
      if (c_ci >= g.cin) {
        c_ci = 0;
        if (++c_tx == g.kw) {
          c_tx = 0;
          ++c_ty;
        }
      }
    }
  };
  // Fast issue path for full k-tiles: every per-lane part of a DMA source offset is fixed over the K loop, the
  // per-tile part is wave-uniform (k0, or the conv tap shift), so a piece costs an add and a select instead of the
  // general path's coordinate math and bounds checks. Invalid lanes keep OOB (+ a uniform offset < 2^31: still out
  // of the 2^31 - 1 byte buffer record). Conv A (cin % KBK == 0): tap validity per lane is a precomputed bit mask.
  int a_v[A_PW], b_v[B_PW];
  unsigned a_tm[A_PW];
#pragma unroll
  for (int j = 0; j < A_PW; ++j) {
    a_tm[j] = 0u;
    if (AM == SDMI_A_ROWMAJOR) a_v[j] = a_ok[j] ? (a_base[j] + a_kk[j]) * 2 : OOB;
    else if (A_MN) a_v[j] = a_ok[j] ? (a_kk[j] * g.lda + a_base[j]) * 2 : OOB;
    else {
      a_v[j] = (a_pix[j] + a_kk[j]) * 2;
      if (cin64) {
        const int taps = g.k_split / g.cin;  // <= 16 (4x4 kernels)
        for (int tp = 0, ty = 0, tx = 0; tp < taps; ++tp) {
          const int iy = a_iy[j] + ty, ix = a_ix[j] + tx;
          if (a_ok[j] && (unsigned)iy < (unsigned)g.ih && (unsigned)ix < (unsigned)g.iw) a_tm[j] |= 1u << tp;
          if (++tx == g.kw) { tx = 0; ++ty; }
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < B_PW; ++j) {
    if (BMODE == SDMI_B_NK) b_v[j] = b_ok[j] ? (b_base[j] + b_kk[j]) * 2 : OOB;
    else if (BMODE == SDMI_B_KN) b_v[j] = b_ok[j] ? (b_kk[j] * g.ldb + b_base[j]) * 2 : OOB;
    else b_v[j] = 0;
  }

  // general issue path (ragged k-tiles, the fused second source, conv with cin % KBK != 0, the B im2col gather)
  auto issue_general_a = [&](int k0, char* sa) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < A_PW; ++j) {
      char* dst = sa + (wave * A_PW + j) * 1024;
      int off;
      if (AM == SDMI_A_ROWMAJOR) {
        int k = k0 + a_kk[j];
        off = (a_ok[j] && k < g.K) ? (a_base[j] + k) * 2 : OOB;
      } else if (A_MN) {
        int k = k0 + a_kk[j];
        off = (a_ok[j] && k < g.K) ? (k * g.lda + a_base[j]) * 2 : OOB;
      } else {
        int k = k0 + a_kk[j];
        if (k0 >= g.k_split) {  // fused 1x1 second source, tile-uniform (k_split % KBK == 0 on this path)
          off = (a_ok[j] && k < g.K) ? (a_base[j] + (k - g.k_split)) * 2 : OOB;
          dma16(rsA2, dst, off);
          continue;
        } else if (cin64) {
          // tap, and with it the (ty, tx) shift, is uniform over the tile (tracked incrementally)
          const int ty = c_ty, tx = c_tx;
          const int sh = (ty * g.iw + tx) * g.ldx + c_ci;
          int iy = a_iy[j] + ty, ix = a_ix[j] + tx;
          bool ok = a_ok[j] && (unsigned)iy < (unsigned)g.ih && (unsigned)ix < (unsigned)g.iw;
          off = ok ? (a_pix[j] + sh + a_kk[j]) * 2 : OOB;
        } else {
          int tap = k / g.cin;
          int ci = k - tap * g.cin;
          int ty = tap / g.kw, tx = tap - (tap / g.kw) * g.kw;
          int iy = a_iy[j] + ty, ix = a_ix[j] + tx;
          bool ok = a_ok[j] && k < g.k_split && (unsigned)iy < (unsigned)g.ih && (unsigned)ix < (unsigned)g.iw;
          off = ok ? (((a_pb[j] + iy) * g.iw + ix) * g.ldx + ci) * 2 : OOB;
        }
      }
      dma16(rsA, dst, off);
    }
    if (AM == SDMI_A_CONV && cin64 && k0 < g.k_split) advance_tap();
  };
  auto issue_general_b = [&](int k0, char* sb) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < B_PW; ++j) {
      char* dst = sb + (wave * B_PW + j) * 1024;
      int off;
      if (BMODE == SDMI_B_NK) {
        int k = k0 + b_kk[j];
        off = (b_ok[j] && k < g.K) ? (b_base[j] + k) * 2 : OOB;
      } else if (BMODE == SDMI_B_KN) {
        int k = k0 + b_kk[j];
        off = (b_ok[j] && k < g.K) ? (k * g.ldb + b_base[j]) * 2 : OOB;
      } else {
        int p = k0 + b_kk[j];
        int b, oy, ox;
        pixel_coords(g, p, b, oy, ox);
        int iy = oy * g.sy + g.oy0 + b_ty[j], ix = ox * g.sx + g.ox0 + b_tx[j];
        bool ok = b_ok[j] && p < g.K && (unsigned)iy < (unsigned)g.ih && (unsigned)ix < (unsigned)g.iw;
        off = ok ? (((b * g.ih + iy) * g.iw + ix) * g.ldx + b_base[j]) * 2 : OOB;
      }
      dma16(rsB, dst, off);
    }
  };

  // full k-tile of implicit-im2col B at pixel k0 (k0 % KBK == 0), bform != 0: the tile's image (and first output row)
  // are wave-uniform scalars
  auto issue_fast_b = [&](int k0, char* sb) __attribute__((always_inline)) {
    const int b = (int)g.ohw_d.div((unsigned)k0);
    const int sbase = b * g.ih * g.iw * g.ldx * 2;
    if (bform == 1) {
      const int soy = (int)g.ow_d.div((unsigned)(k0 - b * g.ohw_d.d())) * g.sy;
      const int rowb = g.iw * g.ldx * 2;
#pragma unroll
      for (int j = 0; j < B_PW; ++j) {
        const int iy = bf_y[j] + soy;
        dma16(rsB, sb + (wave * B_PW + j) * 1024, (unsigned)iy < (unsigned)g.ih ? sbase + iy * rowb + bf_c[j] : OOB);
      }
    } else {
#pragma unroll
      for (int j = 0; j < B_PW; ++j) dma16(rsB, sb + (wave * B_PW + j) * 1024, bf_c[j] + sbase);  // OOB stays OOB
    }
  };

  auto issue = [&](int kt, int stage) __attribute__((always_inline)) {
    char* sa = ring + stage * STAGE_BYTES;
    char* sb = sa + A_BYTES;
    const int k0 = kt * KBK;
    if (k0 + KBK <= g.K && (AM != SDMI_A_CONV || (cin64 && k0 + KBK <= g.k_split))) {
      const int tap = c_ty * g.kw + c_tx;
      const int ash = AM == SDMI_A_ROWMAJOR ? k0 * 2
                      : A_MN              ? k0 * g.lda * 2
                                          : ((c_ty * g.iw + c_tx) * g.ldx + c_ci) * 2;
#pragma unroll
      for (int j = 0; j < A_PW; ++j) {
        int off;
        if (AM == SDMI_A_CONV) off = ((a_tm[j] >> tap) & 1u) ? a_v[j] + ash : OOB;
        else off = a_v[j] + ash;
        dma16(rsA, sa + (wave * A_PW + j) * 1024, off);
      }
      if (AM == SDMI_A_CONV) advance_tap();
      if (BMODE != SDMI_B_KN_CONV) {
        const int bsh = BMODE == SDMI_B_NK ? k0 * 2 : k0 * g.ldb * 2;
#pragma unroll
        for (int j = 0; j < B_PW; ++j) dma16(rsB, sb + (wave * B_PW + j) * 1024, b_v[j] + bsh);
        return;
      }
      if (bform) {
        issue_fast_b(k0, sb);
        return;
      }
    } else {
      issue_general_a(k0, sa);
    }
    issue_general_b(k0, sb);
  };

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // reduction tiles r = (wave % NWN) + rr * NWN of the tiles in column-tile 0 (workgroup-uniform)
  const bool red_tile = RED != 0 && n0 == 0;
  const int nred = RED == 0 ? 0 : (RED == 1 ? 1 : (8 + e.ngrp + 15) / 16);
  f32x4 accr[RPW > 0 ? RPW : 1][4];
#pragma unroll
  for (int rr = 0; rr < (RPW > 0 ? RPW : 1); ++rr)
#pragma unroll
    for (int i = 0; i < 4; ++i) accr[rr][i] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // this k-group's tiles of the split: local tile t is k-tile kt0 + t * KG + kg (KG == 1: all of them, in order)
  const int nt_all = kt1 - kt0;
  const int nt = nt_all > kg ? (nt_all - kg + KG - 1) / KG : 0;
  const int nt_loop = (nt_all + KG - 1) / KG;  // barrier count: every k-group runs the first group's trip count
  // Transposed (MN-contiguous) fragment reads: the lane's address at stage 0, k-step 0 is loop-invariant (one VGPR per
  // 16-row / 16-column fragment); stage, k-step and the +4-row half are immediates of ds_read_b64_tr_b16 when the ring
  // fits the 16-bit offset field, else the stage part is one add per fragment and stage. The loop body is unrolled
  // over the ring's stages so the stage index is a compile-time constant. (The round-4 loop recomputed every read
  // address from a runtime stage base: 44 VALU adds per 32 MFMAs in the weight-gradient kernel.)
  const unsigned ring_lds = (unsigned)(uintptr_t)(SDMI_LDS const char*)ring;
  unsigned fa_base[4], fb_base[NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int mb = wm + 16 * i;
    fa_base[i] = ring_lds + (mb >> 7) * SUB + frag_tr_lane(mb & 127, lane);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nb = wn + 16 * j;
    fb_base[j] = ring_lds + A_BYTES + (nb >> 7) * SUB + frag_tr_lane(nb & 127, lane);
  }
  // largest immediate: last stage + last k-step + the +4-row half
  constexpr bool STAGE_IMM = (STAGES - 1) * STAGE_BYTES + (KS - 1) * 8192 + 1024 < 65536;
  static_assert(STAGES <= 6, "stage-unrolled loop");

  // one k-tile of this k-group at ring stage st_c (IC: compile time; RT: run time): wait, barrier, refill, MFMAs
  auto step = [&](int t, auto st_c) __attribute__((always_inline)) {
    using SC = decltype(st_c);
    constexpr bool CST = !std::is_same<SC, RT>::value;
    const int ST = st_c.value;
    // tile t landed for this thread: at most (tiles issued after t) x (A_PW + B_PW) DMA instructions outstanding
    // (in the last STAGES-2 tiles fewer are in flight: wait for all)
    if (STAGES > 2 && t + STAGES - 2 < nt)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"((STAGES > 2 ? STAGES - 2 : 0) * (A_PW + B_PW)) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMA for tile t done; every wave done with tile t-1
    if (t == 0) SDMI_TRACE_T(1);
    if (KG > 1 && t >= nt) return;  // this k-group has no tile t (its last barriers only)
    if (t + STAGES - 1 < nt) issue(kt0 + (t + STAGES - 1) * KG + kg, (ST + STAGES - 1) % STAGES);
    const char* ta = ring + ST * STAGE_BYTES;
    const char* tb = ta + A_BYTES;
    (void)ta;
    (void)tb;
    constexpr int SOFF = [] {
      if constexpr (CST) return STAGE_IMM ? SC::value * STAGE_BYTES : 0;
      else return 0;
    }();
    unsigned fa_b[4], fb_b[NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa_b[i] = STAGE_IMM ? fa_base[i] : fa_base[i] + ST * STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < NJ; ++j) fb_b[j] = STAGE_IMM ? fb_base[j] : fb_base[j] + ST * STAGE_BYTES;
    __builtin_amdgcn_s_setprio(1);
    auto kstep = [&](auto ks_c) __attribute__((always_inline)) {
      constexpr int ks = decltype(ks_c)::value;
      s16x8 fa[4], fb[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mb = wm + 16 * i;
        if constexpr (A_MN) fa[i] = frag_tr_off<SOFF + ks * 8192>(fa_b[i]);
        else fa[i] = frag_kc_k<KBK>(ta, mb, ks, lane);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int nb = wn + 16 * j;
        if constexpr (B_MN) fb[j] = frag_tr_off<SOFF + ks * 8192>(fb_b[j]);
        else fb[j] = frag_kc_k<KBK>(tb, nb, ks, lane);
      }
      if constexpr (A_MN) lds_wait_frags(fa);
      if constexpr (B_MN) lds_wait_frags(fb);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if (RED != 0 && red_tile) {
        const int kb = (kt0 + t * KG + kg) * KBK + ks * 32 + (lane >> 4) * 8;
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) {
          const int r = wave % NWN + rr * NWN;
          if (r < nred) {
            const s16x8 fr = reduce_frag<RED>(g, r, kb, lane);
#pragma unroll
            for (int i = 0; i < 4; ++i)
              accr[rr][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fr, accr[rr][i], 0, 0, 0);
          }
        }
      }
    };
    kstep(IC<0>{});
    if constexpr (KS > 1) kstep(IC<1>{});
    __builtin_amdgcn_s_setprio(0);
  };

  if (nt_loop > 0) {
    // prologue: STAGES-1 tiles in flight
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nt) issue(kt0 + s * KG + kg, s);
    // tile t sits in ring stage t % STAGES: with transposed reads the loop advances STAGES tiles per trip with the
    // stage as a constant; the K-contiguous-only kernels keep the plain loop (their reads fold the stage base
    // themselves, and the unrolled form measured slower for the 32^2 conv forward: 88 -> 93 us)
    if constexpr (!A_MN && !B_MN) {
      for (int t = 0; t < nt_loop; ++t) step(t, RT{t % STAGES});
    } else
    for (int t0 = 0; t0 < nt_loop; t0 += STAGES) {
      step(t0, IC<0>{});
      if constexpr (STAGES > 1) if (t0 + 1 < nt_loop) step(t0 + 1, IC<1 % STAGES>{});
      if constexpr (STAGES > 2) if (t0 + 2 < nt_loop) step(t0 + 2, IC<2 % STAGES>{});
      if constexpr (STAGES > 3) if (t0 + 3 < nt_loop) step(t0 + 3, IC<3 % STAGES>{});
      if constexpr (STAGES > 4) if (t0 + 4 < nt_loop) step(t0 + 4, IC<4 % STAGES>{});
      if constexpr (STAGES > 5) if (t0 + 5 < nt_loop) step(t0 + 5, IC<5 % STAGES>{});
    }
  }
  SDMI_TRACE_T(2);
  __syncthreads();
  SDMI_TRACE_T(4);
  if constexpr (KG > 1) {
    // k-group g > 0 hands its accumulators (and reduction-tile sums) to k-group 0 through LDS, one group after the
    // other in group order: a fixed summation order, so the result does not depend on timing. Lane-linear 16-B slots
    // (conflict-free ds_write_b128 / ds_read_b128); NE4 float4 per lane, one [NE4][64] block per wave.
    constexpr int NE4 = 4 * NJ + (RPW > 0 ? RPW : 1) * 4;
    float4* xs = (float4*)smem + (long long)wave * NE4 * 64 + lane;
#pragma unroll 1
    for (int src = 1; src < KG; ++src) {
      if (kg == src) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) xs[(i * NJ + j) * 64] = __builtin_bit_cast(float4, acc[i][j]);
        if constexpr (RED != 0) {
#pragma unroll
          for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
            for (int i = 0; i < 4; ++i) xs[(4 * NJ + rr * 4 + i) * 64] = __builtin_bit_cast(float4, accr[rr][i]);
        }
      }
      __syncthreads();
      if (kg == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] += __builtin_bit_cast(f32x4, xs[(i * NJ + j) * 64]);
        if constexpr (RED != 0) {
#pragma unroll
          for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
            for (int i = 0; i < 4; ++i) accr[rr][i] += __builtin_bit_cast(f32x4, xs[(4 * NJ + rr * 4 + i) * 64]);
        }
      }
      __syncthreads();
    }
  }
  EpiArgs ev = epi_args_late();  // epilogue arguments loaded only from here on (see gemm_kernel)
  if (grp) group_epi(ev, g.Cg[grp], g.sum_g[grp], grp);
  // The column tiles of this kernel cover only the n GEMM columns; the reduction columns [n_x0, n_gemm) of a split-K
  // slab belong to the reduction tiles below. The last column tile's padding (n % TBN != 0) must not store its zero
  // accumulators there: it raced with the reduction tile's stores of the same slab entries (round-4 gsum probe).
  if (RED == 2) ev.n_gemm = ev.n_x0;
  const EpiArgs* ep = &ev;
  if (RED != 0 && red_tile && kg == 0) {
    // lane holds C[wm + 16i + 4(lane>>4) + q][r*16 + (lane & 15)]: column 0 = row sums, 8 + j = group j
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int col = (wave % NWN + rr * NWN) * 16 + (lane & 15);
      if (!(col == 0 || (RED == 2 && col >= 8 && col - 8 < ep->ngrp))) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + q;
          if (row >= ep->M) continue;
          const float v = accr[rr][i][q];
          if (ep->raw) ((float*)ep->ws)[(long long)z * ep->split_stride + (long long)row * ep->N + ep->n_x0 + col] = v;
          else Epi::extra(*ep, row, ep->n_x0 + col, &v, 1);
        }
    }
  }
  // only k-group 0 holds the tile (wm = -1: the other groups' waves stage nothing, but share the stores)
  SDMI_TRACE_T(5);
  gemm_epilogue<TBN, false, TBM, NJ, NTH, GNE>(*ep, acc, smem, m0, n0, kg == 0 ? wm : -1, wn, lane, z);
#ifdef SDMI_GEMM_TRACE
  SDMI_TRACE_T(3);
  if (threadIdx.x == 0) {
    const unsigned d = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (d < (1u << 17)) {
#pragma unroll
      for (int i = 0; i < 8; ++i) g_gemm_trace[d * 8 + i] = tr_t[i];
    }
  }
#endif
}

// Sum split-K slabs and apply the epilogue, N % 8 == 0 (16-B slab reads). A workgroup owns 256/SL consecutive
// 8-column items; its SL slab lanes sum disjoint slab subsets (a wave reads 64 consecutive items of ONE slab:
// contiguous 2 KiB) and are merged in LDS in a fixed order, so the result is deterministic. SL > 1 spreads the
// deep split-K of small weight gradients (a 128 x 128 dW = 2048 items) over enough workgroups to fill the chip.
template <int SL>
__global__ __launch_bounds__(256) void splitk_reduce_n8_kernel(const EpiArgs g0) {
  EpiArgs g = g0;  // grid.y = problem of a grouped launch
  if (blockIdx.y) group_epi(g, g0.Cg[blockIdx.y], g0.sum_g[blockIdx.y], blockIdx.y);
  constexpr int IPB = 256 / SL;
  __shared__ float4 part[SL > 1 ? SL : 1][IPB][2];
  const float* ws = g.ws;
  const unsigned N8 = g.N >> 3;
  const unsigned total = (unsigned)g.M * N8;
  const int zs = (int)g.split_stride;
  const int li = threadIdx.x % IPB, sl = threadIdx.x / IPB;
  for (unsigned i0 = blockIdx.x * IPB; i0 < total; i0 += gridDim.x * IPB) {  // uniform trip count per block
    const unsigned idx = i0 + li;
    // 32-bit index math (slabs are < 2^31 bytes) and a multiply-high row split: no 64-bit division per chunk
    const unsigned r = g.n8_magic ? __umulhi(idx, g.n8_magic) : (N8 == 1 ? idx : idx / N8);
    const int row = (int)r, col = (int)(idx - r * N8) * 8;
    const int base = row * g.N + col;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (idx < total) {
      for (int zz = sl; zz < g.nsplit; zz += SL) {
        const float* p = ws + zz * zs + base;
        const float4 x = *(const float4*)p, y = *(const float4*)(p + 4);
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
        b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
      }
    }
    if constexpr (SL > 1) {
      part[sl][li][0] = a;
      part[sl][li][1] = b;
      __syncthreads();
      if (sl == 0) {
#pragma unroll
        for (int q = 1; q < SL; ++q) {
          const float4 x = part[q][li][0], y = part[q][li][1];
          a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
          b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
        }
      }
      __syncthreads();
    }
    if (sl == 0 && idx < total) {
      float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      if (g.n_x0 && col >= g.n_x0) {
        Epi::extra(g, row, col, v, 8);
      } else if (g.vec) {
        if (row < g.m_store && col < g.n_store) Epi::finish8(g, row, col, v);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) Epi::store_final(g, row, col + e, v[e]);
      }
    }
  }
}

// Sum split-K slabs, store bf16(alpha * sum) and the GroupNorm-backward statistics (EpiArgs::gn_part): grid
// (ceil(N / 256), M / gn_rb); 256 threads = 32 column chunks x 8 row lanes, the row lanes summed in LDS in a fixed
// order into the segment's column partials (same arithmetic as epi_gn_half).
__global__ __launch_bounds__(256) void splitk_reduce_gn_kernel(const EpiArgs e) {
  __shared__ float red[8][256][2];
  const int t = threadIdx.x, c8 = t & 31, rl0 = t >> 5;
  const int col = blockIdx.x * 256 + c8 * 8;
  const int r0 = blockIdx.y * e.gn_rb;
  const bool on = col < e.N;
  float u[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, w[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (on) {
    const int b = (int)e.gn_pd.div((unsigned)r0);
    float4 tb[8];
    const float4* tp = e.gn_tab + (long long)b * e.N + col;
#pragma unroll
    for (int q = 0; q < 8; ++q) tb[q] = tp[q];
    const int zs = (int)e.split_stride;
#pragma unroll 1
    for (int rl = rl0; rl < e.gn_rb; rl += 8) {
      const int row = r0 + rl;
      // the slab sum in splitk_reduce_n8_kernel<gn_sl>'s order: lane l sums slabs l, l + SL, ... in order, then the
      // lanes are added in lane order -- so the stored dy is bitwise the reducer's without the statistics
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
      const float* p = e.ws + (long long)row * e.N + col;
#pragma unroll 1
      for (int l = 0; l < e.gn_sl; ++l) {
        float4 pa = make_float4(0.f, 0.f, 0.f, 0.f), pc = pa;
#pragma unroll 4
        for (int zz = l; zz < e.nsplit; zz += e.gn_sl) {
          const float4 x = *(const float4*)(p + (long long)zz * zs), y = *(const float4*)(p + (long long)zz * zs + 4);
          pa.x += x.x; pa.y += x.y; pa.z += x.z; pa.w += x.w;
          pc.x += y.x; pc.y += y.y; pc.z += y.z; pc.w += y.w;
        }
        if (l == 0) {
          a = pa;
          c = pc;
        } else {
          a.x += pa.x; a.y += pa.y; a.z += pa.z; a.w += pa.w;
          c.x += pc.x; c.y += pc.y; c.z += pc.z; c.w += pc.w;
        }
      }
      float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] *= e.alpha;
      const uint4 xr = *(const uint4*)(e.gn_x + (long long)row * e.gn_ldx + col);
      const uint4 pk = pack8(v);
      *(uint4*)((bf16_t*)e.C + (long long)row * e.ldc + col) = pk;
      unpack8(pk, v);
      gn_accum(e, v, xr, tb, u, w);
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    red[rl0][c8 * 8 + q][0] = u[q];
    red[rl0][c8 * 8 + q][1] = w[q];
  }
  __syncthreads();
  const int j = blockIdx.x * 256 + t;
  if (j < e.N) {
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      a1 += red[r][t][0];
      a2 += red[r][t][1];
    }
    *(float2*)(e.gn_part + ((long long)blockIdx.y * e.N + j) * 2) = make_float2(a1, a2);
  }
}

// Sum split-K slabs and apply the epilogue, general N (one element per thread).
__global__ void splitk_reduce_kernel(const EpiArgs g0) {
  EpiArgs g = g0;  // grid.y = problem of a grouped launch
  if (blockIdx.y) group_epi(g, g0.Cg[blockIdx.y], g0.sum_g[blockIdx.y], blockIdx.y);
  const float* ws = g.ws;
  long long stride = (long long)gridDim.x * blockDim.x;
  long long total = (long long)g.M * g.N;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += stride) {
    float s = 0.f;
    for (int zz = 0; zz < g.nsplit; ++zz) s += ws[(long long)zz * g.split_stride + idx];
    int row = (int)(idx / g.N), col = (int)(idx - (long long)row * g.N);
    Epi::store(g, row, col, s, 0);
  }
}

// slab lanes of the n8 reducer: aim for >= 1024 workgroups
int reduce_lanes(const EpiArgs& red) {
  const long long items = (long long)red.M * (red.N / 8);
  int sl = 1;
  while (sl < 32 && sl * 2 <= red.nsplit && items * sl / 256 < 1024) sl *= 2;
  return sl;
}

hipError_t launch_reduce(const EpiArgs& red, hipStream_t s, int G = 1) {
  if (red.gn_part) {
    EpiArgs r = red;
    r.gn_sl = reduce_lanes(red);
    sdmi_rt::launch(splitk_reduce_gn_kernel, dim3((unsigned)((red.N + 255) / 256), (unsigned)(red.M / red.gn_rb)),
                    dim3(256), 0, s, r);
    return hipGetLastError();
  }
  if (!red.n8) {
    const long long total = (long long)red.M * red.N;
    sdmi_rt::launch(splitk_reduce_kernel, dim3((unsigned)std::min<long long>((total + 255) / 256, 4096), G), dim3(256),
                       0, s, red);
    return hipGetLastError();
  }
  const long long items = (long long)red.M * (red.N / 8);
  const int sl = reduce_lanes(red);
  const unsigned blocks = (unsigned)std::min<long long>((items * sl + 255) / 256, 8192);
  const dim3 grid(blocks, G);  // y: problem of a grouped launch
  switch (sl) {
    case 1: sdmi_rt::launch(splitk_reduce_n8_kernel<1>, grid, dim3(256), 0, s, red); break;
    case 2: sdmi_rt::launch(splitk_reduce_n8_kernel<2>, grid, dim3(256), 0, s, red); break;
    case 4: sdmi_rt::launch(splitk_reduce_n8_kernel<4>, grid, dim3(256), 0, s, red); break;
    case 8: sdmi_rt::launch(splitk_reduce_n8_kernel<8>, grid, dim3(256), 0, s, red); break;
    case 16: sdmi_rt::launch(splitk_reduce_n8_kernel<16>, grid, dim3(256), 0, s, red); break;
    default: sdmi_rt::launch(splitk_reduce_n8_kernel<32>, grid, dim3(256), 0, s, red); break;
  }
  return hipGetLastError();
}

bool has_reductions(const sdmi_gemm_desc* d) { return d->sum_out || d->sum_out2 || d->gsum_out; }

int reduction_groups(const sdmi_gemm_desc* d) {
  return d->gsum_out && d->sum_group > 0 ? (d->k + d->sum_group - 1) / d->sum_group : 0;
}

// columns the launch computes: n, plus the reduction columns (8 for the sums, then the groups rounded to 8)
int n_total(const sdmi_gemm_desc* d) {
  if (!d->gsum_out) return d->n;  // plain sums: VALU row sums (Args::rowsum), no extra columns
  return (d->n + 7) / 8 * 8 + 8 + (reduction_groups(d) + 7) / 8 * 8;
}

// slab row width with split-K: the produced columns, plus one 8-column chunk carrying the VALU row sums
int slab_n(const sdmi_gemm_desc* d) { return n_total(d) + ((has_reductions(d) && !d->gsum_out) ? 8 : 0); }

// Mainloop choice (SDMI_GEMM_VARIANT overrides for A/B runs): 0 register-staged; LDS-DMA rings: 2 / 3 stages of
// 64-deep 128-row tiles (4 waves), 4 = 128 x {256, 384} tiles on 8 waves with a 4-stage ring of 32-deep stages (3
// tiles, 96 KiB, in flight per CU), 5 = 128 x {128, 192} tiles on 4 waves with a 3-stage ring of 32-deep stages (two
// workgroups per CU), 6 = 128 x 128 with 4 stages, 7 / 8 = 64 x {64, 128} tiles with 6 stages, 9 / 10 = 64 x 128 tiles
// with 3 / 2 stages. -1 (default) per mode: the DMA ring where it measured faster on the step's shapes (row-major
// and implicit-conv A), register staging for the col-major (weight-gradient) A; the per-shape table
// sdmi/tuned_gemm.json overrides it through variant_hint.
int gemm_variant() {
  static int v = -2;
  if (v == -2) {
    const char* s = getenv("SDMI_GEMM_VARIANT");
    v = s ? atoi(s) : -1;
    if (v != 0 && (v < 2 || v > 11)) v = -1;
  }
  return v;
}

// the DMA kernels form the reduction columns from synthesised B fragments: every group of 8 consecutive k in one
// group (sum_group % 8 == 0) and at most 3 reduction tiles (8 + groups <= 48)
bool dma_reductions_ok(const sdmi_gemm_desc* d) {
  if (!d->gsum_out) return true;
  return d->sum_group % 8 == 0 && 8 + reduction_groups(d) <= 48;
}

int pick_variant(const sdmi_gemm_desc* d) {
  int v = gemm_variant();
  if (v < 0 && d->variant_hint >= 1 && d->variant_hint <= 11) v = d->variant_hint == 1 ? 0 : d->variant_hint;
  if (v < 0) v = 2;  // (col-major A with [n][k] B has no DMA instantiation: register staging below)
  if (has_reductions(d) && (v == 3 || !dma_reductions_ok(d))) v = v == 3 ? 2 : 0;
  if (has_reductions(d) && v != 0 && d->a_mode != SDMI_A_COLMAJOR) v = 0;
  // the DMA path needs a tile-uniform second source (k_split % BK == 0)
  if (d->a_mode == SDMI_A_CONV && d->a2 && d->k_split % BK) v = 0;
  if (v == 4 && d->n % 256 && d->n % 384) v = 2;  // 128 x {256, 384} tiles: N % 384 == 0 or N % 256 == 0
  if (v == 5 && d->a_mode == SDMI_A_CONV && d->a2 && d->k_split % 32) v = 0;
  if (v != 0 && d->a_mode == SDMI_A_COLMAJOR && d->b_mode == SDMI_B_NK) v = 0;  // no DMA instantiation
  // 64-row tiles: K-contiguous images only (row-major / implicit-conv A, [n][k] B), no reduction columns
  if (v >= 7 && v <= 10 && (d->a_mode == SDMI_A_COLMAJOR || d->b_mode != SDMI_B_NK || has_reductions(d))) v = 2;
  // k-groups (128 x 128 tiles of two 4-wave groups): the DMA modes; the conv A's fused second source needs whole
  // 64-deep tiles on either side of k_split (checked above for every DMA variant)
  return v;
}

int tile_m(const sdmi_gemm_desc*, int variant) { return variant >= 7 && variant <= 10 ? 64 : BM; }

// columns the grid covers: the DMA kernels compute the reduction columns outside the column tiles
int n_grid(const sdmi_gemm_desc* d, int variant) { return variant == 0 ? n_total(d) : d->n; }

// Column-tile width: 192 (2-stage DMA, B_NK, N % 192 == 0) when it needs fewer rounds x columns of the
// 512 workgroup slots (2 per CU) than 128 -- e.g. 32768 x 384: 768 tiles = 1.5 rounds at 128, 512 = 1 at 192.
int pick_tbn(const sdmi_gemm_desc* d, int variant) {
  if (variant == 4) return d->n % 384 == 0 ? 384 : 256;
  if (variant == 7) return 64;
  if (variant >= 8 || variant == 6) return BN;  // incl. 11 (k-groups)
  if (variant == 5) return d->b_mode == SDMI_B_NK && d->n % 192 == 0 ? 192 : BN;
  if (variant != 2 || d->b_mode != SDMI_B_NK || d->a_mode == SDMI_A_COLMAJOR) return BN;
  // narrow outputs (N <= 64: the VQVAE's 64-channel convs at 256^2, 4-channel heads, DiT proj_out): a 128-column
  // tile would spend half (or more) of its MFMAs on zero-padded columns
  if (d->n <= 64) return 64;
  // ragged N whose last 128-column tile would be at most half used (DiT hidden size 288: 3 x 128 = 384 columns,
  // 25 % padding; 5 x 64 = 320, 10 %)
  if (d->tile_n_hint != 128 && d->n % 128 && d->n % 128 <= 64 && d->n % 192) return 64;
  if (d->n % 192) return BN;
  if (d->tile_n_hint == 128 || d->tile_n_hint == 192) return d->tile_n_hint;
  const long long mt = (d->m + BM - 1) / BM;
  const long long r128 = (mt * ((d->n + BN - 1) / BN) + 511) / 512, r192 = (mt * (d->n / 192) + 511) / 512;
  return r192 * 192 <= r128 * 128 ? 192 : BN;
}

template <int AM, int BMODE, int STAGES, int TBN, int TBM, int NWN, int RED, int KBK = BK, int KG = 1>
hipError_t launch_dma(const Args& a, const EpiArgs& e, dim3 grid, hipStream_t s) {
  constexpr int NTH = dma_threads<TBM, NWN>();
  constexpr size_t ring = (size_t)STAGES * (TBM + TBN) * KBK * 2 * KG, epi = (size_t)64 * (TBN + 4) * 4;
  if constexpr (RED == 0 && AM != SDMI_A_COLMAJOR && BMODE != SDMI_B_KN_CONV) {
    if (e.gn_part && !e.raw) {  // GroupNorm statistics: + the row-lane sums (NTH / (TBN / 8) x TBN x 2 floats)
      const size_t epi_gn = epi + (size_t)(NTH * KG / (TBN / 8)) * TBN * 2 * 4;
      size_t lds = std::max(ring, epi_gn);
      if constexpr (KG > 1) lds = std::max(lds, (size_t)(4 * (TBN / NWN / 16) + 4) * 16 * NTH);
      sdmi_rt::launch((gemm_dma_kernel<AM, BMODE, STAGES, TBN, TBM, NWN, 0, KBK, true, KG>), grid, dim3(NTH * KG), lds, s,
                      a, e);
      return hipGetLastError();
    }
  }
  if (e.gn_part && !e.raw) return hipErrorInvalidValue;
  if constexpr (KG > 1) {
    // + the k-group hand-off of the accumulators: (4 NJ + 4 RPW) float4 per lane, per wave of one group
    constexpr int NJ = TBN / NWN / 16, RPW = RED == 0 ? 1 : (RED == 1 ? 1 : (3 + NWN - 1) / NWN);
    constexpr size_t xs = (size_t)(4 * NJ + 4 * RPW) * 16 * NTH;
    static_assert(std::max(ring, std::max(epi, xs)) <= 160 * 1024, "LDS");
    sdmi_rt::launch((gemm_dma_kernel<AM, BMODE, STAGES, TBN, TBM, NWN, RED, KBK, false, KG>), grid, dim3(NTH * KG),
                    std::max(ring, std::max(epi, xs)), s, a, e);
    return hipGetLastError();
  }
  sdmi_rt::launch((gemm_dma_kernel<AM, BMODE, STAGES, TBN, TBM, NWN, RED, KBK>), grid, dim3(NTH), std::max(ring, epi), s,
                  a, e);
  return hipGetLastError();
}

template <int AM, int BMODE, int RED>
hipError_t launch_dma_red(const Args& a, const EpiArgs& e, dim3 grid, hipStream_t s, int v, int tbn) {
  if (v == 3 && RED == 0) return launch_dma<AM, BMODE, 3, BN, BM, 2, 0>(a, e, grid, s);
  // two k-groups of 4 waves on one 128 x 128 tile, 2-stage 64-deep rings (128 KiB): one 8-wave workgroup per CU
  if (v == 11) return launch_dma<AM, BMODE, 2, BN, BM, 2, RED, BK, 2>(a, e, grid, s);
  if (v == 6) return launch_dma<AM, BMODE, 4, BN, BM, 2, RED>(a, e, grid, s);  // 4-stage 128 x 128 (128 KiB ring)
  if constexpr (BMODE == SDMI_B_NK && AM != SDMI_A_COLMAJOR && RED == 0) {
    if (v == 7) return launch_dma<AM, BMODE, 6, 64, 64, 4, 0>(a, e, grid, s);    // 64 x 64, 6 stages (96 KiB)
    if (v == 8) return launch_dma<AM, BMODE, 6, 128, 64, 4, 0>(a, e, grid, s);   // 64 x 128, 6 stages (144 KiB)
    // 64 x 128 with 3 / 2 stages (72 / 48 KiB: two or three workgroups per CU) -- the M = 2048-8192 GEMMs whose
    // 128 x 128 grid is one tile per CU (8192 x 512: 256 tiles)
    if (v == 9) return launch_dma<AM, BMODE, 3, 128, 64, 4, 0>(a, e, grid, s);
    if (v == 10) return launch_dma<AM, BMODE, 2, 128, 64, 4, 0>(a, e, grid, s);
  }
  if (v == 4) {  // 128 x {256, 384} on 8 waves, 32-deep stages, 4-stage ring (3 tiles in flight)
    if (tbn == 384) return launch_dma<AM, BMODE, 4, 384, BM, 4, RED, 32>(a, e, grid, s);
    if (tbn == 256) return launch_dma<AM, BMODE, 4, 256, BM, 4, RED, 32>(a, e, grid, s);
    return hipErrorInvalidValue;
  }
  if (v == 5) {  // 128 x {128, 192} on 4 waves, 32-deep stages, 3-stage ring, two workgroups per CU
    if (tbn == BN) return launch_dma<AM, BMODE, 3, BN, BM, 2, RED, 32>(a, e, grid, s);
    if constexpr (BMODE == SDMI_B_NK && RED == 0) {
      if (tbn == 192) return launch_dma<AM, BMODE, 3, 192, BM, 2, 0, 32>(a, e, grid, s);
    }
    return hipErrorInvalidValue;
  }
  if (tbn == BN) return launch_dma<AM, BMODE, 2, BN, BM, 2, RED>(a, e, grid, s);
  if constexpr (BMODE == SDMI_B_NK && AM != SDMI_A_COLMAJOR && RED == 0) {
    if (tbn == 64) return launch_dma<AM, BMODE, 2, 64, BM, 2, 0>(a, e, grid, s);
    if (tbn == 192) return launch_dma<AM, BMODE, 2, 192, BM, 2, 0>(a, e, grid, s);
  }
  return hipErrorInvalidValue;
}

template <int AM, int BMODE>
hipError_t launch_t(const Args& a, const EpiArgs& e, dim3 grid, hipStream_t s, int v, int tbn) {
  if (v == 0) {
    if constexpr (AM == SDMI_A_COLMAJOR) {
      if (a.rowsum) {
        sdmi_rt::launch((gemm_kernel<AM, BMODE, 1>), grid, dim3(NT), 0, s, a, e);
        return hipGetLastError();
      }
      if (a.n_x0) {
        sdmi_rt::launch((gemm_kernel<AM, BMODE, 2>), grid, dim3(NT), 0, s, a, e);
        return hipGetLastError();
      }
    }
    if constexpr (AM != SDMI_A_COLMAJOR && BMODE != SDMI_B_KN_CONV) {
      if (e.gn_part && !e.raw) {
        sdmi_rt::launch((gemm_kernel<AM, BMODE, 0, true>), grid, dim3(NT), 0, s, a, e);
        return hipGetLastError();
      }
    }
    if (e.gn_part && !e.raw) return hipErrorInvalidValue;
    sdmi_rt::launch((gemm_kernel<AM, BMODE>), grid, dim3(NT), 0, s, a, e);
    return hipGetLastError();
  }
  if constexpr (AM == SDMI_A_COLMAJOR && BMODE != SDMI_B_NK) {
    if (a.n_x0) return launch_dma_red<AM, BMODE, 2>(a, e, grid, s, v, tbn);
    if (a.rowsum) return launch_dma_red<AM, BMODE, 1>(a, e, grid, s, v, tbn);
  }
  return launch_dma_red<AM, BMODE, 0>(a, e, grid, s, v, tbn);
}

int fill_args(const sdmi_gemm_desc* d, Args& a, EpiArgs& e) {
  if (!d || d->m <= 0 || d->n <= 0 || d->k <= 0) return -1;
  // K is the contiguous (16-B chunked) dimension of row-major / conv A and of [n][k] B only
  if ((d->a_mode != SDMI_A_COLMAJOR || d->b_mode == SDMI_B_NK) && (d->k % 8)) return -2;
  if ((d->a_mode == SDMI_A_COLMAJOR) && (d->m % 8)) return -3;
  if ((d->b_mode != SDMI_B_NK) && (d->n % 8)) return -4;
  if (d->a_mode == SDMI_A_CONV || d->b_mode == SDMI_B_KN_CONV) {
    const sdmi_conv_geom& q = d->geom;
    if (q.cin <= 0 || q.cin % 8 || q.kw <= 0 || q.ldx % 8) return -5;
  }
  if (d->a2 && (d->k_split % 8 || d->lda2 % 8)) return -7;
  memset(&a, 0, sizeof(a));
  memset(&e, 0, sizeof(e));
  a.M = d->m; a.N = d->n; a.K = d->k;
  a.A = (const bf16_t*)d->a; a.lda = d->lda;
  a.B = (const bf16_t*)d->b; a.ldb = d->ldb;
  a.ih = d->geom.ih; a.iw = d->geom.iw; a.cin = d->geom.cin; a.ldx = d->geom.ldx; a.kw = d->geom.kw;
  if ((d->a_mode == SDMI_A_CONV || d->b_mode == SDMI_B_KN_CONV) && (d->geom.oh <= 0 || d->geom.ow <= 0)) return -5;
  a.ohw_d = FastDiv::make(std::max(1, d->geom.oh * d->geom.ow));
  a.ow_d = FastDiv::make(std::max(1, d->geom.ow));
  a.sy = d->geom.sy; a.sx = d->geom.sx; a.oy0 = d->geom.oy0; a.ox0 = d->geom.ox0;
  if (d->b_mode == SDMI_B_KN_CONV) {
    const int ohw = d->geom.oh * d->geom.ow, ow = d->geom.ow;
    for (int sh = 0; sh < 2; ++sh) {  // KBK 64, then 32
      const int kb = sh ? 32 : 64;
      const int f = (ohw % kb == 0 && kb % ow == 0) ? 1 : (kb % ohw == 0 ? 2 : 0);
      a.bfast |= f << (2 * sh);
    }
  }
  a.A2 = (const bf16_t*)d->a2; a.lda2 = d->lda2;
  a.k_split = (d->a_mode == SDMI_A_CONV && d->a2) ? d->k_split : d->k;
  e.M = d->m; e.N = d->n;
  e.n_gemm = n_total(d);
  e.C = d->c; e.ldc = d->ldc; e.c_f32 = d->c_f32;
  e.bias = d->bias; e.bias2 = d->bias2;
  e.rowbias = (const bf16_t*)d->rowbias; e.rb_ld = d->rb_ld;
  e.resid = (const bf16_t*)d->resid; e.ldr = d->ldr;
  e.alpha = d->alpha; e.act = d->act;
  e.remap = d->remap; e.r_oh = d->r_oh; e.r_ow = d->r_ow;
  if (d->remap && (d->r_gh <= 0 || d->r_gw <= 0)) return -11;
  if (d->remap && d->rowbias && std::max(1, d->rb_div) != d->r_gh * d->r_gw) return -12;
  e.pix_d = FastDiv::make(d->remap ? d->r_gh * d->r_gw : std::max(1, d->rb_div));
  e.gw_d = FastDiv::make(d->remap ? d->r_gw : 1);
  e.r_sy = d->r_sy; e.r_sx = d->r_sx; e.r_oy = d->r_oy; e.r_ox = d->r_ox;
  e.perm = d->perm; e.p_cin = d->p_cin; e.p_taps = d->p_taps;
  if (d->perm && (d->p_cin < 8 || d->p_cin % 8)) return -10;
  e.p_magic = d->perm ? (unsigned)(((1ULL << 32) + d->p_cin - 1) / d->p_cin) : 0u;
  {  // multiply-high division by N/8 is exact for idx < 2^32 / (N/8), i.e. when M * (N/8)^2 < 2^32
    const unsigned long long n8 = (unsigned long long)(d->n >> 3);
    e.n8_magic = (n8 > 1 && (unsigned long long)d->m * n8 * n8 < (1ULL << 32)) ? (unsigned)(((1ULL << 32) + n8 - 1) / n8)
                                                                               : 0u;
  }
  e.p_cvalid = d->p_cvalid > 0 ? d->p_cvalid : d->p_cin;
  e.m_store = d->m_store > 0 ? d->m_store : d->m;
  e.n_store = d->n_store > 0 ? d->n_store : d->n;
  e.n8 = d->n % 8 == 0;
  e.rb_mod = d->rb_mod;
  e.aux = (const bf16_t*)d->aux; e.ld_aux = d->ld_aux;
  if (has_reductions(d)) {
    if (d->a_mode != SDMI_A_COLMAJOR || d->b_mode == SDMI_B_NK) return -13;
    if (d->gsum_out && (d->sum_group <= 0 || d->gsum_ld <= 0)) return -14;
    if (d->gsum_out) {
      a.n_x0 = e.n_x0 = (d->n + 7) / 8 * 8;
      a.grp_d = FastDiv::make(std::max(1, d->sum_group));
    } else {
      a.rowsum = 1;
      e.n_x0 = d->n;  // slab chunk of the row sums (split-K); never produced by the MFMA tiles
    }
    e.ngrp = reduction_groups(d);
    e.gsum_ld = d->gsum_ld;
    e.sum_out = d->sum_out;
    e.sum_out2 = d->sum_out2;
    e.gsum = (bf16_t*)d->gsum_out;
    e.N = slab_n(d);  // split-K slabs cover the reduction columns too
    const unsigned long long n8 = (unsigned long long)(e.N >> 3);
    e.n8_magic = (n8 > 1 && (unsigned long long)d->m * n8 * n8 < (1ULL << 32)) ? (unsigned)(((1ULL << 32) + n8 - 1) / n8)
                                                                              : 0u;
  }
  if (d->act == 3 && !d->aux) return -8;
  if (d->act < 0 || d->act > 3) return -9;
  e.vec = !d->perm && d->n % 8 == 0 && e.n_store % 8 == 0 && d->ldc % 8 == 0 &&
          (!d->resid || d->ldr % 8 == 0) && (!d->rowbias || d->rb_ld % 8 == 0) &&
          ((uintptr_t)d->c % 16 == 0) && (!d->bias || (uintptr_t)d->bias % 16 == 0) &&
          (!d->bias2 || (uintptr_t)d->bias2 % 16 == 0) && (!d->resid || (uintptr_t)d->resid % 16 == 0) &&
          (!d->rowbias || (uintptr_t)d->rowbias % 16 == 0) &&
          (d->act != 3 || (d->ld_aux % 8 == 0 && (uintptr_t)d->aux % 16 == 0));
  if (d->gn_part) {  // GroupNorm-backward statistics: plain bf16 epilogue, whole segments inside one sample
    if (!d->gn_x || !d->gn_tab || d->gn_P <= 0 || d->m % d->gn_P || (d->gn_rb != 16 && d->gn_rb != 32 && d->gn_rb != 64) ||
        d->gn_P % d->gn_rb || d->gn_P >= (1 << 24))
      return -20;
    if (d->bias || d->bias2 || d->rowbias || d->resid || d->act || d->remap || d->perm || has_reductions(d) || d->c_f32 ||
        !e.vec || e.m_store != d->m || e.n_store != d->n || (uintptr_t)d->gn_part % 8 || d->gn_ldx % 8 ||
        (uintptr_t)d->gn_x % 16 || (uintptr_t)d->gn_tab % 16)
      return -21;
    e.gn_x = (const bf16_t*)d->gn_x;
    e.gn_ldx = d->gn_ldx;
    e.gn_tab = (const float4*)d->gn_tab;
    e.gn_part = d->gn_part;
    e.gn_rb = d->gn_rb;
    e.gn_silu = d->gn_silu;
    e.gn_pd = FastDiv::make(d->gn_P);
  }
  return 0;
}

// split-K slices: the measured per-shape count (splits_hint, sdmi/tuned_gemm.json) where there is one, else a shallow
// default (>= 8 k-tiles per slice, at most 16 slices, until the grid has 384 tiles)
int plan_splits(const sdmi_gemm_desc* d) {
  const int v = pick_variant(d), tbn = pick_tbn(d, v), tbm = tile_m(d, v);
  const long long tiles = (long long)((d->m + tbm - 1) / tbm) * ((n_grid(d, v) + tbn - 1) / tbn);
  const int nkt = (d->k + BK - 1) / BK;
  if (d->splits_hint > 0) {
    int s = std::min(d->splits_hint, nkt);
    while (s > 1 && (long long)s * d->m * slab_n(d) * 4 >= (1LL << 31)) s >>= 1;
    return std::max(s, 1);
  }
  int s = 1;
  while (tiles * s < 384 && nkt / (s * 2) >= 8 && s < 16) s *= 2;
  return s;
}

}  // namespace

// which mainloop / column-tile width a launch of this descriptor uses (variant: 0 register-staged, 2 .. 5 the LDS-DMA
// rings of gemm_variant(); tile_n: 64 .. 384) -- for profiling / roofline attribution
extern "C" int sdmi_gemm_kernel_info(const sdmi_gemm_desc* d, int* variant, int* tile_n) {
  if (!d) return -1;
  const int v = pick_variant(d);
  if (variant) *variant = v;
  if (tile_n) *tile_n = pick_tbn(d, v);
  return 0;
}

extern "C" int sdmi_gemm_plan(const sdmi_gemm_desc* d, int* splits, size_t* ws) {
  Args a;
  EpiArgs e;
  int rc = fill_args(d, a, e);
  if (rc) return rc;
  int s = plan_splits(d);
  if (splits) *splits = s;
  if (ws) *ws = s > 1 ? (size_t)s * d->m * slab_n(d) * sizeof(float) : 0;
  return 0;
}

namespace {
// descriptors that may share one grouped launch: identical in every field but the operand / output pointers
bool same_problem_shape(const sdmi_gemm_desc* a, const sdmi_gemm_desc* b) {
  sdmi_gemm_desc x = *a, y = *b;
  x.a = y.a = nullptr;
  x.b = y.b = nullptr;
  x.c = y.c = nullptr;
  x.sum_out = y.sum_out = nullptr;
  return memcmp(&x, &y, sizeof(x)) == 0;
}

// split count of a launch carrying G problems: the single problem's (tuned / heuristic) count shared out over them
int group_splits(const sdmi_gemm_desc* d, int G) {
  const int s = plan_splits(d);
  return G > 1 ? std::max(1, (s + G / 2) / G) : s;
}

int run_gemm(const sdmi_gemm_desc* d, int G, void* workspace, size_t ws_bytes, hipStream_t s) {
  Args a;
  EpiArgs e;
  int rc = fill_args(&d[0], a, e);
  if (rc) return rc;
  if (G < 1 || G > SDMI_GEMM_GROUP_MAX) return -15;
  if (G > 1) {
    // grouped: plain / bias-summing GEMMs only (no second A source, no per-row / residual / auxiliary inputs)
    if (d[0].a2 || d[0].resid || d[0].rowbias || d[0].aux || d[0].bias || d[0].bias2 || d[0].sum_out2 || d[0].gsum_out)
      return -16;
    for (int i = 1; i < G; ++i)
      if (!same_problem_shape(&d[0], &d[i]) || (!d[i].sum_out) != (!d[0].sum_out)) return -17;
  }
  a.ngroups = G;
  for (int i = 0; i < G; ++i) {
    a.Ag[i] = (const bf16_t*)d[i].a;
    a.Bg[i] = (const bf16_t*)d[i].b;
    a.Cg[i] = e.Cg[i] = d[i].c;
    a.sum_g[i] = e.sum_g[i] = d[i].sum_out;
  }
  int splits = group_splits(d, G);
  const int nt = n_total(d), ns = slab_n(d);
  const long long slab = (long long)d->m * ns;  // floats per split slab of one problem
  if (splits > 1 && (!workspace || ws_bytes < (size_t)G * splits * slab * sizeof(float))) splits = 1;
  if ((long long)G * splits * slab * 4 >= (1LL << 31)) splits = 1;  // slab offsets are 32-bit
  int nkt = (d->k + BK - 1) / BK;
  a.ktiles_per_split = (nkt + splits - 1) / splits;
  splits = (nkt + a.ktiles_per_split - 1) / a.ktiles_per_split;
  a.nsplit = splits;
  EpiArgs run = e;
  const int variant = pick_variant(d), tbn = pick_tbn(d, variant), tbm = tile_m(d, variant);
  const int ng = n_grid(d, variant);
  dim3 grid((ng + tbn - 1) / tbn, (d->m + tbm - 1) / tbm, splits * G);
  if (splits > 1) {
    run.raw = 1;
    run.ws = (const float*)workspace;
    run.nsplit = splits;
    run.split_stride = slab;
    run.ws_gstride = (long long)splits * slab;
  }
  hipError_t err;
  int key = d->a_mode * 3 + d->b_mode;
  switch (key) {
    case SDMI_A_ROWMAJOR * 3 + SDMI_B_NK: err = launch_t<SDMI_A_ROWMAJOR, SDMI_B_NK>(a, run, grid, s, variant, tbn); break;
    case SDMI_A_ROWMAJOR * 3 + SDMI_B_KN: err = launch_t<SDMI_A_ROWMAJOR, SDMI_B_KN>(a, run, grid, s, variant, tbn); break;
    case SDMI_A_CONV * 3 + SDMI_B_NK: err = launch_t<SDMI_A_CONV, SDMI_B_NK>(a, run, grid, s, variant, tbn); break;
    case SDMI_A_COLMAJOR * 3 + SDMI_B_KN: err = launch_t<SDMI_A_COLMAJOR, SDMI_B_KN>(a, run, grid, s, variant, tbn); break;
    case SDMI_A_COLMAJOR * 3 + SDMI_B_KN_CONV: err = launch_t<SDMI_A_COLMAJOR, SDMI_B_KN_CONV>(a, run, grid, s, variant, tbn); break;
    default: return -6;
  }
  if (err != hipSuccess) return (int)err;
  if (splits > 1) {
    EpiArgs red = e;
    red.raw = 0;
    red.nsplit = splits;
    red.split_stride = slab;
    red.ws_gstride = (long long)splits * slab;
    red.ws = (const float*)workspace;
    err = launch_reduce(red, s, G);
    if (err != hipSuccess) return (int)err;
  }
  return 0;
}
}  // namespace

extern "C" int sdmi_gemm(const sdmi_gemm_desc* d, void* workspace, size_t ws_bytes, sdmi_stream_t stream) {
  if (!d) return -1;
  return run_gemm(d, 1, workspace, ws_bytes, (hipStream_t)stream);
}

extern "C" int sdmi_gemm_grouped_plan(const sdmi_gemm_desc* d, int ngroups, int* splits, size_t* ws) {
  if (!d || ngroups < 1 || ngroups > SDMI_GEMM_GROUP_MAX) return -1;
  Args a;
  EpiArgs e;
  int rc = fill_args(d, a, e);
  if (rc) return rc;
  for (int i = 1; i < ngroups; ++i)
    if (!same_problem_shape(&d[0], &d[i])) return -17;
  const int sp = group_splits(d, ngroups);
  if (splits) *splits = sp;
  if (ws) *ws = sp > 1 ? (size_t)ngroups * sp * d->m * slab_n(d) * sizeof(float) : 0;
  return 0;
}

extern "C" int sdmi_gemm_grouped(const sdmi_gemm_desc* d, int ngroups, void* workspace, size_t ws_bytes,
                                 sdmi_stream_t stream) {
  if (!d) return -1;
  return run_gemm(d, ngroups, workspace, ws_bytes, (hipStream_t)stream);
}

#ifdef SDMI_GEMM_TRACE
// probe build only: copy the first n_u64 words of the phase-timestamp buffer to host memory (device synchronised)
extern "C" int sdmi_gemm_trace_clear(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_gemm_trace)) != hipSuccess) return -1;
  return hipMemset(p, 0, sizeof(g_gemm_trace)) == hipSuccess ? 0 : -2;
}

extern "C" int sdmi_gemm_trace_copy(void* host_dst, long long n_u64) {
  if (!host_dst || n_u64 < 0 || n_u64 > (1 << 20)) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_gemm_trace), (size_t)n_u64 * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : -3;
}
#endif
