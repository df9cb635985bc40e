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
// All three kernels share one structure: 4 waves x 32 rows (two 16-row groups per wave) = 128 rows
// per workgroup stay on the MFMA lanes, the other operand is streamed through a double-buffered LDS
// ring of 64-row tiles (next tile prefetched into registers while the current one is consumed, one
// barrier per tile); every LDS fragment is read once and used by both row groups.
//
// Forward  : queries on lanes, "swapped" S^T = K Q^T so the softmax statistics are per lane and P^T
//            feeds the PV MFMA straight from the accumulator registers (the key order inside a 32-key
//            step is permuted identically in both operands; V is read with ds_read_b64_tr_b16).
// Backward : two kernels, no atomics:
//            dkv: keys on lanes (S = Q K^T): dV^T += dO^T P, dK^T += Q^T dS
//            dq : queries on lanes (S^T = K Q^T): dQ^T += K^T dS^T
//            with P recomputed from the forward's log-sum-exp and delta = rowsum(dO * O).
#include "common.h"
#include "../../include/sdmi.h"
#include <cstdlib>
#include <algorithm>
#include <type_traits>

namespace {

constexpr int NT = 256, ROWS = 128, TILE = 64;
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* o; const bf16_t* dout;
  bf16_t* out; bf16_t* dq; bf16_t* dk; bf16_t* dv;
  float* lse;          // [B*H][N]  base-2 log-sum-exp of (score * scale * log2e)
  const float* delta;  // [B*H][N]
  int ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv;
  int B, H, N, S, d;
  float scale;  // 1/sqrt(d)
  float* dq_part;     // fused backward: per-key-block fp32 dQ partials [nkb][B*H][N][d] (nkb > 1)
  unsigned* ctr;      // fused backward: per-(b*h, query tile) arrival counters (zero between launches)
  int nblk;           // row blocks per (b, h) of the launch (the grid is 1-D: nblk * B * H workgroups)
};

// XCD-local block order. Workgroups are dealt round-robin over the 8 XCDs (dispatch id d runs on XCD d % 8, each XCD
// has its own 4 MiB L2). A (blocks, B*H) grid put the 8 query (key) blocks of one head on 8 different XCDs, so every
// XCD's L2 fetched that head's whole K / V (Q / dO) from HBM: 4.8x the algorithmic reads in the 32^2 backward
// (profiles/pmc_r04j_summary.txt). The 1-D grid is re-numbered so every XCD owns a CONTIGUOUS band of logical ids
// (bijective for any grid size), logical id = bh * nblk + block: the blocks of one head share one L2.
__device__ __forceinline__ void xcd_block(int nblk, int& blk, int& bh) {
  const int total = gridDim.x, d = blockIdx.x;
  const int xcd = d & 7, q = total >> 3, r = total & 7;
  const int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (d >> 3);
  bh = l / nblk;
  blk = l - bh * nblk;
}

template <int DP> struct Tile {
  static constexpr int LD = DP;  // unpadded rows; the 16-B chunks are XOR-swizzled per row (toff)
  static constexpr int ELEMS = 64 * LD;
  static constexpr int CPT = 64 * DP / 8 / NT;  // 16-B chunks per thread per tile (1 or 2)
};

// Element offset of 16-B chunk c (8 columns) of row r in a tile image with DP-column rows. The chunk is stored at slot
// c ^ f(r) so that every accessor is conflict-free on the LDS banks (MI355X guide, LDS table; checked for all three
// access shapes by scripts/lds_banks.py): frag_rows' ds_read_b128 (rows rbase + lane&15, chunk lane>>4: 4 lane groups
// x 16 lanes), frag_tr's ds_read_b64_tr_b16 (rows rbase + 8-row block, a 32-B column strip: 2 x 32 lanes) and
// tile_store's ds_write_b128 (8 lanes = 128 contiguous bytes). 128-B rows (DP 64): f = r & 7; 64-B rows (DP 32):
// f = {0, 2, 3, 1}[(r >> 2) & 3]. The padded rows used before (LD = DP + 8) cost 2x on every read (8 vs 4 cycles per
// ds_read_b128, 4 vs 2 per transposed read).
template <int DP>
__device__ __forceinline__ int toff(int r, int c) {
  if constexpr (DP == 64) return r * 64 + ((c ^ (r & 7)) << 3);
  return r * 32 + ((c ^ ((0x1320 >> (((r >> 2) & 3) * 4)) & 3)) << 3);
}

// register prefetch of one 64-row x DP tile (zero outside rows < nrows, head columns < d)
template <int DP>
__device__ __forceinline__ void tile_fetch(uint4 (&r)[Tile<DP>::CPT], const bf16_t* src, int ld, int row0, int nrows,
                                           int col0, int d) {
  constexpr int CPR = DP / 8;
#pragma unroll
  for (int j = 0; j < Tile<DP>::CPT; ++j) {
    int c = threadIdx.x + j * NT;
    int rr = c / CPR, ch = c - rr * CPR;
    r[j] = make_uint4(0, 0, 0, 0);
    if (row0 + rr < nrows && ch * 8 < d) r[j] = *(const uint4*)(src + (long long)(row0 + rr) * ld + col0 + ch * 8);
  }
}

template <int DP>
__device__ __forceinline__ void tile_store(bf16_t* t, const uint4 (&r)[Tile<DP>::CPT]) {
  constexpr int CPR = DP / 8;
#pragma unroll
  for (int j = 0; j < Tile<DP>::CPT; ++j) {
    int c = threadIdx.x + j * NT;
    int rr = c / CPR, ch = c - rr * CPR;
    *(uint4*)(t + toff<DP>(rr, ch)) = r[j];
  }
}

// fragment with MFMA row = tile row (rbase + lane&15), k = tile columns kbase + 8*(lane>>4) .. +7
template <int DP>
__device__ __forceinline__ s16x8 frag_rows(const bf16_t* t, int rbase, int kbase, int lane) {
  return *(const s16x8*)(t + toff<DP>(rbase + (lane & 15), (kbase >> 3) + (lane >> 4)));
}

// transposed fragment: MFMA row = tile column (cbase + lane&15), k = tile rows permuted as
// {rbase + 4g + j (j<4), rbase + 16 + 4g + j-4 (j>=4)} for lane group g = lane>>4 (rbase % 8 == 0, cbase % 16 == 0)
template <int DP>
__device__ __forceinline__ s16x8 frag_tr(const bf16_t* t, int rbase, int cbase, int lane) {
  int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r = rbase + 4 * g + q, c = (cbase >> 3) + (p >> 1), w = (p & 1) * 4;
  const bf16_t* a1 = t + toff<DP>(r, c) + w;
  const bf16_t* a2 = t + toff<DP>(r + 16, c) + w;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)a1);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)a2);
  s16x8 r8;
  r8[0] = lo[0]; r8[1] = lo[1]; r8[2] = lo[2]; r8[3] = lo[3];
  r8[4] = hi[0]; r8[5] = hi[1]; r8[6] = hi[2]; r8[7] = hi[3];
  return r8;
}

// B-operand fragment from two accumulator tiles (rows = k): elements j<4 from a[j], j>=4 from b[j-4]
__device__ __forceinline__ s16x8 pack_acc(const f32x4& a, const f32x4& b) {
  uint4 u;
  u.x = pack2bf(a[0], a[1]);
  u.y = pack2bf(a[2], a[3]);
  u.z = pack2bf(b[0], b[1]);
  u.w = pack2bf(b[2], b[3]);
  return __builtin_bit_cast(s16x8, u);
}

// register fragment of one row (row on lane&15): d = 32*ks + 8*(lane>>4) .. +7
template <int DP>
__device__ __forceinline__ void row_frags(s16x8 (&f)[DP / 32], const bf16_t* src, int ld, int row, int nrows, int col0,
                                          int d, int lane) {
#pragma unroll
  for (int ks = 0; ks < DP / 32; ++ks) {
    int dd = ks * 32 + (lane >> 4) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < nrows && dd < d) v = *(const uint4*)(src + (long long)row * ld + col0 + dd);
    f[ks] = __builtin_bit_cast(s16x8, v);
  }
}

__device__ __forceinline__ f32x4 mfma(const s16x8& a, const s16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void store4(bf16_t* dst, const f32x4& v, float s) {
  uint2 w;
  w.x = pack2bf(v[0] * s, v[1] * s);
  w.y = pack2bf(v[2] * s, v[3] * s);
  *(uint2*)dst = w;
}

// max / sum over the four lanes l, l^16, l^32, l^48 (the four 4-key row groups of one query column):
// v_permlane16_swap then v_permlane32_swap, no LDS round trip
__device__ __forceinline__ float xmax4(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r2[0]), __uint_as_float(r2[1]));
}
__device__ __forceinline__ float xsum4(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
}

__device__ __forceinline__ void scale4(f32x4& v, float a) {
  v[0] = v[0] * a;
  v[1] = v[1] * a;
  v[2] = v[2] * a;
  v[3] = v[3] * a;
}

// P = exp2(score * c + nl[i]) and dS = P * dp (element-wise, scalar VALU); nl: per-element negated log-sum-exp
__device__ __forceinline__ void p_ds(f32x4& p, f32x4& ds, float c, const float* nl) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float e = fast_exp2(fmaf(p[i], c, nl[i]));
    p[i] = e;
    ds[i] = e * ds[i];
  }
}

// DT = ceil(d / 16) output column tiles (compile time: no per-tile branches); DP = contraction width over d
template <int DT> struct Dim {
  static constexpr int DP = DT <= 2 ? 32 : 64;
  static constexpr int KS = DP / 32;
};
using Full = std::false_type;
using Ragged = std::true_type;

// =============================================================================================
// forward
// =============================================================================================
// ONES (d % 16 == 8: the last output tile has free padded columns): column d of every valid V row is 1, so the
// PV MFMA accumulates the softmax row sum into o[g][DT-1] (tile row 8: lane group 2, element 0) -- no per-score
// VALU row-sum adds in the loop; the sum is of the bf16 P the MFMA consumes, i.e. exactly what O accumulated
template <int DT, bool ONES>
__global__ __launch_bounds__(NT, 2) void attn_fwd_kernel(AttnArgs a) {
  constexpr int DP = Dim<DT>::DP, KS = Dim<DT>::KS;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * Tile<DP>::ELEMS];  // [buf][K|V]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int blk, bh;
  xcd_block(a.nblk, blk, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const float c = a.scale * LOG2E;
  const bf16_t* Q = a.q + (long long)b * a.N * a.ldq;
  const bf16_t* K = a.k + (long long)b * a.S * a.ldk;
  const bf16_t* V = a.v + (long long)b * a.S * a.ldv;

  int myq[2];
  s16x8 qf[2][KS];
  float m[2], l[2];
  f32x4 o[2][DT];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    myq[g] = blk * ROWS + wave * 32 + g * 16 + (lane & 15);
    row_frags<DP>(qf[g], Q, a.ldq, myq[g], a.N, h * a.d, a.d, lane);
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[g][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  uint4 rk[Tile<DP>::CPT], rv[Tile<DP>::CPT];
  // ONES: the 8-column chunk of V starting at column d (all padding) becomes {1, 0, ..., 0} on valid key rows
  auto fetch_v = [&](int row0) __attribute__((always_inline)) {
    tile_fetch<DP>(rv, V, a.ldv, row0, a.S, h * a.d, a.d);
    if constexpr (ONES) {
      constexpr int CPR = DP / 8;
#pragma unroll
      for (int j = 0; j < Tile<DP>::CPT; ++j) {
        const int c = threadIdx.x + j * NT, rr = c / CPR, ch = c - rr * CPR;
        if (ch * 8 == a.d && row0 + rr < a.S) rv[j].x = 0x3F80u;  // bf16 1.0 in the chunk's first element
      }
    }
  };
  tile_fetch<DP>(rk, K, a.ldk, 0, a.S, h * a.d, a.d);
  fetch_v(0);
  tile_store<DP>(smem, rk);
  tile_store<DP>(smem + Tile<DP>::ELEMS, rv);
  __syncthreads();
  int cur = 0;
  auto step = [&](int k0, auto rag) __attribute__((always_inline)) {
    const bool more = k0 + TILE < a.S;
    if (more) {
      tile_fetch<DP>(rk, K, a.ldk, k0 + TILE, a.S, h * a.d, a.d);
      fetch_v(k0 + TILE);
    }
    const bf16_t* sK = smem + cur * 2 * Tile<DP>::ELEMS;
    const bf16_t* sV = sK + Tile<DP>::ELEMS;
    f32x4 s[2][4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[0][kb] = s[1][kb] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s16x8 kf = frag_rows<DP>(sK, kb * 16, ks * 32, lane);
        s[0][kb] = mfma(kf, qf[0][ks], s[0][kb]);
        s[1][kb] = mfma(kf, qf[1][ks], s[1][kb]);
      }
    }
    if constexpr (decltype(rag)::value) {  // last key tile of a ragged S (cross-attention S = 77): keys >= S out
      const int lim = a.S - k0 - (lane >> 4) * 4;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (kb * 16 + i >= lim) s[0][kb][i] = s[1][kb][i] = -INFINITY;
    }
    s16x8 pf[2][2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      float mx = fmaxf(fmaxf(s[g][0][0], s[g][0][1]), s[g][0][2]);
      mx = fmaxf(fmaxf(mx, s[g][0][3]), s[g][1][0]);
#pragma unroll
      for (int j = 5; j < 16; j += 2) mx = fmaxf(fmaxf(mx, s[g][j >> 2][j & 3]), s[g][(j + 1) >> 2][(j + 1) & 3]);
      mx = xmax4(mx);
      const float mn = fmaxf(m[g], mx * c);
      const float alpha = fast_exp2(m[g] - mn);
      m[g] = mn;
      // scalar f32 VALU only (no v_pk_*_f32): beside MFMAs a packed f32 op costs ~3x two scalar ones (MI355X guide,
      // 'price of one filler beside MFMAs'); the file is built with -fno-slp-vectorize so none are re-formed
      const float nm = -mn;
      float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        float e[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) e[i] = fast_exp2(fmaf(s[g][kb][i], c, nm));
        if constexpr (!ONES) {
          ls0 += e[0] + e[1];
          ls1 += e[2] + e[3];
        }
        s[g][kb] = (f32x4){e[0], e[1], e[2], e[3]};
      }
      if constexpr (!ONES) l[g] = fmaf(l[g], alpha, ls0 + ls1);
#pragma unroll
      for (int t = 0; t < DT; ++t) scale4(o[g][t], alpha);
      pf[g][0] = pack_acc(s[g][0], s[g][1]);
      pf[g][1] = pack_acc(s[g][2], s[g][3]);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        s16x8 vf = frag_tr<DP>(sV, 32 * s2, 16 * t, lane);
        o[0][t] = mfma(vf, pf[0][s2], o[0][t]);
        o[1][t] = mfma(vf, pf[1][s2], o[1][t]);
      }
    if (more) {
      bf16_t* nK = smem + (cur ^ 1) * 2 * Tile<DP>::ELEMS;
      tile_store<DP>(nK, rk);
      tile_store<DP>(nK + Tile<DP>::ELEMS, rv);
    }
    __syncthreads();
    cur ^= 1;
  };
  int k0 = 0;
  for (; k0 + TILE <= a.S; k0 += TILE) step(k0, Full{});
  if (k0 < a.S) step(k0, Ragged{});
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    // ONES: the row sum sits in lane group 2 of the last output tile; every lane of the query column takes it
    const float lt = ONES ? __shfl(o[g][DT - 1][0], 32 + (lane & 15)) : xsum4(l[g]);
    if (myq[g] < a.N) {
      const float inv = 1.f / lt;
      bf16_t* O = a.out + ((long long)b * a.N + myq[g]) * a.ldo + h * a.d;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        int d0 = 16 * t + (lane >> 4) * 4;
        if (d0 < a.d) store4(O + d0, o[g][t], inv);
      }
      if ((lane >> 4) == 0) a.lse[(long long)bh * a.N + myq[g]] = m[g] + __log2f(lt);
    }
  }
}

// =============================================================================================
// backward: dK, dV (keys on lanes, 128 keys per workgroup, query tiles streamed)
// =============================================================================================
// G: 16-key groups per wave (2: 128 keys per workgroup; 4: 256, every staged Q / dO tile and LDS fragment serves twice
// the keys). The query tile is consumed in two 32-query halves so the live P / dS accumulators stay at G x 2.
template <int DT, int G = 2>
__global__ __launch_bounds__(NT, 2) void attn_bwd_dkv_kernel(AttnArgs a) {
  constexpr int DP = Dim<DT>::DP, KS = Dim<DT>::KS;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * Tile<DP>::ELEMS];  // [buf][Q|dO]
  __shared__ __attribute__((aligned(16))) float sLD[2][2][64];               // [buf][-lse|-delta]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int blk, bh;
  xcd_block(a.nblk, blk, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const float c = a.scale * LOG2E;
  const bf16_t* Q = a.q + (long long)b * a.N * a.ldq;
  const bf16_t* dO = a.dout + (long long)b * a.N * a.lddo;

  int mykey[G];
  s16x8 kf[G][KS], vf[G][KS];
  f32x4 dk[G][DT], dv[G][DT];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    mykey[g] = blk * (64 * G) + wave * 16 * G + g * 16 + (lane & 15);
    row_frags<DP>(kf[g], a.k + (long long)b * a.S * a.ldk, a.ldk, mykey[g], a.S, h * a.d, a.d, lane);
    row_frags<DP>(vf[g], a.v + (long long)b * a.S * a.ldv, a.ldv, mykey[g], a.S, h * a.d, a.d, lane);
#pragma unroll
    for (int t = 0; t < DT; ++t) dk[g][t] = dv[g][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  uint4 rq[Tile<DP>::CPT], ro[Tile<DP>::CPT];
  float rl = 0.f, rd = 0.f;
  auto fetch = [&](int q0) __attribute__((always_inline)) {
    tile_fetch<DP>(rq, Q, a.ldq, q0, a.N, h * a.d, a.d);
    tile_fetch<DP>(ro, dO, a.lddo, q0, a.N, h * a.d, a.d);
    if (threadIdx.x < 64) {
      int q = q0 + threadIdx.x;
      rl = q < a.N ? -a.lse[(long long)bh * a.N + q] : -INFINITY;  // invalid rows: p = 0
      rd = q < a.N ? -a.delta[(long long)bh * a.N + q] : 0.f;
    }
  };
  auto put = [&](int buf) __attribute__((always_inline)) {
    tile_store<DP>(smem + buf * 2 * Tile<DP>::ELEMS, rq);
    tile_store<DP>(smem + buf * 2 * Tile<DP>::ELEMS + Tile<DP>::ELEMS, ro);
    if (threadIdx.x < 64) {
      sLD[buf][0][threadIdx.x] = rl;
      sLD[buf][1][threadIdx.x] = rd;
    }
  };
  fetch(0);
  put(0);
  __syncthreads();
  int cur = 0;
  for (int q0 = 0; q0 < a.N; q0 += TILE) {
    const bool more = q0 + TILE < a.N;
    if (more) fetch(q0 + TILE);
    const bf16_t* sQ = smem + cur * 2 * Tile<DP>::ELEMS;
    const bf16_t* sO = sQ + Tile<DP>::ELEMS;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {  // query rows 32*s2 .. +32 of the tile
      f32x4 p[G][2], ds[G][2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int qb = 2 * s2 + h2;
        const int qi = qb * 16 + (lane >> 4) * 4;
        const f32x4 nL = *(const f32x4*)&sLD[cur][0][qi], nD = *(const f32x4*)&sLD[cur][1][qi];
        // dP accumulates on top of -delta: the MFMA yields dP - delta directly (no per-element subtraction)
#pragma unroll
        for (int g = 0; g < G; ++g) {
          p[g][h2] = (f32x4){0.f, 0.f, 0.f, 0.f};
          ds[g][h2] = nD;
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          s16x8 qa = frag_rows<DP>(sQ, qb * 16, ks * 32, lane);
          s16x8 oa = frag_rows<DP>(sO, qb * 16, ks * 32, lane);
#pragma unroll
          for (int g = 0; g < G; ++g) p[g][h2] = mfma(qa, kf[g][ks], p[g][h2]);
#pragma unroll
          for (int g = 0; g < G; ++g) ds[g][h2] = mfma(oa, vf[g][ks], ds[g][h2]);
        }
        const float nl[4] = {nL[0], nL[1], nL[2], nL[3]};
#pragma unroll
        for (int g = 0; g < G; ++g) p_ds(p[g][h2], ds[g][h2], c, nl);
      }
      s16x8 pf[G], df[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        pf[g] = pack_acc(p[g][0], p[g][1]);
        df[g] = pack_acc(ds[g][0], ds[g][1]);
      }
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        s16x8 ot = frag_tr<DP>(sO, 32 * s2, 16 * t, lane);
#pragma unroll
        for (int g = 0; g < G; ++g) dv[g][t] = mfma(ot, pf[g], dv[g][t]);
        s16x8 qt = frag_tr<DP>(sQ, 32 * s2, 16 * t, lane);
#pragma unroll
        for (int g = 0; g < G; ++g) dk[g][t] = mfma(qt, df[g], dk[g][t]);
      }
    }
    if (more) put(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int g = 0; g < G; ++g)
    if (mykey[g] < a.S) {
      bf16_t* DK = a.dk + ((long long)b * a.S + mykey[g]) * a.lddk + h * a.d;
      bf16_t* DV = a.dv + ((long long)b * a.S + mykey[g]) * a.lddv + h * a.d;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        int d0 = 16 * t + (lane >> 4) * 4;
        if (d0 < a.d) {
          store4(DK + d0, dk[g][t], a.scale);
          store4(DV + d0, dv[g][t], 1.f);
        }
      }
    }
}

// =============================================================================================
// backward: dQ (queries on lanes, 64 * G queries per workgroup, key tiles streamed)
// =============================================================================================
template <int DT, int G = 2>
__global__ __launch_bounds__(NT, 2) void attn_bwd_dq_kernel(AttnArgs a) {
  constexpr int DP = Dim<DT>::DP, KS = Dim<DT>::KS;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * Tile<DP>::ELEMS];  // [buf][K|V]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int blk, bh;
  xcd_block(a.nblk, blk, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const float c = a.scale * LOG2E;
  const bf16_t* K = a.k + (long long)b * a.S * a.ldk;
  const bf16_t* V = a.v + (long long)b * a.S * a.ldv;

  int myq[G];
  s16x8 qf[G][KS], of[G][KS];
  float nlse[G], ndlt[G];
  f32x4 dq[G][DT];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    myq[g] = blk * (64 * G) + wave * 16 * G + g * 16 + (lane & 15);
    row_frags<DP>(qf[g], a.q + (long long)b * a.N * a.ldq, a.ldq, myq[g], a.N, h * a.d, a.d, lane);
    row_frags<DP>(of[g], a.dout + (long long)b * a.N * a.lddo, a.lddo, myq[g], a.N, h * a.d, a.d, lane);
    const bool ok = myq[g] < a.N;
    const float L = ok ? -a.lse[(long long)bh * a.N + myq[g]] : -INFINITY;
    // delta = rowsum(dO * O) of this query row: the four lane groups hold disjoint 8-column chunks of the row
    float D = 0.f;
    {
      s16x8 orow[KS];
      row_frags<DP>(orow, a.o + (long long)b * a.N * a.ldo, a.ldo, myq[g], a.N, h * a.d, a.d, lane);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float x[8], y[8];
        unpack8(__builtin_bit_cast(uint4, orow[ks]), x);
        unpack8(__builtin_bit_cast(uint4, of[g][ks]), y);
#pragma unroll
        for (int e = 0; e < 8; ++e) D = fmaf(x[e], y[e], D);
      }
      D = xsum4(D);
      if (ok && (lane >> 4) == 0) ((float*)a.delta)[(long long)bh * a.N + myq[g]] = D;
      D = -D;
    }
    nlse[g] = L;
    ndlt[g] = D;
#pragma unroll
    for (int t = 0; t < DT; ++t) dq[g][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  uint4 rk[Tile<DP>::CPT], rv[Tile<DP>::CPT];
  tile_fetch<DP>(rk, K, a.ldk, 0, a.S, h * a.d, a.d);
  tile_fetch<DP>(rv, V, a.ldv, 0, a.S, h * a.d, a.d);
  tile_store<DP>(smem, rk);
  tile_store<DP>(smem + Tile<DP>::ELEMS, rv);
  __syncthreads();
  int cur = 0;
  auto step = [&](int k0, auto rag) __attribute__((always_inline)) {
    const bool more = k0 + TILE < a.S;
    if (more) {
      tile_fetch<DP>(rk, K, a.ldk, k0 + TILE, a.S, h * a.d, a.d);
      tile_fetch<DP>(rv, V, a.ldv, k0 + TILE, a.S, h * a.d, a.d);
    }
    const bf16_t* sK = smem + cur * 2 * Tile<DP>::ELEMS;
    const bf16_t* sV = sK + Tile<DP>::ELEMS;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {  // keys 32*s2 .. +32 of the tile
      f32x4 ds[G][2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int kb = 2 * s2 + h2;
        f32x4 sc[G], dp[G];
        // dP accumulates on top of -delta (per query = per lane): the MFMA yields dP - delta directly
#pragma unroll
        for (int g = 0; g < G; ++g) {
          sc[g] = (f32x4){0.f, 0.f, 0.f, 0.f};
          dp[g] = (f32x4){ndlt[g], ndlt[g], ndlt[g], ndlt[g]};
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          s16x8 ka = frag_rows<DP>(sK, kb * 16, ks * 32, lane);
          s16x8 va = frag_rows<DP>(sV, kb * 16, ks * 32, lane);
#pragma unroll
          for (int g = 0; g < G; ++g) sc[g] = mfma(ka, qf[g][ks], sc[g]);
#pragma unroll
          for (int g = 0; g < G; ++g) dp[g] = mfma(va, of[g][ks], dp[g]);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
          float e[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) e[i] = fast_exp2(fmaf(sc[g][i], c, nlse[g]));
          if constexpr (decltype(rag)::value) {  // keys >= S of the last ragged tile contribute nothing
            const int lim = a.S - k0 - kb * 16 - (lane >> 4) * 4;
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (i >= lim) e[i] = 0.f;
          }
          ds[g][h2] = (f32x4){e[0] * dp[g][0], e[1] * dp[g][1], e[2] * dp[g][2], e[3] * dp[g][3]};
        }
      }
      s16x8 df[G];
#pragma unroll
      for (int g = 0; g < G; ++g) df[g] = pack_acc(ds[g][0], ds[g][1]);
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        s16x8 kt = frag_tr<DP>(sK, 32 * s2, 16 * t, lane);
#pragma unroll
        for (int g = 0; g < G; ++g) dq[g][t] = mfma(kt, df[g], dq[g][t]);
      }
    }
    if (more) {
      bf16_t* nK = smem + (cur ^ 1) * 2 * Tile<DP>::ELEMS;
      tile_store<DP>(nK, rk);
      tile_store<DP>(nK + Tile<DP>::ELEMS, rv);
    }
    __syncthreads();
    cur ^= 1;
  };
  int k0 = 0;
  for (; k0 + TILE <= a.S; k0 += TILE) step(k0, Full{});
  if (k0 < a.S) step(k0, Ragged{});
#pragma unroll
  for (int g = 0; g < G; ++g)
    if (myq[g] < a.N) {
      bf16_t* DQ = a.dq + ((long long)b * a.N + myq[g]) * a.lddq + h * a.d;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        int d0 = 16 * t + (lane >> 4) * 4;
        if (d0 < a.d) store4(DQ + d0, dq[g][t], a.scale);
      }
    }
}

// =============================================================================================
// backward, fused: dK, dV AND dQ in one pass (keys on lanes, 128 keys per workgroup, query tiles streamed) --
// P and dS are computed once per score instead of once in each of the two kernels above (the exp, the scale FMA,
// the dS product and the dS conversion per score halve; two MFMA products of five are not recomputed).
// dQ = dS K needs the contraction over keys, which sit on the lanes: every wave writes its dS tile transposed
// (dS^T [key][query], bf16, the same values the dK product consumes) into LDS, and after one barrier wave w forms
// dQ^T for queries 16w .. 16w+15 of the tile over all 128 keys of the workgroup from transposed reads of dS^T and
// of the workgroup's key block (staged once). One key block (S <= 128: cross-attention over the 77 text tokens)
// stores dQ directly; otherwise every key block writes an fp32 partial and the LAST of the nblk key blocks to
// finish a (b*h, query tile) -- device-scope arrival counter, no spinning -- sums the partials in key-block order
// (deterministic) and stores dQ. Partials are written and read with sc1 (device-coherent) buffer operations: the
// summing workgroup may run on another XCD. delta = rowsum(dO * O) comes from attn_delta_kernel.
// =============================================================================================
constexpr int LDQ = TILE + 8;  // dS^T image row: 64 queries + 16 B of padding

template <int LD>
__device__ __forceinline__ s16x8 frag_tr_ld(const bf16_t* t, int rbase, int cbase, int lane) {
  int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16_t* a1 = t + (rbase + 4 * g + q) * LD + cbase + 4 * p;
  const bf16_t* a2 = a1 + 16 * LD;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)a1);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SDMI_LDS s16x4*)a2);
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
constexpr int ATTN_CPOL_SC1 = 16;  // buffer cache policy: device (agent) scope coherence

template <int DT>
__global__ __launch_bounds__(NT, 2) void attn_bwd_fused_kernel(AttnArgs a) {
  constexpr int DP = Dim<DT>::DP, KS = Dim<DT>::KS;
  constexpr int LDK = Tile<DP>::LD;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * Tile<DP>::ELEMS];  // [buf][Q|dO]
  __shared__ __attribute__((aligned(16))) bf16_t sK[ROWS * LDK];             // this workgroup's key block
  __shared__ __attribute__((aligned(16))) bf16_t sDS[ROWS * LDQ];            // dS^T of the current query tile
  __shared__ __attribute__((aligned(16))) float sLD[2][2][64];               // [buf][-lse|-delta]
  __shared__ int sflag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int kb, bh;
  xcd_block(a.nblk, kb, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const int nkb = a.nblk;
  const float c = a.scale * LOG2E;
  const bf16_t* Q = a.q + (long long)b * a.N * a.ldq;
  const bf16_t* dO = a.dout + (long long)b * a.N * a.lddo;
  const bf16_t* Kb = a.k + (long long)b * a.S * a.ldk;

  {  // the workgroup's 128 keys (rows >= S zero) for the dQ products
    uint4 rk[Tile<DP>::CPT];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      tile_fetch<DP>(rk, Kb, a.ldk, kb * ROWS + half * TILE, a.S, h * a.d, a.d);
      tile_store<DP>(sK + half * Tile<DP>::ELEMS, rk);
    }
  }
  int mykey[2];
  bool kok[2];
  s16x8 kf[2][KS], vf[2][KS];
  f32x4 dk[2][DT], dv[2][DT];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    mykey[g] = kb * ROWS + wave * 32 + g * 16 + (lane & 15);
    kok[g] = mykey[g] < a.S;
    row_frags<DP>(kf[g], Kb, a.ldk, mykey[g], a.S, h * a.d, a.d, lane);
    row_frags<DP>(vf[g], a.v + (long long)b * a.S * a.ldv, a.ldv, mykey[g], a.S, h * a.d, a.d, lane);
#pragma unroll
    for (int t = 0; t < DT; ++t) dk[g][t] = dv[g][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  uint4 rq[Tile<DP>::CPT], ro[Tile<DP>::CPT];
  float rl = 0.f, rd = 0.f;
  auto fetch = [&](int q0) __attribute__((always_inline)) {
    tile_fetch<DP>(rq, Q, a.ldq, q0, a.N, h * a.d, a.d);
    tile_fetch<DP>(ro, dO, a.lddo, q0, a.N, h * a.d, a.d);
    if (threadIdx.x < 64) {
      int q = q0 + threadIdx.x;
      rl = q < a.N ? -a.lse[(long long)bh * a.N + q] : -INFINITY;  // invalid rows: p = 0
      rd = q < a.N ? -a.delta[(long long)bh * a.N + q] : 0.f;
    }
  };
  auto put = [&](int buf) __attribute__((always_inline)) {
    tile_store<DP>(smem + buf * 2 * Tile<DP>::ELEMS, rq);
    tile_store<DP>(smem + buf * 2 * Tile<DP>::ELEMS + Tile<DP>::ELEMS, ro);
    if (threadIdx.x < 64) {
      sLD[buf][0][threadIdx.x] = rl;
      sLD[buf][1][threadIdx.x] = rd;
    }
  };
  const __amdgpu_buffer_rsrc_t rsP = __builtin_amdgcn_make_buffer_rsrc((void*)a.dq_part, (short)0, 0x7fffffff, 0x00020000);
  const int ntq = (a.N + TILE - 1) / TILE;
  fetch(0);
  put(0);
  __syncthreads();
  int cur = 0;
  for (int q0 = 0; q0 < a.N; q0 += TILE) {
    const bool more = q0 + TILE < a.N;
    if (more) fetch(q0 + TILE);
    const bf16_t* sQ = smem + cur * 2 * Tile<DP>::ELEMS;
    const bf16_t* sO = sQ + Tile<DP>::ELEMS;
    f32x4 p[2][4], ds[2][4];
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
      const int qi = qb * 16 + (lane >> 4) * 4;
      const f32x4 nL = *(const f32x4*)&sLD[cur][0][qi], nD = *(const f32x4*)&sLD[cur][1][qi];
      p[0][qb] = p[1][qb] = (f32x4){0.f, 0.f, 0.f, 0.f};
      ds[0][qb] = ds[1][qb] = nD;  // dP accumulates on top of -delta
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s16x8 qa = frag_rows<DP>(sQ, qb * 16, ks * 32, lane);
        s16x8 oa = frag_rows<DP>(sO, qb * 16, ks * 32, lane);
        p[0][qb] = mfma(qa, kf[0][ks], p[0][qb]);
        p[1][qb] = mfma(qa, kf[1][ks], p[1][qb]);
        ds[0][qb] = mfma(oa, vf[0][ks], ds[0][qb]);
        ds[1][qb] = mfma(oa, vf[1][ks], ds[1][qb]);
      }
      const float nl[4] = {nL[0], nL[1], nL[2], nL[3]};
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        p_ds(p[g][qb], ds[g][qb], c, nl);
        if (!kok[g]) p[g][qb] = ds[g][qb] = (f32x4){0.f, 0.f, 0.f, 0.f};  // keys >= S (zero K rows) must not reach dQ
        uint2 w;
        w.x = pack2bf(ds[g][qb][0], ds[g][qb][1]);
        w.y = pack2bf(ds[g][qb][2], ds[g][qb][3]);
        *(uint2*)(sDS + (wave * 32 + g * 16 + (lane & 15)) * LDQ + qb * 16 + (lane >> 4) * 4) = w;
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s16x8 pf0 = pack_acc(p[0][2 * s2], p[0][2 * s2 + 1]), pf1 = pack_acc(p[1][2 * s2], p[1][2 * s2 + 1]);
      s16x8 df0 = pack_acc(ds[0][2 * s2], ds[0][2 * s2 + 1]), df1 = pack_acc(ds[1][2 * s2], ds[1][2 * s2 + 1]);
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        s16x8 ot = frag_tr<DP>(sO, 32 * s2, 16 * t, lane);
        dv[0][t] = mfma(ot, pf0, dv[0][t]);
        dv[1][t] = mfma(ot, pf1, dv[1][t]);
        s16x8 qt = frag_tr<DP>(sQ, 32 * s2, 16 * t, lane);
        dk[0][t] = mfma(qt, df0, dk[0][t]);
        dk[1][t] = mfma(qt, df1, dk[1][t]);
      }
    }
    __syncthreads();  // dS^T of every wave in LDS
    // dQ^T[d][q] for the tile's queries 16*wave .. +15 over the workgroup's 128 keys: lane holds d = 16t + 4(lane>>4)
    // .. +3 of query 16*wave + (lane & 15)
    f32x4 dq[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) dq[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < ROWS / 32; ++ks) {
      s16x8 sb = frag_tr_ld<LDQ>(sDS, ks * 32, wave * 16, lane);
#pragma unroll
      for (int t = 0; t < DT; ++t) dq[t] = mfma(frag_tr<DP>(sK, ks * 32, t * 16, lane), sb, dq[t]);
    }
    const int myq = q0 + wave * 16 + (lane & 15);
    if (nkb == 1) {
      if (myq < a.N) {
        bf16_t* DQ = a.dq + ((long long)b * a.N + myq) * a.lddq + h * a.d;
#pragma unroll
        for (int t = 0; t < DT; ++t) {
          const int d0 = 16 * t + (lane >> 4) * 4;
          if (d0 < a.d) store4(DQ + d0, dq[t], a.scale);
        }
      }
    } else {
      if (myq < a.N) {
#pragma unroll
        for (int t = 0; t < DT; ++t) {
          const int d0 = 16 * t + (lane >> 4) * 4;
          if (d0 < a.d) {
            const int off = ((((kb * a.B * a.H + bh) * a.N) + myq) * a.d + d0) * 4;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, dq[t]), rsP, off, 0, ATTN_CPOL_SC1);
          }
        }
      }
      // arrival: the partial stores (and the next tile's loads) complete, then one relaxed device-scope increment;
      // the last key block of this (b*h, query tile) sums the partials
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned* ctr = a.ctr + (long long)bh * ntq + q0 / TILE;
        const unsigned prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == (unsigned)(nkb - 1);
        if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sflag = last;
      }
      __syncthreads();
      if (sflag) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the other key blocks' partials: acquire before reading
        const int c4 = a.d / 4;
        for (int i = threadIdx.x; i < TILE * c4; i += NT) {
          const int r = i / c4, d0 = (i - r * c4) * 4, q = q0 + r;
          if (q >= a.N) continue;
          f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
          for (int z = 0; z < nkb; ++z) {
            const int off = ((((z * a.B * a.H + bh) * a.N) + q) * a.d + d0) * 4;
            acc += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsP, off, 0, ATTN_CPOL_SC1));
          }
          store4(a.dq + ((long long)b * a.N + q) * a.lddq + h * a.d + d0, acc, a.scale);
        }
      }
    }
    if (more) put(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int g = 0; g < 2; ++g)
    if (kok[g]) {
      bf16_t* DK = a.dk + ((long long)b * a.S + mykey[g]) * a.lddk + h * a.d;
      bf16_t* DV = a.dv + ((long long)b * a.S + mykey[g]) * a.lddv + h * a.d;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        int d0 = 16 * t + (lane >> 4) * 4;
        if (d0 < a.d) {
          store4(DK + d0, dk[g][t], a.scale);
          store4(DV + d0, dv[g][t], 1.f);
        }
      }
    }
}

// delta[b*h][q] = rowsum(dO * O) over the head's d columns (fp32), one thread per (b, q, h)
__global__ __launch_bounds__(NT) void attn_delta_kernel(AttnArgs a) {
  const long long i = (long long)blockIdx.x * NT + threadIdx.x;
  const long long total = (long long)a.B * a.N * a.H;
  if (i >= total) return;
  const int h = (int)(i % a.H);
  const long long bq = i / a.H;
  const int q = (int)(bq % a.N), b = (int)(bq / a.N);
  const bf16_t* o = a.o + bq * a.ldo + h * a.d;
  const bf16_t* g = a.dout + bq * a.lddo + h * a.d;
  float D = 0.f;
  for (int c0 = 0; c0 < a.d; c0 += 8) {
    float x[8], y[8];
    unpack8(*(const uint4*)(o + c0), x);
    unpack8(*(const uint4*)(g + c0), y);
#pragma unroll
    for (int e = 0; e < 8; ++e) D = fmaf(x[e], y[e], D);
  }
  ((float*)a.delta)[((long long)b * a.H + h) * a.N + q] = D;
}

constexpr int ATTN_CTR_SLOTS = 4, ATTN_CTR_SLOT = 1 << 16;
__device__ unsigned g_attn_counters[ATTN_CTR_SLOTS * ATTN_CTR_SLOT];

int check_args(const AttnArgs& a) {
  if (a.B <= 0 || a.H <= 0 || a.N <= 0 || a.S <= 0 || a.d <= 0) return -1;
  if (a.d % 8 || a.d > 64) return -2;
  return 0;
}

}  // namespace

extern "C" int sdmi_attn_fwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* out, int ldo,
                             float* lse, int B, int H, int N, int S, int d, sdmi_stream_t stream) {
  AttnArgs a = {};
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.out = (bf16_t*)out; a.lse = lse;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
  a.B = B; a.H = H; a.N = N; a.S = S; a.d = d; a.scale = 1.0f / sqrtf((float)d);
  int rc = check_args(a);
  if (rc) return rc;
  a.nblk = (N + ROWS - 1) / ROWS;
  dim3 grid(a.nblk * B * H);
  hipStream_t s = (hipStream_t)stream;
  // ONES: the softmax row sum through the PV MFMA where the padded head dim leaves a free column (d % 16 == 8)
  const bool ones = d % 16 == 8;
#define SDMI_ATTN_FWD(DT)                                                           \
  if (ones) sdmi_rt::launch(attn_fwd_kernel<DT, true>, grid, dim3(NT), 0, s, a);    \
  else sdmi_rt::launch(attn_fwd_kernel<DT, false>, grid, dim3(NT), 0, s, a);
  switch ((d + 15) / 16) {
    case 1: SDMI_ATTN_FWD(1) break;
    case 2: SDMI_ATTN_FWD(2) break;
    case 3: SDMI_ATTN_FWD(3) break;
    default: SDMI_ATTN_FWD(4) break;
  }
#undef SDMI_ATTN_FWD
  SDMI_CHECK_LAUNCH();
  return 0;
}

extern "C" int sdmi_attn_bwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, const void* o,
                             int ldo, const void* dout, int lddo, const float* lse, float* delta_ws, void* dq, int lddq,
                             void* dk, int lddk, void* dv, int lddv, int B, int H, int N, int S, int d,
                             sdmi_stream_t stream) {
  AttnArgs a = {};
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (const bf16_t*)o;
  a.dout = (const bf16_t*)dout; a.lse = (float*)lse; a.delta = delta_ws;
  a.dq = (bf16_t*)dq; a.dk = (bf16_t*)dk; a.dv = (bf16_t*)dv;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo; a.lddo = lddo; a.lddq = lddq; a.lddk = lddk; a.lddv = lddv;
  a.B = B; a.H = H; a.N = N; a.S = S; a.d = d; a.scale = 1.0f / sqrtf((float)d);
  int rc = check_args(a);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  // the dQ kernel also produces delta = rowsum(dO * O) (written to delta_ws) for the dK/dV kernel after it.
  // 16-row groups per wave of both kernels (head dims <= 32): 4 (256 rows per workgroup) when N, S <= 256 -- measured
  // at B = 32, 16 heads: 16^2 d = 24 56.7 -> 48.6 us, d = 32 49.0 -> 44.2 us -- else 2 (128 rows; at 32^2 the two
  // forms measured equal: 279 / 291 / 352 vs 270 / 292 / 348 us at d = 8 / 16 / 24)
  // (and only while the 256-row grids keep >= 512 workgroups, two per CU: DiT-12L's 9-head 16^2 attention, 288
  // workgroups, measured 3.90 / 3.91 -> 3.92 / 3.92 ms per step with G = 4)
  const long long wg4 = (long long)B * H * ((std::min(N, S) + 255) / 256);
  const int g4 = d <= 32 && N <= 256 && S <= 256 && wg4 >= 512;
  const int rows = g4 ? 256 : ROWS;
  AttnArgs aq = a, ak = a;
  aq.nblk = (N + rows - 1) / rows;
  ak.nblk = (S + rows - 1) / rows;
  dim3 gk(ak.nblk * B * H), gq(aq.nblk * B * H);
  switch ((d + 15) / 16) {
#define SDMI_ATTN_BWD(DT)                                                               \
  case DT:                                                                              \
    if constexpr (DT <= 2) {                                                            \
      if (g4) {                                                                         \
        sdmi_rt::launch(attn_bwd_dq_kernel<DT, 4>, gq, dim3(NT), 0, s, aq);             \
        sdmi_rt::launch(attn_bwd_dkv_kernel<DT, 4>, gk, dim3(NT), 0, s, ak);            \
        break;                                                                          \
      }                                                                                 \
    }                                                                                   \
    sdmi_rt::launch(attn_bwd_dq_kernel<DT, 2>, gq, dim3(NT), 0, s, aq);                 \
    sdmi_rt::launch(attn_bwd_dkv_kernel<DT, 2>, gk, dim3(NT), 0, s, ak);                \
    break;
    SDMI_ATTN_BWD(1)
    SDMI_ATTN_BWD(2)
    SDMI_ATTN_BWD(3)
    default: SDMI_ATTN_BWD(4)
#undef SDMI_ATTN_BWD
  }
  SDMI_CHECK_LAUNCH();
  return 0;
}

// fused backward (attn_bwd_fused_kernel): fp32 dQ partial workspace bytes (0 when the keys fit one key block)
extern "C" size_t sdmi_attn_bwd_workspace(int B, int H, int N, int S, int d) {
  const long long nkb = (S + ROWS - 1) / ROWS;
  return nkb > 1 ? (size_t)(nkb * B * H * (long long)N * d * 4) : 0;
}

extern "C" int sdmi_attn_bwd_fused(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                                   const void* o, int ldo, const void* dout, int lddo, const float* lse,
                                   float* delta_ws, void* ws, size_t ws_bytes, void* dq, int lddq, void* dk,
                                   int lddk, void* dv, int lddv, int B, int H, int N, int S, int d,
                                   sdmi_stream_t stream) {
  AttnArgs a = {};
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (const bf16_t*)o;
  a.dout = (const bf16_t*)dout; a.lse = (float*)lse; a.delta = delta_ws;
  a.dq = (bf16_t*)dq; a.dk = (bf16_t*)dk; a.dv = (bf16_t*)dv;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo; a.lddo = lddo; a.lddq = lddq; a.lddk = lddk; a.lddv = lddv;
  a.B = B; a.H = H; a.N = N; a.S = S; a.d = d; a.scale = 1.0f / sqrtf((float)d);
  int rc = check_args(a);
  if (rc) return rc;
  const size_t need = sdmi_attn_bwd_workspace(B, H, N, S, d);
  const long long ntq = (N + TILE - 1) / TILE;
  // partial offsets are 32-bit buffer offsets; counters: one slot region per launch
  if (need && (!ws || ws_bytes < need || need >= (1ull << 31) || (long long)B * H * ntq > ATTN_CTR_SLOT)) return -3;
  static unsigned* ctr_base = nullptr;
  static int next = 0;
  if (need) {
    if (!ctr_base) {
      void* p = nullptr;
      if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_attn_counters)) != hipSuccess) return -4;
      ctr_base = (unsigned*)p;
    }
    a.ctr = ctr_base + (size_t)(next++ % ATTN_CTR_SLOTS) * ATTN_CTR_SLOT;
    a.dq_part = (float*)ws;
  }
  hipStream_t s = (hipStream_t)stream;
  const long long rows = (long long)B * N * H;
  sdmi_rt::launch(attn_delta_kernel, dim3((unsigned)((rows + NT - 1) / NT)), dim3(NT), 0, s, a);
  a.nblk = (S + ROWS - 1) / ROWS;
  dim3 gk(a.nblk * B * H);
  switch ((d + 15) / 16) {
    case 1: sdmi_rt::launch(attn_bwd_fused_kernel<1>, gk, dim3(NT), 0, s, a); break;
    case 2: sdmi_rt::launch(attn_bwd_fused_kernel<2>, gk, dim3(NT), 0, s, a); break;
    case 3: sdmi_rt::launch(attn_bwd_fused_kernel<3>, gk, dim3(NT), 0, s, a); break;
    default: sdmi_rt::launch(attn_bwd_fused_kernel<4>, gk, dim3(NT), 0, s, a); break;
  }
  SDMI_CHECK_LAUNCH();
  return 0;
}
