// Edge-reduction GEMM for weight gradients: C = A^T B (+ colsum(A)) with A (K, M), B (K, N)
// row-major and K = number of edges (~1M), M = N = d.  This is the dW of a per-edge Linear
// (egnn_layer.py:28-39 mlp_msg / mlp_pos: dW = sum_e dpre_e (x) x_e, db = sum_e dpre_e).
//
// Split-K over workgroups (each a contiguous edge range) with the edge index as the MFMA k
// dimension, partial slabs in a workspace and an ordered second pass (bitwise deterministic; no
// atomics); reads A and B once.  Two arithmetic paths: wide edge-level products run on the bf16
// MFMA over exact three-plane splits of the f32 operands (outer_sum_x3_kernel, below); narrow
// products, node-level row counts and gmp_wgrad_set_f32_mfma(1) use the f32 MFMA 16x16x4
// kernels (outer_sum_kernel, outer_sum_rect_kernel).
#include <stdlib.h>

#include "gmp_common.h"

namespace gmp {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kT = 256;      // threads (4 waves)
constexpr int kKT = 32;      // edges per LDS tile

template <int D>
struct WCfg {
  static constexpr int TW = D / 32;  // 16x16 tiles per wave per dim (wave owns a D/2 x D/2 block)
};

// B-operand prologue: PRO = 0: B as stored; 1: relu(B*w + b); 2: silu(B*w + b) (per column
// w, b) — the EGNN activations y1 / m rebuilt from the saved LayerNorm outputs at load time.
template <int PRO>
__device__ __forceinline__ f32x4 prologue(f32x4 v, f32x4 w, f32x4 b) {
  if constexpr (PRO == 0) {
    return v;
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float z = v[c] * w[c] + b[c];
      if constexpr (PRO == 1) v[c] = z > 0.f ? z : 0.f;
      else v[c] = z * (1.f / (1.f + __expf(-z)));
    }
    return v;
  }
}

// One workgroup: edges [k0, k1) -> partial[blockIdx] = A^T pro(B) (D x D) and colsum(A) (D).
template <int D, int PRO>
__global__ __launch_bounds__(kT, 2) void outer_sum_kernel(const float* __restrict__ A,
                                                          const float* __restrict__ B, int64_t K,
                                                          int64_t lda, int64_t ldb,
                                                          int64_t k_per_block,
                                                          float* __restrict__ partial,
                                                          const float* __restrict__ bw,
                                                          const float* __restrict__ bb) {
  constexpr int TW = WCfg<D>::TW;
  constexpr int LD = D + 16;
  __shared__ __attribute__((aligned(16))) float sA[2][kKT * LD];
  __shared__ __attribute__((aligned(16))) float sB[2][kKT * LD];
  __shared__ float sColsum[kT / (D / 4)][D];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, kk = lane >> 4;
  const int m0 = (w >> 1) * (D / 2), n0 = (w & 1) * (D / 2);
  const int64_t k0 = (int64_t)blockIdx.x * k_per_block;
  const int64_t k1 = (k0 + k_per_block < K) ? k0 + k_per_block : K;

  f32x4 acc[TW][TW];
#pragma unroll
  for (int a = 0; a < TW; ++a)
#pragma unroll
    for (int b = 0; b < TW; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // loader mapping: thread -> (row r0 + j*RS, column group c4) ; fixed column => colsum in regs
  constexpr int CG = D / 4;            // float4 column groups per row
  constexpr int RS = kT / CG;          // rows loaded per pass
  const int c4 = tid % CG, r0 = tid / CG;
  f32x4 csum = {0.f, 0.f, 0.f, 0.f};

  constexpr int NL = kKT / RS;  // float4 loads per thread per tile, per operand
  f32x4 ra[NL], rb[NL];
  f32x4 pw = {0.f, 0.f, 0.f, 0.f}, pb = {0.f, 0.f, 0.f, 0.f};
  if constexpr (PRO != 0) {
    pw = *reinterpret_cast<const f32x4*>(bw + 4 * c4);
    pb = *reinterpret_cast<const f32x4*>(bb + 4 * c4);
  }
  unsigned vmask = 0;  // rows of the fetched tile that exist (prologue only on those)
  auto fetch = [&](int64_t kb) {  // global -> registers (stays in flight; no use here)
    vmask = 0;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int64_t k = kb + r0 + j * RS;
      ra[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      rb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k < k1) {
        ra[j] = *reinterpret_cast<const f32x4*>(A + k * lda + 4 * c4);
        rb[j] = *reinterpret_cast<const f32x4*>(B + k * ldb + 4 * c4);
        vmask |= 1u << j;
      }
    }
  };
  auto stash = [&](int buf) {  // registers -> LDS (+ colsum of A), B prologue applied here
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int r = r0 + j * RS;
      if (PRO != 0 && (vmask >> j) & 1u) rb[j] = prologue<PRO>(rb[j], pw, pb);
      csum += ra[j];
      *reinterpret_cast<f32x4*>(&sA[buf][r * LD + 4 * c4]) = ra[j];
      *reinterpret_cast<f32x4*>(&sB[buf][r * LD + 4 * c4]) = rb[j];
    }
  };

  int buf = 0;
  if (k0 < k1) {
    fetch(k0);
    stash(0);
  }
  __syncthreads();
  for (int64_t kb = k0; kb < k1; kb += kKT) {
    const bool more = kb + kKT < k1;
    if (more) fetch(kb + kKT);  // in flight while this tile is computed
    const float* a_s = sA[buf];
    const float* b_s = sB[buf];
#pragma unroll
    for (int s = 0; s < kKT / 4; ++s) {
      const int e = 4 * s + kk;
      float af[TW], bf[TW];
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        af[t] = a_s[e * LD + m0 + 16 * t + li];
        bf[t] = b_s[e * LD + n0 + 16 * t + li];
      }
#pragma unroll
      for (int a = 0; a < TW; ++a)
#pragma unroll
        for (int b = 0; b < TW; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
    if (more) stash(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // C/D map of 16x16x4: col = lane & 15, row = 4*(lane >> 4) + r
  float* out = partial + (int64_t)blockIdx.x * (D * D + D);
#pragma unroll
  for (int a = 0; a < TW; ++a)
#pragma unroll
    for (int b = 0; b < TW; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(m0 + 16 * a + 4 * kk + r) * D + n0 + 16 * b + li] = acc[a][b][r];
  // colsum(A): threads sharing a column group add in row-group order (deterministic)
  *reinterpret_cast<f32x4*>(&sColsum[r0][4 * c4]) = csum;
  __syncthreads();
  for (int c = tid; c < D; c += kT) {
    float sacc = 0.f;
    for (int r = 0; r < RS; ++r) sacc += sColsum[r][c];
    out[D * D + c] = sacc;
  }
}

constexpr int kGC = 16;  // slab loads in flight per lane in the ordered partial sums (default)

// One-pass ordered sum of the G partial slabs (replaces l1 + l2 on the split-K paths): a
// workgroup owns 64 columns x; its SW waves each add a contiguous 1/SW of the slabs (slab
// order, GC loads in flight per lane), then wave 0 adds the SW partial sums in wave order -- a
// fixed order independent of timing (deterministic).  The split-K sums use SW = 4, GC = 32
// (256 threads, a 256-slab reduction in two bursts of loads per lane): these sums run on the
// side stream beside the main stream's edge kernels, and a 256-thread workgroup fits beside
// those kernels' waves on a CU where the r03-r05 1024-thread form (SW = 16, one burst) had to
// wait for a whole CU to drain -- up to 0.9 ms per sum behind the GVP message backward in the
// r05 trace.  A/B on one box (r05): C2 EGNN 113.4 vs 112.2 M edges/s, C3 GVP 28.38 vs 28.47 M
// (neutral).
template <int SW, int GC = kGC>
__global__ __launch_bounds__(64 * SW) void sum_partials_one(const float* __restrict__ part,
                                                            int64_t G, int64_t X,
                                                            float* __restrict__ out,
                                                            float* __restrict__ colsum,
                                                            int64_t DD, int64_t n, int64_t ldc) {
  __shared__ float red[SW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t x = blockIdx.x * (int64_t)64 + lane;
  const int64_t q = (G + SW - 1) / SW, g0 = wv * q, g1 = (g0 + q < G) ? g0 + q : G;
  float s = 0.f;
  if (x < X) {
    for (int64_t c0 = g0; c0 < g1; c0 += GC) {
      float v[GC];
#pragma unroll
      for (int u = 0; u < GC; ++u) v[u] = (c0 + u < g1) ? part[(c0 + u) * X + x] : 0.f;
#pragma unroll
      for (int u = 0; u < GC; ++u)
        if (c0 + u < g1) s += v[u];
    }
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv != 0 || x >= X) return;
#pragma unroll
  for (int w = 1; w < SW; ++w) s += red[w][lane];
  if (x < DD) out[(x / n) * ldc + x % n] = s;
  else if (colsum) colsum[x - DD] = s;
}

// Narrow outputs (X of a few thousand floats: the GVP message-GVP products 16 x 128, 16 x 48,
// 48 x 48, ...): sum_partials_one's 64 columns per workgroup leave X / 64 ~ 30 workgroups, each
// lane walking G / 4 ~ 128 slabs in dependent bursts (34 us per finish in the r05 GVP step, 128
// finishes per step).  Here a workgroup owns 16 columns and its 16 lane groups (4 per wave) each
// add a contiguous 1/16 of the slabs in one burst of loads (64-byte row pieces), then one lane
// group adds the 16 group sums in group order: X / 16 workgroups, a fixed order (deterministic).
template <int GC>
__global__ __launch_bounds__(256) void sum_partials_narrow(const float* __restrict__ part,
                                                           int64_t G, int64_t X,
                                                           float* __restrict__ out,
                                                           float* __restrict__ colsum,
                                                           int64_t DD, int64_t n, int64_t ldc) {
  __shared__ float red[16][16];
  const int q = threadIdx.x >> 4, c = threadIdx.x & 15;
  const int64_t x = blockIdx.x * (int64_t)16 + c;
  const int64_t per = (G + 15) / 16, g0 = q * per, g1 = (g0 + per < G) ? g0 + per : G;
  float s = 0.f;
  if (x < X) {
    for (int64_t c0 = g0; c0 < g1; c0 += GC) {
      float v[GC];
#pragma unroll
      for (int u = 0; u < GC; ++u) v[u] = (c0 + u < g1) ? part[(c0 + u) * X + x] : 0.f;
#pragma unroll
      for (int u = 0; u < GC; ++u)
        if (c0 + u < g1) s += v[u];
    }
  }
  red[q][c] = s;
  __syncthreads();
  if (q != 0 || x >= X) return;
#pragma unroll
  for (int w = 1; w < 16; ++w) s += red[w][c];
  if (x < DD) out[(x / n) * ldc + x % n] = s;
  else if (colsum) colsum[x - DD] = s;
}

// out (row stride ldc, n columns) = the ordered sum of G slabs of X = DD (+ colsum) floats.
// (r03: a two-level form with single-wave workgroups measured neutral on the EGNN step; removed)
void sum_partials(const float* part, int64_t G, int64_t X, float* out, float* colsum,
                  int64_t DD, int64_t n, int64_t ldc, hipStream_t s) {
  if (X < 8192 && G >= 64) {  // narrow: < 128 workgroups of 64 columns
    sum_partials_narrow<32><<<(unsigned)ceil_div(X, 16), 256, 0, s>>>(part, G, X, out, colsum,
                                                                      DD, n, ldc);
    return;
  }
  const unsigned grid = (unsigned)ceil_div(X, 64);
  sum_partials_one<4, 32><<<grid, 256, 0, s>>>(part, G, X, out, colsum, DD, n, ldc);
}

// Rectangular variant for the other per-edge Linears (GVP message GVPs: 128 x 144, 128 x 80,
// 16 x 128, 16 x 48, 16 x 16): C (M x N) = A^T B with M, N multiples of 16.  Wave tiling: with
// >= 4 row tiles a wave owns row tiles {w, w+4, ..} x all column tiles, otherwise all row tiles x
// column tiles {w, w+4, ..}; operands are read from LDS once per tile row / column (register
// reuse across the wave's tiles).  Register-staged double buffering of kKT-edge tiles; same
// split-K / ordered partial-sum scheme as above.
// LDS row stride = 16 mod 64 floats: the 4 edge rows (kk) of an MFMA operand read fall on
// disjoint 16-bank groups (conflict-free for all 64 lanes)
__host__ __device__ __forceinline__ int rect_ld(int x) { return x + ((16 - x) % 64 + 64) % 64; }
constexpr int kMaxL = 9;     // float4 loads per thread per tile (kKT * (M + N) / 4 / kT)

template <int MR, int MC, int NL, int OCC>
__global__ __launch_bounds__(kT, OCC) void outer_sum_rect_kernel(
    const float* __restrict__ A, const float* __restrict__ B, int64_t K, int M, int N,
    int64_t lda, int64_t ldb, int64_t k_per_block, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int LDA = rect_ld(M), LDB = rect_ld(N);
  const int TILE = kKT * (LDA + LDB);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, kk = lane >> 4;
  const int TM = M >> 4, TN = N >> 4;
  const bool rows_mode = TM >= 4;
  const int RT = rows_mode ? (TM - w + 3) / 4 : TM;
  const int CT = rows_mode ? TN : (TN - w + 3) / 4;
  const int64_t k0 = (int64_t)blockIdx.x * k_per_block;
  const int64_t k1 = (k0 + k_per_block < K) ? k0 + k_per_block : K;
  f32x4 acc[MR][MC];
#pragma unroll
  for (int r = 0; r < MR; ++r)
#pragma unroll
    for (int c = 0; c < MC; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float cs[MR];
#pragma unroll
  for (int r = 0; r < MR; ++r) cs[r] = 0.f;
  const int CA = M >> 2, CTOT = (M + N) >> 2;
  f32x4 reg[NL];
  // element tid + q*kT of the tile's (row, float4 column) list: (r0 + q*dR + carry, x...)
  // computed incrementally — one division per thread, not per element
  int rq[NL], xq[NL];
  {
    const int dR = kT / CTOT, dX = kT - dR * CTOT;
    int r = tid / CTOT, x = tid - (tid / CTOT) * CTOT;
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      rq[q] = r;
      xq[q] = x;
      r += dR;
      x += dX;
      if (x >= CTOT) {
        x -= CTOT;
        ++r;
      }
    }
  }
  auto fetch = [&](int64_t kb) {
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      reg[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int64_t k = kb + rq[q];
      if (rq[q] < kKT && k < k1) {
        const int x = xq[q];
        reg[q] = (x < CA) ? *reinterpret_cast<const f32x4*>(A + k * lda + 4 * x)
                          : *reinterpret_cast<const f32x4*>(B + k * ldb + 4 * (x - CA));
      }
    }
  };
  auto stash = [&](float* buf) {
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      if (rq[q] < kKT) {
        const int r = rq[q], x = xq[q];
        float* dst = (x < CA) ? buf + r * LDA + 4 * x : buf + kKT * LDA + r * LDB + 4 * (x - CA);
        *reinterpret_cast<f32x4*>(dst) = reg[q];
      }
    }
  };
  int cur = 0;
  if (k0 < k1) {
    fetch(k0);
    stash(sm);
  }
  __syncthreads();
  for (int64_t kb = k0; kb < k1; kb += kKT) {
    const bool more = kb + kKT < k1;
    if (more) fetch(kb + kKT);
    const float* sA = sm + cur * TILE;
    const float* sB = sA + kKT * LDA;
#pragma unroll
    for (int st = 0; st < kKT / 4; ++st) {
      const int e = 4 * st + kk;
      float af[MR], bf[MC];
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const int tm = rows_mode ? w + 4 * r : r;
        af[r] = (r < RT) ? sA[e * LDA + 16 * tm + li] : 0.f;
      }
#pragma unroll
      for (int c = 0; c < MC; ++c) {
        const int tn = rows_mode ? c : w + 4 * c;
        bf[c] = (c < CT) ? sB[e * LDB + 16 * tn + li] : 0.f;
      }
      // colsum(A) from the A operands already in registers (edges e = kk mod 4 of this lane)
#pragma unroll
      for (int r = 0; r < MR; ++r) cs[r] += af[r];
      // no per-tile guard: out-of-range tiles multiply zero operands (a wave's time is set by
      // the wave with the most tiles anyway) and are never stored — branch-free MFMA stream
#pragma unroll
      for (int r = 0; r < MR; ++r)
#pragma unroll
        for (int c = 0; c < MC; ++c)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[r], bf[c], acc[r][c], 0, 0, 0);
    }
    if (more) stash(sm + (cur ^ 1) * TILE);
    __syncthreads();
    cur ^= 1;
  }
  float* out = partial + (int64_t)blockIdx.x * ((int64_t)M * N + M);
#pragma unroll
  for (int r = 0; r < MR; ++r)
#pragma unroll
    for (int c = 0; c < MC; ++c)
      if (r < RT && c < CT) {
        const int tm = rows_mode ? w + 4 * r : r;
        const int tn = rows_mode ? c : w + 4 * c;
#pragma unroll
        for (int q = 0; q < 4; ++q) out[(16 * tm + 4 * kk + q) * N + 16 * tn + li] = acc[r][c][q];
      }
  // colsum: add the 4 edge-phase lane groups (l, l^16, l^32, l^48) in a fixed order; each
  // row tile is owned by one wave (rows mode) or by wave 0 (columns mode: all waves hold it)
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    float v = cs[r];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    const int tm = rows_mode ? w + 4 * r : r;
    if (kk == 0 && r < RT && (rows_mode || w == 0)) out[(int64_t)M * N + 16 * tm + li] = v;
  }
}

// ------------------------------------------------------------------ f32 through three bf16 planes
// The edge reduction runs on the bf16 MFMA (16x the f32 MFMA rate on gfx950) without giving up
// f32 accuracy: every f32 operand is split exactly into three bf16 planes x = x0 + x1 + x2
// (RNE splits: |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|, each product of two planes exact in the f32
// accumulator) and the six partial products of order <= 2^-16 are accumulated,
//     C += A2 B0 + A1 B1 + A0 B2 + A1 B0 + A0 B1 + A0 B0,
// dropping A1 B2, A2 B1, A2 B2 (<= 2^-26 |a b| together).  Measured error vs fp64
// (tests/test_gpu_wgrad.py, K = 1M): 1.2e-8 of sum |a b| per entry, 2x the f32-MFMA split-K
// kernel's, 20x below rocBLAS's f32 GEMM's (f32 unit roundoff: 6e-8).
// Six 16x16x32 bf16 MFMAs (16 cycles each) replace eight 16x16x4 f32 MFMAs (32 cycles each) per
// 32 edges x 16 x 16 outputs: 2.7x less matrix time, so the kernel becomes HBM-bound.
//
// Layout: 512 threads (8 waves, a WM x WN grid of RT x CT output tiles of 16 x 16 each), one
// 32-edge stage per MFMA k step.  A thread loads a (4 edges x 4 channels) unit of A or B with
// four 16-byte loads (8 lanes cover 128 contiguous bytes of a row), splits it and writes each
// channel's 4 edges per plane as 8 bytes into an LDS image [plane][channel][32 edges] of 64-byte
// rows whose 16-byte chunk q sits at q ^ ((row >> 1) & 3): 8 lanes fill one row per ds_write_b64
// and the MFMA operand read (lane: channel l & 15, edges 8(l >> 4) .. +7) is one conflict-free
// ds_read_b128.  Loads run PD stages ahead in a register ring (branch-free: counted vmcnt
// waits); two LDS stages.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int kXT = 512;  // threads (8 waves)
constexpr int kXK = 32;   // edges per stage (= the bf16 MFMA k)
constexpr int kXPad = 64; // LDS padding rows per plane (>= 16 * (WN * CT - TN) of any tiling)

__device__ __forceinline__ void split3(f32x2 x, unsigned& h, unsigned& m, unsigned& l) {
  const bf16x2 bh = __builtin_convertvector(x, bf16x2);
  const f32x2 r1 = x - __builtin_convertvector(bh, f32x2);   // exact
  const bf16x2 bm = __builtin_convertvector(r1, bf16x2);
  const f32x2 r2 = r1 - __builtin_convertvector(bm, f32x2);  // exact, <= 8 significant bits
  const bf16x2 bl = __builtin_convertvector(r2, bf16x2);     // exact
  h = __builtin_bit_cast(unsigned, bh);
  m = __builtin_bit_cast(unsigned, bm);
  l = __builtin_bit_cast(unsigned, bl);
}
__device__ __forceinline__ int xoff(int row, int chunk) {
  return row * 64 + 16 * (chunk ^ ((row >> 1) & 3));
}

// HF form (NP = 2; gmp_edge_outer_sum_act_hf_f32): two fp16 planes (x = hi + lo, 22 bits) of
// the operands scaled by powers of two, three products lo*hi + hi*lo + hi*hi per stage, partial
// slabs scaled back exactly.  A's scale from a device max word (the EGNN backward kernel folds
// max |dpre| into it); B = act(X w + b) of LayerNorm rows X (|X| <= sqrt(N)): bounded by
// sqrt(N) max|w| + max|b|, computed per block from w, b.
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void split2h(f32x2 x, unsigned& h, unsigned& l) {
  const h16x2 hh = __builtin_convertvector(x, h16x2);
  const f32x2 r = x - __builtin_convertvector(hh, f32x2);  // exact
  const h16x2 hl = __builtin_convertvector(r, h16x2);
  h = __builtin_bit_cast(unsigned, hh);
  l = __builtin_bit_cast(unsigned, hl);
}
__device__ __forceinline__ int hf_scale_exp(float mx) {
  if (!(mx > 0.f) || !(mx < 3.0e38f)) return 0;
  int e;
  (void)frexpf(mx, &e);
  const int s = 15 - e;
  return s < -120 ? -120 : (s > 120 ? 120 : s);
}

template <int RT, int CT, int PRO, int NL, int NP = 3, int PD = (NL == 1 ? 4 : 2)>
__global__ __launch_bounds__(kXT, 1) void outer_sum_x3_kernel(
    const float* __restrict__ A, const float* __restrict__ B, int64_t K, int M, int N,
    int64_t lda, int64_t ldb, int64_t k_per_block, float* __restrict__ partial,
    const float* __restrict__ bw, const float* __restrict__ bb, int WN,
    const float* __restrict__ B2, int64_t ldb2, int N1, int64_t a_col_step,
    const unsigned* __restrict__ amaxA) {
  // B may be two column blocks [B (N1 columns) | B2 (N - N1 columns)] of different tensors.
  // blockIdx.y > 0 (gmp_outer_sum_cols_f32): column block y of a wide A, A + y a_col_step, its
  // own row of partial slabs
  A += (int64_t)blockIdx.y * a_col_step;
  partial += (int64_t)blockIdx.y * gridDim.x * ((int64_t)M * N + M);
  extern __shared__ __attribute__((aligned(16))) unsigned char smx[];
  const int R = M + N;  // LDS rows per plane: A channels, then B channels
  // + 64 padding rows: written by idle loader lanes (row R), read by the ragged tiles
  const int PLANE = (R + kXPad) * 64, STAGE = NP * PLANE;
  const int tid = threadIdx.x, lane = tid & 63;
  // HF scales: fa = 2^sa (A), fb = 2^sb (B), partials x 2^-sa x 2^-sb (two exact steps)
  float fa = 1.f, fb = 1.f, da = 1.f, db = 1.f;
  if constexpr (NP == 2) {
    __shared__ unsigned bmx[2];
    if (tid < 2) bmx[tid] = 0u;
    __syncthreads();
    if (tid < N) {
      atomicMax(&bmx[0], __float_as_uint(fabsf(bw[tid])));
      atomicMax(&bmx[1], __float_as_uint(fabsf(bb[tid])));
    }
    __syncthreads();
    const int sa = hf_scale_exp(__uint_as_float(amaxA[0]));
    const int sb = hf_scale_exp(sqrtf((float)N) * __uint_as_float(bmx[0]) +
                                __uint_as_float(bmx[1]));
    fa = ldexpf(1.f, sa);
    fb = ldexpf(1.f, sb);
    da = ldexpf(1.f, -sa);
    db = ldexpf(1.f, -sb);
  }
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar tile branches
  const int li = lane & 15, g = lane >> 4;
  const int wm = w / WN, wn = w - (w / WN) * WN;
  const int TM = M >> 4, TN = N >> 4;
  const int64_t k0 = (int64_t)blockIdx.x * k_per_block;
  const int64_t k1 = (k0 + k_per_block < K) ? k0 + k_per_block : K;

  f32x4 acc[RT][CT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // loader units u = tid + q * kXT: [0, UA) A units, [UA, UA + UB) B units, each range padded
  // to whole waves (a wave loads from one operand); unit v of an operand: edge quad v % 8,
  // channel group v / 8
  const int UA = (2 * M + 63) & ~63, UB = (2 * N + 63) & ~63;
  int ucg[NL], ueq[NL], lrow[NL];
  bool uok[NL], isA[NL];
  f32x4 pw[NL], pb[NL], csum[NL];
#pragma unroll
  for (int q = 0; q < NL; ++q) {
    const int u = tid + q * kXT;
    isA[q] = 64 * w + q * kXT < UA;  // wave-uniform by the padding
    const int v = isA[q] ? u : u - UA;
    uok[q] = isA[q] ? v < 2 * M : (v < 2 * N && u < UA + UB);
    ueq[q] = uok[q] ? (v & 7) : 0;   // edge quad fastest: 8 lanes fill one 64-B LDS row
    ucg[q] = uok[q] ? (v >> 3) : 0;  // (conflict-free ds_write_b64), 128-B global row runs
    // idle lanes load zeros (out-of-range offset) and write them to the spare rows R .. R+3
    lrow[q] = !uok[q] ? R : (isA[q] ? 4 * ucg[q] : M + 4 * ucg[q]);
    csum[q] = pw[q] = pb[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (PRO != 0 && uok[q] && !isA[q]) {
      pw[q] = *reinterpret_cast<const f32x4*>(bw + 4 * ucg[q]);
      pb[q] = *reinterpret_cast<const f32x4*>(bb + 4 * ucg[q]);
    }
  }
  // global -> register ring, PD stages ahead.  Every load is issued (rows clamped to the
  // block's last row, idle lanes read row k0) and masked to zero in stash: no branches, so the
  // compiler's vmcnt waits are counted
  const float* ubase[NL];
  int64_t uld[NL];
#pragma unroll
  for (int q = 0; q < NL; ++q) {
    const bool second = !isA[q] && 4 * ucg[q] >= N1;
    uld[q] = isA[q] ? lda : (second ? ldb2 : ldb);
    ubase[q] = isA[q] ? A + 4 * ucg[q] : (second ? B2 + (4 * ucg[q] - N1) : B + 4 * ucg[q]);
  }
  f32x4 ring[PD][NL][4];
  auto fetch = [&](f32x4 (&reg)[NL][4], int st) {
#pragma unroll
    for (int q = 0; q < NL; ++q) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int64_t k = k0 + st * kXK + 4 * ueq[q] + j;
        k = k < k1 ? k : k1 - 1;
        reg[q][j] = *reinterpret_cast<const f32x4*>(ubase[q] + k * uld[q]);
      }
    }
  };
  auto stash = [&](f32x4 (&reg)[NL][4], unsigned char* buf, int st) {
#pragma unroll
    for (int q = 0; q < NL; ++q) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool valid = uok[q] && k0 + st * kXK + 4 * ueq[q] + j < k1;
        const f32x4 y = (PRO != 0 && !isA[q]) ? prologue<PRO>(reg[q][j], pw[q], pb[q]) : reg[q][j];
        reg[q][j] = valid ? y : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) csum[q] += reg[q][j];  // used for A units only
      const int eq = ueq[q];
      const float fs = isA[q] ? fa : fb;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int off = xoff(lrow[q] + c, eq >> 1) + 8 * (eq & 1);
        if constexpr (NP == 3) {
          unsigned h0, m0, l0, h1, m1, l1;
          split3(f32x2{reg[q][0][c], reg[q][1][c]}, h0, m0, l0);
          split3(f32x2{reg[q][2][c], reg[q][3][c]}, h1, m1, l1);
          *reinterpret_cast<u32x2*>(buf + off) = u32x2{h0, h1};
          *reinterpret_cast<u32x2*>(buf + PLANE + off) = u32x2{m0, m1};
          *reinterpret_cast<u32x2*>(buf + 2 * PLANE + off) = u32x2{l0, l1};
        } else {
          unsigned h0, l0, h1, l1;
          split2h(f32x2{reg[q][0][c] * fs, reg[q][1][c] * fs}, h0, l0);
          split2h(f32x2{reg[q][2][c] * fs, reg[q][3][c] * fs}, h1, l1);
          *reinterpret_cast<u32x2*>(buf + off) = u32x2{h0, h1};
          *reinterpret_cast<u32x2*>(buf + PLANE + off) = u32x2{l0, l1};
        }
      }
    }
  };
  // branch-free: tiles past TM / TN (ragged wave grids) multiply rows of the LDS padding or of
  // the other operand and are never stored, so compute and stash form one basic block and the
  // scheduler can overlap the MFMAs with the next stage's split
  auto compute = [&](const unsigned char* buf) {
    if constexpr (NP == 3) {
      bf16x8 a[RT][3];
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int off = xoff(16 * (wm * RT + r) + li, g);
#pragma unroll
        for (int p = 0; p < 3; ++p) a[r][p] = *reinterpret_cast<const bf16x8*>(buf + p * PLANE + off);
      }
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const int off = xoff(M + 16 * (wn * CT + c) + li, g);
        bf16x8 b[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) b[p] = *reinterpret_cast<const bf16x8*>(buf + p * PLANE + off);
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          f32x4 t = acc[r][c];
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][2], b[0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][1], b[1], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][0], b[2], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][1], b[0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][0], b[1], t, 0, 0, 0);
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][0], b[0], t, 0, 0, 0);
        }
      }
    } else {
      h16x8 a[RT][2];
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int off = xoff(16 * (wm * RT + r) + li, g);
#pragma unroll
        for (int p = 0; p < 2; ++p) a[r][p] = *reinterpret_cast<const h16x8*>(buf + p * PLANE + off);
      }
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const int off = xoff(M + 16 * (wn * CT + c) + li, g);
        h16x8 b[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) b[p] = *reinterpret_cast<const h16x8*>(buf + p * PLANE + off);
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          f32x4 t = acc[r][c];
          t = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[r][1], b[0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[r][0], b[1], t, 0, 0, 0);
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[r][0], b[0], t, 0, 0, 0);
        }
      }
    }
  };

  // stages rounded up to whole ring turns and every fetch / stash unconditional (stages past
  // the block's rows load zeros and add nothing): the same loads are in flight at every wait,
  // so the compiler's vmcnt waits are counted, PD - 1 stages deep
  const int nst = k1 > k0 ? (int)((k1 - k0 + kXK - 1) / kXK) : 0;
  const int nst_pad = (nst + PD - 1) / PD * PD;
  if (nst > 0) {
#pragma unroll
    for (int j = 0; j < PD; ++j) fetch(ring[j], j);
    stash(ring[0], smx, 0);
  }
  __syncthreads();
  for (int s0 = 0; s0 < nst_pad; s0 += PD) {
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      const int st = s0 + j;
      fetch(ring[j], st + PD);  // slot j was stashed for stage st
      compute(smx + (st & 1) * STAGE);
      stash(ring[(j + 1) % PD], smx + ((st + 1) & 1) * STAGE, st + 1);
      __syncthreads();
    }
  }

  // C/D map of 16x16x32: col = lane & 15, row = 4 * (lane >> 4) + r
  float* out = partial + (int64_t)blockIdx.x * ((int64_t)M * N + M);
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int tm = wm * RT + r, tn = wn * CT + c;
      if (tm < TM && tn < TN) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          out[(int64_t)(16 * tm + 4 * g + q) * N + 16 * tn + li] =
              NP == 3 ? acc[r][c][q] : (acc[r][c][q] * da) * db;
      }
    }
  // colsum(A): the 8 edge quads of a channel group added in quad order (deterministic)
  float* scs = reinterpret_cast<float*>(smx);  // [8][M], after the loop's final barrier
#pragma unroll
  for (int q = 0; q < NL; ++q) {
    if (!uok[q] || !isA[q]) continue;
    float* d = scs + ueq[q] * M + 4 * ucg[q];
    d[0] = csum[q][0];
    d[1] = csum[q][1];
    d[2] = csum[q][2];
    d[3] = csum[q][3];
  }
  __syncthreads();
  for (int m = tid; m < M; m += kXT) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += scs[e * M + m];
    out[(int64_t)M * N + m] = s;
  }
}

// (RT, CT) tile shape per wave for an M x N problem: the first of the compiled shapes whose
// wave grid fits in 8 waves; returns the index into kX3 or -1
struct X3Shape { int rt, ct; };
// ({1, 1} would only fit m n <= 2048, which stays on the f32-MFMA kernels)
constexpr X3Shape kX3[] = {{1, 2}, {2, 2}, {2, 4}, {2, 5}};
int x3_pick(int64_t m, int64_t n, int* wn) {
  const int64_t TM = m / 16, TN = n / 16;
  for (int i = 0; i < 4; ++i) {
    const int64_t WM = ceil_div(TM, (int64_t)kX3[i].rt), WN = ceil_div(TN, (int64_t)kX3[i].ct);
    if (WM * WN <= kXT / 64) {
      *wn = (int)WN;
      return i;
    }
  }
  return -1;
}
// 1: the f32-MFMA kernels (numerics studies, the exact-f32 bench leg); gmp_wgrad_set_f32_mfma
int g_wgrad_mode = 0;
bool wgrad_f32_mfma() { return g_wgrad_mode == 1; }
// minimum edge tiles per workgroup of the f32-MFMA split-K sums
constexpr int kMinTiles = 16;

// smallest K (rows) routed to the split-plane sums (below: the node-level quadrant sums)
constexpr int64_t kX3MinK = 262144;
int64_t x3_blocks_for(int64_t K) {
  // one 8-wave workgroup per CU (LDS ~100 KB)
  int64_t g = (int64_t)device_cu_count();
  const int64_t min_per = 4 * kXK;
  if (g * min_per > K) g = ceil_div(K, min_per);
  return g < 1 ? 1 : g;
}

// C (m x n, row stride ldc) = A^T pro(B), colsum(A): split-K over x3 blocks + ordered sums.
// Returns GMP_ERR_UNSUPPORTED for shapes outside the compiled tilings.
int outer_sum_x3_launch(int64_t K, int64_t m, int64_t n, const float* A, int64_t lda,
                        const float* B, int64_t ldb, int pro, const float* bw, const float* bb,
                        float* C, int64_t ldc, float* colsum_A, void* workspace, hipStream_t s,
                        const float* B2 = nullptr, int64_t ldb2 = 0, int64_t n1 = -1,
                        const unsigned* amaxA = nullptr) {
  const bool hf = amaxA != nullptr;  // HF form: act prologue (pro != 0), single B operand
  if (hf && (pro == 0 || B2 || n > kXT)) return GMP_ERR_UNSUPPORTED;
  if (n1 < 0) n1 = n;  // single B operand
  // Narrow products (m n < 4096) stay on the f32-MFMA kernels: too little matrix work per
  // loaded byte for the split's VALU and LDS staging to pay (measured: 16 x 128, 48 x 48 slower).
  // Node-level sums (K ~ 50k rows) stay there too: a few stages per block, and the 1-block-per-
  // CU LDS footprint keeps them from sharing CUs with the concurrent main-stream kernels.
  if (m * n < 4096 || K < kX3MinK) return GMP_ERR_UNSUPPORTED;
  int wn = 0;
  const int shape = x3_pick(m, n, &wn);
  const int64_t R = m + n;
  if (shape < 0 || R + kXPad > 416) return GMP_ERR_UNSUPPORTED;  // 2 x 3 x (R + pad) x 64 B
  GMP_CHECK_ARG(pro == 0 || ((reinterpret_cast<uintptr_t>(bw) | reinterpret_cast<uintptr_t>(bb)) % 16 == 0));
  const int64_t units = ((2 * m + 63) & ~63) + ((2 * n + 63) & ~63);
  if (units > 2 * kXT) return GMP_ERR_UNSUPPORTED;
  const int nl = units <= kXT ? 1 : 2;
  const int64_t G = x3_blocks_for(K);
  const int64_t per = ceil_div(ceil_div(K, G), kXK) * kXK;
  const int64_t Gr = ceil_div(K, per);
  float* part = reinterpret_cast<float*>(workspace);
  const size_t smem = (size_t)2 * (hf ? 2 : 3) * (R + kXPad) * 64;
  int rc = 0;
#define LAUNCH_X3(RT, CT, PP, NL)                                                                \
  {                                                                                           \
    auto k = hf ? outer_sum_x3_kernel<RT, CT, PP, NL, 2> : outer_sum_x3_kernel<RT, CT, PP, NL>; \
    if ((rc = hip_check(hipFuncSetAttribute((const void*)k,                                   \
                                            hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                            (int)smem))))                                     \
      return rc;                                                                              \
    k<<<(unsigned)Gr, kXT, smem, s>>>(A, B, K, (int)m, (int)n, lda, ldb, per, part, bw, bb,  \
                                      wn, B2, ldb2, (int)n1, 0, amaxA);                       \
  }
#define LAUNCH_X3_NL(RT, CT, PP) \
  if (nl == 1) LAUNCH_X3(RT, CT, PP, 1) else LAUNCH_X3(RT, CT, PP, 2)
#define LAUNCH_X3_PRO(RT, CT)                   \
  if (pro == 0) { LAUNCH_X3_NL(RT, CT, 0) }     \
  else if (pro == 1) { LAUNCH_X3_NL(RT, CT, 1) } \
  else { LAUNCH_X3_NL(RT, CT, 2) }
  switch (shape) {
    case 0: LAUNCH_X3_PRO(1, 2) break;
    case 1: LAUNCH_X3_PRO(2, 2) break;
    case 2: LAUNCH_X3_PRO(2, 4) break;
    default: LAUNCH_X3_PRO(2, 5) break;
  }
#undef LAUNCH_X3_PRO
#undef LAUNCH_X3_NL
#undef LAUNCH_X3
  rc = launch_status();
  if (rc) return rc;
  const int64_t X = m * n + m;
  sum_partials(part, Gr, X, C, colsum_A, m * n, n, ldc, s);
  return launch_status();
}

// Wide A: C (m_total x n, row stride ldc) = A^T B for m_total a multiple of 128 (the TP path
// GEMM dW2p = S^T G: S (K rows x mul1 H), G (K rows x mul_out)), column blocks of 128 on
// blockIdx.y, split-K over Gr row ranges per block, then one ordered pass over the Gr slabs.
constexpr int kColBlk = 128;
int64_t cols_groups(int64_t K, int64_t Y) {
  int64_t g = ceil_div(2 * (int64_t)device_cu_count(), Y);
  const int64_t cap = ceil_div(K, 4 * kXK);
  if (g > cap) g = cap;
  return g < 1 ? 1 : g;
}

__global__ void sum_partials_cols(const float* __restrict__ part, int64_t Gr, int64_t X, int m,
                                  int n, float* __restrict__ C, int64_t ldc) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t y = blockIdx.y;
  if (x >= (int64_t)m * n) return;
  const float* p = part + y * Gr * X + x;
  float s = 0.f;
  for (int64_t g0 = 0; g0 < Gr; g0 += kGC) {  // kGC loads in flight, added in slab order
    float v[kGC];
#pragma unroll
    for (int u = 0; u < kGC; ++u) v[u] = (g0 + u < Gr) ? p[(g0 + u) * X] : 0.f;
#pragma unroll
    for (int u = 0; u < kGC; ++u)
      if (g0 + u < Gr) s += v[u];
  }
  const int64_t r = x / n, c = x - r * n;
  C[(y * m + r) * ldc + c] = s;
}

// dW2p column-block outer sum with G pre-split ("pre-split G once per pass
// instead of per column block"): B = three bf16 planes of G in MFMA fragment order, k padded
// to 32 (split_g_kernel, once per call), read straight into registers PD stages ahead; only A
// (the S columns of the block) goes through LDS.  The r03 kernel staged and split both operands
// per column block: ~196 KB of LDS traffic per 32-deep stage against 1536 MFMA cycles (LDS-
// bound, 29 % bank conflicts).  Here: 24 KB of A writes + 96 KB of A fragment reads per stage.
// 512 threads, wave grid 2 (M) x 4 (N): wave tile 64 x 16 CT.
__device__ __forceinline__ int64_t gfrag_index(int64_t p, int64_t n, int64_t k, int64_t ct_total) {
  return ((((k >> 5) * ct_total + (n >> 4)) * 3 + p) * 64 + (n & 15) + 16 * ((k & 31) >> 3)) * 8 +
         (k & 7);
}
// lane l of block (k step ks, column tile ct): rows 32 ks + 8 (l >> 4) .. + 7 of column
// 16 ct + (l & 15) -> three 16-byte plane pieces (coalesced reads along G rows, contiguous writes)
__global__ __launch_bounds__(256) void split_g_kernel(const float* __restrict__ G, int64_t K,
                                                      int64_t nks, int n,
                                                      unsigned short* __restrict__ Bp) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // (ks, ct) block per wave
  const int ct_total = n >> 4;
  if (t >= nks * ct_total) return;
  const int64_t ks = t / ct_total, ct = t - ks * ct_total;
  const int l = threadIdx.x & 63;
  const int64_t col = 16 * ct + (l & 15), k0 = 32 * ks + 8 * (l >> 4);
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = k0 + i < K ? G[(k0 + i) * n + col] : 0.f;
  u32x4 pl[3];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned h, m, lo;
    split3(f32x2{v[2 * i], v[2 * i + 1]}, h, m, lo);
    pl[0][i] = h;
    pl[1][i] = m;
    pl[2][i] = lo;
  }
#pragma unroll
  for (int p = 0; p < 3; ++p)
    *reinterpret_cast<u32x4*>(Bp + ((t * 3 + p) * 64 + l) * 8) = pl[p];
}

template <int CT, int PD, int OCC>
__global__ __launch_bounds__(kXT, OCC) void outer_cols_x3g_kernel(
    const float* __restrict__ A, int64_t K, int64_t lda, const unsigned short* __restrict__ Bp,
    int n, int64_t k_per_block, int64_t X, float* __restrict__ partial) {
  constexpr int RT = 4;
  constexpr int PL = kColBlk * 64, STG = 3 * PL;  // one plane image: 128 rows x 32 bf16
  __shared__ __attribute__((aligned(16))) unsigned char sa[2 * STG];
  A += (int64_t)blockIdx.y * kColBlk;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wm = w >> 2, wn = w & 3;
  const int64_t k0 = (int64_t)blockIdx.x * k_per_block;
  const int64_t k1 = (k0 + k_per_block < K) ? k0 + k_per_block : K;
  const int nst = k1 > k0 ? (int)((k1 - k0 + kXK - 1) / kXK) : 0;
  // A loader (waves 0-3): edge quad eq (4 rows k), channel group cg (4 columns); measured
  // faster than spreading the block over all 8 waves (12.8 vs 11.7 ms at the MACE lo = 2
  // shape: twice the LDS store instructions at half the width)
  const bool loader = w < 4;
  const int eq = tid & 7, cg = (tid >> 3) & 31;
  const float* abase = A + 4 * cg;
  f32x4 ra[PD][4];
  auto fetch_a = [&](int slot, int st) {
    if (!loader) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t k = k0 + (int64_t)st * kXK + 4 * eq + j;
      k = k < k1 ? k : k1 - 1;
      ra[slot][j] = *reinterpret_cast<const f32x4*>(abase + k * lda);
    }
  };
  auto stash_a = [&](int slot, unsigned char* buf, int st) {
    if (!loader) return;
    f32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool ok = k0 + (int64_t)st * kXK + 4 * eq + j < k1;
      v[j] = ok ? ra[slot][j] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // column 4 cg + c goes to image row 4 cg + (c ^ (cg & 1)): the two channel groups of a
    // 16-lane ds_write_b64 group (banks (a / 4) mod 32: a 128-byte period) then land 3 or 5
    // rows apart (64 B mod 128) instead of 4 (the same banks: a 2-way conflict on every store);
    // the epilogue undoes the permutation
    const int cx = cg & 1;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int off = xoff(4 * cg + (c ^ cx), eq >> 1) + 8 * (eq & 1);
      unsigned h0, m0, l0, h1, m1, l1;
      split3(f32x2{v[0][c], v[1][c]}, h0, m0, l0);
      split3(f32x2{v[2][c], v[3][c]}, h1, m1, l1);
      *reinterpret_cast<u32x2*>(buf + off) = u32x2{h0, h1};
      *reinterpret_cast<u32x2*>(buf + PL + off) = u32x2{m0, m1};
      *reinterpret_cast<u32x2*>(buf + 2 * PL + off) = u32x2{l0, l1};
    }
  };
  const int64_t ct_total = n >> 4;
  const unsigned short* bl = Bp + 8 * lane;
  u32x4 rb[PD][CT][3];
  auto fetch_b = [&](int slot, int st) {
    const int64_t ks = (k0 >> 5) + (st < nst ? st : (nst > 0 ? nst - 1 : 0));
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        rb[slot][c][p] = *reinterpret_cast<const u32x4*>(
            bl + ((ks * ct_total + wn * CT + c) * 3 + p) * 512);
  };
  f32x4 acc[RT][CT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const unsigned char* buf, int slot) {
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int off = xoff(64 * wm + 16 * r + li, g);
      bf16x8 a[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8*>(buf + p * PL + off);
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        f32x4 t = acc[r][c];
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], __builtin_bit_cast(bf16x8, rb[slot][c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], __builtin_bit_cast(bf16x8, rb[slot][c][1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], __builtin_bit_cast(bf16x8, rb[slot][c][2]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], __builtin_bit_cast(bf16x8, rb[slot][c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], __builtin_bit_cast(bf16x8, rb[slot][c][1]), t, 0, 0, 0);
        acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], __builtin_bit_cast(bf16x8, rb[slot][c][0]), t, 0, 0, 0);
      }
    }
  };
  if (nst > 0) {
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      fetch_a(q, q);
      fetch_b(q, q);
    }
    stash_a(0, sa, 0);
  }
  __syncthreads();
  const int nst_pad = (nst + PD - 1) / PD * PD;
  for (int s0 = 0; s0 < nst_pad; s0 += PD) {
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      const int st = s0 + j;
      fetch_a(j, st + PD);  // slot j was stashed for stage st
      compute(sa + (st & 1) * STG, j);
      __builtin_amdgcn_sched_barrier(0);
      fetch_b(j, st + PD);  // the slot the MFMAs above just read
      stash_a((j + 1) % PD, sa + ((st + 1) & 1) * STG, st + 1);
      __syncthreads();
    }
  }
  // C/D map of 16x16x32: col = lane & 15, row = 4 (lane >> 4) + q; slab layout as the r03
  // kernel's (X floats per (column block, range): m n values, the colsum tail unused here)
  float* out = partial + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * X;
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        // image row 64 wm + 16 r + 4 g + q holds column 64 wm + 16 r + 4 g + (q ^ (g & 1))
        out[(int64_t)(64 * wm + 16 * r + 4 * g + (q ^ (g & 1))) * n + 16 * (wn * CT + c) + li] =
            acc[r][c][q];
}

// Node-level sums (r04): C (m x n, m, n multiples of 64, <= 256) = A^T B (+ colsum(A)) over K
// rows with the OUTPUT split into 64 x 64 quadrants as well as K into row ranges: 4-wave
// workgroups (32 KB of LDS, two per CU) of ~400 rows each, so a 50k-row sum spreads over ~512
// short workgroups instead of ~100 long ones (r03: outer_sum_kernel<128, 0> 107-115 us per 50k x
// 128 x 128 sum on the side stream, holding CUs the critical path's node kernels wait for).
// f32 MFMA 16x16x4 (exact f32 products, the rows as the MFMA k dimension), stages of 32 rows
// double-buffered through LDS; slabs summed in range order by sum_partials_one<4>.
constexpr int kQT = 256;
constexpr int kQK = 32;
constexpr int kQLd = 64 + 4;
__global__ __launch_bounds__(kQT, 2) void outer_sum_quad_kernel(
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb, int64_t K,
    int m, int n, int64_t per, float* __restrict__ part, int64_t X) {
  __shared__ __attribute__((aligned(16))) float sA[2][kQK * kQLd];
  __shared__ __attribute__((aligned(16))) float sB[2][kQK * kQLd];
  __shared__ float sCol[16][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, kk = lane >> 4;
  const int nq = n >> 6;
  const int qm = blockIdx.y / nq, qn = blockIdx.y - qm * nq;
  const int m0 = 64 * qm, n0 = 64 * qn;
  const int64_t k0 = (int64_t)blockIdx.x * per;
  const int64_t k1 = (k0 + per < K) ? k0 + per : K;
  const int wm = w >> 1, wn = w & 1;
  const bool colsum = qn == 0;
  // loader: v = tid + 256 q (q < 2) -> stage row v / 16, float4 column group v % 16 (the same
  // column group for both q: the thread's colsum stays in registers)
  const int cq = tid & 15, r0 = tid >> 4;
  f32x4 ra[2], rb[2], csum = {0.f, 0.f, 0.f, 0.f};
  auto fetch = [&](int64_t kb) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t k = kb + r0 + 16 * q;
      ra[q] = rb[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k < k1) {
        ra[q] = *reinterpret_cast<const f32x4*>(A + k * lda + m0 + 4 * cq);
        rb[q] = *reinterpret_cast<const f32x4*>(B + k * ldb + n0 + 4 * cq);
      }
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = r0 + 16 * q;
      csum += ra[q];
      *reinterpret_cast<f32x4*>(&sA[buf][r * kQLd + 4 * cq]) = ra[q];
      *reinterpret_cast<f32x4*>(&sB[buf][r * kQLd + 4 * cq]) = rb[q];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) acc[a][0] = acc[a][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  int buf = 0;
  if (k0 < k1) {
    fetch(k0);
    stash(0);
  }
  __syncthreads();
  for (int64_t kb = k0; kb < k1; kb += kQK) {
    const bool more = kb + kQK < k1;
    if (more) fetch(kb + kQK);  // in flight while this stage is computed
    const float* a_s = sA[buf];
    const float* b_s = sB[buf];
#pragma unroll
    for (int st = 0; st < kQK / 4; ++st) {
      const int e = 4 * st + kk;
      float af[2], bf[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        af[t] = a_s[e * kQLd + 32 * wm + 16 * t + li];
        bf[t] = b_s[e * kQLd + 32 * wn + 16 * t + li];
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
    if (more) stash(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // C/D map of 16x16x4: col = lane & 15, row = 4 (lane >> 4) + r
  float* out = part + (int64_t)blockIdx.x * X;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(int64_t)(m0 + 32 * wm + 16 * a + 4 * kk + r) * n + n0 + 32 * wn + 16 * b + li] =
            acc[a][b][r];
  if (colsum) {  // the 16 row groups of each column group, added in row-group order
    *reinterpret_cast<f32x4*>(&sCol[r0][4 * cq]) = csum;
    __syncthreads();
    if (tid < 64) {
      float t = 0.f;
#pragma unroll
      for (int g2 = 0; g2 < 16; ++g2) t += sCol[g2][tid];
      out[(int64_t)m * n + m0 + tid] = t;
    }
  }
}

// node-level (K < kX3MinK) sums: split over about two workgroups per CU
int64_t quad_splits(int64_t K, int64_t quads) {
  int64_t s = ceil_div((int64_t)2 * device_cu_count(), quads);
  const int64_t cap = ceil_div(K, 256);                          // >= 256 rows each
  if (s > cap) s = cap;
  return s < 1 ? 1 : s;
}
// (r06: up to 1024 x 1024 -- the quadrants are grid blocks, nothing in LDS scales with m, n --
// so K17's combined weight-sum operands, e.g. 576 x 192, are one launch)
bool quad_ok(int64_t K, int64_t m, int64_t n, int pro, int64_t lda, int64_t ldb) {
  return pro == 0 && K < kX3MinK && K > 0 && m % 64 == 0 && n % 64 == 0 &&
         m <= 1024 && n <= 1024 && lda % 4 == 0 && ldb % 4 == 0;
}
size_t quad_workspace(int64_t K, int64_t m, int64_t n) {
  return (size_t)quad_splits(K, (m / 64) * (n / 64)) * (size_t)(m * n + m) * sizeof(float);
}
int outer_sum_quad_launch(int64_t K, int64_t m, int64_t n, const float* A, int64_t lda,
                          const float* B, int64_t ldb, float* C, int64_t ldc, float* colsum_A,
                          void* workspace, hipStream_t s) {
  const int64_t quads = (m / 64) * (n / 64);
  const int64_t S = quad_splits(K, quads);
  const int64_t per = ceil_div(ceil_div(K, S), kQK) * kQK;
  const int64_t Sr = ceil_div(K, per);
  const int64_t X = m * n + m;
  float* part = reinterpret_cast<float*>(workspace);
  outer_sum_quad_kernel<<<dim3((unsigned)Sr, (unsigned)quads), kQT, 0, s>>>(A, lda, B, ldb, K,
                                                                           (int)m, (int)n, per,
                                                                           part, X);
  int rc = launch_status();
  if (rc) return rc;
  sum_partials(part, Sr, X, C, colsum_A, m * n, n, ldc, s);
  return launch_status();
}

// capacity bucket for (M, N): returns 0 if unsupported
// Tile bucket of an M x N problem: the smallest compiled (MR, MC) covering the per-wave tile
// counts (the MFMA stream is branch-free, so oversized buckets cost real MFMAs), and the
// per-thread load count NL in {5, 7, 9}.  Returns MR * 100 + MC * 10 + NL / 2, or 0.
int rect_bucket(int64_t m, int64_t n) {
  const int64_t TM = m / 16, TN = n / 16;
  int64_t RT, CT;
  if (TM >= 4) { RT = (TM + 3) / 4; CT = TN; }
  else { RT = TM; CT = (TN + 3) / 4; }
  const int64_t loads = ceil_div((m + n) / 4 * kKT, kT);
  if (loads > kMaxL) return 0;
  const int nl = loads <= 5 ? 5 : (loads <= 7 ? 7 : 9);
  static const int kMR[] = {1, 1, 1, 2, 2, 2, 2, 2, 3, 3, 3, 4};
  static const int kMC[] = {1, 2, 3, 1, 2, 3, 5, 9, 1, 2, 3, 4};
  for (int b = 0; b < 12; ++b)
    if (RT <= kMR[b] && CT <= kMC[b]) return kMR[b] * 100 + kMC[b] * 10 + nl / 2;
  return 0;
}

// out[c] = sum_e sum_x A[e, 3c + x] v[e, x] for A (E, 3C) contiguous, v (E, 3): the xyz
// contractions of per-edge vector gradients with the edge vectors in the GVP first-message
// weight sums (u = sum dvpre . ev, dwev = sum dvh . ev).  A workgroup streams tiles of kXdRows
// whole rows as float4s (kXdRows x W3 / 4 / kXdT float4 per thread): the (thread, slot) ->
// column map is the same in every tile, so each thread accumulates fixed columns in registers;
// the tile rows are then added per column in row order through LDS, the three x of a column
// group in order: one partial row of C floats per workgroup (deterministic), summed by
// sum_partials.
constexpr int kXdT = 256, kXdRows = 64;
template <int W3>
__global__ __launch_bounds__(kXdT) void xyz_dot_kernel(const float* __restrict__ A,
                                                       const float* __restrict__ v, int64_t E,
                                                       int64_t per, float* __restrict__ part) {
  constexpr int U = kXdRows * W3 / 4 / kXdT;  // float4 per thread per tile
  static_assert(kXdRows * W3 % (4 * kXdT) == 0, "tile must split into whole float4 per thread");
  __shared__ float sT[kXdRows][W3];
  const int t = threadIdx.x;
  f32x4 acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t k0 = (int64_t)blockIdx.x * per;
  const int64_t k1 = (k0 + per < E) ? k0 + per : E;
  for (int64_t r0 = k0; r0 < k1; r0 += kXdRows) {
    f32x4 a[U];
    float w[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = t + kXdT * u, row = 4 * f / W3, col = 4 * f - row * W3;
      const int64_t e = r0 + row;
      const bool ok = e < k1;
      a[u] = ok ? *reinterpret_cast<const f32x4*>(A + e * W3 + col) : f32x4{0.f, 0.f, 0.f, 0.f};
      const int64_t ec = ok ? e : k0;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[u][i] = v[3 * ec + (col + i) % 3];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[u][i] += a[u][i] * w[u][i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int f = t + kXdT * u, row = 4 * f / W3, col = 4 * f - row * W3;
#pragma unroll
    for (int i = 0; i < 4; ++i) sT[row][col + i] = acc[u][i];
  }
  __syncthreads();
  if (t < W3 / 3) {
    float s = 0.f;
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      float c = 0.f;
      for (int r = 0; r < kXdRows; ++r) c += sT[r][3 * t + x];
      s += c;
    }
    part[(int64_t)blockIdx.x * (W3 / 3) + t] = s;
  }
}

int64_t blocks_for(int64_t K) {
  int64_t g = (int64_t)device_cu_count() * 2;  // two resident workgroups per CU
  // >= 16 edge tiles per workgroup: a node-level sum (K = 50k rows) then takes ~100 CUs and
  // writes ~100 partial slabs instead of 391 (r03 trace: the 391-slab form and its reduction
  // held the side stream 3.3 ms per EGNN step, beside the critical path's kernels)
  const int64_t min_per = kMinTiles * kKT;
  if (g * min_per > K) g = ceil_div(K, min_per);
  return g < 1 ? 1 : g;
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_wgrad_set_f32_mfma(int on) {
  const int prev = wgrad_f32_mfma() ? 1 : 0;
  g_wgrad_mode = on ? 1 : 0;
  return prev;
}

size_t gmp_edge_outer_sum_workspace_size(int64_t K, int64_t d) {
  const int64_t G = blocks_for(K);
  const size_t ws = (size_t)(G + ceil_div(G, kGC)) * (size_t)(d * d + d) * sizeof(float);
  const size_t wq = quad_ok(K, d, d, 0, d, d) ? quad_workspace(K, d, d) : 0;
  return ws > wq ? ws : wq;
}

static int outer_sum_launch(int64_t K, int64_t d, const float* A, int64_t lda, const float* B,
                            int64_t ldb, int pro, const float* bw, const float* bb, float* C,
                            int64_t ldc, float* colsum_A, void* workspace, size_t workspace_bytes,
                            void* stream) {
  if (!(d == 32 || d == 64 || d == 128)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(K >= 0 && C && pro >= 0 && pro <= 2 && (pro == 0 || (bw && bb)));
  GMP_CHECK_ARG(lda >= d && ldb >= d && ldc >= d && lda % 4 == 0 && ldb % 4 == 0);
  hipStream_t s = as_stream(stream);
  if (K == 0) {
    int rc = hip_check(hipMemset2DAsync(C, ldc * sizeof(float), 0, d * sizeof(float), d, s));
    if (!rc && colsum_A) rc = hip_check(hipMemsetAsync(colsum_A, 0, d * sizeof(float), s));
    return rc;
  }
  GMP_CHECK_ARG(A && B && workspace);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(A) % 16 == 0 && reinterpret_cast<uintptr_t>(B) % 16 == 0);
  GMP_CHECK_ARG(pro == 0 || (reinterpret_cast<uintptr_t>(bw) % 16 == 0 &&
                             reinterpret_cast<uintptr_t>(bb) % 16 == 0));
  if (workspace_bytes < gmp_edge_outer_sum_workspace_size(K, d)) return GMP_ERR_WORKSPACE;
  if (!wgrad_f32_mfma()) {
    const int rc = outer_sum_x3_launch(K, d, d, A, lda, B, ldb, pro, bw, bb, C, ldc, colsum_A,
                                       workspace, s);
    if (rc != GMP_ERR_UNSUPPORTED) return rc;
  }
  if (quad_ok(K, d, d, pro, lda, ldb) && d >= 64 &&
      reinterpret_cast<uintptr_t>(A) % 16 == 0 && reinterpret_cast<uintptr_t>(B) % 16 == 0)
    return outer_sum_quad_launch(K, d, d, A, lda, B, ldb, C, ldc, colsum_A, workspace, s);
  const int64_t G = blocks_for(K);
  const int64_t per = ceil_div(ceil_div(K, G), kKT) * kKT;
  const int64_t Gr = ceil_div(K, per);
  float* part = reinterpret_cast<float*>(workspace);
#define LAUNCH_OS(DD, PP) \
  outer_sum_kernel<DD, PP><<<(unsigned)Gr, kT, 0, s>>>(A, B, K, lda, ldb, per, part, bw, bb)
#define LAUNCH_OS_D(PP)                 \
  if (d == 128) LAUNCH_OS(128, PP);     \
  else if (d == 64) LAUNCH_OS(64, PP);  \
  else LAUNCH_OS(32, PP)
  if (pro == 0) { LAUNCH_OS_D(0); }
  else if (pro == 1) { LAUNCH_OS_D(1); }
  else { LAUNCH_OS_D(2); }
#undef LAUNCH_OS_D
#undef LAUNCH_OS
  int rc = launch_status();
  if (rc) return rc;
  const int64_t X = d * d + d;
  sum_partials(part, Gr, X, C, colsum_A, d * d, d, ldc, s);
  return launch_status();
}

int gmp_edge_outer_sum_f32(int64_t K, int64_t d, const float* A, const float* B, float* C,
                           float* colsum_A, void* workspace, size_t workspace_bytes,
                           void* stream) {
  return outer_sum_launch(K, d, A, d, B, d, 0, nullptr, nullptr, C, d, colsum_A, workspace,
                          workspace_bytes, stream);
}

int gmp_edge_outer_sum_act_f32(int64_t K, int64_t d, const float* A, const float* X,
                               const float* w, const float* b, int act, float* C,
                               float* colsum_A, void* workspace, size_t workspace_bytes,
                               void* stream) {
  if (!(act == 0 || act == 1)) return GMP_ERR_ARG;
  return outer_sum_launch(K, d, A, d, X, d, act + 1, w, b, C, d, colsum_A, workspace,
                          workspace_bytes, stream);
}

int gmp_edge_outer_sum_act_hf_f32(int64_t K, int64_t d, const float* A, const float* X,
                                  const float* w, const float* b, int act, const uint32_t* amax_A,
                                  float* C, float* colsum_A, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  if (!(act == 0 || act == 1)) return GMP_ERR_ARG;
  GMP_CHECK_ARG(amax_A && w && b && C && K >= 0);
  if (!(d == 32 || d == 64 || d == 128)) return GMP_ERR_UNSUPPORTED;
  if (workspace_bytes < gmp_edge_outer_sum_workspace_size(K, d)) return GMP_ERR_WORKSPACE;
  hipStream_t s = as_stream(stream);
  if (K > 0) {
    GMP_CHECK_ARG(A && X && workspace);
    GMP_CHECK_ARG(((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(X) |
                    reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(b)) % 16) == 0);
    if (!wgrad_f32_mfma()) {
      const int rc = outer_sum_x3_launch(K, d, d, A, d, X, d, act + 1, w, b, C, d, colsum_A,
                                         workspace, s, nullptr, 0, -1, amax_A);
      if (rc != GMP_ERR_UNSUPPORTED) return rc;
    }
  }
  return outer_sum_launch(K, d, A, d, X, d, act + 1, w, b, C, d, colsum_A, workspace,
                          workspace_bytes, stream);
}

int64_t rect_blocks_for(int64_t K) {
  int64_t g = (int64_t)device_cu_count() * 2;
  const int64_t min_per = kMinTiles * kKT;  // as blocks_for
  if (g * min_per > K) g = ceil_div(K, min_per);
  return g < 1 ? 1 : g;
}

size_t gmp_edge_outer_sum_rect_workspace_size(int64_t K, int64_t m, int64_t n) {
  const int64_t G = rect_blocks_for(K);
  const size_t ws = (size_t)(G + ceil_div(G, kGC)) * (size_t)(m * n + m) * sizeof(float);
  const size_t wq = quad_ok(K, m, n, 0, m, n) ? quad_workspace(K, m, n) : 0;
  return ws > wq ? ws : wq;
}

static int outer_sum_rect_launch(int64_t K, int64_t m, int64_t n, const float* A, int64_t lda,
                                 const float* B, int64_t ldb, float* C, int64_t ldc,
                                 float* colsum_A, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  GMP_CHECK_ARG(K >= 0 && C && m > 0 && n > 0 && m % 16 == 0 && n % 16 == 0);
  GMP_CHECK_ARG(lda >= m && ldb >= n && ldc >= n && lda % 4 == 0 && ldb % 4 == 0);
  GMP_CHECK_ARG(m <= kT || quad_ok(K, m, n, 0, lda, ldb));
  const int bucket = m <= kT ? rect_bucket(m, n) : 0;
  if (!bucket && !quad_ok(K, m, n, 0, lda, ldb)) return GMP_ERR_UNSUPPORTED;
  hipStream_t s = as_stream(stream);
  if (K == 0) {
    int rc = hip_check(hipMemset2DAsync(C, ldc * sizeof(float), 0, n * sizeof(float), m, s));
    if (!rc && colsum_A) rc = hip_check(hipMemsetAsync(colsum_A, 0, m * sizeof(float), s));
    return rc;
  }
  GMP_CHECK_ARG(A && B && workspace);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(A) % 16 == 0 && reinterpret_cast<uintptr_t>(B) % 16 == 0);
  if (workspace_bytes < gmp_edge_outer_sum_rect_workspace_size(K, m, n)) return GMP_ERR_WORKSPACE;
  if (!wgrad_f32_mfma()) {
    const int rc2 = outer_sum_x3_launch(K, m, n, A, lda, B, ldb, 0, nullptr, nullptr, C, ldc,
                                        colsum_A, workspace, s);
    if (rc2 != GMP_ERR_UNSUPPORTED) return rc2;
  }
  if (quad_ok(K, m, n, 0, lda, ldb))
    return outer_sum_quad_launch(K, m, n, A, lda, B, ldb, C, ldc, colsum_A, workspace, s);
  if (!bucket) return GMP_ERR_UNSUPPORTED;
  const int64_t G = rect_blocks_for(K);
  const int64_t per = ceil_div(ceil_div(K, G), kKT) * kKT;
  const int64_t Gr = ceil_div(K, per);
  float* part = reinterpret_cast<float*>(workspace);
  const size_t smem = (size_t)2 * kKT * (rect_ld((int)m) + rect_ld((int)n)) * sizeof(float);
  int rc;
#define LAUNCH_RECT(MR, MC, NL, OCC)                                                             \
  {                                                                                           \
    auto k = outer_sum_rect_kernel<MR, MC, NL, OCC>;                                          \
    if ((rc = hip_check(hipFuncSetAttribute((const void*)k,                                   \
                                            hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                            (int)smem))))                                     \
      return rc;                                                                              \
    k<<<(unsigned)Gr, kT, smem, s>>>(A, B, K, (int)m, (int)n, lda, ldb, per, part);           \
  }
#define LAUNCH_RECT_NL(MR, MC)                                   \
  case MR * 100 + MC * 10 + 2: LAUNCH_RECT(MR, MC, 5, 2) break;  \
  case MR * 100 + MC * 10 + 3: LAUNCH_RECT(MR, MC, 7, 2) break;  \
  case MR * 100 + MC * 10 + 4: LAUNCH_RECT(MR, MC, 9, 2) break;
// the widest buckets need > 256 VGPRs at 7-9 loads per thread: one workgroup per CU (the
// compiler then has the AGPRs as well; at two per CU they spilled 40-152 B/lane to scratch)
#define LAUNCH_RECT_NL_WIDE(MR, MC)                              \
  case MR * 100 + MC * 10 + 2: LAUNCH_RECT(MR, MC, 5, 2) break;  \
  case MR * 100 + MC * 10 + 3: LAUNCH_RECT(MR, MC, 7, 1) break;  \
  case MR * 100 + MC * 10 + 4: LAUNCH_RECT(MR, MC, 9, 1) break;
  switch (bucket) {
    LAUNCH_RECT_NL(1, 1) LAUNCH_RECT_NL(1, 2) LAUNCH_RECT_NL(1, 3)
    LAUNCH_RECT_NL(2, 1) LAUNCH_RECT_NL(2, 2) LAUNCH_RECT_NL(2, 3) LAUNCH_RECT_NL(2, 5) LAUNCH_RECT_NL_WIDE(2, 9)
    LAUNCH_RECT_NL(3, 1) LAUNCH_RECT_NL(3, 2) LAUNCH_RECT_NL(3, 3)
    LAUNCH_RECT_NL_WIDE(4, 4)
    default: return GMP_ERR_UNSUPPORTED;
  }
#undef LAUNCH_RECT_NL_WIDE
#undef LAUNCH_RECT_NL
#undef LAUNCH_RECT
  rc = launch_status();
  if (rc) return rc;
  const int64_t X = m * n + m;
  sum_partials(part, Gr, X, C, colsum_A, m * n, n, ldc, s);
  return launch_status();
}

int gmp_edge_outer_sum_rect_f32(int64_t K, int64_t m, int64_t n, const float* A, const float* B,
                                float* C, float* colsum_A, void* workspace,
                                size_t workspace_bytes, void* stream) {
  return outer_sum_rect_launch(K, m, n, A, m, B, n, C, n, colsum_A, workspace, workspace_bytes,
                               stream);
}

size_t gmp_edge_outer_sum_ex_workspace_size(int64_t K, int64_t m, int64_t n) {
  if (m == n && (m == 32 || m == 64 || m == 128)) return gmp_edge_outer_sum_workspace_size(K, m);
  return gmp_edge_outer_sum_rect_workspace_size(K, m, n);
}

int gmp_edge_outer_sum_ex2_f32(int64_t K, int64_t m, int64_t n1, int64_t n2, const float* A,
                               int64_t lda, const float* B1, int64_t ldb1, const float* B2,
                               int64_t ldb2, float* C, int64_t ldc, float* colsum_A,
                               void* workspace, size_t workspace_bytes, void* stream) {
  const int64_t n = n1 + n2;
  GMP_CHECK_ARG(K >= 0 && C && m > 0 && n1 > 0 && n2 > 0 && m % 16 == 0 && n1 % 4 == 0 &&
                n2 % 4 == 0 && n % 16 == 0);
  GMP_CHECK_ARG(lda >= m && ldb1 >= n1 && ldb2 >= n2 && ldc >= n && lda % 4 == 0 &&
                ldb1 % 4 == 0 && ldb2 % 4 == 0);
  if (K == 0 || wgrad_f32_mfma()) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(A && B1 && B2 && workspace);
  GMP_CHECK_ARG((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B1) |
                 reinterpret_cast<uintptr_t>(B2)) % 16 == 0);
  if (workspace_bytes < gmp_edge_outer_sum_rect_workspace_size(K, m, n)) return GMP_ERR_WORKSPACE;
  return outer_sum_x3_launch(K, m, n, A, lda, B1, ldb1, 0, nullptr, nullptr, C, ldc, colsum_A,
                             workspace, as_stream(stream), B2, ldb2, n1);
}

int gmp_edge_outer_sum_ex_f32(int64_t K, int64_t m, int64_t n, const float* A, int64_t lda,
                              const float* B, int64_t ldb, int act, const float* w, const float* b,
                              float* C, int64_t ldc, float* colsum_A, void* workspace,
                              size_t workspace_bytes, void* stream) {
  GMP_CHECK_ARG(act >= -1 && act <= 1);
  if (m == n && (m == 32 || m == 64 || m == 128))
    return outer_sum_launch(K, m, A, lda, B, ldb, act + 1, w, b, C, ldc, colsum_A, workspace,
                            workspace_bytes, stream);
  if (act != -1) return GMP_ERR_UNSUPPORTED;  // activation prologue: square shapes only
  return outer_sum_rect_launch(K, m, n, A, lda, B, ldb, C, ldc, colsum_A, workspace,
                               workspace_bytes, stream);
}


size_t gmp_outer_sum_cols_workspace_size(int64_t K, int64_t m_total, int64_t n) {
  if (m_total <= 0 || n <= 0 || m_total % kColBlk) return 0;
  const int64_t Y = m_total / kColBlk;
  // partial slabs, then (pre-split path) G's three bf16 planes with k padded to 32
  return (size_t)(Y * cols_groups(K, Y) * (kColBlk * n + kColBlk)) * sizeof(float) +
         (size_t)3 * n * ceil_div(K, kXK) * kXK * sizeof(unsigned short) + 16;
}

int gmp_outer_sum_cols_f32(int64_t K, int64_t m_total, int64_t n, const float* A, int64_t lda,
                           const float* B, int64_t ldb, float* C, int64_t ldc, void* workspace,
                           size_t workspace_bytes, void* stream) {
  GMP_CHECK_ARG(K >= 0 && m_total > 0 && m_total % kColBlk == 0 && n > 0 && n % 16 == 0);
  GMP_CHECK_ARG(lda >= m_total && ldb >= n && ldc >= n && lda % 4 == 0 && ldb % 4 == 0);
  GMP_CHECK_ARG(A && B && C);
  GMP_CHECK_ARG((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) % 16 == 0);
  const int64_t m = kColBlk, R = m + n;
  int wn = 0;
  const int shape = x3_pick(m, n, &wn);
  const int64_t units = ((2 * m + 63) & ~63) + ((2 * n + 63) & ~63);
  if (shape < 0 || shape > 2 || R + kXPad > 416 || units > kXT) return GMP_ERR_UNSUPPORTED;
  const int64_t Y = m_total / kColBlk;
  GMP_CHECK_ARG(Y < 65536);
  hipStream_t s = as_stream(stream);
  if (K == 0) {
    for (int64_t r = 0; r < m_total; ++r) {
      int rc = hip_check(hipMemsetAsync(C + r * ldc, 0, n * sizeof(float), s));
      if (rc) return rc;
    }
    return GMP_OK;
  }
  GMP_CHECK_ARG(workspace);
  if (workspace_bytes < gmp_outer_sum_cols_workspace_size(K, m_total, n)) return GMP_ERR_WORKSPACE;
  const int64_t G = cols_groups(K, Y);
  const int64_t per = ceil_div(ceil_div(K, G), kXK) * kXK;
  const int64_t Gr = ceil_div(K, per);
  float* part = reinterpret_cast<float*>(workspace);
  if ((n == 64 || n == 128) && ldb == n) {
    const int64_t X = m * n + m;
    const int64_t nks = ceil_div(K, kXK);
    unsigned short* planes = reinterpret_cast<unsigned short*>(
        reinterpret_cast<unsigned char*>(workspace) +
        ((Y * Gr * X * sizeof(float) + 15) & ~(size_t)15));
    split_g_kernel<<<(unsigned)ceil_div(nks * (n / 16), 4), 256, 0, s>>>(B, K, nks, (int)n,
                                                                          planes);
    int rc = launch_status();
    if (rc) return rc;
    if (n == 128)
      outer_cols_x3g_kernel<2, 3, 1><<<dim3((unsigned)Gr, (unsigned)Y), kXT, 0, s>>>(
          A, K, lda, planes, (int)n, per, X, part);
    else
      outer_cols_x3g_kernel<1, 3, 2><<<dim3((unsigned)Gr, (unsigned)Y), kXT, 0, s>>>(
          A, K, lda, planes, (int)n, per, X, part);
    rc = launch_status();
    if (rc) return rc;
    sum_partials_cols<<<dim3((unsigned)ceil_div(m * n, 256), (unsigned)Y), 256, 0, s>>>(
        part, Gr, X, (int)m, (int)n, C, ldc);
    return launch_status();
  }
  const size_t smem = (size_t)2 * 3 * (R + kXPad) * 64;
  auto k = shape == 2   ? outer_sum_x3_kernel<2, 4, 0, 1>
           : shape == 1 ? outer_sum_x3_kernel<2, 2, 0, 1>
                        : outer_sum_x3_kernel<1, 2, 0, 1>;
  int rc = hip_check(hipFuncSetAttribute((const void*)k,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  if (rc) return rc;
  k<<<dim3((unsigned)Gr, (unsigned)Y), kXT, smem, s>>>(A, B, K, (int)m, (int)n, lda, ldb, per,
                                                      part, nullptr, nullptr, wn, nullptr, 0,
                                                      (int)n, m, nullptr);
  rc = launch_status();
  if (rc) return rc;
  const int64_t X = m * n + m;
  sum_partials_cols<<<dim3((unsigned)ceil_div(m * n, 256), (unsigned)Y), 256, 0, s>>>(
      part, Gr, X, (int)m, (int)n, C, ldc);
  return launch_status();
}

size_t gmp_edge_xyz_dot_workspace_size(int64_t K) {
  return (size_t)(2 * device_cu_count()) * 48 * sizeof(float);
}

int gmp_edge_xyz_dot_f32(int64_t K, int64_t C, const float* A, const float* v, float* out,
                         void* workspace, size_t workspace_bytes, void* stream) {
  GMP_CHECK_ARG(K >= 0 && out);
  if (!(C == 16 || C == 48)) return GMP_ERR_UNSUPPORTED;
  hipStream_t s = as_stream(stream);
  if (K == 0) return hip_check(hipMemsetAsync(out, 0, C * sizeof(float), s));
  GMP_CHECK_ARG(A && v && workspace);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(A) % 16 == 0);
  if (workspace_bytes < gmp_edge_xyz_dot_workspace_size(K)) return GMP_ERR_WORKSPACE;
  int64_t G = 2 * (int64_t)device_cu_count();
  const int64_t per = ceil_div(ceil_div(K, G), (int64_t)kXdRows) * kXdRows;
  G = ceil_div(K, per);
  float* part = reinterpret_cast<float*>(workspace);
  if (C == 48)
    xyz_dot_kernel<144><<<(unsigned)G, kXdT, 0, s>>>(A, v, K, per, part);
  else
    xyz_dot_kernel<48><<<(unsigned)G, kXdT, 0, s>>>(A, v, K, per, part);
  int rc = launch_status();
  if (rc) return rc;
  sum_partials(part, G, C, out, nullptr, C, C, C, s);
  return launch_status();
}

}  // extern "C"
