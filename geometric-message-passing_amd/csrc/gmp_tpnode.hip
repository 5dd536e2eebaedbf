// K7 receiver-factorised form, per-receiver MFMA kernels (see gmp_tp.hip "node form"):
//
//   outer:  S[n, r, j] = sum_{e -> n} Z[e, r] A[e, j],   Sb[n, r] = sum_{e -> n} Z[e, r]
//   apply:  dZ[e, r] = sum_j T[n, r, j] A[e, j] + Tb[n, r],   dA[e, j] += sum_r Z[e, r] T[n, r, j]
//
// for the receiver chunk's edges (receiver-sorted, chunk-local offsets eoff[n] .. eoff[n+1]),
// with Z = z rows of one path (w = (2lo+1) mul1 columns), A = hidden radial features a_e (H
// columns, H % 16 == 0), T = G [W2_p]^T and Tb = G b2_p^T from the path GEMMs.  Replaces the
// degree-padded batched GEMMs (K = max in-degree, output-bound) by MFMA tiles with the edge index
// as the k dimension; every receiver's sums are formed inside one workgroup in edge order
// (deterministic).  f32 MFMA 16x16x4: lane l supplies A[i = l&15][k = l>>4] and B[k = l>>4][j =
// l&15]; D[row = 4(l>>4) + q][col = l&15].
#include <cstring>
#include <type_traits>

#include "gmp_common.h"

namespace gmp {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kNT = 256;          // 4 waves
constexpr int kRowsPerBlock = 64; // outer: rows (r) per workgroup (one 16-row tile per wave)
constexpr int kEdgeStage = 32;    // outer: edges staged per LDS pass (in-degree ~20: one pass)
constexpr int kMaxH = 256;

// ---------------------------------------------------------------------------------- outer
// grid (ceil(w / (64 kOuterRB)), receivers): the workgroup stages the receiver's hidden radial
// rows a_e once and produces up to kOuterRB 64-row blocks of S from them (one workgroup per
// receiver for kOuterRB >= w / 64; measured slower than one 64-row block per workgroup: 10.1
// vs 9.1 ms for the 32.8 GB MACE-128 lo = 2 path -- fewer workgroups in flight per CU)
constexpr int kOuterRB = 1;
// RMAX: each wave's max |S|, |Sb| over its 16 rows r0 .. r0 + 15 (all H columns) into
// rmax[n (w / 16) + r0 / 16] (w % 16 == 0), no atomics: with mul1 % 16 == 0 the path GEMM's A
// row (n, k) (columns (u, j) ++ u) owns the mul1 / 16 consecutive words from (n d3 + k) mul1 / 16
// -- the per-row scales of its H2 form (gmp_tp_gemm_h2_f32)
__device__ __forceinline__ void rmax_commit(float* rmax, int64_t n, int w, int r0, float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  if ((threadIdx.x & 63) == 0 && r0 < w) rmax[n * (w >> 4) + (r0 >> 4)] = v;
}

// CS: the workgroup covers H / CS of the columns (grid.x = row blocks x CS, column part fastest):
// CS = 2 halves the staged a rows (18 KB of LDS: 8 workgroups per CU instead of 4) at the cost
// of loading each Z column twice (Z is ~1/H of the S bytes).
// STG: the common branch's S rows leave through LDS (after the MFMAs, sA is free): per 64-column
// chunk each wave parks its 16 x 64 tile and stores it back as whole 256-byte row segments (four
// rows per store instruction) instead of sixteen 64-byte pieces per instruction.
template <bool RMAX, bool STG, int CS>
__global__ __launch_bounds__(kNT, CS == 2 ? 5 : 1) void tp_node_outer_kernel(int w, int H,
                                                            const int64_t* __restrict__ eoff,
                                                            const float* __restrict__ Z,
                                                            const float* __restrict__ A,
                                                            float* __restrict__ S,
                                                            float* __restrict__ Sb,
                                                            float* __restrict__ rmax) {
  static_assert(!RMAX || CS == 1, "row maxima need every column of the row block");
  constexpr int kMaxT = kMaxH / 16 / CS;  // 16-column tiles per workgroup (max)
  __shared__ __attribute__((aligned(16))) float sA[kEdgeStage * (kMaxH / CS + 16)];
  const int n = blockIdx.y;
  const int hc = H / CS, c0 = (CS == 1 ? 0 : (int)(blockIdx.x % CS)) * hc;
  const int LDA = hc + 16;  // 16 mod 64 floats: the 4 edge rows of an MFMA read hit disjoint banks
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, i = lane & 15, kk = lane >> 4;
  const int64_t e0 = eoff[n], deg = eoff[n + 1] - e0;
  // CS = 2 runs at H = kMaxH only, with the tile count a constant (a runtime bound on the
  // predicated MFMAs made the compiler shuffle accumulators through thousands of moves)
  const int TJ = CS > 1 ? kMaxT : hc >> 4;
  const bool sb_out = c0 == 0;  // one column part writes Sb
  float* Sn = S + (int64_t)n * w * H + c0;
  const float* Ac = A + c0;
  const int rb0 = (int)(blockIdx.x / CS) * kOuterRB;
  const int rb1 = min(rb0 + kOuterRB, (w + kRowsPerBlock - 1) / kRowsPerBlock);
  if (deg <= kEdgeStage) {
    // common case (one edge stage): this lane's Z column values for every k step of the next
    // row block are loaded while the current block's MFMAs run (register double buffer), the a
    // rows are staged once; no dependent global load inside the MFMA loop
    const int ns = (int)deg, nst = (ns + 3) >> 2;
    float zr[2][kEdgeStage / 4];
    auto zload = [&](int buf, int rb) {  // (the guarded loads issue back to back: one wait)
      const int r = rb * kRowsPerBlock + wv * 16 + i;
#pragma unroll
      for (int s = 0; s < kEdgeStage / 4; ++s) {
        const int el = 4 * s + kk;
        zr[buf][s] = (el < ns && r < w) ? Z[(e0 + el) * w + r] : 0.f;
      }
    };
    zload(0, rb0);
    // The a rows are staged with every load issued (at a clamped, valid row) before any is
    // used, then masked: one memory round trip.  r05's staging loop (`if (e < ns) v = ..; sA =
    // v` per iteration) waited vmcnt(0) in every iteration: up to 4 dependent round trips per
    // workgroup.  (A has no pad row: a receiver without edges skips the loads.)
    constexpr int kSI = (kEdgeStage * (kMaxH / CS) / 4 + kNT - 1) / kNT;  // float4s per thread
    const int q4 = hc >> 2, cnt = 4 * nst * q4;                            // (padding rows zeroed)
    if (ns > 0) {
      f32x4 av[kSI];
#pragma unroll
      for (int it = 0; it < kSI; ++it) {
        const int x = tid + it * kNT, e = x / q4, q = x - e * q4;
        const int ec = e < ns ? e : ns - 1;
        av[it] = *reinterpret_cast<const f32x4*>(Ac + (e0 + ec) * H + 4 * q);
      }
#pragma unroll
      for (int it = 0; it < kSI; ++it) {
        const int x = tid + it * kNT, e = x / q4, q = x - e * q4;
        if (x < cnt)
          *reinterpret_cast<f32x4*>(&sA[e * LDA + 4 * q]) =
              e < ns ? av[it] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    __syncthreads();
    for (int rb = rb0; rb < rb1; ++rb) {
      const int cur = (rb - rb0) & 1;
      if (rb + 1 < rb1) zload(cur ^ 1, rb + 1);
      const int r = rb * kRowsPerBlock + wv * 16 + i;
      float lmax = 0.f;
      f32x4 acc[kMaxT];
#pragma unroll
      for (int t = 0; t < kMaxT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      float zsum = 0.f;
#pragma unroll
      for (int s = 0; s < kEdgeStage / 4; ++s) {
        if (s < nst) {
          const int el = 4 * s + kk;
          const float zv = zr[cur][s];
          zsum += zv;
#pragma unroll
          for (int t = 0; t < kMaxT; ++t)
            if (t < TJ) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(sA[el * LDA + 16 * t + i], zv, acc[t], 0, 0, 0);
          // keep the LDS operand reads inside their k step (hoisted, the narrow CS = 2 form
          // held all of them at once: 246 VGPRs, one wave per SIMD)
          if constexpr (CS > 1) asm volatile("" ::: "memory");
        }
      }
      if (RMAX && r < w) {
#pragma unroll
        for (int t = 0; t < kMaxT; ++t)
          if (t < TJ)
            lmax = fmaxf(lmax, fmaxf(fmaxf(fabsf(acc[t][0]), fabsf(acc[t][1])),
                                     fmaxf(fabsf(acc[t][2]), fabsf(acc[t][3]))));
      }
      if constexpr (STG) {
        static_assert(kOuterRB == 1, "the parked tiles overwrite the staged a rows");
        constexpr int LDW = 68;  // 64 + 4 floats: the 16 rows of a parked tile spread banks
        static_assert(4 * 16 * LDW <= kEdgeStage * (kMaxH / CS + 16), "park fits in sA");
        float* park = sA + wv * 16 * LDW;
        const int r0 = rb * kRowsPerBlock + wv * 16;
#pragma unroll
        for (int h = 0; h < (kMaxT + 3) / 4; ++h) {
          if (4 * h >= TJ) break;  // uniform
          __syncthreads();  // every wave is done with sA (MFMA operands / previous chunk)
#pragma unroll
          for (int t = 4 * h; t < 4 * h + 4; ++t)
            if (t < TJ)
              *reinterpret_cast<f32x4*>(park + i * LDW + 16 * (t - 4 * h) + 4 * kk) = acc[t];
          __syncthreads();
          const int cols = 16 * (min(TJ, 4 * h + 4) - 4 * h);  // this chunk's columns (<= 64)
#pragma unroll
          for (int it = 0; it < 4; ++it) {
            const int idx = it * 64 + lane, row = idx >> 4, c4 = 4 * (idx & 15);
            if (c4 < cols && r0 + row < w)
              *reinterpret_cast<f32x4*>(Sn + (int64_t)(r0 + row) * H + 64 * h + c4) =
                  *reinterpret_cast<const f32x4*>(park + row * LDW + c4);
          }
        }
      } else if (r < w) {
#pragma unroll
        for (int t = 0; t < kMaxT; ++t)
          if (t < TJ) *reinterpret_cast<f32x4*>(Sn + (int64_t)r * H + 16 * t + 4 * kk) = acc[t];
      }
      zsum += __shfl_xor(zsum, 16);
      zsum += __shfl_xor(zsum, 32);
      if (kk == 0 && r < w && sb_out) Sb[(int64_t)n * w + r] = zsum;
      if (RMAX) {
        if (r < w) lmax = fmaxf(lmax, fabsf(zsum));
        rmax_commit(rmax, n, w, rb * kRowsPerBlock + wv * 16, lmax);
      }
    }
    return;
  }
  for (int rb = rb0; rb < rb1; ++rb) {
    // D = S^T tile: D[j][r] = sum_e A[e, j] Z[e, r]  (A op = a columns, B op = Z columns), so a
    // lane holds 4 consecutive j of one row r and stores them as one float4
    const int r = rb * kRowsPerBlock + wv * 16 + i;  // this lane's output row
    float lmax = 0.f;
    f32x4 acc[kMaxT];
#pragma unroll
    for (int t = 0; t < kMaxT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float zsum = 0.f;  // Sb[n, r]: this lane's edges (k phase kk) of the Z column
    for (int64_t eb = 0; eb < deg; eb += kEdgeStage) {
      const int ns = (int)((deg - eb) < kEdgeStage ? (deg - eb) : kEdgeStage);
      const int ns4 = (ns + 3) & ~3;
      __syncthreads();
      for (int x = tid; x < ns4 * (hc >> 2); x += kNT) {  // padding rows zeroed
        const int e = x / (hc >> 2), q = x - e * (hc >> 2);
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (e < ns) v = *reinterpret_cast<const f32x4*>(Ac + (e0 + eb + e) * H + 4 * q);
        *reinterpret_cast<f32x4*>(&sA[e * LDA + 4 * q]) = v;
      }
      __syncthreads();
      for (int s = 0; s < (ns4 >> 2); ++s) {
        const int el = 4 * s + kk;
        const float zv = (el < ns && r < w) ? Z[(e0 + eb + el) * w + r] : 0.f;
        zsum += zv;
#pragma unroll
        for (int t = 0; t < kMaxT; ++t)
          if (t < TJ) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(sA[el * LDA + 16 * t + i], zv, acc[t], 0, 0, 0);
      }
    }
    if (r < w) {
#pragma unroll
      for (int t = 0; t < kMaxT; ++t)
        if (t < TJ) {
          *reinterpret_cast<f32x4*>(Sn + (int64_t)r * H + 16 * t + 4 * kk) = acc[t];
          if (RMAX)
            lmax = fmaxf(lmax, fmaxf(fmaxf(fabsf(acc[t][0]), fabsf(acc[t][1])),
                                     fmaxf(fabsf(acc[t][2]), fabsf(acc[t][3]))));
        }
    }
    zsum += __shfl_xor(zsum, 16);
    zsum += __shfl_xor(zsum, 32);
    if (kk == 0 && r < w && sb_out) Sb[(int64_t)n * w + r] = zsum;
    if (RMAX) {
      if (r < w) lmax = fmaxf(lmax, fabsf(zsum));
      rmax_commit(rmax, n, w, rb * kRowsPerBlock + wv * 16, lmax);
    }
  }
}

// ---------------------------------------------------------------------------------- apply
// One workgroup per receiver; edges in groups of 32 (a rows staged in LDS), rows of the path in
// blocks of 32 (T rows staged in LDS, the only large stream: read once).  Per row block:
//   dZ tile (32 rows x 32 edges, K = H) : waves own one (row tile, edge tile) each
//   dA tile (32 edges x H, K = 32 rows) : waves own j tiles {wv, wv+4, wv+8, wv+12} x 2 edge tiles
constexpr int kAR = 32;          // rows per block
constexpr int kAE = 32;          // edges per group
constexpr int kLdT = kMaxH + 4;  // LDS stride for T / A rows
constexpr int kLdZ = kAR + 4;

__global__ __launch_bounds__(kNT, 2) void tp_node_apply_kernel(int w, int H,
                                                               const int64_t* __restrict__ eoff,
                                                               const float* __restrict__ Z,
                                                               const float* __restrict__ A,
                                                               const float* __restrict__ T,
                                                               const float* __restrict__ Tb,
                                                               float* __restrict__ dZ,
                                                               float* __restrict__ dA) {
  __shared__ __attribute__((aligned(16))) float sT[kAR * kLdT];
  __shared__ __attribute__((aligned(16))) float sA[kAE * kLdT];
  __shared__ __attribute__((aligned(16))) float sZ[kAE * kLdZ];
  __shared__ __attribute__((aligned(16))) float sDZ[kAE * kLdZ];  // dZ tile, written row-wise
  const int n = blockIdx.x;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, i = lane & 15, kk = lane >> 4;
  const int64_t e0 = eoff[n], deg = eoff[n + 1] - e0;
  const float* Tn = T + (int64_t)n * w * H;
  const int TJ = H >> 4, H4 = H >> 2;
  const int rt = wv >> 1, et = wv & 1;  // dZ tile of this wave
  for (int64_t g0 = 0; g0 < deg; g0 += kAE) {
    const int ng = (int)((deg - g0) < kAE ? (deg - g0) : kAE);
    __syncthreads();
    for (int x = tid; x < kAE * H4; x += kNT) {
      const int e = x / H4, q = x - e * H4;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (e < ng) v = *reinterpret_cast<const f32x4*>(A + (e0 + g0 + e) * H + 4 * q);
      *reinterpret_cast<f32x4*>(&sA[e * kLdT + 4 * q]) = v;
    }
    f32x4 accA[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a) accA[a][0] = accA[a][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // register-staged prefetch of the next row block (T rows and Z columns) so its HBM latency
    // overlaps the current block's MFMAs
    constexpr int kTL = kAR * (kMaxH / 4) / kNT;   // float4 T loads per thread (8)
    constexpr int kZL = kAE * kAR / kNT;           // Z loads per thread (4)
    f32x4 regT[kTL];
    float regZ[kZL];
    // Tb[n, rb + (tid & 31)]: the one bias row value this thread adds in the dZ store loop
    // (x = tid + kNT q there, so rr = tid & 31), prefetched with the row block instead of a
    // dependent load after the block's last barrier
    float regTb = 0.f;
    static_assert(kNT % kAR == 0, "store-loop row of a thread is tid % kAR");
    auto fetch = [&](int rb) {
      {
        const int rr = tid & (kAR - 1);
        const int nrb0 = (w - rb) < kAR ? (w - rb) : kAR;
        regTb = rr < nrb0 ? Tb[(int64_t)n * w + rb + rr] : 0.f;
      }
      const int nrb = (w - rb) < kAR ? (w - rb) : kAR;
#pragma unroll
      for (int q = 0; q < kTL; ++q) {
        const int x = tid + kNT * q;
        const int rr = x / H4, c4 = x - rr * H4;
        regT[q] = (x < kAR * H4 && rr < nrb)
                      ? *reinterpret_cast<const f32x4*>(Tn + (int64_t)(rb + rr) * H + 4 * c4)
                      : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int q = 0; q < kZL; ++q) {
        const int x = tid + kNT * q;
        const int e = x / kAR, rr = x - e * kAR;
        regZ[q] = (e < ng && rr < nrb) ? Z[(e0 + g0 + e) * w + rb + rr] : 0.f;
      }
    };
    fetch(0);
    for (int r0 = 0; r0 < w; r0 += kAR) {
      const int nr = (w - r0) < kAR ? (w - r0) : kAR;
      __syncthreads();
#pragma unroll
      for (int q = 0; q < kTL; ++q) {
        const int x = tid + kNT * q;
        if (x < kAR * H4) {
          const int rr = x / H4, c4 = x - rr * H4;
          *reinterpret_cast<f32x4*>(&sT[rr * kLdT + 4 * c4]) = regT[q];
        }
      }
#pragma unroll
      for (int q = 0; q < kZL; ++q) {
        const int x = tid + kNT * q;
        const int e = x / kAR, rr = x - e * kAR;
        sZ[e * kLdZ + rr] = regZ[q];
      }
      const float tb_cur = regTb;  // this row block's bias value (regTb is refilled below)
      __syncthreads();
      if (r0 + kAR < w) fetch(r0 + kAR);
      // dZ[e, r] = sum_j T[r, j] a[e, j]   (D[row][e]; A op = T rows, B op = a rows)
      if (16 * rt < nr && 16 * et < ng) {
        // four independent accumulation chains over j (MFMA latency), summed in fixed order
        f32x4 z4[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) z4[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* tr = sT + (16 * rt + i) * kLdT + kk;
        const float* ar = sA + (16 * et + i) * kLdT + kk;
        for (int j0 = 0; j0 < H; j0 += 16) {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            z4[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(tr[j0 + 4 * c], ar[j0 + 4 * c], z4[c],
                                                         0, 0, 0);
        }
        const f32x4 accZ = (z4[0] + z4[1]) + (z4[2] + z4[3]);
        *reinterpret_cast<f32x4*>(&sDZ[(16 * et + i) * kLdZ + 16 * rt + 4 * kk]) = accZ;
      }
      // dA[e, j] += sum_r Z[e, r] T[r, j]   (D[e][j]; A op = Z rows, B op = T columns)
#pragma unroll
      for (int s = 0; s < kAR / 4; ++s) {
        const int rr = 4 * s + kk;
        const float z0 = sZ[i * kLdZ + rr], z1 = sZ[(16 + i) * kLdZ + rr];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const int jt = wv + 4 * a;
          if (jt < TJ) {
            const float tv = sT[rr * kLdT + 16 * jt + i];
            accA[a][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(z0, tv, accA[a][0], 0, 0, 0);
            accA[a][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(z1, tv, accA[a][1], 0, 0, 0);
          }
        }
      }
      __syncthreads();  // sDZ complete: coalesced row-wise store (+ Tb)
      for (int x = tid; x < kAE * kAR; x += kNT) {
        const int e = x / kAR, rr = x - e * kAR;
        if (e < ng && rr < nr)
          dZ[(e0 + g0 + e) * w + r0 + rr] = sDZ[e * kLdZ + rr] + tb_cur;
      }
    }
    // accumulate into dA (per-path launches on one stream: ordered RMW, deterministic)
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int jt = wv + 4 * a;
      if (jt < TJ) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e = 16 * b + 4 * kk + q;
            if (e < ng) dA[(e0 + g0 + e) * H + 16 * jt + i] += accA[a][b][q];
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------- apply v2
// The same contraction on the bf16 MFMA over exact three-plane f32 splits (gmp_tpgemm.hip's
// arithmetic: six plane products, f32 accumulation).  One 512-thread workgroup per receiver edge
// group (<= 32 edges); rows of T in blocks of 32 (one k = 2lo+1 row, 32 consecutive u: a
// contiguous 32 H-float block), split once into an LDS image that serves both products
// (H % 64 == 0: every thread stages whole float4 units of the block):
//   dZ tile D[r][e] = sum_j T[r][j] A[e][j]   (waves 0-3: T row reads, ds_read_b128)
//   dA tile D[e][j] += sum_r Z[e][r] T[r][j]  (waves 4-7: T column reads, ds_read_b64_tr_b16)
// T image: [plane][half (128 j)][32 rows][256 B] with chunk c of row r at c ^ ((r&3)<<2 |
// (r>>2)&3) (the dual row / transposed-read image of the CDNA4 guide).  A_n and Z as [plane][k
// step][32 edges][64 B] (chunk q at q ^ ((row >> 1) & 3)).  T streams through registers two
// blocks ahead (a double-buffered LDS image with one barrier per block measured slower: 19.7
// vs 13.2 ms at the MACE-128 lo = 2 shape, 254 VGPRs); 13.2 ms against 13.75 for the f32-MFMA
// kernel: both wait on the T stream and LDS (2.5-3 TB/s of T).  Requires w % 32 == 0,
// H % 64 == 0, H <= 256.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));

constexpr int kV2T = 512;
constexpr int kV2R = 32;                    // T rows per block
constexpr int kV2E = 32;                    // edges per group
constexpr int kTPlane = 2 * kV2R * 256;     // bytes of one T plane image (two 128-j halves)
constexpr int kSPlane = kV2E * 64;          // bytes of one 32 x 32 bf16 image

__device__ __forceinline__ void split3v(f32x2_t x, unsigned& h, unsigned& m, unsigned& l) {
  const bf16x2_t bh = __builtin_convertvector(x, bf16x2_t);
  const f32x2_t r1 = x - __builtin_convertvector(bh, f32x2_t);
  const bf16x2_t bm = __builtin_convertvector(r1, bf16x2_t);
  const f32x2_t r2 = r1 - __builtin_convertvector(bm, f32x2_t);
  const bf16x2_t bl = __builtin_convertvector(r2, bf16x2_t);
  h = __builtin_bit_cast(unsigned, bh);
  m = __builtin_bit_cast(unsigned, bm);
  l = __builtin_bit_cast(unsigned, bl);
}
__device__ __forceinline__ int toff(int r, int ch) {  // ch: 16-byte chunk 0..31 of a 512-B row
  const int c = ch & 15;
  return (ch >> 4) * (kV2R * 256) + 256 * r + 16 * (c ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}
__device__ __forceinline__ int soff(int row, int chunk) {
  return row * 64 + 16 * (chunk ^ ((row >> 1) & 3));
}
// split an f32x4 and write its three 8-byte plane pieces
__device__ __forceinline__ void put3(unsigned char* base, int plane_bytes, int off, f32x4 v) {
  unsigned h0, m0, l0, h1, m1, l1;
  split3v(f32x2_t{v[0], v[1]}, h0, m0, l0);
  split3v(f32x2_t{v[2], v[3]}, h1, m1, l1);
  *reinterpret_cast<u32x2_t*>(base + off) = u32x2_t{h0, h1};
  *reinterpret_cast<u32x2_t*>(base + plane_bytes + off) = u32x2_t{m0, m1};
  *reinterpret_cast<u32x2_t*>(base + 2 * plane_bytes + off) = u32x2_t{l0, l1};
}
__device__ __forceinline__ f32x4 mma6(const bf16x8_t (&a)[3], const bf16x8_t (&b)[3], f32x4 t) {
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], t, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], t, 0, 0, 0);
}

template <int HS>  // H / 32 k steps (H <= 256)
__global__ __launch_bounds__(kV2T, 1) void tp_node_apply_x3_kernel(
    int w, const int64_t* __restrict__ eoff, const float* __restrict__ Z,
    const float* __restrict__ A, const float* __restrict__ T, const float* __restrict__ Tb,
    float* __restrict__ dZ, float* __restrict__ dA) {
  constexpr int H = 32 * HS, H4 = H / 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm2[];
  unsigned char* sT = sm2;                                // 3 x kTPlane
  unsigned char* sA = sm2 + 3 * kTPlane;                  // 3 x HS x kSPlane
  unsigned char* sZ = sA + 3 * HS * kSPlane;              // 3 x kSPlane
  const int n = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int64_t e0 = eoff[n], deg = eoff[n + 1] - e0;
  const float* Tn = T + (int64_t)n * w * H;
  const int nblk = w / kV2R;
  constexpr int TL = kV2R * H4 / kV2T;  // T float4 units per thread per block (H = 256: 4)
  for (int64_t g0 = 0; g0 < deg; g0 += kV2E) {
    const int ng = (int)((deg - g0) < kV2E ? (deg - g0) : kV2E);
    __syncthreads();  // previous group's readers of sA done
    // A_n rows (edges x H) -> planes [s][e][32 j]
    for (int v = tid; v < kV2E * H4; v += kV2T) {
      const int e = v / H4, c4 = v - e * H4, j = 4 * c4;
      f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
      if (e < ng) x = *reinterpret_cast<const f32x4*>(A + (e0 + g0 + e) * H + j);
      const int sstep = j >> 5, cq = (j & 31) >> 2;
      put3(sA + sstep * kSPlane, HS * kSPlane, soff(e, cq >> 1) + 8 * (cq & 1), x);
    }
    // register ring: T block (TL float4 per thread) and Z block (one float4, threads < 256)
    f32x4 rT[2][TL], rZ[2];
    auto fetch = [&](int slot, int b) {
      const int bc = b < nblk ? b : nblk - 1;
      const float* tb = Tn + (int64_t)bc * kV2R * H;
#pragma unroll
      for (int q = 0; q < TL; ++q)
        rT[slot][q] = *reinterpret_cast<const f32x4*>(tb + 4 * (tid + kV2T * q));
      const int e = (tid >> 3) & 31, c4 = tid & 7;
      const int64_t ee = (e < ng ? e : 0) + e0 + g0;
      rZ[slot] = *reinterpret_cast<const f32x4*>(Z + ee * w + bc * kV2R + 4 * c4);
    };
    auto stash = [&](int slot) {
#pragma unroll
      for (int q = 0; q < TL; ++q) {
        const int v = tid + kV2T * q;
        const int r = v / H4, c4 = v - r * H4;
        put3(sT, kTPlane, toff(r, c4 >> 1) + 8 * (c4 & 1), rT[slot][q]);
      }
      if (tid < 256) {
        const int e = tid >> 3, c4 = tid & 7;
        f32x4 x = rZ[slot];
        if (e >= ng) x = f32x4{0.f, 0.f, 0.f, 0.f};
        put3(sZ, kSPlane, soff(e, c4 >> 1) + 8 * (c4 & 1), x);
      }
    };
    f32x4 accA[HS];  // dA tiles of waves 4-7: e tile (wv - 4) >> 1, j tiles HS ((wv - 4) & 1) + t
#pragma unroll
    for (int t = 0; t < HS; ++t) accA[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    fetch(0, 0);
    fetch(1, 1);
    for (int b = 0; b < nblk; ++b) {
      const int slot = b & 1;
      __syncthreads();  // readers of the previous block's images done (and sA written)
      stash(slot);
      __syncthreads();
      fetch(slot, b + 2);
      if (wv < 4) {
        // dZ tile: rows r = 16 rt + .., edges 16 et + ..
        const int rt = wv & 1, et = wv >> 1;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < HS; ++st) {
          bf16x8_t a[3], bb[3];
          const int ta = toff(16 * rt + li, 4 * st + g);
          const int sb = st * kSPlane + soff(16 * et + li, g);
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            a[p] = *reinterpret_cast<const bf16x8_t*>(sT + p * kTPlane + ta);
            bb[p] = *reinterpret_cast<const bf16x8_t*>(sA + p * HS * kSPlane + sb);
          }
          acc = mma6(a, bb, acc);
        }
        // lane: D[r = 4g + q][e = li] -> dZ[e][r0 + 16 rt + 4g .. + 3] (+ Tb)
        const int e = 16 * et + li;
        if (e < ng) {
          const int r = b * kV2R + 16 * rt + 4 * g;
          const f32x4 tb = *reinterpret_cast<const f32x4*>(Tb + (int64_t)n * w + r);
          *reinterpret_cast<f32x4*>(dZ + (e0 + g0 + e) * w + r) = acc + tb;
        }
      } else {
        const int v = wv - 4, et = v >> 1;
        bf16x8_t a[3];
        const int za = soff(16 * et + li, g);
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8_t*>(sZ + p * kSPlane + za);
        const int q = li >> 2, pp = li & 3;
#pragma unroll
        for (int t = 0; t < HS; ++t) {
          const int jt = HS * (v & 1) + t;  // 16-column tile of j
          bf16x8_t bb[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const unsigned char* base = sT + p * kTPlane;
            const int o0 = toff(8 * g + q, 2 * jt + (pp >> 1)) + 8 * (pp & 1);
            const int o1 = toff(8 * g + 4 + q, 2 * jt + (pp >> 1)) + 8 * (pp & 1);
            const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) i16x4_t*)(base + o0));
            const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) i16x4_t*)(base + o1));
            bb[p] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4,
                                                                           5, 6, 7));
          }
          accA[t] = mma6(a, bb, accA[t]);
        }
      }
    }
    if (wv >= 4) {  // dA[e][j] += (per-path launches on one stream: ordered RMW, deterministic)
      const int v = wv - 4, et = v >> 1;
#pragma unroll
      for (int t = 0; t < HS; ++t) {
        const int j = 16 * (HS * (v & 1) + t) + li;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = 16 * et + 4 * g + q;
          if (e < ng) dA[(e0 + g0 + e) * H + j] += accA[t][q];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------- apply v3
// The same contraction and arithmetic as v2, re-partitioned so that T never passes through a
// workgroup-shared LDS image: 256 threads (4 waves) per receiver edge group (<= 32 edges), wave
// q owns the j quarter [64q, 64q + 64) of H = 256.  Per 32-row block of T_n:
//   * each wave loads ITS 32 x 64 quarter of the block straight from HBM into registers in the
//     A-operand fragment order of the dZ product (lane: row 16 rt + (l & 15), 8 consecutive j),
//     one block ahead of use, and splits it into the three bf16 planes in registers;
//   * dZ partial D[r][e] = sum_{j in quarter} T[r][j] A[e][j] on those registers (A_n's planes
//     for the quarter stay in registers for the whole receiver); the four quarter partials are
//     summed in fixed order through a double-buffered LDS slab (one barrier per block) and the
//     wave owning tile (rt, et) adds Tb and stores dZ;
//   * dA D[e][j] += sum_r Z[e][r] T[r][j] for the quarter's 4 j tiles: the planes go to a
//     wave-private LDS slab and come back transposed (ds_read_b64_tr_b16), no barrier.
// v2 staged the whole block for all 8 waves behind two barriers and re-read A_n from LDS for
// every block (~300 KB of LDS reads per 32-row block); here ~24 KB per wave, the T stream
// overlaps the MFMAs of the previous block, and 80 KB of LDS lets two workgroups share a CU.
// Edge groups with <= 16 edges run half the MFMAs.  Requires H == 256, w % 64 == 0 (an even
// number of 32-row blocks: the block loop is unrolled by two without a guard), 16-byte aligned
// Z, A, T, Tb, dZ.
constexpr int kV3T = 256;
constexpr int kV3H = 256;
constexpr int kV3Q = kV3H / 4;                 // j per wave
constexpr int kV3Plane = 32 * 128;             // one plane of a wave's slab: 32 rows x 64 bf16
constexpr int kV3Slab = 3 * kV3Plane;          // a wave's transposition slab
constexpr int kV3Red = 4 * 4 * 64 * 16;        // [wave][tile][lane] f32x4 partials
constexpr int kV3Smem = 4 * kV3Slab + 2 * kV3Red;
constexpr int kV3Zd = 1;

// byte offset of (row, bf16 column jc) in a slab plane: 16-byte chunk jc / 8 XOR f(row) with
// f = (row & 7) ^ ((row & 8) >> 1) -- rows 0..7 of a ds_write_b128 lane group hit 8 distinct
// chunks of a 128-byte bank row, and the 8 rows of a ds_read_b64_tr_b16 half-wave (8g + 0..3,
// 8g + 8 .. 11) cover all 64 banks once
__device__ __forceinline__ int v3off(int row, int jc) {
  const int f = (row & 7) ^ ((row & 8) >> 1);
  return row * 128 + 16 * ((jc >> 3) ^ f) + 2 * (jc & 7);
}

// 8 consecutive f32 (two float4) -> the three bf16x8 planes of one MFMA fragment
__device__ __forceinline__ void split8(f32x4 x0, f32x4 x1, bf16x8_t (&p)[3]) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  unsigned h0, m0, l0, h1, m1, l1, h2, m2, l2, h3, m3, l3;
  split3v(f32x2_t{x0[0], x0[1]}, h0, m0, l0);
  split3v(f32x2_t{x0[2], x0[3]}, h1, m1, l1);
  split3v(f32x2_t{x1[0], x1[1]}, h2, m2, l2);
  split3v(f32x2_t{x1[2], x1[3]}, h3, m3, l3);
  p[0] = __builtin_bit_cast(bf16x8_t, u32x4_t{h0, h1, h2, h3});
  p[1] = __builtin_bit_cast(bf16x8_t, u32x4_t{m0, m1, m2, m3});
  p[2] = __builtin_bit_cast(bf16x8_t, u32x4_t{l0, l1, l2, l3});
}

template <int V>
using ic_t = std::integral_constant<int, V>;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ f32x4 ld4(rsrc_t r, unsigned voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// T (the large stream) and Z run two blocks ahead in a register ring whose slot is a
// compile-time index (the block loop is unrolled by two); A_n's quarter is held as raw f32 and
// split per use (VALU is idle beside the MFMAs; the registers go to the ring)
template <int ZD>  // Z / Tb ring depth (T: 2)
__global__ __launch_bounds__(kV3T, 2) void tp_node_apply_v3_kernel(
    int w, const int64_t* __restrict__ eoff, const float* __restrict__ Z,
    const float* __restrict__ A, const float* __restrict__ T, const float* __restrict__ Tb,
    float* __restrict__ dZ, float* __restrict__ dA) {
  constexpr int H = kV3H;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm3[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  unsigned char* slab = sm3 + wv * kV3Slab;
  unsigned char* red = sm3 + 4 * kV3Slab;
  const int n = blockIdx.x;
  const int64_t e0 = eoff[n], deg = eoff[n + 1] - e0;
  const rsrc_t tr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(T) + (int64_t)n * w * H,
                                                      0, w * H * 4, 0x00020000);
  const rsrc_t tbr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Tb) + (int64_t)n * w, 0,
                                                       w * 4, 0x00020000);
  const int jq = wv * kV3Q;
  const int nblk = w >> 5;
  const int my_rt = wv & 1, my_et = wv >> 1;  // the dZ tile this wave reduces and stores
  const f32x4 zero4 = f32x4{0.f, 0.f, 0.f, 0.f};
  int parity = 0;
  for (int64_t g0 = 0; g0 < deg; g0 += 32) {
    const int ng = (int)((deg - g0) < 32 ? (deg - g0) : 32);
    const bool two = ng > 16;  // uniform
    const int64_t eb = e0 + g0;
    // buffer descriptors over this group's rows (edges past ng read as zeros: the range check)
    // and 32-bit lane offsets: one address VGPR per stream instead of a 64-bit pointer per load
    const rsrc_t zr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Z) + eb * w, 0,
                                                        ng * w * 4, 0x00020000);
    const rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A) + eb * H, 0,
                                                        ng * H * 4, 0x00020000);
    // A_n's quarter (dZ's B operand: k = j, n = edge), split once per group
    bf16x8_t pa[2][2][3];
#pragma unroll
    for (int et = 0; et < 2; ++et) {
      const unsigned off = ((16 * et + li) * H + jq + 8 * g) * 4;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        split8(ld4(ar, off + 128 * ks, 0), ld4(ar, off + 128 * ks + 16, 0), pa[et][ks]);
    }
    f32x4 rT[2][2][2][2], rZ[ZD][2][2], rTb[ZD];
    const unsigned t_off = (li * H + jq + 8 * g) * 4;
    const unsigned z_off = (li * w + 8 * g) * 4;
    auto fetch_t = [&](auto slot, int b, int rt) {
      const int so = (32 * b + 16 * rt) * H * 4;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        rT[slot][rt][ks][0] = ld4(tr, t_off + 128 * ks, so);
        rT[slot][rt][ks][1] = ld4(tr, t_off + 128 * ks + 16, so);
      }
    };
    auto fetch_z = [&](auto slot, int b) {
#pragma unroll
      for (int et = 0; et < 2; ++et) {
        const int so = (16 * et * w + 32 * b) * 4;
        rZ[slot][et][0] = ld4(zr, z_off, so);
        rZ[slot][et][1] = ld4(zr, z_off + 16, so);
      }
      rTb[slot] = ld4(tbr, (16 * my_rt + 4 * g) * 4, 32 * b * 4);
    };
    f32x4 accA[2][4];
#pragma unroll
    for (int et = 0; et < 2; ++et)
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) accA[et][jt] = zero4;
    // The ring loads are unconditional: past the receiver's rows (the last two blocks' look-ahead)
    // the buffer range check returns zeros and no memory is touched.  r05 guarded them with
    // `if (b + 2 < nblk)`: the guarded registers then met the unguarded ones in PHI copies at
    // the unrolled loop's back edge, each behind a full vmcnt(0) wait, so the T ring prefetched
    // nothing across iterations.
    auto body = [&](auto slot, int b) {
      constexpr int zs = ZD == 2 ? decltype(slot)::value : 0;
      bf16x8_t pz[2][3];
#pragma unroll
      for (int et = 0; et < 2; ++et) split8(rZ[zs][et][0], rZ[zs][et][1], pz[et]);
      const f32x4 tb = rTb[zs];
      fetch_z(ic_t<zs>{}, b + ZD);
      unsigned char* rb = red + parity * kV3Red;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        bf16x8_t pt[2][3];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) split8(rT[slot][rt][ks][0], rT[slot][rt][ks][1], pt[ks]);
        fetch_t(slot, b + 2, rt);
        // planes into the wave's slab ([plane][row][64 j]); read back transposed below (one
        // wave's LDS operations complete in order: no barrier, no wait)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int p = 0; p < 3; ++p)
            *reinterpret_cast<bf16x8_t*>(slab + p * kV3Plane +
                                         v3off(16 * rt + li, 32 * ks + 8 * g)) = pt[ks][p];
        // dZ quarter partials -> reduction buffer [wave][tile = rt + 2 et][lane]
#pragma unroll
        for (int et = 0; et < 2; ++et) {
          f32x4 acc = zero4;
          if (et == 0 || two) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) acc = mma6(pt[ks], pa[et][ks], acc);
          }
          *reinterpret_cast<f32x4*>(rb + ((wv * 4 + rt + 2 * et) * 64 + lane) * 16) = acc;
        }
      }
      __asm__ volatile("" ::: "memory");
      // dA for the quarter's 4 j tiles (B operand: rows 8g .. 8g + 7 of column 16 jt + li)
      {
        const int q = li >> 2, pp = li & 3;
#pragma unroll
        for (int jt = 0; jt < 4; ++jt) {
          bf16x8_t bt[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            unsigned char* base = slab + p * kV3Plane;
            const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) i16x4_t*)(base +
                                                             v3off(8 * g + q, 16 * jt + 4 * pp)));
            const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) i16x4_t*)(base +
                                                             v3off(8 * g + 4 + q, 16 * jt + 4 * pp)));
            bt[p] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5,
                                                                           6, 7));
          }
          accA[0][jt] = mma6(pz[0], bt, accA[0][jt]);
          if (two) accA[1][jt] = mma6(pz[1], bt, accA[1][jt]);
          __asm__ volatile("" ::: "memory");  // one j tile's transposed reads live at a time
        }
      }
      __syncthreads();  // all quarter partials of this block are in rb
      {
        const int t = my_rt + 2 * my_et;
        f32x4 s = *reinterpret_cast<const f32x4*>(rb + ((0 * 4 + t) * 64 + lane) * 16);
        s += *reinterpret_cast<const f32x4*>(rb + ((1 * 4 + t) * 64 + lane) * 16);
        s += *reinterpret_cast<const f32x4*>(rb + ((2 * 4 + t) * 64 + lane) * 16);
        s += *reinterpret_cast<const f32x4*>(rb + ((3 * 4 + t) * 64 + lane) * 16);
        const int e = 16 * my_et + li;
        if (e < ng)
          *reinterpret_cast<f32x4*>(dZ + (eb + e) * w + 32 * b + 16 * my_rt + 4 * g) = s + tb;
      }
      parity ^= 1;
    };
    fetch_t(ic_t<0>{}, 0, 0);
    fetch_t(ic_t<0>{}, 0, 1);
    fetch_z(ic_t<0>{}, 0);
    fetch_t(ic_t<1>{}, 1, 0);
    fetch_t(ic_t<1>{}, 1, 1);
    if constexpr (ZD == 2) fetch_z(ic_t<ZD - 1>{}, 1);
    for (int b = 0; b < nblk; b += 2) {  // nblk even (w % 64 == 0, checked at the launch)
      body(ic_t<0>{}, b);
      body(ic_t<1>{}, b + 1);
    }
    // dA[e][j] += (per-path launches on one stream: ordered RMW, deterministic), through a
    // buffer descriptor over the group's ng rows: rows past ng load zeros and drop their stores,
    // so the 32 loads issue back to back and meet one wait (r05's per-element `if (e < ng)`
    // RMW was 32 dependent round trips per group and wave, each behind a vmcnt(0))
    {
      const rsrc_t dar = __builtin_amdgcn_make_buffer_rsrc(dA + eb * H, 0, ng * H * 4, 0x00020000);
      float old[2][4][4];
#pragma unroll
      for (int et = 0; et < 2; ++et)
#pragma unroll
        for (int jt = 0; jt < 4; ++jt)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            old[et][jt][q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                dar, ((16 * et + 4 * g + q) * H + jq + 16 * jt + li) * 4, 0, 0));
#pragma unroll
      for (int et = 0; et < 2; ++et)
#pragma unroll
        for (int jt = 0; jt < 4; ++jt)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(
                __float_as_uint(old[et][jt][q] + accA[et][jt][q]), dar,
                ((16 * et + 4 * g + q) * H + jq + 16 * jt + li) * 4, 0, 0);
    }
  }
}

}  // namespace
}  // namespace gmp

using namespace gmp;

namespace gmp {
// apply kernel: 2 = v3 (per-wave j quarters, T straight to registers; default where the shape
// allows), 1 = v2 (bf16x3, shared LDS image), 0 = the f32-MFMA kernel (gmp_tp_apply_set_x3:
// the tests run every form)
int g_apply_x3 = 2;
}  // namespace gmp

extern "C" {

int gmp_tp_apply_set_x3(int on) {
  const int old = g_apply_x3;
  g_apply_x3 = on < 0 ? 0 : (on > 2 ? 2 : on);
  return old;
}


int gmp_tp_node_outer_f32(int64_t n_recv, int64_t w, int64_t H, const int64_t* eoff,
                          const float* Z, const float* A, float* S, float* Sb, void* stream) {
  GMP_CHECK_ARG(n_recv >= 0 && w > 0 && H > 0 && H <= kMaxH && H % 16 == 0);
  GMP_CHECK_ARG(n_recv <= 65535 * 1024);
  if (n_recv == 0) return GMP_OK;
  GMP_CHECK_ARG(eoff && Z && A && S && Sb);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(A) % 16 == 0);
  if (n_recv > 65535) return GMP_ERR_UNSUPPORTED;  // grid.y limit: caller chunks receivers
  // two column parts for the widest H; S stored through LDS
  const int cs = H == kMaxH ? 2 : 1;
  const dim3 grid((unsigned)(ceil_div(w, kRowsPerBlock * kOuterRB) * cs), (unsigned)n_recv);
  auto k = cs == 2 ? tp_node_outer_kernel<false, true, 2> : tp_node_outer_kernel<false, true, 1>;
  k<<<grid, kNT, 0, as_stream(stream)>>>((int)w, (int)H, eoff, Z, A, S, Sb, nullptr);
  return launch_status();
}

int gmp_tp_node_apply_f32(int64_t n_recv, int64_t w, int64_t H, const int64_t* eoff,
                          const float* Z, const float* A, const float* T, const float* Tb,
                          float* dZ, float* dA, void* stream) {
  GMP_CHECK_ARG(n_recv >= 0 && w > 0 && H > 0 && H <= kMaxH && H % 16 == 0);
  if (n_recv == 0) return GMP_OK;
  GMP_CHECK_ARG(eoff && Z && A && T && Tb && dZ && dA);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(T) % 16 == 0);
  const bool a16 = ((reinterpret_cast<uintptr_t>(Z) | reinterpret_cast<uintptr_t>(A) |
                     reinterpret_cast<uintptr_t>(Tb) | reinterpret_cast<uintptr_t>(dZ)) % 16) == 0;
  if (g_apply_x3 == 2 && H == kV3H && w % 64 == 0 && a16) {
    auto k = tp_node_apply_v3_kernel<kV3Zd>;
    int rc = 0;
    if ((rc = hip_check(hipFuncSetAttribute((const void*)k,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, kV3Smem))))
      return rc;
    k<<<(unsigned)n_recv, kV3T, kV3Smem, as_stream(stream)>>>((int)w, eoff, Z, A, T, Tb, dZ, dA);
    return launch_status();
  }
  // x3 form only for wide paths: measured (scripts/mb_apply_shapes.py, 50k receivers x 20
  // edges, H = 256) 13.3 vs 13.7 ms at w = 640, but slower at w <= 384 (9.1 vs 8.9 ms at 384,
  // 3.8 vs 3.2 at 64)
  if (w >= 512 && w % kV2R == 0 && H % 64 == 0 && a16 && g_apply_x3) {  // whole float4 units
    const int hs = (int)(H / 32);
    const size_t smem = (size_t)3 * kTPlane + (size_t)3 * hs * kSPlane + 3 * kSPlane;
    int rc = 0;
#define LAUNCH_AV2(HS)                                                                              \
  {                                                                                              \
    auto k = tp_node_apply_x3_kernel<HS>;                                                        \
    if ((rc = hip_check(hipFuncSetAttribute((const void*)k,                                      \
                                            hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                            (int)smem))))                                        \
      return rc;                                                                                 \
    k<<<(unsigned)n_recv, kV2T, smem, as_stream(stream)>>>((int)w, eoff, Z, A, T, Tb, dZ, dA);   \
  }
    switch (hs) {
      case 2: LAUNCH_AV2(2) break;
      case 4: LAUNCH_AV2(4) break;
      case 6: LAUNCH_AV2(6) break;
      default: LAUNCH_AV2(8) break;
    }
#undef LAUNCH_AV2
    return launch_status();
  }
  tp_node_apply_kernel<<<(unsigned)n_recv, kNT, 0, as_stream(stream)>>>(
      (int)w, (int)H, eoff, Z, A, T, Tb, dZ, dA);
  return launch_status();
}

}  // extern "C"
