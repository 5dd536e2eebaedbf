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
// rows a_e once and produces kOuterRB 64-row blocks of S from them
constexpr int kOuterRB = 1;
__global__ __launch_bounds__(kNT) void tp_node_outer_kernel(int w, int H,
                                                            const int64_t* __restrict__ eoff,
                                                            const float* __restrict__ Z,
                                                            const float* __restrict__ A,
                                                            float* __restrict__ S,
                                                            float* __restrict__ Sb) {
  __shared__ __attribute__((aligned(16))) float sA[kEdgeStage * (kMaxH + 16)];
  const int n = blockIdx.y;
  const int LDA = H + 16;  // 16 mod 64 floats: the 4 edge rows of an MFMA read hit disjoint banks
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, i = lane & 15, kk = lane >> 4;
  const int64_t e0 = eoff[n], deg = eoff[n + 1] - e0;
  const int TJ = H >> 4;
  float* Sn = S + (int64_t)n * w * H;
  if (kOuterRB == 1 && deg <= kEdgeStage) {
    // common case (one edge stage): this lane's Z column values for every k step are loaded
    // up front, in flight together with the a-row staging — no dependent global load inside the
    // MFMA loop (the block's latency chain was load -> MFMA per step, ~5 HBM round trips)
    const int ns = (int)deg, nst = (ns + 3) >> 2;
    const int r = blockIdx.x * kRowsPerBlock + wv * 16 + i;
    float zr[kEdgeStage / 4];
#pragma unroll
    for (int s = 0; s < kEdgeStage / 4; ++s) {
      const int el = 4 * s + kk;
      zr[s] = (el < ns && r < w) ? Z[(e0 + el) * w + r] : 0.f;
    }
    for (int x = tid; x < 4 * nst * (H >> 2); x += kNT) {  // padding rows zeroed
      const int e = x / (H >> 2), q = x - e * (H >> 2);
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (e < ns) v = *reinterpret_cast<const f32x4*>(A + (e0 + e) * H + 4 * q);
      *reinterpret_cast<f32x4*>(&sA[e * LDA + 4 * q]) = v;
    }
    __syncthreads();
    f32x4 acc[kMaxH / 16];
#pragma unroll
    for (int t = 0; t < kMaxH / 16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float zsum = 0.f;
#pragma unroll
    for (int s = 0; s < kEdgeStage / 4; ++s) {
      if (s < nst) {
        const int el = 4 * s + kk;
        zsum += zr[s];
#pragma unroll
        for (int t = 0; t < kMaxH / 16; ++t)
          if (t < TJ) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(sA[el * LDA + 16 * t + i], zr[s], acc[t], 0, 0, 0);
      }
    }
    if (r < w) {
#pragma unroll
      for (int t = 0; t < kMaxH / 16; ++t)
        if (t < TJ) *reinterpret_cast<f32x4*>(Sn + (int64_t)r * H + 16 * t + 4 * kk) = acc[t];
    }
    zsum += __shfl_xor(zsum, 16);
    zsum += __shfl_xor(zsum, 32);
    if (kk == 0 && r < w) Sb[(int64_t)n * w + r] = zsum;
    return;
  }
  if (deg <= kEdgeStage) {  // stage a once for all row blocks
    const int ns = (int)deg, ns4 = (ns + 3) & ~3;
    for (int x = tid; x < ns4 * (H >> 2); x += kNT) {  // padding rows zeroed (0 * garbage = NaN)
      const int e = x / (H >> 2), q = x - e * (H >> 2);
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (e < ns) v = *reinterpret_cast<const f32x4*>(A + (e0 + e) * H + 4 * q);
      *reinterpret_cast<f32x4*>(&sA[e * LDA + 4 * q]) = v;
    }
    __syncthreads();
  }
  for (int rbi = 0; rbi < kOuterRB; ++rbi) {
    const int rb = blockIdx.x * kOuterRB + rbi;
    if (rb * kRowsPerBlock >= w) break;
    // D = S^T tile: D[j][r] = sum_e A[e, j] Z[e, r]  (A op = a columns, B op = Z columns), so a
    // lane holds 4 consecutive j of one row r and stores them as one float4
    const int r = rb * kRowsPerBlock + wv * 16 + i;  // this lane's output row
    f32x4 acc[kMaxH / 16];
#pragma unroll
    for (int t = 0; t < kMaxH / 16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float zsum = 0.f;  // Sb[n, r]: this lane's edges (k phase kk) of the Z column
    for (int64_t eb = 0; eb < deg; eb += kEdgeStage) {
      const int ns = (int)((deg - eb) < kEdgeStage ? (deg - eb) : kEdgeStage);
      const int ns4 = (ns + 3) & ~3;
      if (deg > kEdgeStage) {
        __syncthreads();
        for (int x = tid; x < ns4 * (H >> 2); x += kNT) {
          const int e = x / (H >> 2), q = x - e * (H >> 2);
          f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
          if (e < ns) v = *reinterpret_cast<const f32x4*>(A + (e0 + eb + e) * H + 4 * q);
          *reinterpret_cast<f32x4*>(&sA[e * LDA + 4 * q]) = v;
        }
        __syncthreads();
      }
      for (int s = 0; s < (ns4 >> 2); ++s) {
        const int el = 4 * s + kk;
        const float zv = (el < ns && r < w) ? Z[(e0 + eb + el) * w + r] : 0.f;
        zsum += zv;
#pragma unroll
        for (int t = 0; t < kMaxH / 16; ++t)
          if (t < TJ) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(sA[el * LDA + 16 * t + i], zv, acc[t], 0, 0, 0);
      }
    }
    if (r < w) {  // streaming stores: S (GBs per chunk) is consumed by the next GEMM from HBM
#pragma unroll
      for (int t = 0; t < kMaxH / 16; ++t)
        if (t < TJ)
          *reinterpret_cast<f32x4*>(Sn + (int64_t)r * H + 16 * t + 4 * kk) = acc[t];
    }
    zsum += __shfl_xor(zsum, 16);
    zsum += __shfl_xor(zsum, 32);
    if (kk == 0 && r < w) Sb[(int64_t)n * w + r] = zsum;
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

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_tp_node_outer_f32(int64_t n_recv, int64_t w, int64_t H, const int64_t* eoff,
                          const float* Z, const float* A, float* S, float* Sb, void* stream) {
  GMP_CHECK_ARG(n_recv >= 0 && w > 0 && H > 0 && H <= kMaxH && H % 16 == 0);
  GMP_CHECK_ARG(n_recv <= 65535 * 1024);
  if (n_recv == 0) return GMP_OK;
  GMP_CHECK_ARG(eoff && Z && A && S && Sb);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(A) % 16 == 0);
  if (n_recv > 65535) return GMP_ERR_UNSUPPORTED;  // grid.y limit: caller chunks receivers
  const dim3 grid((unsigned)ceil_div(w, kRowsPerBlock * kOuterRB), (unsigned)n_recv);
  tp_node_outer_kernel<<<grid, kNT, 0, as_stream(stream)>>>((int)w, (int)H, eoff, Z, A, S, Sb);
  return launch_status();
}

int gmp_tp_node_apply_f32(int64_t n_recv, int64_t w, int64_t H, const int64_t* eoff,
                          const float* Z, const float* A, const float* T, const float* Tb,
                          float* dZ, float* dA, void* stream) {
  GMP_CHECK_ARG(n_recv >= 0 && w > 0 && H > 0 && H <= kMaxH && H % 16 == 0);
  if (n_recv == 0) return GMP_OK;
  GMP_CHECK_ARG(eoff && Z && A && T && Tb && dZ && dA);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(T) % 16 == 0);
  tp_node_apply_kernel<<<(unsigned)n_recv, kNT, 0, as_stream(stream)>>>(
      (int)w, (int)H, eoff, Z, A, T, Tb, dZ, dA);
  return launch_status();
}

}  // extern "C"
