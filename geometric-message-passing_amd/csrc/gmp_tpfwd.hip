// K7s: the forward of the receiver-factorised tensor-product convolution with the S intermediate
// built inside the path GEMM (tfn_layer.py:73-87 regrouped, see gmp_tp.hip "node form"):
//
//   out[(n,k), w] += sum_{u,j} S[(n,k), (u,j)] W2p[(u,j), w] + sum_u Sb[(n,k), u] b2p[u, w],
//   S[(n,k), (u,j)] = sum_{e -> n} Z[e, k mul1 + u] A[e, j],   Sb[(n,k), u] = sum_{e -> n} Z[e, ..]
//
// The unfused forward writes S (N (2lo+1) x mul1 H floats: 32.8 GB for a MACE-128 lo = 2 path at
// 1M edges) with gmp_tp_node_outer_f32 and streams it back through the K7g GEMM: 66 GB of HBM
// traffic per path.  Here a workgroup owns RT = 64 / d3 whole receivers (<= 64 GEMM rows (n, k))
// and all mul_out columns, and walks the GEMM's k range in steps of U = 16 / d3 channels u times
// one 32-wide j chunk.  Per step each wave builds S tiles with the f32 MFMA (16x16x4, the edge
// index as the MFMA k dimension, the arithmetic of the S kernel): rows = the U x d3 (u, k) combos
// of one receiver (15 of 16 MFMA rows for d3 = 3, 5), columns = 16 j; the results are split into
// three bf16 planes into a double-buffered LDS A image while the other buffer feeds the bf16
// MFMA GEMM (six plane products, f32 accumulation: the K7g arithmetic, gmp_tpgemm.hip).  B (W2p,
// b2p) comes straight from global memory in MFMA fragment order (the forward planes of
// gmp_tp_split_w2_f32, read in this kernel's chunk order).  S never reaches HBM: per path the
// kernel reads Z and A (and W2p from the caches) and accumulates into out.
//
// Step order: the bias chunks (Sb: VALU sums of Z rows) first, then u-steps outer, j chunks inner
// (the Z columns of a u-step are reused across its j chunks from L1/L2).  Deterministic: every
// S value is one MFMA chain over the receiver's edges in edge order; every output element is one
// accumulator chain over the k range in a fixed order.
#include <type_traits>

#include "gmp_common.h"

namespace gmp {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kFT = 512;        // threads (8 waves)
constexpr int kFM = 64;         // GEMM rows per workgroup (RT receivers x d3, padded)
constexpr int kChunkB = kFM * 64;  // bytes of one plane of one 32-k chunk image (64 rows x 32 bf16)

__device__ __forceinline__ void split3p(f32x2 x, unsigned& h, unsigned& m, unsigned& l) {
  const bf16x2 bh = __builtin_convertvector(x, bf16x2);
  const f32x2 r1 = x - __builtin_convertvector(bh, f32x2);
  const bf16x2 bm = __builtin_convertvector(r1, bf16x2);
  const f32x2 r2 = r1 - __builtin_convertvector(bm, f32x2);
  const bf16x2 bl = __builtin_convertvector(r2, bf16x2);
  h = __builtin_bit_cast(unsigned, bh);
  m = __builtin_bit_cast(unsigned, bm);
  l = __builtin_bit_cast(unsigned, bl);
}

// [row][32 k] bf16 image with 64-byte rows, 16-byte chunk q at q ^ ((row >> 1) & 3) (the K7g
// layout: the MFMA operand read row = lane & 15, k = 8 (lane >> 4) .. + 7 is conflict-free)
__device__ __forceinline__ int ioff(int row, int k) {
  return row * 64 + 16 * ((k >> 3) ^ ((row >> 1) & 3)) + 2 * (k & 7);
}
__device__ __forceinline__ int ioffc(int row, int chunk16) {
  return row * 64 + 16 * (chunk16 ^ ((row >> 1) & 3));
}
__device__ __forceinline__ bf16x8 asb(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

// compile-time loop: f(integral_constant<int, I>) for I in [B, E)
template <int B, int E, class Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>());
    static_for<B + 1, E>(f);
  }
}

template <int D3>
struct FCfg {
  static constexpr int U = 16 / D3;          // channels u per step (U x d3 <= 16 MFMA rows)
  static constexpr int NC = U * D3;          // live S-MFMA rows (combos (k, u))
  static constexpr int RT = kFM / D3;        // receivers per workgroup
  static constexpr int ROWS = RT * D3;       // live GEMM rows
  static constexpr int NCH = (2 * RT + 7) / 8;  // S chains (receiver x 16-wide j block) per wave
  static constexpr int PF = NCH <= 3 ? 6 : 4;   // MFMA steps (4 edges each) of operands prefetched
  static constexpr int STG = U * 3 * kChunkB;   // LDS bytes of one step image (U chunks, 3 planes)
};

// Every wave both consumes (the GEMM on the current step image) and produces (S chains of the
// next step into the other image), one barrier per step.  The B fragments of two consecutive
// 32-k chunks are in registers (the next chunk's loads in flight during the current chunk's
// MFMAs, across step boundaries; the step loop is unrolled by two so the register set of a chunk
// is a compile-time choice); the S operands of step s + 2 are loaded during step s + 1.
template <int D3, int NBW>
__global__ __launch_bounds__(kFT, 1) void tp_node_fwd_fused_kernel(
    int n_recv, int mul1, int H, const int64_t* __restrict__ eoff, const float* __restrict__ Z,
    int64_t zrows, const float* __restrict__ A, const unsigned short* __restrict__ Bf,
    float* __restrict__ C, int64_t cldg) {
  using F = FCfg<D3>;
  constexpr int U = F::U, RT = F::RT, NCH = F::NCH, PF = F::PF;
  constexpr int WN = NBW / 16, WM = 8 / WN, RTW = 4 / WM;  // consumer wave grid (1 column tile)
  extern __shared__ __attribute__((aligned(16))) unsigned char smf[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WN, wn = wv % WN;
  const int li = lane & 15, g = lane >> 4;
  const int HB = H >> 5;                    // 32-wide j chunks
  const int QB = mul1 >> 5;                 // bias chunks
  const int NBS = (QB + U - 1) / U;         // bias steps
  const int NUS = (mul1 + U - 1) / U;       // u steps
  const int nsteps = NBS + NUS * HB;
  const int64_t K1 = (int64_t)mul1 * H;
  const int ct_total = NBW / 16;            // forward B planes of this path: N = mul_out = NBW
  const int n0 = blockIdx.x * RT;           // first receiver of the tile

  // zero both step images (rows past ROWS stay zero; chains of absent receivers write zeros)
  for (int x = tid; x < 2 * F::STG / 16; x += kFT)
    reinterpret_cast<u32x4*>(smf)[x] = u32x4{0u, 0u, 0u, 0u};

  // step -> (bias?, u0, jc)
  auto step_u0 = [&](int s) { return s < NBS ? s * U : ((s - NBS) / HB) * U; };
  auto step_jc = [&](int s) { return s < NBS ? -1 : (s - NBS) % HB; };
  // original k chunk (the forward B plane order, k = u H + j, bias k = K1 + u) of chunk uu of
  // step s, or -1 when absent
  auto chunk_of = [&](int s, int uu) -> int64_t {
    if (s >= nsteps) return -1;
    if (s < NBS) {
      const int q = s * U + uu;
      return q < QB ? (K1 >> 5) + q : -1;
    }
    const int u = step_u0(s) + uu;
    return u < mul1 ? ((int64_t)u * H >> 5) + step_jc(s) : -1;
  };

  // ================= producer state: chains c = wv + 8 i -> receiver rho = c % RT, j block
  // jb = c / RT.  Z in the K7s layout (gmp_tp_z_fused_layout_f32): per u step us, a row of 16
  // floats per edge holding the d3 x U combos c = k U + uu (z[e][k mul1 + us U + uu]; the 16th
  // and any past mul1 zero): one S-MFMA operand load is 4 edges x 64 contiguous bytes.  The
  // tile's rows go through buffer descriptors (32-bit lane offsets from the tile's first edge; an
  // offset past the descriptor (kOobF) loads 0: absent edges need no branch or select).
  int ce0[NCH], ce1[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = wv + 8 * i, rho = c % RT, n = n0 + rho;
    const bool live = c < 2 * RT && n < n_recv;
    ce0[i] = live ? (int)eoff[n] : 0;
    ce1[i] = live ? (int)eoff[n + 1] : 0;
  }
  const int nlast = min(n0 + RT, n_recv);
  const int64_t te0 = eoff[n0], te1 = eoff[nlast];
  auto zrs_of = [&](int us) {
    return __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(Z) + ((int64_t)us * zrows + te0) * 16, 0, (int)((te1 - te0) * 64),
        0x00020000);
  };
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A) + te0 * H, 0, (int)((te1 - te0) * H * 4), 0x00020000);
  constexpr unsigned kOobF = 0x80000000u;
  // byte offsets of this lane's operands of MFMA step t of chain i (recomputed per use: the
  // producer's VALU is idle beside the consumer's MFMAs, its registers are not)
  auto zoff = [&](int i, int t) {
    const int el = ce0[i] - (int)te0 + 4 * t + g;
    return ce0[i] + 4 * t + g < ce1[i] ? (unsigned)(el * 16 + li) * 4u : kOobF;
  };
  auto aoff = [&](int i, int t, unsigned as) {
    const int el = ce0[i] - (int)te0 + 4 * t + g;
    const int jb = (wv + 8 * i) / RT;
    return ce0[i] + 4 * t + g < ce1[i] ? (unsigned)(el * H + jb * 16 + li) * 4u + as : kOobF;
  };
  float zp[NCH][PF], ap[NCH][PF];  // prefetched operands of the first PF MFMA steps per chain
  auto prefetch = [&](int s) {
    if (s >= nsteps || s < NBS) return;
    const __amdgpu_buffer_rsrc_t zrs = zrs_of(step_u0(s) / U);
    const unsigned as = 128u * step_jc(s);
#pragma unroll
    for (int i = 0; i < NCH; ++i)
#pragma unroll
      for (int t = 0; t < PF; ++t) {
        zp[i][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zrs, zoff(i, t), 0, 0));
        ap[i][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ars, aoff(i, t, as), 0, 0));
      }
  };
  auto produce = [&](int s, unsigned char* img) {
    if (s >= nsteps) return;
    if (s < NBS) {
      // bias chunks: Sb[(rho, k), u] by VALU; thread -> row tid / 8, 4 u's
      const int u4 = 4 * (tid & 7);
      for (int uu = 0; uu < U; ++uu) {
        const int q = s * U + uu;
        if (q >= QB) break;
        {
          const int r = tid >> 3;
          const int rho = r / D3, k = r - rho * D3, n = n0 + rho;
          const bool live = r < F::ROWS && n < n_recv;
          const int e0 = live ? (int)eoff[n] : 0, e1 = live ? (int)eoff[n + 1] : 0;
          // z[e][k mul1 + u] for u = 32 q + u4 + x at ((u / U) zrows + e) 16 + k U + u % U
          const float* zc[4];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            const int u = 32 * q + u4 + x;
            zc[x] = Z + (int64_t)(u / U) * zrows * 16 + k * U + u % U;
          }
          f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
          for (int e = e0; e < e1; ++e)
#pragma unroll
            for (int x = 0; x < 4; ++x) acc[x] += zc[x][(int64_t)e * 16];
          unsigned p[3][2];
          split3p(f32x2{acc[0], acc[1]}, p[0][0], p[1][0], p[2][0]);
          split3p(f32x2{acc[2], acc[3]}, p[0][1], p[1][1], p[2][1]);
          const int off = ioff(r, u4);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            *reinterpret_cast<u32x2*>(img + (uu * 3 + pl) * kChunkB + off) = u32x2{p[pl][0], p[pl][1]};
        }
      }
      return;
    }
    const __amdgpu_buffer_rsrc_t zrs = zrs_of(step_u0(s) / U);
    const unsigned as = 128u * step_jc(s);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = wv + 8 * i;
      if (c >= 2 * RT) break;  // wave-uniform
      const int rho = c % RT, jb = c / RT;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const int nq = (ce1[i] - ce0[i] + 3) >> 2;
#pragma unroll
      for (int t = 0; t < PF; ++t)
        if (t < nq) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ap[i][t], zp[i][t], acc, 0, 0, 0);
      for (int t = PF; t < nq; ++t)  // in-degree > 4 PF: the rest directly
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ars, aoff(i, t, as), 0, 0)),
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zrs, zoff(i, t), 0, 0)),
            acc, 0, 0, 0);
      // S transposed (MFMA rows = j, columns = combos): lane (li, g) holds S[combo li][j = jb 16 +
      // 4 g .. + 3], four consecutive k of one image row -> one 8-byte store per plane
      if (li < F::NC) {
        unsigned ph[2], pm[2], pl[2];
        split3p(f32x2{acc[0], acc[1]}, ph[0], pm[0], pl[0]);
        split3p(f32x2{acc[2], acc[3]}, ph[1], pm[1], pl[1]);
        const int k = li / U, uu = li - (li / U) * U;
        unsigned char* base = img + uu * 3 * kChunkB + ioff(rho * D3 + k, jb * 16 + 4 * g);
        *reinterpret_cast<u32x2*>(base) = u32x2{ph[0], ph[1]};
        *reinterpret_cast<u32x2*>(base + kChunkB) = u32x2{pm[0], pm[1]};
        *reinterpret_cast<u32x2*>(base + 2 * kChunkB) = u32x2{pl[0], pl[1]};
      }
    }
  };

  // ================= consumer state: row tiles RTW wm .. + RTW - 1, column tile wn
  f32x4 acc[RTW];
#pragma unroll
  for (int r = 0; r < RTW; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
  // B planes through a descriptor: the lane / column-tile part of the offset is fixed, the chunk
  // part is wave-uniform (scalar offset): no per-load address arithmetic
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(Bf), 0, 0x7fffffff, 0x00020000);
  const unsigned bvo = 16u * lane + (unsigned)wn * 3u * 1024u;
  // B ring: R register sets of one 32-k chunk each, chunk q in set q % R, loaded R - 1 chunks
  // ahead (R = 3 for U = 3: the set of a step's chunks is static; else R = 2 and the step loop's
  // unroll by two keeps it static)
  constexpr int R = (U % 3 == 0) ? 3 : 2;
  u32x4 bset[R][3];
  auto load_b = [&](u32x4 (&b)[3], int s, int uu) {
    int64_t ch = chunk_of(s, uu);
    if (ch < 0) ch = 0;  // absent chunk: a valid address, never consumed
    const int so = (int)(ch * ct_total * 3 * 1024);
#pragma unroll
    for (int p = 0; p < 3; ++p)
      b[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(brs, bvo, so + p * 1024, 0));
  };
  // the chunk's A fragments (all row tiles of this wave) are read from LDS before its MFMAs (one
  // exposed LDS round trip per chunk instead of one per row tile)
  auto load_a = [&](u32x4 (&a)[RTW][3], const unsigned char* cimg) {
#pragma unroll
    for (int r = 0; r < RTW; ++r) {
      const int off = ioffc(16 * (wm * RTW + r) + li, g);
#pragma unroll
      for (int p = 0; p < 3; ++p) a[r][p] = *reinterpret_cast<const u32x4*>(cimg + p * kChunkB + off);
    }
  };
  // step s's chunks from image img; P0 = the B set of the step's first chunk
  auto consume = [&](int s, const unsigned char* img, auto par0) {
    constexpr int P0 = decltype(par0)::value;
    static_for<0, U>([&](auto uu_c) {
      constexpr int uu = decltype(uu_c)::value;
      constexpr int cur = (P0 + uu) % R;
      constexpr int du = uu + R - 1;  // chunk q + R - 1 (the next step's when du >= U)
      load_b(bset[(cur + R - 1) % R], s + du / U, du % U);
      if (chunk_of(s, uu) < 0) return;  // absent chunk (wave-uniform)
      u32x4 a[RTW][3];
      load_a(a, img + uu * 3 * kChunkB);
      const u32x4 (&b)[3] = bset[cur];
#pragma unroll
      for (int r = 0; r < RTW; ++r) {
        f32x4 t = acc[r];
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[r][2]), asb(b[0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[r][1]), asb(b[1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[r][0]), asb(b[2]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[r][1]), asb(b[0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[r][0]), asb(b[1]), t, 0, 0, 0);
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[r][0]), asb(b[0]), t, 0, 0, 0);
      }
    });
  };

  __syncthreads();  // zeroed images
  // the B set of step s's first chunk is (s U) % R: static within the unrolled pair
  constexpr int PA = 0, PB = U % R;
  prefetch(0);
  produce(0, smf);
  prefetch(1);
  static_for<0, R - 1>([&](auto q_c) {
    constexpr int q = decltype(q_c)::value;
    load_b(bset[q], q / U, q % U);
  });
  __syncthreads();
  for (int s = 0; s < nsteps; s += 2) {
    consume(s, smf, std::integral_constant<int, PA>());
    __builtin_amdgcn_sched_barrier(0);
    produce(s + 1, smf + F::STG);  // its operands were loaded a whole step ago
    __builtin_amdgcn_sched_barrier(0);
    prefetch(s + 2);
    __syncthreads();
    if (s + 1 < nsteps) {
      consume(s + 1, smf + F::STG, std::integral_constant<int, PB>());
      __builtin_amdgcn_sched_barrier(0);
      produce(s + 2, smf);
      __builtin_amdgcn_sched_barrier(0);
      prefetch(s + 3);
    }
    __syncthreads();
  }

  // epilogue: row (rho, k) of receiver n0 + rho, column w' -> out[n, w' d3 + k] (+=)
#pragma unroll
  for (int r = 0; r < RTW; ++r) {
    const int col = 16 * wn + li;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * (wm * RTW + r) + 4 * g + q;
      const int rho = row / D3, k = row - rho * D3;
      if (row < F::ROWS && n0 + rho < n_recv)
        C[(int64_t)(n0 + rho) * cldg + col * D3 + k] += acc[r][q];
    }
  }
}

// Z (rows x d3 mul1, z[e][k mul1 + u]) -> the K7s layout Zf[us][e][16] (combo c = k U + uu,
// u = us U + uu; zeros at c >= d3 U and u >= mul1).  A workgroup stages kZE consecutive rows in
// LDS (coalesced float4 reads), then writes each u step's kZE x 16 block as one contiguous run.
constexpr int kZE = 16;
__global__ __launch_bounds__(256) void z_fused_layout_kernel(const float* __restrict__ Z,
                                                             int64_t rows, int d3, int mul1,
                                                             int U, int nus,
                                                             float* __restrict__ Zf) {
  extern __shared__ __attribute__((aligned(16))) float zs[];
  const int w = d3 * mul1;
  const int64_t e0 = (int64_t)blockIdx.x * kZE;
  const int ne = (int)min((int64_t)kZE, rows - e0);
  const int w4 = w >> 2;
  for (int x = threadIdx.x; x < ne * w4; x += 256) {
    const int e = x / w4, q = x - e * w4;
    reinterpret_cast<f32x4*>(zs)[e * w4 + q] =
        *reinterpret_cast<const f32x4*>(Z + (e0 + e) * w + 4 * q);
  }
  __syncthreads();
  const int el = threadIdx.x >> 4, c = threadIdx.x & 15;
  const int k = c / U, uu = c - (c / U) * U;
  if (el >= ne) return;
  for (int us = 0; us < nus; ++us) {
    const int u = us * U + uu;
    Zf[((int64_t)us * rows + e0 + el) * 16 + c] = (k < d3 && u < mul1) ? zs[el * w + k * mul1 + u] : 0.f;
  }
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int64_t gmp_tp_z_fused_layout_floats(int64_t rows, int64_t d3, int64_t mul1) {
  if (d3 < 1 || d3 > 16 || rows < 0 || mul1 <= 0) return -1;
  const int64_t U = 16 / d3;
  return ceil_div(mul1, U) * rows * 16;
}

int gmp_tp_z_fused_layout_f32(const float* Z, int64_t rows, int64_t d3, int64_t mul1,
                              float* Zf, void* stream) {
  GMP_CHECK_ARG(rows >= 0 && d3 >= 1 && d3 <= 16 && mul1 > 0);
  const int64_t n = gmp_tp_z_fused_layout_floats(rows, d3, mul1);
  if (n == 0) return GMP_OK;
  GMP_CHECK_ARG(Z && Zf);
  const int U = (int)(16 / d3);
  GMP_CHECK_ARG((d3 * mul1) % 4 == 0 && d3 * mul1 * kZE * 4 <= 160 * 1024);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(Z) % 16 == 0);
  const int smem = (int)(d3 * mul1 * kZE * 4);
  int rc = hip_check(hipFuncSetAttribute((const void*)z_fused_layout_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  if (rc) return rc;
  z_fused_layout_kernel<<<(unsigned)ceil_div(rows, kZE), 256, smem, as_stream(stream)>>>(
      Z, rows, (int)d3, (int)mul1, U, (int)ceil_div(mul1, U), Zf);
  return launch_status();
}

int gmp_tp_node_fwd_fused_f32(int64_t n_recv, int64_t d3, int64_t mul1, int64_t H,
                              int64_t mul_out, const int64_t* eoff, const float* Zf,
                              int64_t zrows, const float* A, const void* Bf, float* C,
                              int64_t cldg, void* stream) {
  GMP_CHECK_ARG(n_recv >= 0 && mul1 > 0 && H > 0 && cldg > 0);
  if (!(d3 == 3 || d3 == 5 || d3 == 7)) return GMP_ERR_UNSUPPORTED;
  if (!(mul_out == 128 || mul_out == 64)) return GMP_ERR_UNSUPPORTED;
  if (mul1 % 32 != 0 || H % 32 != 0) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(mul1 * d3 <= (1 << 20) && H <= (1 << 16));
  if (n_recv == 0) return GMP_OK;
  GMP_CHECK_ARG(eoff && Zf && A && Bf && C && zrows >= 1);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(Bf) % 16 == 0 && reinterpret_cast<uintptr_t>(Zf) % 16 == 0);
  hipStream_t s = as_stream(stream);
  int rc = 0;
#define GMP_FF(DD, NB)                                                                        \
  {                                                                                           \
    auto k = tp_node_fwd_fused_kernel<DD, NB>;                                                \
    const int smem = 2 * FCfg<DD>::STG;                                                       \
    if ((rc = hip_check(hipFuncSetAttribute((const void*)k,                                   \
                                            hipFuncAttributeMaxDynamicSharedMemorySize, smem)))) \
      return rc;                                                                              \
    const int64_t tiles = ceil_div(n_recv, FCfg<DD>::RT);                                     \
    GMP_CHECK_ARG(tiles < (1LL << 31));                                                       \
    k<<<(unsigned)tiles, kFT, smem, s>>>((int)n_recv, (int)mul1, (int)H, eoff, Zf, zrows, A,  \
                                         static_cast<const unsigned short*>(Bf), C, cldg);    \
  }
  if (mul_out == 128) {
    if (d3 == 3) GMP_FF(3, 128) else if (d3 == 5) GMP_FF(5, 128) else GMP_FF(7, 128)
  } else {
    if (d3 == 3) GMP_FF(3, 64) else if (d3 == 5) GMP_FF(5, 64) else GMP_FF(7, 64)
  }
#undef GMP_FF
  return launch_status();
}

}  // extern "C"
