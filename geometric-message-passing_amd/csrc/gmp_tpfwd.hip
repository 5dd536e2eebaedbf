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

__device__ __forceinline__ void split3v(float x, unsigned short& h, unsigned short& m,
                                        unsigned short& l) {
  const bf16x2 bh = __builtin_convertvector(f32x2{x, 0.f}, bf16x2);
  const f32x2 r1 = f32x2{x, 0.f} - __builtin_convertvector(bh, f32x2);
  const bf16x2 bm = __builtin_convertvector(r1, bf16x2);
  const f32x2 r2 = r1 - __builtin_convertvector(bm, f32x2);
  const bf16x2 bl = __builtin_convertvector(r2, bf16x2);
  h = (unsigned short)(__builtin_bit_cast(unsigned, bh) & 0xffffu);
  m = (unsigned short)(__builtin_bit_cast(unsigned, bm) & 0xffffu);
  l = (unsigned short)(__builtin_bit_cast(unsigned, bl) & 0xffffu);
}
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

template <int D3>
struct FCfg {
  static constexpr int U = 16 / D3;          // channels u per step (U x d3 <= 16 MFMA rows)
  static constexpr int NC = U * D3;          // live S-MFMA rows (combos (k, u))
  static constexpr int RT = kFM / D3;        // receivers per workgroup
  static constexpr int ROWS = RT * D3;       // live GEMM rows
  static constexpr int NCH = (2 * RT + 7) / 8;  // S chains (receiver x 16-wide j block) per wave
  static constexpr int PF = NCH <= 3 ? 6 : 2;   // MFMA steps (4 edges each) of operands prefetched
  static constexpr int STG = U * 3 * kChunkB;   // LDS bytes of one step image (U chunks, 3 planes)
};

template <int D3, int NBW>
__global__ __launch_bounds__(kFT, 1) void tp_node_fwd_fused_kernel(
    int n_recv, int mul1, int H, const int64_t* __restrict__ eoff, const float* __restrict__ Z,
    const float* __restrict__ A, const unsigned short* __restrict__ Bf, float* __restrict__ C,
    int64_t cldg) {
  using F = FCfg<D3>;
  constexpr int U = F::U, RT = F::RT, NCH = F::NCH, PF = F::PF;
  constexpr int WN = NBW / 16, WM = 8 / WN, RTW = 4 / WM;  // wave grid; row tiles per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smf[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wm = wv / WN, wn = wv % WN;
  const int w = D3 * mul1;                  // z row width
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

  // chains of this wave: c = wv + 8 i -> receiver rho = c % RT, j block jb = c / RT
  int ce0[NCH], ce1[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = wv + 8 * i, rho = c % RT, n = n0 + rho;
    const bool live = c < 2 * RT && n < n_recv;
    ce0[i] = live ? (int)eoff[n] : 0;
    ce1[i] = live ? (int)eoff[n + 1] : 0;
  }
  // S-MFMA input row of this lane: combo li -> (k_in, uu_in)
  const int k_in = li / U, uu_in = li - (li / U) * U;
  const bool row_in = li < F::NC;

  // the tile's z / a rows through buffer descriptors (32-bit lane offsets from the tile's first
  // edge; a lane offset past the descriptor (kOobF) loads 0: absent edges and combos need no
  // branch or select).  Z has a pad row after the last edge: the last u step's combos past mul1
  // read at most U - 1 floats past a row (into its image chunks that are never consumed).
  const int nlast = min(n0 + RT, n_recv);
  const int64_t te0 = eoff[n0], te1 = eoff[nlast];
  const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(Z) + te0 * w, 0, (int)((te1 - te0 + 1) * w * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A) + te0 * H, 0, (int)((te1 - te0) * H * 4), 0x00020000);
  constexpr unsigned kOobF = 0x80000000u;
  unsigned zo[NCH][PF], ao[NCH][PF];  // byte offsets of this lane's operands of MFMA step t
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int jb = (wv + 8 * i) / RT;
#pragma unroll
    for (int t = 0; t < PF; ++t) {
      const int el = ce0[i] - (int)te0 + 4 * t + g;
      const bool ok = ce0[i] + 4 * t + g < ce1[i];
      zo[i][t] = (ok && row_in) ? (unsigned)(el * w + k_in * mul1 + uu_in) * 4u : kOobF;
      ao[i][t] = ok ? (unsigned)(el * H + jb * 16 + li) * 4u : kOobF;
    }
  }

  // step -> (bias?, u0, jc)
  auto step_u0 = [&](int s) { return s < NBS ? s * U : ((s - NBS) / HB) * U; };
  auto step_jc = [&](int s) { return s < NBS ? -1 : (s - NBS) % HB; };
  // original k chunk (the forward B plane order, k = u H + j, bias k = K1 + u) of chunk uu of
  // step s, or -1 when absent
  auto chunk_of = [&](int s, int uu) -> int64_t {
    if (s < NBS) {
      const int q = s * U + uu;
      return q < QB ? (K1 >> 5) + q : -1;
    }
    const int u = step_u0(s) + uu;
    return u < mul1 ? ((int64_t)u * H >> 5) + step_jc(s) : -1;
  };

  // ---- producer: S (or Sb) of step s into image buffer buf
  float zp[NCH][PF], ap[NCH][PF];  // prefetched operands of the first PF MFMA steps per chain
  auto prefetch = [&](int s) {
    if (s >= nsteps || s < NBS) return;
    const unsigned zs = 4u * step_u0(s), as = 128u * step_jc(s);
#pragma unroll
    for (int i = 0; i < NCH; ++i)
#pragma unroll
      for (int t = 0; t < PF; ++t) {
        zp[i][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zrs, zo[i][t] + zs, 0, 0));
        ap[i][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ars, ao[i][t] + as, 0, 0));
      }
  };
  auto produce = [&](int s, unsigned char* img) {
    if (s >= nsteps) return;
    if (s < NBS) {
      // bias chunks: Sb[(rho, k), u] by VALU; thread -> (row r = tid / 8, 4 u's)
      const int r = tid >> 3, u4 = 4 * (tid & 7);
      const int rho = r / D3, k = r - rho * D3, n = n0 + rho;
      const bool live = r < F::ROWS && n < n_recv;
      const int e0 = live ? (int)eoff[n] : 0, e1 = live ? (int)eoff[n + 1] : 0;
      for (int uu = 0; uu < U; ++uu) {
        const int q = s * U + uu;
        if (q >= QB) break;
        const float* zc = Z + k * mul1 + 32 * q + u4;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int e = e0; e < e1; ++e) acc += *reinterpret_cast<const f32x4*>(zc + (int64_t)e * w);
        unsigned p[3][2];
        split3p(f32x2{acc[0], acc[1]}, p[0][0], p[1][0], p[2][0]);
        split3p(f32x2{acc[2], acc[3]}, p[0][1], p[1][1], p[2][1]);
        if (r < kFM) {
          const int off = ioff(r, u4);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            *reinterpret_cast<u32x2*>(img + (uu * 3 + pl) * kChunkB + off) = u32x2{p[pl][0], p[pl][1]};
        }
      }
      return;
    }
    const unsigned zs = 4u * step_u0(s), as = 128u * step_jc(s);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = wv + 8 * i;
      if (c >= 2 * RT) break;  // wave-uniform
      const int rho = c % RT, jb = c / RT;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const int nq = (ce1[i] - ce0[i] + 3) >> 2;
#pragma unroll
      for (int t = 0; t < PF; ++t)
        if (t < nq) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(zp[i][t], ap[i][t], acc, 0, 0, 0);
      for (int t = PF; t < nq; ++t) {  // in-degree > 4 PF: the rest directly
        const int el = ce0[i] - (int)te0 + 4 * t + g;
        const bool ok = ce0[i] + 4 * t + g < ce1[i];
        const unsigned zv = ok && row_in ? (unsigned)(el * w + k_in * mul1 + uu_in) * 4u + zs : kOobF;
        const unsigned av = ok ? (unsigned)(el * H + jb * 16 + li) * 4u + as : kOobF;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(zrs, zv, 0, 0)),
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ars, av, 0, 0)), acc,
            0, 0, 0);
      }
      // lane (li, g): S[combo m = 4 g + q][j = jb 16 + li] -> image chunk uu, row rho d3 + k;
      // pairs of values split together (one f32x2 pass), written as 16-bit halves
      unsigned ph[2], pm[2], pl[2];
      split3p(f32x2{acc[0], acc[1]}, ph[0], pm[0], pl[0]);
      split3p(f32x2{acc[2], acc[3]}, ph[1], pm[1], pl[1]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = 4 * g + q;
        if (m < F::NC) {
          const int k = m / U, uu = m - (m / U) * U;
          const int sh = 16 * (q & 1);
          unsigned char* base = img + uu * 3 * kChunkB + ioff(rho * D3 + k, jb * 16 + li);
          *reinterpret_cast<unsigned short*>(base) = (unsigned short)(ph[q >> 1] >> sh);
          *reinterpret_cast<unsigned short*>(base + kChunkB) = (unsigned short)(pm[q >> 1] >> sh);
          *reinterpret_cast<unsigned short*>(base + 2 * kChunkB) = (unsigned short)(pl[q >> 1] >> sh);
        }
      }
    }
  };

  // ---- consumer: GEMM over the U chunks of the step in image buffer img, B fragments of the
  // whole step in registers (loaded during the previous step, BEFORE that step's z / a
  // prefetch: vector-memory counts complete in issue order, so the MFMAs wait only for B)
  f32x4 acc[RTW];
#pragma unroll
  for (int r = 0; r < RTW; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ct = wn;  // this wave's 16-column tile
  // B planes through a descriptor: the lane / column-tile part of the offset is fixed, the chunk
  // part is wave-uniform (scalar offset): no per-load address arithmetic
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(Bf), 0, 0x7fffffff, 0x00020000);
  const unsigned bvo = 16u * lane + (unsigned)ct * 3u * 1024u;
  u32x4 bst[U][3];
  auto load_b_step = [&](int s) {
#pragma unroll
    for (int uu = 0; uu < U; ++uu) {
      int64_t ch = s < nsteps ? chunk_of(s, uu) : -1;
      if (ch < 0) ch = 0;  // absent chunk: a valid address, never consumed
      const int so = (int)(ch * ct_total * 3 * 1024);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bst[uu][p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(brs, bvo, so + p * 1024, 0));
    }
  };
  auto consume = [&](int s, const unsigned char* img) {
#pragma unroll
    for (int uu = 0; uu < U; ++uu) {
      if (chunk_of(s, uu) < 0) break;  // absent chunks are the step's last ones (wave-uniform)
      const unsigned char* cimg = img + uu * 3 * kChunkB;
#pragma unroll
      for (int r = 0; r < RTW; ++r) {
        const int off = ioffc(16 * (wm * RTW + r) + li, g);
        u32x4 a[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const u32x4*>(cimg + p * kChunkB + off);
        f32x4 t = acc[r];
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[2]), asb(bst[uu][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[1]), asb(bst[uu][1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[0]), asb(bst[uu][2]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[1]), asb(bst[uu][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[0]), asb(bst[uu][1]), t, 0, 0, 0);
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[0]), asb(bst[uu][0]), t, 0, 0, 0);
      }
    }
  };

  __syncthreads();  // zeroed images
  prefetch(0);
  produce(0, smf);
  load_b_step(0);
  prefetch(1);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    unsigned char* cur = smf + (s & 1) * F::STG;
    unsigned char* nxt = smf + ((s + 1) & 1) * F::STG;
    consume(s, cur);
    __builtin_amdgcn_sched_barrier(0);
    produce(s + 1, nxt);      // its operands were prefetched a whole step ago
    __builtin_amdgcn_sched_barrier(0);
    load_b_step(s + 1);       // B of the next step first,
    __builtin_amdgcn_sched_barrier(0);
    prefetch(s + 2);          // then the z / a operands of the step after it
    __syncthreads();
  }

  // epilogue: row (rho, k) of receiver n0 + rho, column w' -> out[n, w' d3 + k] (+=)
#pragma unroll
  for (int r = 0; r < RTW; ++r) {
    const int col = 16 * ct + li;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * (wm * RTW + r) + 4 * g + q;
      const int rho = row / D3, k = row - rho * D3;
      if (row < F::ROWS && n0 + rho < n_recv) C[(int64_t)(n0 + rho) * cldg + col * D3 + k] += acc[r][q];
    }
  }
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_tp_node_fwd_fused_f32(int64_t n_recv, int64_t d3, int64_t mul1, int64_t H,
                              int64_t mul_out, const int64_t* eoff, const float* Z,
                              const float* A, const void* Bf, float* C, int64_t cldg,
                              void* stream) {
  GMP_CHECK_ARG(n_recv >= 0 && mul1 > 0 && H > 0 && cldg > 0);
  if (!(d3 == 3 || d3 == 5 || d3 == 7)) return GMP_ERR_UNSUPPORTED;
  if (!(mul_out == 128 || mul_out == 64)) return GMP_ERR_UNSUPPORTED;
  if (mul1 % 32 != 0 || H % 32 != 0) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(mul1 * d3 <= (1 << 20) && H <= (1 << 16));
  if (n_recv == 0) return GMP_OK;
  GMP_CHECK_ARG(eoff && Z && A && Bf && C);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(Bf) % 16 == 0 && reinterpret_cast<uintptr_t>(Z) % 16 == 0);
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
    k<<<(unsigned)tiles, kFT, smem, s>>>((int)n_recv, (int)mul1, (int)H, eoff, Z, A,          \
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
