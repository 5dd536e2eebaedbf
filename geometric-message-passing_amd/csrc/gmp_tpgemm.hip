// K7g: the path GEMMs of the receiver-factorised tensor-product convolution (gmp_tp.hip "node
// form", tfn_layer.py:73-87 regrouped) on the bf16 MFMA through exact three-plane splits:
//
//   forward   out[(n,k), w] += sum_{u,j} S[(n,k), (u,j)] W2p[(u,j), w] + sum_u Sb[(n,k), u] b2p[u, w]
//   backward  T[(n,k), (u,j)] = sum_w G[(n,k), w] W2p[(u,j), w]
//
// as one kernel C (+)= A B^T with A f32 (M x K, split on load) and B pre-split into three bf16
// planes [3][N][K] (gmp_tp_split_w2_f32, once per pass).  Every f32 operand x = x0 + x1 + x2
// exactly (RNE splits), and C accumulates the six plane products of order <= 2^-16,
// A2 B0 + A1 B1 + A0 B2 + A1 B0 + A0 B1 + A0 B0, in f32 (dropped terms <= 2^-26 |ab|; the same
// arithmetic as the K5 edge outer sums, gmp_wgrad.hip, measured f32-class there).  Six
// v_mfma_f32_16x16x32_bf16 (16 cycles each) replace eight v_mfma_f32_16x16x4_f32 (32 cycles)
// per 32-deep k step of a 16 x 16 tile: 2.7x less matrix time than the f32 MFMA (1/16 of the
// bf16 rate on gfx950, no xf32).
//
// Tiling: 512 threads (8 waves as 2 (M) x 4 (N)), a 128 x 128 output tile per workgroup, one
// 32-deep k stage per step, wave tile 64 x 32 (4 x 2 MFMA tiles).  LDS image per stage: A and B
// as [plane][row][32 k] bf16 (64-byte rows, 16-byte chunk q at q ^ ((row >> 1) & 3)): the MFMA
// operand read (row = lane & 15, k = 8 (lane >> 4) .. +7) is one conflict-free ds_read_b128.
// Loads run two stages ahead in a register ring (no branches: clamped addresses, masked in the
// stash), two LDS stages (96 KB, one workgroup per CU).  Tiles are grouped (8 M tiles per group,
// N tiles inside a group) and dealt XCD-contiguously so workgroups that share an operand block
// share an L2.  A second A operand (A2, K2 columns) continues the k range: the bias term of the
// forward rides in the same accumulators.  The epilogue stores C at
//   (r / cgrp) * cldg + (r % cgrp) * cldr + col * cldn
// so the forward adds its (n, k)-row result straight into the receivers' mul_ir output block
// (row stride out_dim, k stride 1, w stride 2lo+1) and the backward writes row-major T.
//
// H2 form (NP = 2, gmp_tp_*_h2_f32): the same kernels over TWO fp16 planes (x = hi + lo,
// 22-bit operands) of the operands scaled by powers of two — B by 2^sb from max |W2p|, A by a
// per-ROW 2^sa(r) (the forward GEMM: from the S kernel's per-wave row-block maxima, max over
// the row's `nparts` words; the widen kernel: one device-side max |G| word) — with three
// products lo*hi + hi*lo + hi*hi per k step (dropped lo*lo ~2^-22 relative) and each output
// row scaled back by 2^-(sa(r) + sb) (exact) in the epilogue: half the MFMAs, two thirds of the
// LDS image and of the split arithmetic of the x3 form.  Per-row scales keep every row at
// 22-bit precision relative to its own magnitude (a launch-wide scale did not: rows far below
// the launch max lost bits and the C4 1M-edge rotation-invariance bound failed).
#include "gmp_common.h"

namespace gmp {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kGT = 512;               // threads (8 waves)
constexpr int kBM = 128, kBN = 128;    // output tile
constexpr int kBK = 32;                // k per stage (= the bf16 MFMA k)
constexpr int kPlane = 128 * 64;       // bytes of one plane image (128 rows x 32 bf16)
constexpr int kGroupM = 8;             // M tiles per tile group

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

// H2: hi / lo fp16 planes of x (already scaled): x = hi + lo to 22 bits
__device__ __forceinline__ void split2h(f32x2 x, unsigned& h, unsigned& l) {
  const h16x2 hh = __builtin_convertvector(x, h16x2);
  const f32x2 r = x - __builtin_convertvector(hh, f32x2);  // exact
  const h16x2 hl = __builtin_convertvector(r, h16x2);
  h = __builtin_bit_cast(unsigned, hh);
  l = __builtin_bit_cast(unsigned, hl);
}

// exponent s with max 2^s < 2^15 (fp16 range with headroom) from a max |x| bit pattern
__device__ __forceinline__ int scale_exp_bits(unsigned mx_bits) {
  const float mx = __uint_as_float(mx_bits);
  if (!(mx > 0.f) || !(mx < 3.0e38f)) return 0;
  int e;
  (void)frexpf(mx, &e);
  const int s = 15 - e;
  return s < -60 ? -60 : (s > 60 ? 60 : s);
}

// per-row A exponent of the H2 forward GEMM: as scale_exp_bits with a +-120 range (applied and
// undone with v_ldexp, so sa + sb never has to be a representable power of two)
__device__ __forceinline__ int row_exp(float mx) {
  if (!(mx > 0.f) || !(mx < 3.0e38f)) return 0;
  int e;
  (void)frexpf(mx, &e);
  const int s = 15 - e;
  return s < -120 ? -120 : (s > 120 ? 120 : s);
}

// split of 4 f32 into NP planes (x3: bf16 hi / mid / lo; H2: fp16 hi / lo of x * fs)
template <int NP>
__device__ __forceinline__ void split_planes(f32x4 v, float fs, unsigned (&p)[3][2]) {
  if constexpr (NP == 3) {
    split3(f32x2{v[0], v[1]}, p[0][0], p[1][0], p[2][0]);
    split3(f32x2{v[2], v[3]}, p[0][1], p[1][1], p[2][1]);
  } else {
    split2h(f32x2{v[0] * fs, v[1] * fs}, p[0][0], p[1][0]);
    split2h(f32x2{v[2] * fs, v[3] * fs}, p[0][1], p[1][1]);
    p[2][0] = p[2][1] = 0u;
  }
}

__device__ __forceinline__ int xoff(int row, int chunk) {
  return row * 64 + 16 * (chunk ^ ((row >> 1) & 3));
}

// One k step's MFMA operands of a wave (64 x 32 output block: 4 row tiles x 2 column tiles,
// three bf16 planes each).  The main loops hold two of them: the fragments of step s + 1 are
// read from LDS while the MFMAs of step s run (one barrier per step).
template <int NP>
struct Frag {
  u32x4 a[4][NP];
  u32x4 b[2][NP];
};

template <int NP>
__device__ __forceinline__ void load_frag(Frag<NP>& f, const unsigned char* aimg,
                                          const unsigned char* bimg, int wm, int wn, int li,
                                          int g) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int off = xoff(64 * wm + 16 * r + li, g);
#pragma unroll
    for (int p = 0; p < NP; ++p) f.a[r][p] = *reinterpret_cast<const u32x4*>(aimg + p * kPlane + off);
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int off = xoff(32 * wn + 16 * c + li, g);
#pragma unroll
    for (int p = 0; p < NP; ++p) f.b[c][p] = *reinterpret_cast<const u32x4*>(bimg + p * kPlane + off);
  }
}

__device__ __forceinline__ bf16x8 asb(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ h16x8 ash(u32x4 v) { return __builtin_bit_cast(h16x8, v); }

// acc += A B over one 32-deep step, smallest products first: x3 the six bf16 plane products,
// H2 the three fp16 ones
template <int NP>
__device__ __forceinline__ void mma_np(f32x4 (&acc)[4][2], const Frag<NP>& f) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      f32x4 t = acc[r][c];
      if constexpr (NP == 3) {
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][2]), asb(f.b[c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][1]), asb(f.b[c][1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][0]), asb(f.b[c][2]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][1]), asb(f.b[c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][0]), asb(f.b[c][1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][0]), asb(f.b[c][0]), t, 0, 0, 0);
      } else {
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ash(f.a[r][1]), ash(f.b[c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ash(f.a[r][0]), ash(f.b[c][1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ash(f.a[r][0]), ash(f.b[c][0]), t, 0, 0, 0);
      }
      acc[r][c] = t;
    }
  }
}

// The forward kernel's B operand comes straight from global memory in MFMA fragment order
// (gmp_tp_split_w2_f32 writes it so): one 16-byte load per lane per (column tile, plane) and
// k step, no LDS image.  Element (plane p, column n, k) of an N-column, K-deep operand sits at
//   ((((k / 32) * (N / 16) + n / 16) * NP + p) * 64 + n % 16 + 16 * ((k % 32) / 8)) * 8 + k % 8
// (ushort units): lane l of the (k step, column tile, plane) block holds B[16 ct + l % 16]
// [32 ks + 8 (l / 16) .. + 7], exactly the B operand of v_mfma_f32_16x16x32_{bf16,f16}.
__host__ __device__ __forceinline__ int64_t bfrag_index(int64_t p, int64_t n, int64_t k,
                                                        int64_t ct_total, int np) {
  return ((((k >> 5) * ct_total + (n >> 4)) * np + p) * 64 + (n & 15) + 16 * ((k & 31) >> 3)) *
             8 + (k & 7);
}
template <int NP>
struct FragA {
  u32x4 a[4][NP];
};
template <int NP>
__device__ __forceinline__ void load_frag_a(FragA<NP>& f, const unsigned char* aimg, int wm,
                                            int li, int g) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int off = xoff(64 * wm + 16 * r + li, g);
#pragma unroll
    for (int p = 0; p < NP; ++p) f.a[r][p] = *reinterpret_cast<const u32x4*>(aimg + p * kPlane + off);
  }
}
template <int NP>
__device__ __forceinline__ void mma_ab(f32x4 (&acc)[4][2], const FragA<NP>& f,
                                       const u32x4 (&b)[2][NP]) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      f32x4 t = acc[r][c];
      if constexpr (NP == 3) {
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][2]), asb(b[c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][1]), asb(b[c][1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][0]), asb(b[c][2]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][1]), asb(b[c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][0]), asb(b[c][1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(f.a[r][0]), asb(b[c][0]), t, 0, 0, 0);
      } else {
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ash(f.a[r][1]), ash(b[c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ash(f.a[r][0]), ash(b[c][1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ash(f.a[r][0]), ash(b[c][0]), t, 0, 0, 0);
      }
      acc[r][c] = t;
    }
  }
}

// H2 scale factors of a launch: x A by 2^sa before the split, results by 2^-(sa + sb)
struct H2Scale {
  float fa, down;
};
template <int NP>
__device__ __forceinline__ H2Scale h2_scale(const unsigned* amax, const unsigned* wmax) {
  if constexpr (NP == 3) {
    return H2Scale{1.f, 1.f};
  } else {
    const int sa = scale_exp_bits(amax[0]), sb = scale_exp_bits(wmax[0]);
    return H2Scale{ldexpf(1.f, sa), ldexpf(1.f, -(sa + sb))};
  }
}

// The forward kernel in two tile shapes: WGM = 2 (waves 2 (M) x 4 (N), a 128 x 128 output tile:
// mul_out = 128) and WGM = 4 (waves 4 x 2, a 256 x 64 tile: the 64-channel paths of config C5,
// which a 128-column tile would run with half of its MFMAs on zero B columns).  The wave tile is
// 64 x 32 in both; the A stage image holds BM = 64 WGM rows.
template <bool ACC, int RA, int RBB, int WGM>
__global__ __launch_bounds__(kGT, 1) void tp_gemm_x3_kernel(
    int64_t M, int N, int64_t K1, const float* __restrict__ A1, int64_t lda1, int64_t K2,
    const float* __restrict__ A2, int64_t lda2, const unsigned short* __restrict__ Bp,
    int64_t ldb, int64_t bplane, float* __restrict__ C, int64_t cgrp, int64_t cldg,
    int64_t cldr, int64_t cldn, int tiles_m, int tiles_n, const float* __restrict__ bias,
    int prio) {
  constexpr int NP = 3;
  constexpr int WGN = 8 / WGM;              // waves along N
  constexpr int BM = 64 * WGM, BN = 32 * WGN;
  constexpr int PL = BM * 64;               // bytes of one plane image (BM rows x 32 bf16)
  constexpr int STG = NP * PL;              // LDS bytes per stage (A planes; B skips LDS)
  constexpr int AU = BM / 64;               // A load units (row, float4) per thread and stage
  extern __shared__ __attribute__((aligned(16))) unsigned char smg[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wm = w / WGN, wn = w % WGN;

  // XCD-contiguous logical id (blocks b, b + 8, ... share an XCD under round-robin dealing;
  // speed only), then grouped tile order
  const int64_t nwg = (int64_t)tiles_m * tiles_n;
  int64_t L;
  {
    const int64_t b = blockIdx.x, x = b & 7, q = nwg >> 3, r = nwg & 7;
    L = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  const int64_t per_group = (int64_t)kGroupM * tiles_n;
  const int64_t grp = L / per_group;
  const int64_t first_m = grp * kGroupM;
  const int64_t gsize = (tiles_m - first_m) < kGroupM ? (tiles_m - first_m) : kGroupM;
  const int64_t in_grp = L - grp * per_group;
  const int64_t tm = first_m + in_grp % gsize, tn = in_grp / gsize;
  const int64_t m0 = tm * BM, n0 = tn * BN;

  const int64_t Ktot = K1 + K2;
  const int nst = (int)(Ktot / kBK);

  // loaders: A units (AU per thread) = (row, float4 of k); B straight into registers
  int arow_[AU], akq[AU];
  bool aok[AU];
  const float* abase1[AU];
  const float* abase2[AU];
#pragma unroll
  for (int q = 0; q < AU; ++q) {
    const int v = tid + kGT * q;
    arow_[q] = v >> 3;
    akq[q] = v & 7;
    const int64_t gr = m0 + arow_[q];
    aok[q] = gr < M;
    const int64_t grc = gr < M ? gr : M - 1;
    abase1[q] = A1 + grc * lda1 + 4 * akq[q];
    abase2[q] = A2 ? A2 + grc * lda2 + 4 * akq[q] : abase1[q];
  }
  // this wave's two B column tiles (fragment order) through a buffer descriptor: a tile past N
  // gets an out-of-range offset (loads zeros, no select); the stage part of the offset is
  // wave-uniform
  const int64_t ct_total = N / 16;
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(Bp), 0, 0x7fffffff, 0x00020000);
  unsigned boff[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int64_t ct = (n0 >> 4) + 2 * wn + c;
    boff[c] = ct < ct_total ? (unsigned)((ct * NP * 512 + 8 * lane) * 2) : 0x80000000u;
  }

  // A ring: RA register slots (slot t % RA holds stage t); a stage's loads are issued RA
  // iterations before its split + LDS write.  RA = 2 kept 32 KB of the A stream (the S rows) in
  // flight per CU; measured at the MACE-128 lo = 2 shape (scripts/mb_tpgemm.py): RA = 2 11.33 ms,
  // 4 10.74 ms, 8 10.55 ms (230 VGPRs, no scratch) -- the A stream was only part of the limit.
  static_assert(RA % RBB == 0, "the unrolled loop indexes both rings statically");
  f32x4 ringA[RA][AU];
  u32x4 ringB[RBB][2][NP];  // B (W2p planes, from the Infinity Cache): RBB steps ahead
  auto fetch = [&](int slot, int st) {
    const int stc = st < nst ? st : nst - 1;
    const int64_t k0 = (int64_t)stc * kBK;
#pragma unroll
    for (int q = 0; q < AU; ++q) {
      const float* p = k0 < K1 ? abase1[q] + k0 : abase2[q] + (k0 - K1);
      ringA[slot][q] = *reinterpret_cast<const f32x4*>(p);
    }
  };
  auto fetch_b = [&](int slot, int st) {
    const int64_t stc = st < nst ? st : nst - 1;
    const int so = (int)(stc * ct_total * NP * 512 * 2);  // bytes, wave-uniform
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        ringB[slot][c][p] = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(brs, boff[c], so + p * 1024, 0));
  };
  auto stash = [&](int slot, unsigned char* buf, int st) {
    const bool live = st < nst;
#pragma unroll
    for (int q = 0; q < AU; ++q) {
      f32x4 v = ringA[slot][q];
      if (!(live && aok[q])) v = f32x4{0.f, 0.f, 0.f, 0.f};
      unsigned pl[3][2];
      split_planes<NP>(v, 1.f, pl);
      const int off = xoff(arow_[q], akq[q] >> 1) + 8 * (akq[q] & 1);
#pragma unroll
      for (int p = 0; p < NP; ++p)
        *reinterpret_cast<u32x2*>(buf + p * PL + off) = u32x2{pl[p][0], pl[p][1]};
    }
  };
  auto load_a = [&](FragA<NP>& f, const unsigned char* aimg) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int off = xoff(64 * wm + 16 * r + li, g);
#pragma unroll
      for (int p = 0; p < NP; ++p)
        f.a[r][p] = *reinterpret_cast<const u32x4*>(aimg + p * PL + off);
    }
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r][0] = acc[r][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Pipeline (stage t's A registers in ring slot t & 1, its LDS image in buffer t & 1; its B
  // fragments in ringB[t & 1], loaded two stages ahead):
  //   iteration s: split + write A of stage s + 2 into the buffer stage s used (its fragments
  //   are in registers, read before the last barrier) | load A of s + 4 | read the A fragments
  //   of s + 1 | MFMAs of s | load B of s + 2 into the slot they read | barrier.
  // Stages past nst load clamped addresses; their A is stashed as zeros.
  const int nst_pad = (nst + RA - 1) / RA * RA;
  FragA<NP> F[2];
#pragma unroll
  for (int q = 0; q < RA; ++q) fetch(q, q);
#pragma unroll
  for (int q = 0; q < RBB; ++q) fetch_b(q, q);
  stash(0, smg, 0);
  fetch(0, RA);
  stash(1, smg + STG, 1);
  fetch(1, RA + 1);
  __syncthreads();
  load_a(F[0], smg);
  __syncthreads();  // every wave holds stage 0's fragments: buffer 0 may be rewritten
  // optional static priority for the second-dispatched half (MI355X_MICROARCH.md, two waves per
  // SIMD, item 4); kGemmPrio
  if ((prio & 1) && w >= 4) __builtin_amdgcn_s_setprio(1);
  // prio bit 1 (A/B): waves 4-7, the SIMD partners of waves 0-3, run each stage's MFMAs before
  // its split / LDS stash, so one wave of a SIMD pair splits while the other multiplies
  const bool late = (prio & 2) && w >= 4;
  for (int s0 = 0; s0 < nst_pad; s0 += RA) {
#pragma unroll
    for (int j = 0; j < RA; ++j) {
      const int st = s0 + j;
      const int sl = (j + 2) % RA;  // ring slot of stage st + 2
      const unsigned char* nb = smg + ((st + 1) & 1) * STG;
      // sched barriers pin the ring discipline: slot sl's registers are consumed by the stash
      // before its next loads are issued, so the stash waits only for loads RA stages old
      // (counted vmcnt) instead of the scheduler hoisting the new loads and draining vmcnt(0)
      if (!late) {
        stash(sl, smg + (st & 1) * STG, st + 2);
        __builtin_amdgcn_sched_barrier(0);
        fetch(sl, st + 2 + RA);
        __builtin_amdgcn_sched_barrier(0);
      }
      load_a(F[(j & 1) ^ 1], nb);
      mma_ab<NP>(acc, F[j & 1], ringB[j % RBB]);
      __builtin_amdgcn_sched_barrier(0);
      fetch_b(j % RBB, st + RBB);  // the slot the MFMAs above just read: RBB stages of lead
      if (late) {  // (the stash writes the buffer stage st used: its fragments are in registers)
        __builtin_amdgcn_sched_barrier(0);
        stash(sl, smg + (st & 1) * STG, st + 2);
        __builtin_amdgcn_sched_barrier(0);
        fetch(sl, st + 2 + RA);
      }
      __syncthreads();
    }
  }

  // C/D map of 16x16x32: col = lane & 15, row = 4 (lane >> 4) + q
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int64_t col = n0 + 32 * wn + 16 * c + li;
      if (col >= N) continue;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int lr = 64 * wm + 16 * r + 4 * g + q;
        const int64_t row = m0 + lr;
        if (row >= M) continue;
        const int64_t grp_r = row / cgrp;
        float* dst = C + grp_r * cldg + (row - grp_r * cgrp) * cldr + col * cldn;
        if (ACC) *dst += acc[r][c][q] + bv;
        else *dst = acc[r][c][q] + bv;
      }
    }
  }
}

// Short-K, wide-N form (the backward T = G W2p^T: K = mul_out <= 128, N = mul1 H ~ 32k): the
// workgroup splits its 128-row block of A ONCE into LDS (K / 32 resident stage images) and sweeps
// a range of 128-column tiles, streaming only B (two LDS stages, register ring two stages
// ahead across tile boundaries); after each tile's K / 32 steps the accumulators go out with
// non-temporal stores (T is consumed by a later kernel, far past the caches) and restart.
// Replaces one workgroup per 128 x 128 tile, whose prologue / epilogue dominated at 4 k steps.
constexpr int kMaxKS = 4;  // K <= 128
constexpr int kParkLd = 36;  // widen epilogue LDS slab row stride (floats): 32 + 4
template <int NKS, int NP, int RB>
__global__ __launch_bounds__(kGT, 1) void tp_gemm_x3_widen_kernel(
    int64_t M, int64_t N, const float* __restrict__ A, int64_t lda,
    const unsigned short* __restrict__ Bp, int64_t ldb, int64_t bplane, float* __restrict__ C,
    int64_t ldc, int tiles_m, int tiles_n, int n_split, const unsigned* __restrict__ amax,
    const unsigned* __restrict__ wmax) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smw[];
  unsigned char* sA = smw;  // NKS x NP planes (B goes straight to registers, fragment order)
  const H2Scale hs = h2_scale<NP>(amax, wmax);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wm = w >> 2, wn = w & 3;
  // XCD-contiguous logical id; M tile fastest so the n_split workgroups of neighbouring M tiles
  // that stream the same B columns run side by side
  const int64_t nwg = (int64_t)tiles_m * n_split;
  int64_t L;
  {
    const int64_t b = blockIdx.x, x = b & 7, q = nwg >> 3, r = nwg & 7;
    L = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  const int64_t tm = L % tiles_m, sp = L / tiles_m;
  const int64_t m0 = tm * kBM;
  const int64_t per = (tiles_n + n_split - 1) / n_split;
  const int64_t t0 = sp * per, t1 = (t0 + per < tiles_n) ? t0 + per : tiles_n;
  if (t0 >= t1) return;

  // A block -> resident split planes (rows beyond M are zero)
#pragma unroll
  for (int q = 0; q < NKS * 2; ++q) {
    const int v = tid + kGT * q;                 // (stage, row, float4)
    const int st = v >> 10, row = (v >> 3) & 127, kq = v & 7;
    const int64_t gr = m0 + row;
    f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
    if (gr < M) x = *reinterpret_cast<const f32x4*>(A + gr * lda + 32 * st + 4 * kq);
    unsigned pl[3][2];
    split_planes<NP>(x, hs.fa, pl);
    unsigned char* img = sA + st * NP * kPlane;
    const int off = xoff(row, kq >> 1) + 8 * (kq & 1);
#pragma unroll
    for (int p = 0; p < NP; ++p)
      *reinterpret_cast<u32x2*>(img + p * kPlane + off) = u32x2{pl[p][0], pl[p][1]};
  }

  const int nst = (int)((t1 - t0) * NKS);
  const int64_t ct_total = N / 16;
  const unsigned short* bl = Bp + 8 * lane;
  // B ring: RB register slots (slot gs % RB holds step gs), loaded RB steps ahead (W2p's planes,
  // 25 MB at the MACE-128 shape, stream from the Infinity Cache, not L2).  Measured at the lo = 2
  // shape: RB = 2 11.70 ms, RB = 4 11.41 ms (238 VGPRs, no scratch); MACE 2314 -> 2278 ms/step
  u32x4 ringB[RB][2][NP];
  // B fragments of global step gs (tile t0 + gs / NKS, k step gs % NKS) for this wave's two
  // column tiles.  Steps past the range and tiles past N read a clamped (valid, finite) block
  // WITHOUT masking: their products land in accumulators that are never stored (columns >= N,
  // or the padded steps after the last tile's store, whose accumulators are discarded).  r05
  // zeroed them with a select after each load; the compiler placed those selects at the
  // unrolled loop's latch, so every RB steps the wave waited for all its B loads (vmcnt(0)) and
  // the ring prefetched almost nothing: MACE-128 lo = 2 shape 11.60 -> 10.68 ms without them.
  auto fetch_b = [&](int slot, int gs) {
    const int gsc = gs < nst ? gs : nst - 1;
    const int64_t ks = gsc % NKS;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int64_t ct = (t0 + gsc / NKS) * (kBN / 16) + 2 * wn + c;
      const int64_t ctc = ct < ct_total ? ct : ct_total - 1;
#pragma unroll
      for (int p = 0; p < NP; ++p)
        ringB[slot][c][p] = *reinterpret_cast<const u32x4*>(bl + ((ks * ct_total + ctc) * NP + p) * 512);
    }
  };
  f32x4 acc[4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r][0] = acc[r][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // epilogue through a wave-private LDS slab (16 rows x 32 columns per row tile): the
  // accumulators (lane: 4 rows of one column) are parked, then leave as whole 128-byte row
  // segments, 16 bytes per lane (direct 4-byte stores of the accumulator layout wrote 64-byte
  // pieces with the non-temporal hint: 2.5-3.2 TB/s of T at the TFN / MACE shapes)
  float* park = reinterpret_cast<float*>(smw + NKS * NP * kPlane) + w * (16 * kParkLd);
  const bool vec_st = (ldc % 4 == 0) && (N % 4 == 0) && (reinterpret_cast<uintptr_t>(C) % 16 == 0);
  auto store_tile = [&](int64_t tn) {
    const int64_t c0 = tn * kBN + 32 * wn;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          park[(4 * g + q) * kParkLd + 16 * c + li] =
              NP == 3 ? acc[r][c][q] : acc[r][c][q] * hs.down;
        acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      __builtin_amdgcn_wave_barrier();  // park is wave-private
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rr = 8 * h + (lane >> 3), c4 = 4 * (lane & 7);
        const int64_t row = m0 + 64 * wm + 16 * r + rr;
        const f32x4 v = *reinterpret_cast<const f32x4*>(park + rr * kParkLd + c4);
        if (row < M && c0 + c4 < N) {
          float* dst = C + row * ldc + c0 + c4;
          if (vec_st) {
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));
          } else {  // unaligned rows (ldc % 4 != 0) or a ragged last column group
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (c0 + c4 + e < N) __builtin_nontemporal_store(v[e], dst + e);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  };

  // over the global step index gs: A fragments from the resident images (read one step ahead),
  // B fragments from global memory two steps ahead (into the ring slot the MFMAs just read);
  // nothing is written to LDS after the A images, so the loop has no barrier
  FragA<NP> F[2];
#pragma unroll
  for (int q = 0; q < RB; ++q) fetch_b(q, q);
  __syncthreads();  // A images
  load_frag_a<NP>(F[0], sA, wm, li, g);
  const int nst_pad = (nst + RB - 1) / RB * RB;
  for (int s0 = 0; s0 < nst_pad; s0 += RB) {
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int gs = s0 + j;
      load_frag_a<NP>(F[(j & 1) ^ 1], sA + ((gs + 1) % NKS) * NP * kPlane, wm, li, g);
      mma_ab<NP>(acc, F[j & 1], ringB[j]);
      __builtin_amdgcn_sched_barrier(0);
      fetch_b(j, gs + RB);
      if (gs < nst && gs % NKS == NKS - 1) store_tile(t0 + gs / NKS);
    }
  }
}

// Planes of one path's second radial Linear block (W2 rows (u, w), H columns; b2 (u, w)):
//   Bf[p][w][u H + j] = W2[(u mo + w), j],  Bf[p][w][mul1 H + u] = b2[u mo + w]   (forward B)
//   Bt[p][u H + j][w] = W2[(u mo + w), j]                                         (backward B)
// grid (H / 64, mul1), 256 threads: the (mo x 64) block of W2 rows u mo .. u mo + mo - 1,
// columns j0 .. j0 + 63 goes through LDS (transpose for Bf); Bt rows are written directly.
// (NP = 2: hi / lo fp16 planes of the values scaled by 2^sb, sb from *wmax = max |W2p|, |b2p|)
template <int NP>
__device__ __forceinline__ void split1(float v, float fs, unsigned (&p)[3]) {
  if constexpr (NP == 3) {
    split3(f32x2{v, 0.f}, p[0], p[1], p[2]);
  } else {
    split2h(f32x2{v * fs, 0.f}, p[0], p[1]);
    p[2] = 0u;
  }
}
template <int NP>
__global__ __launch_bounds__(256) void tp_split_w2_kernel(int mul1, int mo, int H,
                                                          const float* __restrict__ W2,
                                                          const float* __restrict__ b2,
                                                          unsigned short* __restrict__ Bf,
                                                          unsigned short* __restrict__ Bt,
                                                          const unsigned* __restrict__ wmax) {
  __shared__ float tile[128][65];
  const float fs = NP == 3 ? 1.f : ldexpf(1.f, scale_exp_bits(wmax ? wmax[0] : 0u));
  const int u = blockIdx.y, j0 = blockIdx.x * 64, tid = threadIdx.x;
  const int64_t K1 = (int64_t)mul1 * H;
  for (int x = tid; x < mo * 64; x += 256) {
    const int wr = x >> 6, j = x & 63;
    const float v = (j0 + j < H) ? W2[((int64_t)u * mo + wr) * H + j0 + j] : 0.f;
    tile[wr][j] = v;
  }
  __syncthreads();
  // Bf[p][w][u H + j0 + j]: rows w, 64 consecutive k
  for (int x = tid; Bf && x < mo * 64; x += 256) {
    const int wr = x >> 6, j = x & 63;
    if (j0 + j >= H) continue;
    unsigned p[3];
    split1<NP>(tile[wr][j], fs, p);
#pragma unroll
    for (int q = 0; q < NP; ++q)
      Bf[bfrag_index(q, wr, (int64_t)u * H + j0 + j, mo / 16, NP)] = (unsigned short)p[q];
  }
  if (Bt) {  // Bt[p][u H + j0 + j][w]: rows k, mo consecutive w
    for (int x = tid; x < mo * 64; x += 256) {
      const int j = x / mo, wr = x - j * mo;
      if (j0 + j >= H) continue;
      unsigned p[3];
      split1<NP>(tile[wr][j], fs, p);
#pragma unroll
      for (int q = 0; q < NP; ++q)
        Bt[bfrag_index(q, (int64_t)u * H + j0 + j, wr, K1 / 16, NP)] = (unsigned short)p[q];
    }
  }
  if (Bf && blockIdx.x == 0) {  // bias columns of Bf: Bf[p][w][K1 + u]
    for (int wr = tid; wr < mo; wr += 256) {
      unsigned p[3];
      split1<NP>(b2[(int64_t)u * mo + wr], fs, p);
#pragma unroll
      for (int q = 0; q < NP; ++q)
        Bf[bfrag_index(q, wr, K1 + u, mo / 16, NP)] = (unsigned short)p[q];
    }
  }
}

}  // namespace
}  // namespace gmp

using namespace gmp;

// forward path GEMM schedule: s_setprio 1 for waves 4-7 (bit 0), and waves 4-7 run their MFMAs
// before the stage's split / stash (bit 1).  MACE-128 lo = 2 shape, one box: 0: 12.80 / 12.73 ms,
// 2: 12.50, 3: 12.43
constexpr int kGemmPrio = 3;

template <int NP>
int split_w2_launch(int64_t mul1, int64_t mul_out, int64_t H, const float* W2p, const float* b2p,
                    const unsigned* wmax, void* Bf, void* Bt, void* stream) {
  GMP_CHECK_ARG(mul1 > 0 && mul_out > 0 && mul_out <= 128 && H > 0 && mul1 <= 65535);
  GMP_CHECK_ARG(W2p && b2p && (Bf || Bt) && (NP == 3 || wmax));
  // fragment order: Bf (mul_out x (mul1 H + mul1)), Bt (mul1 H x mul_out)
  GMP_CHECK_ARG(!Bf || (mul_out % 16 == 0 && (mul1 * H + mul1) % 32 == 0));
  GMP_CHECK_ARG(!Bt || (mul_out % 32 == 0 && (mul1 * H) % 16 == 0));
  tp_split_w2_kernel<NP><<<dim3((unsigned)ceil_div(H, 64), (unsigned)mul1), 256, 0,
                           as_stream(stream)>>>((int)mul1, (int)mul_out, (int)H, W2p, b2p,
                                                static_cast<unsigned short*>(Bf),
                                                static_cast<unsigned short*>(Bt), wmax);
  return launch_status();
}

int gemm_launch(int64_t M, int64_t N, int64_t K1, const float* A1, int64_t lda1, int64_t K2,
                const float* A2, int64_t lda2, const void* Bp, int64_t ldb, int64_t bplane,
                float* C, int64_t cgrp, int64_t cldg, int64_t cldr, int64_t cldn, int accumulate,
                void* stream, const float* bias = nullptr) {
  GMP_CHECK_ARG(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0 && cgrp >= 1);
  if (M == 0 || N == 0) return GMP_OK;
  GMP_CHECK_ARG(A1 && Bp && C && (K2 == 0 || A2));
  GMP_CHECK_ARG(K1 % kBK == 0 && K2 % kBK == 0 && K1 + K2 > 0 && N % 16 == 0);
  GMP_CHECK_ARG(lda1 % 4 == 0 && (K2 == 0 || lda2 % 4 == 0));
  // B is fragment-ordered (bfrag_index): the row-major strides it replaced must be the dense ones
  GMP_CHECK_ARG(ldb == K1 + K2 && bplane == N * (K1 + K2));
  GMP_CHECK_ARG(lda1 >= K1 && (K2 == 0 || lda2 >= K2));
  GMP_CHECK_ARG(((reinterpret_cast<uintptr_t>(A1) | reinterpret_cast<uintptr_t>(Bp)) % 16) == 0);
  GMP_CHECK_ARG(K2 == 0 || reinterpret_cast<uintptr_t>(A2) % 16 == 0);
  // narrow outputs (mul_out <= 64: C5's 64-channel paths) take the 256 x 64 tile
  const bool narrow = N <= 64;
  const int64_t bm = narrow ? 256 : 128, bn = narrow ? 64 : 128;
  const int64_t tiles_m = ceil_div(M, bm), tiles_n = ceil_div(N, bn);
  GMP_CHECK_ARG(tiles_m < (1LL << 31) && tiles_n < (1LL << 31));
  const int64_t nwg = tiles_m * tiles_n;
  GMP_CHECK_ARG(nwg < (1LL << 32));
  const size_t smem = 2 * (size_t)(3 * bm * 64);
  int rc = 0;
  decltype(&tp_gemm_x3_kernel<true, 8, 2, 2>) k;
  if ((K1 + K2) <= 8 * kBK && !narrow) {
    // short k ranges (node-level Linears, K <= 256): a 2-deep A ring; the deep rings would only
    // prefetch clamped copies of the last stage
    k = accumulate ? tp_gemm_x3_kernel<true, 2, 2, 2> : tp_gemm_x3_kernel<false, 2, 2, 2>;
  } else if (narrow) {  // 4 A units per thread: a 4-deep ring holds the same bytes as 8 x 2
    k = accumulate ? tp_gemm_x3_kernel<true, 4, 2, 4> : tp_gemm_x3_kernel<false, 4, 2, 4>;
  } else {
    // an 8-deep A-stream register ring (r02's 2-deep form measured slower)
    k = accumulate ? tp_gemm_x3_kernel<true, 8, 2, 2> : tp_gemm_x3_kernel<false, 8, 2, 2>;
  }
  if ((rc = hip_check(hipFuncSetAttribute((const void*)k,
                                          hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)smem))))
    return rc;
  k<<<(unsigned)nwg, kGT, smem, as_stream(stream)>>>(
      M, (int)N, K1, A1, lda1, K2, K2 ? A2 : A1, K2 ? lda2 : lda1,
      static_cast<const unsigned short*>(Bp), ldb, bplane, C, cgrp, cldg, cldr, cldn,
      (int)tiles_m, (int)tiles_n, bias, kGemmPrio);
  return launch_status();
}

template <int NP>
int widen_launch(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const void* Bp,
                 int64_t ldb, int64_t bplane, const unsigned* amax, const unsigned* wmax,
                 float* C, int64_t ldc, void* stream) {
  GMP_CHECK_ARG(M >= 0 && N >= 0 && K > 0 && K % kBK == 0 && K <= kBK * kMaxKS);
  if (M == 0 || N == 0) return GMP_OK;
  GMP_CHECK_ARG(A && Bp && C && lda >= K && lda % 4 == 0 && ldc >= N && N % 16 == 0 &&
                (NP == 3 || (amax && wmax)));
  GMP_CHECK_ARG(ldb == K && bplane == N * K);  // B fragment-ordered (bfrag_index)
  GMP_CHECK_ARG(((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(Bp)) % 16) == 0);
  const int64_t tiles_m = ceil_div(M, kBM), tiles_n = ceil_div(N, kBN);
  GMP_CHECK_ARG(tiles_m < (1LL << 30) && tiles_n < (1LL << 30));
  // about four workgroups per CU over the launch, each sweeping >= 8 column tiles
  int64_t n_split = ceil_div(4 * (int64_t)device_cu_count(), tiles_m);
  const int64_t max_split = ceil_div(tiles_n, 8);
  if (n_split > max_split) n_split = max_split;
  if (n_split < 1) n_split = 1;
  const int64_t nwg = tiles_m * n_split;
  GMP_CHECK_ARG(nwg < (1LL << 32));
  const int nks = (int)(K / kBK);
  // resident A planes + the epilogue's per-wave 16 x 32 parking slabs
  const size_t smem = (size_t)(nks * NP) * kPlane + (size_t)(kGT / 64) * 16 * kParkLd * 4;
  hipStream_t s = as_stream(stream);
  const unsigned short* B = static_cast<const unsigned short*>(Bp);
  int rc = 0;
#define LAUNCH_WN(NK)                                                                               \
  {                                                                                              \
    auto k = tp_gemm_x3_widen_kernel<NK, NP, 4>;                                                 \
    if ((rc = hip_check(hipFuncSetAttribute((const void*)k,                                      \
                                            hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                            (int)smem))))                                        \
      return rc;                                                                                 \
    k<<<(unsigned)nwg, kGT, smem, s>>>(M, N, A, lda, B, ldb, bplane, C, ldc, (int)tiles_m,       \
                                       (int)tiles_n, (int)n_split, amax, wmax);                  \
  }
  switch (nks) {
    case 1: LAUNCH_WN(1) break;
    case 2: LAUNCH_WN(2) break;
    case 3: LAUNCH_WN(3) break;
    default: LAUNCH_WN(4) break;
  }
#undef LAUNCH_WN
  return launch_status();
}

extern "C" {

int gmp_tp_split_w2_f32(int64_t mul1, int64_t mul_out, int64_t H, const float* W2p,
                        const float* b2p, void* Bf, void* Bt, void* stream) {
  return split_w2_launch<3>(mul1, mul_out, H, W2p, b2p, nullptr, Bf, Bt, stream);
}

int gmp_tp_gemm_x3_f32(int64_t M, int64_t N, int64_t K1, const float* A1, int64_t lda1,
                       int64_t K2, const float* A2, int64_t lda2, const void* Bp, int64_t ldb,
                       int64_t bplane, float* C, int64_t cgrp, int64_t cldg, int64_t cldr,
                       int64_t cldn, int accumulate, void* stream) {
  return gemm_launch(M, N, K1, A1, lda1, K2, A2, lda2, Bp, ldb, bplane, C, cgrp, cldg, cldr,
                     cldn, accumulate, stream);
}

int gmp_tp_gemm_x3_widen_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                             const void* Bp, int64_t ldb, int64_t bplane, float* C, int64_t ldc,
                             void* stream) {
  return widen_launch<3>(M, N, K, A, lda, Bp, ldb, bplane, nullptr, nullptr, C, ldc, stream);
}

}  // extern "C"
