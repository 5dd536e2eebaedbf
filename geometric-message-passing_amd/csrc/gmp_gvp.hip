// K5g: GVP-GNN message function (models/layers/gvp_layer.py:101-170 GVP applied per edge by
// GVPConv.message :319-324, with the reference configuration activations = (relu, None),
// vector_gate = True, s = 128 scalar / v = 16 vector channels, edge (32, 1)).
//
// Two fused kernels (forward and backward each), one wave per 16-edge chunk, lane l holding
// edge i = l & 15 and feature group g = l >> 4 (features 16p + 4g + q: the register order the
// v_mfma_f32_16x16x4_f32 B operand and C/D accumulator share, as in the EGNN kernels), so each
// GVP's Linears, norms and gates run in registers; the xyz components of a vector channel sit in
// the same lane (norms need no cross-lane traffic):
//   * gvp_msg0: the first message GVP on [s_j, e_s, s_i] / [v_j, e_v, v_i].  Its scalar Linear is
//     split into node projections P = [s W_a^T | s W_b^T] (gathered at j and i) plus the edge
//     terms W_e e_s and W_n |vh|; its vector Linear W_h into node projections Q = [v W_ha^T |
//     v W_hb^T] (33 channels padded to 48) plus the rank-1 e_v term;
//   * gvp_layer: a GVP (128, 16) -> (128, 16) on per-edge rows (message GVPs 2 and 3).
// Backward kernels recompute the forward in registers and write the input gradients plus the
// per-edge factors of every weight gradient (reduced by the deterministic edge outer sum).
#include "gmp_gvp_common.h"

namespace gmp {
namespace {

using namespace gvpk;

constexpr int kGT = 512;   // threads per workgroup (8 waves, 1 workgroup per CU: LDS-bound)
constexpr int S = 128;     // scalar channels
constexpr int V = 16;      // vector channels
constexpr int SE = 32;     // edge scalar channels
constexpr int H0 = 48;     // first GVP hidden vector channels (33 padded)

// LDS row strides (floats): +4 keeps the 16 rows of an A-operand read on distinct banks
constexpr int LD128 = S + 4;
constexpr int LD16 = V + 4;
constexpr int LD32 = SE + 4;
constexpr int LD48 = H0 + 4;

// ------------------------------------------------------------------------------------------
// Generic GVP (128, 16) -> (128, 16) weights and the per-edge forward state
struct LayerW {
  const float *Ws, *bs, *Wsv, *bsv, *Wh, *Wv;
};
struct LayerFwd {
  f32x4 vh[3][1], vn[1], sq[1], spre[S / 16], vpre[3][1], sg[1];
};
struct Chunk {
  int64_t e;
  bool valid;
};
__device__ __forceinline__ Chunk chunk_edge(int64_t c, int i, int64_t E) {
  Chunk k;
  k.e = 16 * c + i;
  k.valid = k.e < E;
  if (!k.valid) k.e = E - 1;  // clamp loads; stores are masked
  return k;
}

// Backward: inputs s_in, v_in, ds_out, dv_out.  Outputs ds_in, dv_in and the weight-gradient
// factors dspre (E,128), spre (E,128), dgate (E,16), vn (E,16), vh (E,48), dvpre (E,48),
// dvh (E,48) (vector tensors in (channel, xyz) layout).
struct LayerGrads {
  float *ds_in, *dv_in, *dspre, *spre, *dgate, *vn, *vh, *dvpre, *dvh;
};

// ------------------------------------------------------------------------------------------
// First message GVP: LDS = We (128 x 32) | Wn (128 x 48) | Wv0 (16 x 48) | Wsv0 (16 x 128) |
// b0 (128) | bsv0 (16) | wev (48)
struct Msg0W {
  const float *We, *Wn, *b, *Wv, *Wsv, *bsv, *wev;  // Wn, Wv, wev zero-padded to 48 channels
};
constexpr int kMsg0Smem = S * LD32 + S * LD48 + V * LD48 + V * LD128 + S + V + H0;

__device__ void msg0_to_lds(float* sm, const Msg0W& P) {
  float* sWe = sm;
  float* sWn = sWe + S * LD32;
  float* sWv = sWn + S * LD48;
  float* sWsv = sWv + V * LD48;
  float* sb = sWsv + V * LD128;
  float* sbsv = sb + S;
  float* swev = sbsv + V;
  for (int x = threadIdx.x; x < S * SE; x += blockDim.x) sWe[(x / SE) * LD32 + x % SE] = P.We[x];
  for (int x = threadIdx.x; x < S * H0; x += blockDim.x) sWn[(x / H0) * LD48 + x % H0] = P.Wn[x];
  for (int x = threadIdx.x; x < V * H0; x += blockDim.x) sWv[(x / H0) * LD48 + x % H0] = P.Wv[x];
  for (int x = threadIdx.x; x < V * S; x += blockDim.x) sWsv[(x / S) * LD128 + x % S] = P.Wsv[x];
  for (int x = threadIdx.x; x < S; x += blockDim.x) sb[x] = P.b[x];
  for (int x = threadIdx.x; x < V; x += blockDim.x) sbsv[x] = P.bsv[x];
  for (int x = threadIdx.x; x < H0; x += blockDim.x) swev[x] = P.wev[x];
}

struct Msg0Fwd {
  f32x4 vh[3][3], vn[3], sq[3], spre[S / 16], vpre[3][1], sg[1];
};

// P row: [Pa (128) | Pb (128)]; Q row: [Qa (48 x 3) | Qb (48 x 3)] in (channel, xyz) layout
__device__ __forceinline__ void msg0_forward(const float* sm, const float* __restrict__ Prow_j,
                                             const float* __restrict__ Prow_i,
                                             const float* __restrict__ Qrow_j,
                                             const float* __restrict__ Qrow_i,
                                             const float* __restrict__ es_row,
                                             const float* __restrict__ ev_row, Msg0Fwd& F, int i,
                                             int g) {
  const float* sWe = sm;
  const float* sWn = sWe + S * LD32;
  const float* sWv = sWn + S * LD48;
  const float* sWsv = sWv + V * LD48;
  const float* sb = sWsv + V * LD128;
  const float* sbsv = sb + S;
  const float* swev = sbsv + V;
  // vh = Qa[j] + Qb[i] + wev (x) ev
  ld_vrow<3>(F.vh, Qrow_j, g);
  f32x4 t[3][3];
  ld_vrow<3>(t, Qrow_i + 3 * H0, g);
  const float ev0 = ev_row[0], ev1 = ev_row[1], ev2 = ev_row[2];
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const f32x4 w = *reinterpret_cast<const f32x4*>(swev + 16 * p + 4 * g);
    F.vh[0][p] += t[0][p] + w * ev0;
    F.vh[1][p] += t[1][p] + w * ev1;
    F.vh[2][p] += t[2][p] + w * ev2;
  }
  vnorm<3>(F.vh, F.vn, F.sq);
  // spre = b + Pa[j] + Pb[i] + We es + Wn vn
  ld_vec<S / 16>(F.spre, sb, g);
  add_row<S / 16>(F.spre, Prow_j, g);
  add_row<S / 16>(F.spre, Prow_i + S, g);
  f32x4 es[2];
  ld_row<2>(es, es_row, g);
  gemm_wx<S / 16, 2>(sWe, LD32, es, F.spre, i, g);
  gemm_wx<S / 16, 3>(sWn, LD48, F.vn, F.spre, i, g);
  // vpre = Wv vh ; gate = bsv + Wsv spre
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    zero(F.vpre[x]);
    gemm_wx<1, 3>(sWv, LD48, F.vh[x], F.vpre[x], i, g);
  }
  f32x4 gate[1];
  ld_vec<1>(gate, sbsv, g);
  gemm_wx<1, S / 16>(sWsv, LD128, F.spre, gate, i, g);
#pragma unroll
  for (int q = 0; q < 4; ++q) F.sg[0][q] = sigm(gate[0][q]);
}

__global__ __launch_bounds__(kGT) void gvp_msg0_fwd_kernel(int64_t E, const int64_t* __restrict__ send,
                                                           const int64_t* __restrict__ recv,
                                                           const float* __restrict__ Pn,
                                                           const float* __restrict__ Qn,
                                                           const float* __restrict__ es,
                                                           const float* __restrict__ ev, Msg0W W,
                                                           float* __restrict__ s_out,
                                                           float* __restrict__ v_out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  msg0_to_lds(sm, W);
  __syncthreads();
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int64_t nchunks = (E + 15) / 16;
  const int64_t wave = (int64_t)blockIdx.x * (kGT / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (kGT / 64);
  for (int64_t c = wave; c < nchunks; c += nwaves) {
    const Chunk k = chunk_edge(c, i, E);
    const int64_t j = send[k.e], r = recv[k.e];
    Msg0Fwd F;
    msg0_forward(sm, Pn + j * 2 * S, Pn + r * 2 * S, Qn + j * 6 * H0, Qn + r * 6 * H0,
                 es + k.e * SE, ev + k.e * 3, F, i, g);
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int q = 0; q < 4; ++q) F.vpre[x][0][q] *= F.sg[0][q];
#pragma unroll
    for (int p = 0; p < S / 16; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) F.spre[p][q] = fmaxf(F.spre[p][q], 0.f);
    if (k.valid) {
      st_row<S / 16>(s_out + k.e * S, F.spre, g);
      st_vrow<1>(v_out + k.e * (3 * V), F.vpre, g);
    }
  }
}

// Backward of the first GVP.  Outputs: dspre (E,128) [= dPa rows at j, dPb rows at i, and the
// dW_e / dW_n / db factor], spre (E,128), dgate (E,16), vn (E,48), vh (E,144), dvpre (E,48),
// dvh (E,144) [= dQa rows at j, dQb rows at i], des (E,32), dev (E,3).
struct Msg0Grads {
  float *dspre, *spre, *dgate, *vn, *vh, *dvpre, *dvh, *des, *dev;
};

// Backward of the first message GVP for this lane's edge e (gathers at j = send[e], r = recv[e]):
// the per-edge outputs (stored here, at row e) and, returned for callers that reduce them over
// the receivers, the rows dspre (ds), dgate, dvpre (dv) and dvh.
struct Msg0Bwd {
  f32x4 ds[S / 16], dgate[1], dv[3][1], dvh[3][3];
};
__device__ __forceinline__ void msg0_bwd_edge(const float* sm, int64_t e, bool valid, int64_t j,
                                              int64_t r, const float* __restrict__ Pn,
                                              const float* __restrict__ Qn,
                                              const float* __restrict__ es,
                                              const float* __restrict__ ev,
                                              const float* __restrict__ ds_out,
                                              const float* __restrict__ dv_out,
                                              const Msg0Grads& O, Msg0Bwd& B, int i, int g) {
  const float* sWe = sm;
  const float* sWn = sWe + S * LD32;
  const float* sWv = sWn + S * LD48;
  const float* sWsv = sWv + V * LD48;
  const float* swev = sWsv + V * LD128 + S + V;
  Msg0Fwd F;
  msg0_forward(sm, Pn + j * 2 * S, Pn + r * 2 * S, Qn + j * 6 * H0, Qn + r * 6 * H0,
               es + e * SE, ev + e * 3, F, i, g);
  ld_row<S / 16>(B.ds, ds_out + e * S, g);
#pragma unroll
  for (int p = 0; p < S / 16; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) B.ds[p][q] = F.spre[p][q] > 0.f ? B.ds[p][q] : 0.f;
  ld_vrow<1>(B.dv, dv_out + e * (3 * V), g);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float dsg = B.dv[0][0][q] * F.vpre[0][0][q] + B.dv[1][0][q] * F.vpre[1][0][q] + B.dv[2][0][q] * F.vpre[2][0][q];
    B.dgate[0][q] = dsg * F.sg[0][q] * (1.f - F.sg[0][q]);
#pragma unroll
    for (int x = 0; x < 3; ++x) B.dv[x][0][q] *= F.sg[0][q];
  }
  gemm_wtx<S / 16, 1>(sWsv, LD128, B.dgate, B.ds, i, g);  // dspre total
  if (valid) {
    st_row<S / 16>(O.dspre + e * S, B.ds, g);
    if (O.spre) st_row<S / 16>(O.spre + e * S, F.spre, g);
    st_row<1>(O.dgate + e * V, B.dgate, g);
    st_row<3>(O.vn + e * H0, F.vn, g);
    if (O.vh) st_vrow<3>(O.vh + e * (3 * H0), F.vh, g);
    st_vrow<1>(O.dvpre + e * (3 * V), B.dv, g);
  }
  // des = We^T dspre ; dvn = Wn^T dspre
  f32x4 des[2], dvn[3];
  zero(des);
  zero(dvn);
  gemm_wtx<2, S / 16>(sWe, LD32, B.ds, des, i, g);
  gemm_wtx<3, S / 16>(sWn, LD48, B.ds, dvn, i, g);
  if (valid) st_row<2>(O.des + e * SE, des, g);
  // dvh = Wv^T dvpre + dvn * vh / vn
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    zero(B.dvh[x]);
    gemm_wtx<3, 1>(sWv, LD48, B.dv[x], B.dvh[x], i, g);
  }
  float dev0 = 0.f, dev1 = 0.f, dev2 = 0.f;
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const f32x4 w = *reinterpret_cast<const f32x4*>(swev + 16 * p + 4 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float f = F.sq[p][q] > 1e-8f ? dvn[p][q] / F.vn[p][q] : 0.f;
      B.dvh[0][p][q] += f * F.vh[0][p][q];
      B.dvh[1][p][q] += f * F.vh[1][p][q];
      B.dvh[2][p][q] += f * F.vh[2][p][q];
      dev0 += w[q] * B.dvh[0][p][q];
      dev1 += w[q] * B.dvh[1][p][q];
      dev2 += w[q] * B.dvh[2][p][q];
    }
  }
  // dev = sum over the 48 channels: reduce the 4 lane groups of this edge (fixed order)
  dev0 += __shfl_xor(dev0, 16);
  dev0 += __shfl_xor(dev0, 32);
  dev1 += __shfl_xor(dev1, 16);
  dev1 += __shfl_xor(dev1, 32);
  dev2 += __shfl_xor(dev2, 16);
  dev2 += __shfl_xor(dev2, 32);
  if (valid) {
    st_vrow<3>(O.dvh + e * (3 * H0), B.dvh, g);
    if (g == 0) {
      O.dev[e * 3 + 0] = dev0;
      O.dev[e * 3 + 1] = dev1;
      O.dev[e * 3 + 2] = dev2;
    }
  }
}

__global__ __launch_bounds__(kGT) void gvp_msg0_bwd_kernel(int64_t E, const int64_t* __restrict__ send,
                                                           const int64_t* __restrict__ recv,
                                                           const float* __restrict__ Pn,
                                                           const float* __restrict__ Qn,
                                                           const float* __restrict__ es,
                                                           const float* __restrict__ ev, Msg0W W,
                                                           const float* __restrict__ ds_out,
                                                           const float* __restrict__ dv_out,
                                                           Msg0Grads O) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  msg0_to_lds(sm, W);
  __syncthreads();
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int64_t nchunks = (E + 15) / 16;
  const int64_t wave = (int64_t)blockIdx.x * (kGT / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (kGT / 64);
  for (int64_t c = wave; c < nchunks; c += nwaves) {
    const Chunk k = chunk_edge(c, i, E);
    Msg0Bwd B;
    msg0_bwd_edge(sm, k.e, k.valid, send[k.e], recv[k.e], Pn, Qn, es, ev, ds_out, dv_out, O, B,
                  i, g);
  }
}

// ------------------------------------------------------------------------------------------
// r04: the GVP layer's 128 x 128 products (W_s's scalar block: Ws[:, :128] s in the forward and
// its recompute, Ws[:, :128]^T dspre in the backward) on the bf16 MFMA over exact three-plane
// splits (x = hi + mid + lo, six products hi.hi + hi.mid + mid.hi + hi.lo + lo.hi + mid.mid in
// f32 accumulation: f32-class, no scaling -- bf16 keeps f32's exponent range).  16x16x32 bf16
// = 16 cycles for 6 x 16 x 16 x 32 products against 8 x 32 cycles of 16x16x4 f32 for the same
// 16 x 16 x 32 f32 product: 2.7x fewer MFMA cycles on the kernel's dominant products.  The small
// products (vn block of Ws, Wsv, Wh, Wv: K = 16 or 16 outputs) stay on the exact f32 MFMA.
// Image: 3 planes x 128 rows x LDH bf16 (272-byte rows: the 16 rows of a 16-byte A read fall on
// distinct banks); columns in the hf_pos order (the 8 halfs a lane feeds one 16x16x32 MFMA,
// k = 8 g + j of block p, are its slots x[2p][0..3], x[2p + 1][0..3]).  The forward kernel
// stores W (rows o); the backward stores W^T (rows k) and reads W for the recompute with
// ds_read_b64_tr_b16 (same address pattern as the EGNN backward's x_hat3 recompute).
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));

// 320-byte rows (80 dwords = 16 mod 64) with the 16-byte chunks of row r XOR-swizzled by
// x3_swz(r): the 16-lane groups of a 16-byte A read (lanes {0-3,12-15,20-27}, ...) hit 64
// distinct banks, and the transposed 8-byte reads are 2-way (the floor for 8-byte pieces of
// 16-byte-aligned rows).  The r04 first form (272-byte rows) measured 0.48 / 0.62 of its LDS
// cycles in bank conflicts (2-way / 4-way).
constexpr int XLDH = S + 32;             // bf16 per image row
constexpr int XPLANE = S * XLDH;         // bf16 per plane
constexpr int kXImgFloats = 3 * XPLANE / 2;
// LDS (floats): image | Ws vn block (128 x LD16) | Wsv (16 x LD128) | Wh | Wv | bs | bsv
constexpr int kLayerSmemX3 = kXImgFloats + S * LD16 + V * LD128 + 2 * V * LD16 + S + V;

__device__ __forceinline__ int x3_pos(int k) {
  const int tt = k >> 4, gg = (k >> 2) & 3, q = k & 3;
  return 32 * (tt >> 1) + 8 * gg + 4 * (tt & 1) + q;
}

__device__ __forceinline__ int x3_swz(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }  // {0,2,3,1}

__device__ __forceinline__ void split3(f32x2_t x, unsigned& h, unsigned& m, unsigned& l) {
  const bf16x2_t bh = __builtin_convertvector(x, bf16x2_t);
  const f32x2_t r1 = x - __builtin_convertvector(bh, f32x2_t);
  const bf16x2_t bm = __builtin_convertvector(r1, bf16x2_t);
  const f32x2_t r2 = r1 - __builtin_convertvector(bm, f32x2_t);
  const bf16x2_t bl = __builtin_convertvector(r2, bf16x2_t);
  h = __builtin_bit_cast(unsigned, bh);
  m = __builtin_bit_cast(unsigned, bm);
  l = __builtin_bit_cast(unsigned, bl);
}
// slots x[2p], x[2p + 1] of this lane -> the three bf16x8 planes of one B fragment
__device__ __forceinline__ void split_slots(const f32x4& x0, const f32x4& x1, bf16x8_t (&b)[3]) {
  unsigned h[4], m[4], l[4];
  split3(f32x2_t{x0[0], x0[1]}, h[0], m[0], l[0]);
  split3(f32x2_t{x0[2], x0[3]}, h[1], m[1], l[1]);
  split3(f32x2_t{x1[0], x1[1]}, h[2], m[2], l[2]);
  split3(f32x2_t{x1[2], x1[3]}, h[3], m[3], l[3]);
  b[0] = __builtin_bit_cast(bf16x8_t, u32x4_t{h[0], h[1], h[2], h[3]});
  b[1] = __builtin_bit_cast(bf16x8_t, u32x4_t{m[0], m[1], m[2], m[3]});
  b[2] = __builtin_bit_cast(bf16x8_t, u32x4_t{l[0], l[1], l[2], l[3]});
}
__device__ __forceinline__ f32x4 mma6(const bf16x8_t (&a)[3], const bf16x8_t (&b)[3], f32x4 t) {
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], t, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], t, 0, 0, 0);
}

// image of Ws[:, :128] (TRANSPOSE: of its transpose), plus the f32 remainder
template <bool TRANSPOSE>
__device__ void layer_to_lds_x3(float* sm, const LayerW& P) {
  __bf16* img = reinterpret_cast<__bf16*>(sm);
  float* sWsV = sm + kXImgFloats;
  float* sWsv = sWsV + S * LD16;
  float* sWh = sWsv + V * LD128;
  float* sWv = sWh + V * LD16;
  float* sbs = sWv + V * LD16;
  float* sbsv = sbs + S;
  for (int x = threadIdx.x; x < S * S / 2; x += blockDim.x) {
    const int o = (2 * x) / S, k = (2 * x) % S;  // W[o][k], W[o][k + 1]
    const f32x2_t w = *reinterpret_cast<const f32x2_t*>(P.Ws + o * (S + V) + k);
    unsigned h, m, l;
    split3(w, h, m, l);
    const unsigned pl[3] = {h, m, l};
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = TRANSPOSE ? k + u : o, c = TRANSPOSE ? o : k + u;
        const int pos = x3_pos(c);
        reinterpret_cast<unsigned short*>(img)[p * XPLANE + r * XLDH + (pos ^ (x3_swz(r) << 3))] =
            (unsigned short)(pl[p] >> (16 * u));
      }
  }
  for (int x = threadIdx.x; x < S * V; x += blockDim.x)
    sWsV[(x / V) * LD16 + x % V] = P.Ws[(x / V) * (S + V) + S + x % V];
  for (int x = threadIdx.x; x < V * S; x += blockDim.x) sWsv[(x / S) * LD128 + x % S] = P.Wsv[x];
  for (int x = threadIdx.x; x < V * V; x += blockDim.x) {
    sWh[(x / V) * LD16 + x % V] = P.Wh[x];
    sWv[(x / V) * LD16 + x % V] = P.Wv[x];
  }
  for (int x = threadIdx.x; x < S; x += blockDim.x) sbs[x] = P.bs[x];
  for (int x = threadIdx.x; x < V; x += blockDim.x) sbsv[x] = P.bsv[x];
}

// y[slot(r)] += sum_c IMG[r][c] x[slot(c)]  (A rows read directly)
__device__ __forceinline__ void gemm_x3(const __bf16* __restrict__ img, const f32x4 (&x)[S / 16],
                                        f32x4 (&y)[S / 16], int i, int g) {
#pragma unroll
  for (int p = 0; p < S / 32; ++p) {
    bf16x8_t b[3];
    split_slots(x[2 * p], x[2 * p + 1], b);
#pragma unroll
    for (int t = 0; t < S / 16; ++t) {
      const __bf16* row = img + (16 * t + i) * XLDH + 32 * p + 8 * (g ^ x3_swz(i));
      bf16x8_t a[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) a[pl] = *reinterpret_cast<const bf16x8_t*>(row + pl * XPLANE);
      y[t] = mma6(a, b, y[t]);
      if (t % 2 == 1) asm volatile("" ::: "memory");  // bounds hoisted A reads (registers)
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ s16x4_t lds_tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}
// y[slot(c)] += sum_r IMG[r][c] x[slot(r)]: the product with the image's transpose, A fragments
// by transposed 8-byte reads (lane 4q + c of group g supplies row 32p + 4g + q (+ 16))
__device__ __forceinline__ void gemm_x3_tr(const __bf16* __restrict__ img, const f32x4 (&x)[S / 16],
                                           f32x4 (&y)[S / 16], int lane, int g) {
  const int q = (lane & 15) >> 2, c = lane & 3;
#pragma unroll
  for (int p = 0; p < S / 32; ++p) {
    bf16x8_t b[3];
    split_slots(x[2 * p], x[2 * p + 1], b);
    const __bf16* rowk = img + (32 * p + 4 * g + q) * XLDH + 8 * (c ^ x3_swz(4 * g));
#pragma unroll
    for (int t = 0; t < S / 16; ++t) {
      const __bf16* a0 = rowk + 32 * (t >> 1) + 4 * (t & 1);
      bf16x8_t a[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const s16x4_t h0 = lds_tr16(a0 + pl * XPLANE), h1 = lds_tr16(a0 + pl * XPLANE + 16 * XLDH);
        a[pl] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      y[t] = mma6(a, b, y[t]);
      if (t % 2 == 1) asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// forward of one GVP layer for this lane's edge on the image (TR: the image holds W^T)
template <bool TR>
__device__ __forceinline__ void layer_forward_x3(const float* sm, const f32x4 (&s)[S / 16],
                                                 const f32x4 (&v)[3][1], LayerFwd& F, int lane,
                                                 int i, int g) {
  const __bf16* img = reinterpret_cast<const __bf16*>(sm);
  const float* sWsV = sm + kXImgFloats;
  const float* sWsv = sWsV + S * LD16;
  const float* sWh = sWsv + V * LD128;
  const float* sWv = sWh + V * LD16;
  const float* sbs = sWv + V * LD16;
  const float* sbsv = sbs + S;
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    zero(F.vh[x]);
    gemm_wx<1, 1>(sWh, LD16, v[x], F.vh[x], i, g);
  }
  vnorm<1>(F.vh, F.vn, F.sq);
  ld_vec<S / 16>(F.spre, sbs, g);
  if constexpr (TR) gemm_x3_tr(img, s, F.spre, lane, g);
  else gemm_x3(img, s, F.spre, i, g);
  gemm_wx<S / 16, 1>(sWsV, LD16, F.vn, F.spre, i, g);
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    zero(F.vpre[x]);
    gemm_wx<1, 1>(sWv, LD16, F.vh[x], F.vpre[x], i, g);
  }
  f32x4 gate[1];
  ld_vec<1>(gate, sbsv, g);
  gemm_wx<1, S / 16>(sWsv, LD128, F.spre, gate, i, g);
#pragma unroll
  for (int q = 0; q < 4; ++q) F.sg[0][q] = sigm(gate[0][q]);
}

template <int ACT>
__global__ __launch_bounds__(kGT) void gvp_layer_fwd_x3_kernel(int64_t E, const float* __restrict__ s_in,
                                                               const float* __restrict__ v_in, LayerW P,
                                                               float* __restrict__ s_out,
                                                               float* __restrict__ v_out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  layer_to_lds_x3<false>(sm, P);
  __syncthreads();
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int64_t nchunks = (E + 15) / 16;
  const int64_t wave = (int64_t)blockIdx.x * (kGT / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (kGT / 64);
  for (int64_t c = wave; c < nchunks; c += nwaves) {
    const Chunk k = chunk_edge(c, i, E);
    f32x4 s[S / 16], v[3][1];
    ld_row<S / 16>(s, s_in + k.e * S, g);
    ld_vrow<1>(v, v_in + k.e * (3 * V), g);
    LayerFwd F;
    layer_forward_x3<false>(sm, s, v, F, lane, i, g);
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int q = 0; q < 4; ++q) F.vpre[x][0][q] *= F.sg[0][q];
    if (ACT) {
#pragma unroll
      for (int p = 0; p < S / 16; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) F.spre[p][q] = fmaxf(F.spre[p][q], 0.f);
    }
    if (k.valid) {
      st_row<S / 16>(s_out + k.e * S, F.spre, g);
      st_vrow<1>(v_out + k.e * (3 * V), F.vpre, g);
    }
  }
}

// ------------------------------------------------------------------------------------------
// r05: the last message GVP fused with the receivers' sum / mean (GVPConv, gvp_layer.py:319-324):
// no (E, S + 3V) per-edge output rows.  Edges are walked in receiver-sorted order (the CSR of
// the receivers: perm = original edge of sorted position k, skey = its receiver, rowptr); each
// wave owns the in-edges of a contiguous receiver range (edge-balanced, as K4), reads its rows
// through perm, runs the layer in registers and sums each receiver's rows by an in-wave
// segmented scan over the chunk's 16 edge lanes (DPP row_shr) with the open segment carried to
// the next chunk through LDS; the last edge of a segment stores the receiver's row (x 1 / count
// for the mean).  Deterministic (fixed order; a tree order inside a chunk, so not bitwise K3's
// sequential sum).  Receivers without in-edges get zero rows.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int OFF, int T>
__device__ __forceinline__ void seg_scan_level(f32x4 (&x)[T], int i, int head) {
  const bool take = (i - OFF) >= head;
#pragma unroll
  for (int p = 0; p < T; ++p)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float u = dpp_mov<0x110 + OFF>(x[p][c]);  // row_shr:OFF = lane i - OFF
      if (take) x[p][c] += u;
    }
}
template <int T>
__device__ __forceinline__ void seg_scan(f32x4 (&x)[T], int i, int head) {
  seg_scan_level<1>(x, i, head);
  seg_scan_level<2>(x, i, head);
  seg_scan_level<4>(x, i, head);
  seg_scan_level<8>(x, i, head);
}
constexpr int kAggCarry = S / 4 + 3 * 4;  // floats per (wave, lane group): scalar + 3 xyz slots
constexpr int kAggSmem = kLayerSmemX3 + (kGT / 64) * 4 * kAggCarry;

// first receiver of wave w under an edge-balanced, receiver-aligned split (K4's node_begin)
__device__ __forceinline__ int64_t agg_node_begin(const int64_t* __restrict__ rowptr,
                                                  int64_t n_nodes, int64_t n_edges, int64_t w,
                                                  int64_t n_waves) {
  if (w >= n_waves) return n_nodes;
  if (w <= 0) return 0;
  const int64_t target = (n_edges * w) / n_waves;
  int64_t lo = 0, hi = n_nodes;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rowptr[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <bool MEAN>
__global__ __launch_bounds__(kGT) void gvp_layer_fwd_agg_kernel(
    int64_t E, int64_t N, const float* __restrict__ s_in, const float* __restrict__ v_in,
    LayerW P, const int64_t* __restrict__ perm, const int64_t* __restrict__ skey,
    const int64_t* __restrict__ rowptr, float* __restrict__ s_agg, float* __restrict__ v_agg) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  layer_to_lds_x3<false>(sm, P);
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* wcarry = sm + kLayerSmemX3 + wid * 4 * kAggCarry;
  for (int k = lane; k < 4 * kAggCarry; k += 64) wcarry[k] = 0.f;
  float* cbuf = wcarry + g * kAggCarry;
  __syncthreads();
  const int64_t n_waves = (int64_t)gridDim.x * (kGT / 64);
  const int64_t wave = (int64_t)blockIdx.x * (kGT / 64) + wid;
  const int64_t nb = agg_node_begin(rowptr, N, E, wave, n_waves);
  const int64_t ne = agg_node_begin(rowptr, N, E, wave + 1, n_waves);
  const int64_t e_lo = (nb < ne) ? rowptr[nb] : 0, e_hi = (nb < ne) ? rowptr[ne] : 0;
  // receivers of this wave's range without in-edges: zero rows (no other writer)
  for (int64_t n = nb + lane; n < ne; n += 64) {
    if (rowptr[n] == rowptr[n + 1]) {
      for (int c = 0; c < S; c += 4)
        *reinterpret_cast<f32x4*>(s_agg + n * S + c) = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int c = 0; c < 3 * V; c += 4)
        *reinterpret_cast<f32x4*>(v_agg + n * (3 * V) + c) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  int64_t carry_node = -1;
  for (int64_t base = e_lo; base < e_hi; base += 16) {
    const int64_t k = base + i;
    const bool valid = k < e_hi;
    const int64_t kc = valid ? k : e_hi - 1;  // clamp loads; stores are masked
    const int64_t e = perm ? perm[kc] : kc;
    int64_t n = skey[kc];
    n = (n >= 0 && n < N) ? n : 0;
    const int64_t seg0 = rowptr[n], seg1 = rowptr[n + 1];
    f32x4 s[S / 16], v[3][1];
    ld_row<S / 16>(s, s_in + e * S, g);
    ld_vrow<1>(v, v_in + e * (3 * V), g);
    LayerFwd F;
    layer_forward_x3<false>(sm, s, v, F, lane, i, g);
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int q = 0; q < 4; ++q) F.vpre[x][0][q] *= F.sg[0][q];
    // open segment carried from the previous chunk (lane 0 of the group only)
    const float tf = (i == 0 && valid && n == carry_node) ? 1.f : 0.f;
#pragma unroll
    for (int p = 0; p < S / 16; ++p) {
      const f32x4 c = *reinterpret_cast<const f32x4*>(cbuf + 4 * p);
#pragma unroll
      for (int q = 0; q < 4; ++q) F.spre[p][q] = __builtin_fmaf(c[q], tf, F.spre[p][q]);
    }
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      const f32x4 c = *reinterpret_cast<const f32x4*>(cbuf + S / 4 + 4 * x);
#pragma unroll
      for (int q = 0; q < 4; ++q) F.vpre[x][0][q] = __builtin_fmaf(c[q], tf, F.vpre[x][0][q]);
    }
    const int head = valid ? (int)((seg0 > base) ? (seg0 - base) : 0) : i;
    seg_scan<S / 16>(F.spre, i, head);
#pragma unroll
    for (int x = 0; x < 3; ++x) seg_scan<1>(F.vpre[x], i, head);
    const bool is_end = valid && (k == seg1 - 1);
    if (i == 15) {  // the (possibly open) segment of lane 15: the next chunk's carry
#pragma unroll
      for (int p = 0; p < S / 16; ++p) *reinterpret_cast<f32x4*>(cbuf + 4 * p) = F.spre[p];
#pragma unroll
      for (int x = 0; x < 3; ++x) *reinterpret_cast<f32x4*>(cbuf + S / 4 + 4 * x) = F.vpre[x][0];
    }
    if (is_end) {
      if (MEAN) {
        const float sc = 1.f / (float)(seg1 - seg0);
#pragma unroll
        for (int p = 0; p < S / 16; ++p) F.spre[p] *= sc;
#pragma unroll
        for (int x = 0; x < 3; ++x) F.vpre[x][0] *= sc;
      }
      st_row<S / 16>(s_agg + n * S, F.spre, g);
      st_vrow<1>(v_agg + n * (3 * V), F.vpre, g);
    }
    carry_node = __builtin_amdgcn_readlane((int)n, 15);
  }
}

// r05: the first message GVP's backward over the receiver-sorted edges, additionally reducing
// dspre, dgate, dvpre and dvh over each receiver in registers (segmented scan, LDS carries; as
// gvp_layer_fwd_agg_kernel): the receiver-side sums dPb = S_i dspre, dQb = S_i dvh and the
// weight sums' S_i dgate, S_i dvpre without re-reading those per-edge rows.  Per-edge outputs
// are stored at the original edge rows (perm), bitwise those of gvp_msg0_bwd_kernel.
constexpr int kM0Carry = S / 4 + 4 + 12 + 36;  // ds | dgate | dvpre (3 x 4) | dvh (3 x 12)
constexpr int kM0AggSmem = kMsg0Smem + (kGT / 64) * 4 * kM0Carry;

__device__ __forceinline__ void carry_in(const float* c, f32x4* x, int n4, float tf) {
  for (int t = 0; t < n4; ++t) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(c + 4 * t);
#pragma unroll
    for (int q = 0; q < 4; ++q) x[t][q] = __builtin_fmaf(v[q], tf, x[t][q]);
  }
}
__device__ __forceinline__ void carry_out(float* c, const f32x4* x, int n4) {
  for (int t = 0; t < n4; ++t) *reinterpret_cast<f32x4*>(c + 4 * t) = x[t];
}

__global__ __launch_bounds__(kGT) void gvp_msg0_bwd_agg_kernel(
    int64_t E, int64_t N, const int64_t* __restrict__ send, const int64_t* __restrict__ recv,
    const int64_t* __restrict__ perm, const int64_t* __restrict__ rowptr,
    const float* __restrict__ Pn, const float* __restrict__ Qn, const float* __restrict__ es,
    const float* __restrict__ ev, Msg0W W, const float* __restrict__ ds_out,
    const float* __restrict__ dv_out, Msg0Grads O, float* __restrict__ dPb,
    float* __restrict__ dQb, float* __restrict__ sgr, float* __restrict__ svr) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  msg0_to_lds(sm, W);
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* wcarry = sm + kMsg0Smem + wid * 4 * kM0Carry;
  for (int k = lane; k < 4 * kM0Carry; k += 64) wcarry[k] = 0.f;
  float* cbuf = wcarry + g * kM0Carry;
  __syncthreads();
  const int64_t n_waves = (int64_t)gridDim.x * (kGT / 64);
  const int64_t wave = (int64_t)blockIdx.x * (kGT / 64) + wid;
  const int64_t nb = agg_node_begin(rowptr, N, E, wave, n_waves);
  const int64_t ne = agg_node_begin(rowptr, N, E, wave + 1, n_waves);
  const int64_t e_lo = (nb < ne) ? rowptr[nb] : 0, e_hi = (nb < ne) ? rowptr[ne] : 0;
  for (int64_t n = nb + lane; n < ne; n += 64) {
    if (rowptr[n] == rowptr[n + 1]) {
      const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int c = 0; c < S; c += 4) *reinterpret_cast<f32x4*>(dPb + n * S + c) = z;
      for (int c = 0; c < 3 * H0; c += 4) *reinterpret_cast<f32x4*>(dQb + n * (3 * H0) + c) = z;
      for (int c = 0; c < V; c += 4) *reinterpret_cast<f32x4*>(sgr + n * V + c) = z;
      for (int c = 0; c < 3 * V; c += 4) *reinterpret_cast<f32x4*>(svr + n * (3 * V) + c) = z;
    }
  }
  int64_t carry_node = -1;
  for (int64_t base = e_lo; base < e_hi; base += 16) {
    const int64_t k = base + i;
    const bool valid = k < e_hi;
    const int64_t kc = valid ? k : e_hi - 1;
    const int64_t e = perm ? perm[kc] : kc;
    const int64_t r = recv[e];
    const int64_t n = (r >= 0 && r < N) ? r : 0;
    const int64_t seg0 = rowptr[n], seg1 = rowptr[n + 1];
    Msg0Bwd B;
    msg0_bwd_edge(sm, e, valid, send[e], r, Pn, Qn, es, ev, ds_out, dv_out, O, B, i, g);
    const float tf = (i == 0 && valid && n == carry_node) ? 1.f : 0.f;
    carry_in(cbuf, B.ds, S / 16, tf);
    carry_in(cbuf + S / 4, B.dgate, 1, tf);
#pragma unroll
    for (int x = 0; x < 3; ++x) carry_in(cbuf + S / 4 + 4 + 4 * x, B.dv[x], 1, tf);
#pragma unroll
    for (int x = 0; x < 3; ++x) carry_in(cbuf + S / 4 + 16 + 12 * x, B.dvh[x], 3, tf);
    const int head = valid ? (int)((seg0 > base) ? (seg0 - base) : 0) : i;
    seg_scan<S / 16>(B.ds, i, head);
    seg_scan<1>(B.dgate, i, head);
#pragma unroll
    for (int x = 0; x < 3; ++x) seg_scan<1>(B.dv[x], i, head);
#pragma unroll
    for (int x = 0; x < 3; ++x) seg_scan<3>(B.dvh[x], i, head);
    if (i == 15) {
      carry_out(cbuf, B.ds, S / 16);
      carry_out(cbuf + S / 4, B.dgate, 1);
#pragma unroll
      for (int x = 0; x < 3; ++x) carry_out(cbuf + S / 4 + 4 + 4 * x, B.dv[x], 1);
#pragma unroll
      for (int x = 0; x < 3; ++x) carry_out(cbuf + S / 4 + 16 + 12 * x, B.dvh[x], 3);
    }
    if (valid && k == seg1 - 1) {
      st_row<S / 16>(dPb + n * S, B.ds, g);
      st_row<1>(sgr + n * V, B.dgate, g);
      st_vrow<1>(svr + n * (3 * V), B.dv, g);
      st_vrow<3>(dQb + n * (3 * H0), B.dvh, g);
    }
    carry_node = __builtin_amdgcn_readlane((int)n, 15);
  }
}

// Upstream gradient of the layer's per-edge outputs.  AGG = 0: per-edge rows ds_out (E, S),
// dv_out (E, 3V).  AGG = 1 / 2: the layer feeds a sum / mean aggregation at the receivers
// (GVPConv, gvp_layer.py:319-324 with aggr "add" / "mean"): the rows are the aggregation's node
// gradient gathered at index[e] (x 1 / max(count, 1) for the mean, count from rowptr; an index
// outside [0, n_nodes) gets zeros) -- K3's sum / mean backward in the load, so the (E, S + 3V)
// per-edge gradient is never written.
struct AggGrad {
  const int64_t* index;
  const int64_t* rowptr;
  int64_t n_nodes;
};
template <int AGG>
__device__ __forceinline__ void ld_grad_rows(const float* __restrict__ ds_out,
                                             const float* __restrict__ dv_out, const AggGrad& A,
                                             int64_t e, int g, f32x4 (&ds)[S / 16],
                                             f32x4 (&dv)[3][1]) {
  if (AGG == 0) {
    ld_row<S / 16>(ds, ds_out + e * S, g);
    ld_vrow<1>(dv, dv_out + e * (3 * V), g);
    return;
  }
  const int64_t n = A.index[e];
  const bool ok = n >= 0 && n < A.n_nodes;
  const int64_t r = ok ? n : 0;
  ld_row<S / 16>(ds, ds_out + r * S, g);
  ld_vrow<1>(dv, dv_out + r * (3 * V), g);
  float sc = ok ? 1.f : 0.f;
  if (AGG == 2 && ok) {
    const int64_t cnt = A.rowptr[r + 1] - A.rowptr[r];
    sc = 1.f / (float)(cnt > 0 ? cnt : 1);
  }
#pragma unroll
  for (int p = 0; p < S / 16; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) ds[p][q] *= sc;
#pragma unroll
  for (int x = 0; x < 3; ++x)
#pragma unroll
    for (int q = 0; q < 4; ++q) dv[x][0][q] *= sc;
}

template <int ACT, int AGG>
__global__ __launch_bounds__(kGT) void gvp_layer_bwd_x3_kernel(int64_t E, const float* __restrict__ s_in,
                                                               const float* __restrict__ v_in, LayerW P,
                                                               const float* __restrict__ ds_out,
                                                               const float* __restrict__ dv_out,
                                                               AggGrad A, LayerGrads O) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  layer_to_lds_x3<true>(sm, P);
  __syncthreads();
  const __bf16* img = reinterpret_cast<const __bf16*>(sm);  // W^T
  const float* sWsV = sm + kXImgFloats;
  const float* sWsv = sWsV + S * LD16;
  const float* sWh = sWsv + V * LD128;
  const float* sWv = sWh + V * LD16;
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int64_t nchunks = (E + 15) / 16;
  const int64_t wave = (int64_t)blockIdx.x * (kGT / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (kGT / 64);
  for (int64_t c = wave; c < nchunks; c += nwaves) {
    const Chunk k = chunk_edge(c, i, E);
    f32x4 s[S / 16], v[3][1];
    ld_row<S / 16>(s, s_in + k.e * S, g);
    ld_vrow<1>(v, v_in + k.e * (3 * V), g);
    LayerFwd F;
    layer_forward_x3<true>(sm, s, v, F, lane, i, g);
    f32x4 dv[3][1];
    ld_grad_rows<AGG>(ds_out, dv_out, A, k.e, g, s, dv);
    if (ACT) {
#pragma unroll
      for (int p = 0; p < S / 16; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) s[p][q] = F.spre[p][q] > 0.f ? s[p][q] : 0.f;
    }
    f32x4 dgate[1];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float dsg = dv[0][0][q] * F.vpre[0][0][q] + dv[1][0][q] * F.vpre[1][0][q] + dv[2][0][q] * F.vpre[2][0][q];
      dgate[0][q] = dsg * F.sg[0][q] * (1.f - F.sg[0][q]);
#pragma unroll
      for (int x = 0; x < 3; ++x) dv[x][0][q] *= F.sg[0][q];  // dvpre
    }
    gemm_wtx<S / 16, 1>(sWsv, LD128, dgate, s, i, g);  // dspre += Wsv^T dgate
    if (k.valid) {
      st_row<S / 16>(O.dspre + k.e * S, s, g);
      if (O.spre) st_row<S / 16>(O.spre + k.e * S, F.spre, g);
      st_row<1>(O.dgate + k.e * V, dgate, g);
      st_row<1>(O.vn + k.e * V, F.vn, g);
      if (O.vh) st_vrow<1>(O.vh + k.e * (3 * V), F.vh, g);
      st_vrow<1>(O.dvpre + k.e * (3 * V), dv, g);
    }
    // ds_in = Ws_s^T dspre (image rows k) ; dvn = Ws_v^T dspre (f32)
    f32x4 dsin[S / 16], dvn[1];
    zero(dsin);
    zero(dvn);
    gemm_x3(img, s, dsin, i, g);
    gemm_wtx<1, S / 16>(sWsV, LD16, s, dvn, i, g);
    if (k.valid) st_row<S / 16>(O.ds_in + k.e * S, dsin, g);
    f32x4 dvh[3][1];
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      zero(dvh[x]);
      gemm_wtx<1, 1>(sWv, LD16, dv[x], dvh[x], i, g);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float f = F.sq[0][q] > 1e-8f ? dvn[0][q] / F.vn[0][q] : 0.f;
#pragma unroll
      for (int x = 0; x < 3; ++x) dvh[x][0][q] += f * F.vh[x][0][q];
    }
    if (k.valid) st_vrow<1>(O.dvh + k.e * (3 * V), dvh, g);
    f32x4 dvin[3][1];
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      zero(dvin[x]);
      gemm_wtx<1, 1>(sWh, LD16, dvh[x], dvin[x], i, g);
    }
    if (k.valid) st_vrow<1>(O.dv_in + k.e * (3 * V), dvin, g);
  }
}

int64_t grid_for(int64_t E) {
  const int64_t chunks = ceil_div(E, (int64_t)16);
  int64_t b = ceil_div(chunks, (int64_t)(kGT / 64));
  const int64_t cap = (int64_t)device_cu_count();
  if (b > cap) b = cap;
  return b < 1 ? 1 : b;
}

template <class K>
int set_smem(K k, size_t bytes) {
  return hip_check(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)bytes));
}

bool al16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_gvp_layer_fwd_f32(int64_t n_edges, int relu, const float* s_in, const float* v_in,
                          const float* Ws, const float* bs, const float* Wsv, const float* bsv,
                          const float* Wh, const float* Wv, float* s_out, float* v_out,
                          void* stream) {
  GMP_CHECK_ARG(n_edges >= 0);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(s_in && v_in && Ws && bs && Wsv && bsv && Wh && Wv && s_out && v_out);
  GMP_CHECK_ARG(al16(s_in) && al16(v_in) && al16(s_out) && al16(v_out));
  const LayerW P{Ws, bs, Wsv, bsv, Wh, Wv};
  const unsigned G = (unsigned)grid_for(n_edges);
  hipStream_t s = as_stream(stream);
  int rc;
  const size_t smx = kLayerSmemX3 * sizeof(float);
  auto k = relu ? gvp_layer_fwd_x3_kernel<1> : gvp_layer_fwd_x3_kernel<0>;
  if ((rc = set_smem(k, smx))) return rc;
  k<<<G, kGT, smx, s>>>(n_edges, s_in, v_in, P, s_out, v_out);
  return launch_status();
}

}  // extern "C"

namespace {
int layer_bwd(int64_t n_edges, int relu, int agg, const AggGrad& A, const float* s_in,
              const float* v_in, const float* Ws, const float* bs, const float* Wsv,
              const float* bsv, const float* Wh, const float* Wv, const float* ds_out,
              const float* dv_out, float* ds_in, float* dv_in, float* dspre, float* spre,
              float* dgate, float* vn, float* vh, float* dvpre, float* dvh, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(s_in && v_in && Ws && bs && Wsv && bsv && Wh && Wv && ds_out && dv_out);
  GMP_CHECK_ARG(ds_in && dv_in && dspre && dgate && vn && dvpre && dvh);  // spre, vh: optional
  GMP_CHECK_ARG(al16(s_in) && al16(v_in) && al16(ds_out) && al16(dv_out) && al16(ds_in) &&
                al16(dv_in) && al16(dspre) && al16(spre) && al16(dgate) && al16(vn) &&
                al16(vh) && al16(dvpre) && al16(dvh));
  const LayerW P{Ws, bs, Wsv, bsv, Wh, Wv};
  const LayerGrads O{ds_in, dv_in, dspre, spre, dgate, vn, vh, dvpre, dvh};
  const unsigned G = (unsigned)grid_for(n_edges);
  hipStream_t s = as_stream(stream);
  int rc;
  const size_t smx = kLayerSmemX3 * sizeof(float);
  auto k = relu ? (agg == 0 ? gvp_layer_bwd_x3_kernel<1, 0>
                            : (agg == 1 ? gvp_layer_bwd_x3_kernel<1, 1>
                                        : gvp_layer_bwd_x3_kernel<1, 2>))
                : (agg == 0 ? gvp_layer_bwd_x3_kernel<0, 0>
                            : (agg == 1 ? gvp_layer_bwd_x3_kernel<0, 1>
                                        : gvp_layer_bwd_x3_kernel<0, 2>));
  if ((rc = set_smem(k, smx))) return rc;
  k<<<G, kGT, smx, s>>>(n_edges, s_in, v_in, P, ds_out, dv_out, A, O);
  return launch_status();
}
}  // namespace

extern "C" {

int gmp_gvp_layer_bwd_f32(int64_t n_edges, int relu, const float* s_in, const float* v_in,
                          const float* Ws, const float* bs, const float* Wsv, const float* bsv,
                          const float* Wh, const float* Wv, const float* ds_out,
                          const float* dv_out, float* ds_in, float* dv_in, float* dspre,
                          float* spre, float* dgate, float* vn, float* vh, float* dvpre,
                          float* dvh, void* stream) {
  return layer_bwd(n_edges, relu, 0, AggGrad{nullptr, nullptr, 0}, s_in, v_in, Ws, bs, Wsv, bsv,
                   Wh, Wv, ds_out, dv_out, ds_in, dv_in, dspre, spre, dgate, vn, vh, dvpre, dvh,
                   stream);
}

int gmp_gvp_msg0_bwd_agg_f32(int64_t n_edges, int64_t n_nodes, const int64_t* send,
                             const int64_t* recv, const int64_t* perm, const int64_t* rowptr,
                             const float* P, const float* Q, const float* es, const float* ev,
                             const float* We, const float* Wn, const float* b, const float* Wv,
                             const float* Wsv, const float* bsv, const float* wev,
                             const float* ds_out, const float* dv_out, float* dspre, float* spre,
                             float* dgate, float* vn, float* vh, float* dvpre, float* dvh,
                             float* des, float* dev, float* dPb, float* dQb, float* sgate_recv,
                             float* svpre_recv, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && n_edges < (1LL << 31) && n_nodes < (1LL << 31));
  if (n_nodes == 0) return GMP_OK;
  GMP_CHECK_ARG(rowptr && dPb && dQb && sgate_recv && svpre_recv && al16(dPb) && al16(dQb) &&
                al16(sgate_recv) && al16(svpre_recv));
  if (n_edges > 0) {
    GMP_CHECK_ARG(send && recv && P && Q && es && ev && We && Wn && b && Wv && Wsv && bsv &&
                  wev && ds_out && dv_out);
    GMP_CHECK_ARG(dspre && dgate && vn && dvpre && dvh && des && dev);  // spre, vh: optional
    GMP_CHECK_ARG(al16(P) && al16(Q) && al16(es) && al16(ds_out) && al16(dv_out) &&
                  al16(dspre) && al16(spre) && al16(dgate) && al16(vn) && al16(vh) &&
                  al16(dvpre) && al16(dvh) && al16(des));
  }
  const Msg0W W{We, Wn, b, Wv, Wsv, bsv, wev};
  const Msg0Grads O{dspre, spre, dgate, vn, vh, dvpre, dvh, des, dev};
  int64_t G = (int64_t)device_cu_count();
  const int64_t cap = ceil_div(n_edges, (int64_t)(kGT / 64) * 64);
  if (G > cap) G = cap;
  if (G < 1) G = 1;
  const size_t smem = kM0AggSmem * sizeof(float);
  int rc;
  if ((rc = set_smem(gvp_msg0_bwd_agg_kernel, smem))) return rc;
  gvp_msg0_bwd_agg_kernel<<<(unsigned)G, kGT, smem, as_stream(stream)>>>(
      n_edges, n_nodes, send, recv, perm, rowptr, P, Q, es, ev, W, ds_out, dv_out, O, dPb, dQb,
      sgate_recv, svpre_recv);
  return launch_status();
}

int gmp_gvp_layer_fwd_agg_f32(int64_t n_edges, int64_t n_nodes, int reduce, const int64_t* perm,
                              const int64_t* skey, const int64_t* rowptr, const float* s_in,
                              const float* v_in, const float* Ws, const float* bs,
                              const float* Wsv, const float* bsv, const float* Wh,
                              const float* Wv, float* s_agg, float* v_agg, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && n_edges < (1LL << 31) && n_nodes < (1LL << 31));
  GMP_CHECK_ARG(reduce == GMP_REDUCE_SUM || reduce == GMP_REDUCE_MEAN);
  if (n_nodes == 0) return GMP_OK;
  GMP_CHECK_ARG(rowptr && s_agg && v_agg && al16(s_agg) && al16(v_agg));
  GMP_CHECK_ARG(n_edges == 0 || (skey && s_in && v_in && al16(s_in) && al16(v_in) && Ws && bs &&
                                 Wsv && bsv && Wh && Wv));
  const LayerW P{Ws, bs, Wsv, bsv, Wh, Wv};
  // enough waves for the chip, but whole receiver ranges of >= ~4 chunks each
  int64_t G = (int64_t)device_cu_count();
  const int64_t cap = ceil_div(n_edges, (int64_t)(kGT / 64) * 64);
  if (G > cap) G = cap;
  if (G < 1) G = 1;
  hipStream_t s = as_stream(stream);
  const size_t smem = kAggSmem * sizeof(float);
  auto k = reduce == GMP_REDUCE_MEAN ? gvp_layer_fwd_agg_kernel<true> : gvp_layer_fwd_agg_kernel<false>;
  int rc;
  if ((rc = set_smem(k, smem))) return rc;
  k<<<(unsigned)G, kGT, smem, s>>>(n_edges, n_nodes, s_in, v_in, P, perm, skey, rowptr, s_agg,
                                    v_agg);
  return launch_status();
}

int gmp_gvp_layer_bwd_agg_f32(int64_t n_edges, int64_t n_nodes, int reduce, const int64_t* index,
                              const int64_t* rowptr, int relu, const float* s_in,
                              const float* v_in, const float* Ws, const float* bs,
                              const float* Wsv, const float* bsv, const float* Wh,
                              const float* Wv, const float* ds_node, const float* dv_node,
                              float* ds_in, float* dv_in, float* dspre, float* spre,
                              float* dgate, float* vn, float* vh, float* dvpre, float* dvh,
                              void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0 && index && (reduce == GMP_REDUCE_SUM ||
                                          (reduce == GMP_REDUCE_MEAN && rowptr)));
  if (n_edges > 0) GMP_CHECK_ARG(n_nodes > 0);
  return layer_bwd(n_edges, relu, reduce == GMP_REDUCE_MEAN ? 2 : 1,
                   AggGrad{index, rowptr, n_nodes}, s_in, v_in, Ws, bs, Wsv, bsv, Wh, Wv, ds_node,
                   dv_node, ds_in, dv_in, dspre, spre, dgate, vn, vh, dvpre, dvh, stream);
}

int gmp_gvp_msg0_fwd_f32(int64_t n_edges, const int64_t* send, const int64_t* recv,
                         const float* P, const float* Q, const float* es, const float* ev,
                         const float* We, const float* Wn, const float* b, const float* Wv,
                         const float* Wsv, const float* bsv, const float* wev, float* s_out,
                         float* v_out, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(send && recv && P && Q && es && ev && We && Wn && b && Wv && Wsv && bsv && wev &&
                s_out && v_out);
  GMP_CHECK_ARG(al16(P) && al16(Q) && al16(es) && al16(s_out) && al16(v_out));
  const Msg0W W{We, Wn, b, Wv, Wsv, bsv, wev};
  const size_t smem = kMsg0Smem * sizeof(float);
  int rc;
  if ((rc = set_smem(gvp_msg0_fwd_kernel, smem))) return rc;
  gvp_msg0_fwd_kernel<<<(unsigned)grid_for(n_edges), kGT, smem, as_stream(stream)>>>(
      n_edges, send, recv, P, Q, es, ev, W, s_out, v_out);
  return launch_status();
}

int gmp_gvp_msg0_bwd_f32(int64_t n_edges, const int64_t* send, const int64_t* recv,
                         const float* P, const float* Q, const float* es, const float* ev,
                         const float* We, const float* Wn, const float* b, const float* Wv,
                         const float* Wsv, const float* bsv, const float* wev,
                         const float* ds_out, const float* dv_out, float* dspre, float* spre,
                         float* dgate, float* vn, float* vh, float* dvpre, float* dvh,
                         float* des, float* dev, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(send && recv && P && Q && es && ev && We && Wn && b && Wv && Wsv && bsv && wev &&
                ds_out && dv_out);
  GMP_CHECK_ARG(dspre && dgate && vn && dvpre && dvh && des && dev);  // spre, vh: optional
  GMP_CHECK_ARG(al16(P) && al16(Q) && al16(es) && al16(ds_out) && al16(dv_out) && al16(dspre) &&
                al16(spre) && al16(dgate) && al16(vn) && al16(vh) && al16(dvpre) && al16(dvh) &&
                al16(des));
  const Msg0W W{We, Wn, b, Wv, Wsv, bsv, wev};
  const Msg0Grads O{dspre, spre, dgate, vn, vh, dvpre, dvh, des, dev};
  const size_t smem = kMsg0Smem * sizeof(float);
  int rc;
  if ((rc = set_smem(gvp_msg0_bwd_kernel, smem))) return rc;
  gvp_msg0_bwd_kernel<<<(unsigned)grid_for(n_edges), kGT, smem, as_stream(stream)>>>(
      n_edges, send, recv, P, Q, es, ev, W, ds_out, dv_out, O);
  return launch_status();
}

}  // extern "C"
