// K4: EGNN fused edge message + segmented aggregation (forward and backward), gfx950.
//
// Reference: models/layers/egnn_layer.py:62-80 (message / aggregate) with the MLPs of :28-39.
// Design:
//  * edges are receiver-sorted (CSR); every wave owns a node-aligned, edge-balanced range and
//    walks it in 16-edge chunks, so each receiver's sum is formed inside one wave in a fixed
//    order (deterministic, no atomics);
//  * lane l holds edge e = l & 15 and feature group g = l >> 4: features 16p + 4g + c
//    (p < d/16, c < 4) — exactly the register order that v_mfma_f32_16x16x4_f32 uses for its B
//    operand AND produces as its C/D accumulator when computing out^T = W . x^T, so the chain
//    Linear -> LN -> act -> Linear -> LN -> act -> Linear -> LN -> act -> dot stays in
//    registers with no LDS transpose (exact fp32: the f32 MFMA is a k-ordered fmaf chain);
//  * W2 / W3 (d x d, row-major) live in LDS with row stride d+4 floats; W.x reads W rows with
//    ds_read_b128, W^T.g reads W columns with conflict-free ds_read_b32;
//  * the first Linear(2d+1 -> d) is split into per-node projections AB = [h W1a^T | h W1b^T]
//    (a node-level GEMM done once per node by the caller) plus a rank-1 distance term;
//  * HF path (default): the two d x d products per chunk run on v_mfma_f32_16x16x32_f16 over
//    2-plane fp16 splits (hi + lo, 22-bit operands; products hi*hi + hi*lo + lo*hi, f32
//    accumulation) with power-of-two scaling (W per matrix, x per edge) that keeps the planes
//    in fp16 range; the planes of W take the LDS of the f32 W (gemm_h2 below).  The f32 path
//    (exact fmaf chains on the f32 MFMA) stays selectable: gmp_egnn_set_f32_mfma(1).
#include <mutex>
#include <set>
#include <tuple>

#include "gmp_egnn_common.h"

namespace gmp {
namespace {

// ================================================================================== forward
// SAVE (training): also write the LayerNorm outputs x_hat1, x_hat2 (and x_hat3 when save_planes
// is 3) into xsave ((save_planes, E, d), rows in receiver-sorted edge order) and their 1/std
// (rsave, (E, 3)) for the backward.
template <int D, int ACT, bool MSG_MEAN, bool SAVE, bool HF>
__global__ __launch_bounds__(fwd_waves<HF>() * 64, fwd_waves<HF>() / 4) void egnn_fwd_kernel(
    int64_t n_nodes, int64_t n_edges, const float* __restrict__ AB, const float* __restrict__ pos,
    const int64_t* __restrict__ rowptr, const int64_t* __restrict__ recv,
    const int64_t* __restrict__ send, gmp_egnn_params P, float eps, int64_t n_waves,
    float* __restrict__ m_aggr, float* __restrict__ pos_aggr, float* __restrict__ xsave,
    float* __restrict__ rsave, int save_planes) {
  constexpr int T = Cfg<D>::T, LDW = Cfg<D>::LDW;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const float* sW2 = smem;
  const float* sW3 = smem + D * LDW;
  _Float16* hW = reinterpret_cast<_Float16*>(smem + smem_mats_off<D, fwd_waves<HF>(), HF>());
  const _Float16* hW2 = hW;
  const _Float16* hW3 = hW + HCfg<D>::MAT;
  float* sVw = smem + smem_vec_off<D, fwd_waves<HF>(), HF>();
  const float* sV = sVw;
  float* carry0 = smem + smem_carry_off<D, fwd_waves<HF>(), HF>();
  if constexpr (HF) load_params_hf<D, false, 3, ACT>(sVw, hW, carry0, P);
  else load_params_to_lds<D>(smem, P);
  __syncthreads();
  const int sw2 = HF ? (int)sV[NV * D] : 0, sw3 = HF ? (int)sV[NV * D + 1] : 0;
  const int ex2 = HF ? (int)sV[NV * D + 2] : 0, ex3 = HF ? (int)sV[NV * D + 3] : 0;
  constexpr bool XS = ACT == GMP_ACT_RELU;  // relu: y1 comes pre-scaled for the W2 product

  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* cbuf = carry0 + (wid * 4 + g) * carry_stride<D>();
  carry_clear<D>(carry0 + wid * 4 * carry_stride<D>(), lane);
  const WaveRange wr = wave_range(rowptr, n_nodes, n_edges, n_waves, wid, fwd_waves<HF>());
  zero_isolated<D>(wr, rowptr, m_aggr, pos_aggr, lane);
  const float b4 = P.b4[0];
  int carry_node = -1;
  EdgeIJ nxt = load_ij(wr.e_lo, li, wr.e_hi, recv, send);
  // land the first ids before the loop, so that the wait at the loop head only has to cover
  // the ids prefetched by the previous chunk (a counted vmcnt, not a full drain)
  asm volatile("" ::"v"(nxt.i), "v"(nxt.j));

  for (int base = wr.e_lo; base < wr.e_hi; base += 16) {
    asm volatile("" ::: "memory");  // keep LDS parameter reads inside the loop
    const EdgeIJ cur = nxt;
    nxt = load_ij(base + 16, li, wr.e_hi, recv, send);
    EdgeCtx c = edge_ctx(cur, base, li, wr.e_hi, (int)n_nodes, rowptr, pos);

    const size_t ED = (size_t)n_edges * D;
    f32x4 x[T];  // y1 = act(LN1(pre1))
    load_pre1<D, HF>(x, rowp(AB, c.i, 2 * D), rowp(AB, c.j, 2 * D) + D, sV, c, g);
    const float r1 = ln_normalize<D, HF>(x, eps);
    // chunk windows: edges [base, base + ne) of the saved tensors, receivers [i0, i1]
    const int ne = __builtin_amdgcn_readfirstlane(min(16, wr.e_hi - base));
    const int i0 = __builtin_amdgcn_readfirstlane(c.i);
    const int i1 = __builtin_amdgcn_readlane(c.i, 15);
    const unsigned eoff = c.valid ? (unsigned)(li * D * 4) : kOob;
    if (SAVE) store_row_w<D, kAuxNT>(rows_window(xsave, base, ne, D), eoff, x, g);
    affine_act<D, ACT>(x, sV, HF ? V_LN1WS : V_LN1W, HF ? V_LN1BS : V_LN1B, g);

    f32x4 m[T];  // m = act(LN2(W2 y1 + b2))
    float r2;
    if constexpr (HF) {
      load_vec<D>(m, sV, V_B2S, g);
      gemm_h2s<D, XS>(hW2, ex2, x, m, li, g);
      r2 = ln_rms<D>(m, eps, ex2 + sw2);
    } else {
      load_vec<D>(m, sV, V_B2, g);
      gemm_wx<D>(sW2, x, m, li, g);
      r2 = ln_normalize<D, false>(m, eps);
    }
    if (SAVE) store_row_w<D, kAuxNT>(rows_window(xsave + ED, base, ne, D), eoff, m, g);
    affine_act<D, ACT>(m, sV, V_LN2W, V_LN2B, g);  // (unscaled: m is also the message)

    // y3 = act(LN3(W3 m + b3)); s = w4 . y3 + b4   (x reused)
    float r3;
    if constexpr (HF) {
      load_vec<D>(x, sV, V_B3S, g);
      gemm_h2s<D, false>(hW3, ex3, m, x, li, g);
      r3 = ln_rms<D>(x, eps, ex3 + sw3);
    } else {
      load_vec<D>(x, sV, V_B3, g);
      gemm_wx<D>(sW3, m, x, li, g);
      r3 = ln_normalize<D, false>(x, eps);
    }
    if (SAVE) {
      if (save_planes == 3)
        store_row_w<D, kAuxNT>(rows_window(xsave + 2 * ED, base, ne, D), eoff, x, g);
      store3_w<kAuxNT>(rows_window(rsave, base, ne, 3), (g == 0 && c.valid) ? li * 12u : kOob,
                       r1, r2, r3);
    }
    affine_act<D, ACT>(x, sV, V_LN3W, V_LN3B, g);
    float sp = 0.f;
#pragma unroll
    for (int p = 0; p < T; ++p) {
      const f32x4 w = vec4<D>(sV, V_W4, p, g);
      sp += w[0] * x[p][0] + w[1] * x[p][1] + w[2] * x[p][2] + w[3] * x[p][3];
    }
    const float s_e = sum_groups(sp) + b4;

    // segmented sums over receivers: m -> m_aggr (sum / mean), rel*s -> pos_aggr (mean)
    const int head = c.valid ? (int)((c.seg0 > base) ? (c.seg0 - base) : 0) : li;
    const bool is_end = c.valid && (c.e == c.seg1 - 1);
    const bool take = (li == 0) && c.valid && (c.i == carry_node);
    float pv[3] = {c.rx * s_e, c.ry * s_e, c.rz * s_e};
    carry_apply<D>(cbuf, m, pv, take);
    seg_scan<T>(m, li, head);
    {
      f32x4 pw[1] = {{pv[0], pv[1], pv[2], 0.f}};
      seg_scan<1>(pw, li, head);
      pv[0] = pw[0][0]; pv[1] = pw[0][1]; pv[2] = pw[0][2];
    }
    {  // receiver rows, stored by the last edge of each segment
      const float deg = (float)(c.seg1 - c.seg0);
      // 1/deg: v_rcp_f32 (~1 ulp) on the HF path, the correctly rounded quotient on the f32 one
      const float rdeg = HF ? __builtin_amdgcn_rcpf(deg) : 1.f / deg;
      if (MSG_MEAN) {  // only segment ends (an open segment's m is the next chunk's carry)
        const float sc = is_end ? rdeg : 1.f;
#pragma unroll
        for (int p = 0; p < T; ++p) m[p] *= sc;
      }
      const int nn = max(i1 - i0 + 1, 0);  // (receiver-sorted: i0 <= i <= i1)
      store_row_w<D, 0>(rows_window(m_aggr, i0, nn, D), is_end ? (unsigned)((c.i - i0) * D * 4) : kOob,
                        m, g);
      store3_w<0>(rows_window(pos_aggr, i0, nn, 3),
                  (is_end && g == 0) ? (unsigned)((c.i - i0) * 12) : kOob,
                  HF ? pv[0] * rdeg : pv[0] / deg, HF ? pv[1] * rdeg : pv[1] / deg,
                  HF ? pv[2] * rdeg : pv[2] / deg);
    }
    if (li == 15) carry_store<D>(cbuf, m, pv);
    carry_node = __builtin_amdgcn_readlane(c.i, 15);
  }
}

// ================================================================================== backward
// max |x| over the wave's 16 edges x d features (row_ror butterfly inside each 16-lane row,
// then the 4 lane groups), folded into an LDS word by one lane
template <int D>
__device__ __forceinline__ void fold_max(unsigned* word, const f32x4 (&x)[D / 16], int lane) {
  float v = 0.f;
#pragma unroll
  for (int p = 0; p < D / 16; ++p)
    v = fmaxf(v, fmaxf(fmaxf(fabsf(x[p][0]), fabsf(x[p][1])), fmaxf(fabsf(x[p][2]), fabsf(x[p][3]))));
  v = fmaxf(v, dpp<0x128>(v));
  v = fmaxf(v, dpp<0x124>(v));
  v = fmaxf(v, dpp<0x122>(v));
  v = fmaxf(v, dpp<0x121>(v));
  v = max_groups(v);
  if (lane == 0) atomicMax(word, __float_as_uint(v));
}

constexpr int NVG = 8;  // vector-gradient outputs: ln1w ln1b ln2w ln2b ln3w ln3b w4 w1d
enum GradVec { G_LN1W = 0, G_LN1B, G_LN2W, G_LN2B, G_LN3W, G_LN3B, G_W4, G_W1D };

template <int D>
__device__ __forceinline__ float slot(const f32x4 (&x)[D / 16], int s) { return x[s >> 2][s & 3]; }
template <int D>
__device__ __forceinline__ float vslot(const float* sV, int v, int s, int g) {
  return sV[v * D + featq(s, g)];
}

// Backward from the forward's saved x_hat1..3 / rstd (no forward recompute, no AB gathers):
// two transposed GEMMs (W3^T, W2^T) per 16-edge chunk.
// AMAX: fold max |dpre2|, |dpre3| into amax[0], amax[1] (float bit patterns; the scales of the
// HF weight-gradient outer sums, gmp_edge_outer_sum_act_hf_f32)
// RC (what the backward recomputes instead of reading; bitwise the forward's values, with the
// forward's saved 1/std and W3 from the W3^T image by transposed reads):
//   0: nothing (the forward saved x_hat1..3: save_planes 3);
//   1: x_hat3 from x_hat2 (the forward saved x_hat1, x_hat2: save_planes 2, the default).
// (r03 also measured rebuilding x_hat1 / x_hat2 from the node projections AB: slower, removed.)
template <int D, int ACT, bool MSG_MEAN, bool HF, bool AMAX, int RC>
__global__ __launch_bounds__(kBwdWaves * 64, 2) void egnn_bwd_kernel(
    int64_t n_nodes, int64_t n_edges, const float* __restrict__ pos,
    const int64_t* __restrict__ rowptr, const int64_t* __restrict__ recv,
    const int64_t* __restrict__ send, gmp_egnn_params P, int64_t n_waves,
    const float* __restrict__ xsave, const float* __restrict__ rsave,
    const float* __restrict__ g_maggr, const float* __restrict__ g_paggr, float* __restrict__ dA,
    float* __restrict__ dpos_recv, float* __restrict__ dpre1_out, float* __restrict__ gdiff_out,
    float* __restrict__ dpre2_out, float* __restrict__ dpre3_out, float* __restrict__ partials,
    unsigned* __restrict__ amax) {
  constexpr int T = Cfg<D>::T, LDW = Cfg<D>::LDW, K = VecAcc<D>::K;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const float* sW2t = smem;  // W2^T
  const float* sW3t = smem + D * LDW;  // W3^T
  _Float16* hW = reinterpret_cast<_Float16*>(smem + smem_mats_off<D, kBwdWaves, HF>());
  const _Float16* hW2t = hW;
  const _Float16* hW3t = hW + HCfg<D>::MAT;
  float* sVw = smem + smem_vec_off<D, kBwdWaves, HF>();
  const float* sV = sVw;
  // (HF: W3^T centred as the forward's W3, so the x_hat3 recompute is bitwise the forward's; W2 as
  // given)
  if constexpr (HF) load_params_hf<D, true, 2, ACT>(sVw, hW, smem + smem_carry_off<D, kBwdWaves, HF>(), P);
  else load_params_to_lds<D, true>(smem, P);
  __syncthreads();
  const int sw2 = HF ? (int)sV[NV * D] : 0, sw3 = HF ? (int)sV[NV * D + 1] : 0;
  const int ex3 = HF ? (int)sV[NV * D + 3] : 0;  // the forward's static W3 input exponent
  const float* xr1 = xsave;
  const float* xr2 = xsave + (size_t)n_edges * D;
  // AMAX: per-chunk wave maxima go to two LDS words (no loop-carried registers: the kernel sits
  // at 256 VGPRs), folded into amax[] once per workgroup at the end
  unsigned* lmx = reinterpret_cast<unsigned*>(const_cast<float*>(sV) + NV * D + 10);
  if (AMAX) {
    if (threadIdx.x < 2) lmx[threadIdx.x] = 0u;
    __syncthreads();
  }

  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* cbuf = smem + smem_carry_off<D, kBwdWaves, HF>() + (wid * 4 + g) * carry_stride<D>();
  carry_clear<D>(smem + smem_carry_off<D, kBwdWaves, HF>() + wid * 4 * carry_stride<D>(), lane);
  const WaveRange wr = wave_range(rowptr, n_nodes, n_edges, n_waves, wid, kBwdWaves);
  zero_isolated<D>(wr, rowptr, dA, dpos_recv, lane);
  const float b4 = P.b4[0];
  const size_t ED = (size_t)n_edges * D;

  float vacc[NVG][K];
#pragma unroll
  for (int v = 0; v < NVG; ++v)
#pragma unroll
    for (int k = 0; k < K; ++k) vacc[v][k] = 0.f;
  float db4 = 0.f;
  int carry_node = -1;
  EdgeIJ nxt = load_ij(wr.e_lo, li, wr.e_hi, recv, send);
  // land the first ids before the loop, so that the wait at the loop head only has to cover
  // the ids prefetched by the previous chunk (a counted vmcnt, not a full drain)
  asm volatile("" ::"v"(nxt.i), "v"(nxt.j));

  for (int base = wr.e_lo; base < wr.e_hi; base += 16) {
    asm volatile("" ::: "memory");
    const EdgeIJ cur = nxt;
    nxt = load_ij(base + 16, li, wr.e_hi, recv, send);
    EdgeCtx c = edge_ctx(cur, base, li, wr.e_hi, (int)n_nodes, rowptr, pos);
    // every per-chunk load below is issued branch-free at the clamped edge / receiver (one
    // round trip); lanes past the range are zeroed through ds / gscale / rstd = 0
    const float rs1 = rsave[3 * (size_t)c.ec + 0];
    const float rs2 = rsave[3 * (size_t)c.ec + 1];
    const float rs3 = rsave[3 * (size_t)c.ec + 2];
    const float gp0 = g_paggr[3 * c.i + 0], gp1 = g_paggr[3 * c.i + 1], gp2 = g_paggr[3 * c.i + 2];
    f32x4 x[T], xh2[T], z[T];
    if constexpr (RC == 1) load_row<D>(x, rowp(xsave + ED, c.ec, D), g);  // x = xhat2
    else load_row<D>(z, rowp(xsave + 2 * ED, c.ec, D), g);               // z = xhat3
    __builtin_amdgcn_sched_barrier(0);
    edge_geom<HF>(c);
    const float rstd1 = c.valid ? rs1 : 0.f;
    const float rstd2 = c.valid ? rs2 : 0.f;
    const float rstd3 = c.valid ? rs3 : 0.f;
    if constexpr (RC == 1) {
      // z = xhat3 = LN3(W3 act(LN2 affine(xhat2)) + b3) with the forward's 1/std: the forward's
      // products (same operands, planes, scales and MFMA order) -> bitwise its x_hat3
      if constexpr (HF) {
        affine_act<D, ACT>(x, sV, V_LN2W, V_LN2B, g);
        load_vec<D>(z, sV, V_B3S, g);
        gemm_h2s_tr<D, false>(hW3t, ex3, x, z, lane, g);
        const float r = ldexpf(rs3, -(ex3 + sw3));  // ln_rms's multiplier
#pragma unroll
        for (int p = 0; p < T; ++p) z[p] *= r;
      } else {
        affine_act<D, ACT>(x, sV, V_LN2W, V_LN2B, g);
        load_vec<D>(z, sV, V_B3, g);
        gemm_wtx<D>(sW3t, x, z, li, g);
        ln_recenter<D>(z, rs3);
      }
    }

  // ---------------- pos-branch backward
    const float inv_deg = c.valid ? 1.f / (float)(c.seg1 - c.seg0) : 0.f;
    const float gscale = MSG_MEAN ? inv_deg : (c.valid ? 1.f : 0.f);
    const float gpx = gp0 * inv_deg;
    const float gpy = gp1 * inv_deg;
    const float gpz = gp2 * inv_deg;
    const float ds = gpx * c.rx + gpy * c.ry + gpz * c.rz;  // dL/ds_e
    if (g == 0) db4 += ds;

    float sp = 0.f;
#pragma unroll
    for (int p = 0; p < T; ++p) {
      const f32x4 w3 = vec4<D>(sV, V_LN3W, p, g), b3 = vec4<D>(sV, V_LN3B, p, g);
      const f32x4 w4 = vec4<D>(sV, V_W4, p, g);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float zz = z[p][q] * w3[q] + b3[q];
        sp += w4[q] * act_f<ACT>(zz);
        x[p][q] = ds * w4[q] * act_df<ACT>(zz);  // dz3 (m already stored)
      }
    }
    const float s_e = sum_groups(sp) + b4;
    accumulate_vec<D>([&](int s) {
      return ds * act_f<ACT>(slot<D>(z, s) * vslot<D>(sV, V_LN3W, s, g) + vslot<D>(sV, V_LN3B, s, g));
    }, vacc[G_W4], li);
    accumulate_vec<D>([&](int s) { return slot<D>(x, s) * slot<D>(z, s); }, vacc[G_LN3W], li);
    accumulate_vec<D>([&](int s) { return slot<D>(x, s); }, vacc[G_LN3B], li);
    load_row<D>(xh2, rowp(g_maggr, c.i, D), g);  // g_m_aggr[i] (dm seed, below)
    __builtin_amdgcn_sched_barrier(0);             // issue it here, ahead of the LN backward
#pragma unroll
    for (int p = 0; p < T; ++p) x[p] *= vec4<D>(sV, V_LN3W, p, g);
    ln_backward<D>(x, z, rstd3);  // x = dpre3
    if (AMAX) fold_max<D>(lmx + 1, x, lane);
    const int ne = __builtin_amdgcn_readfirstlane(min(16, wr.e_hi - base));
    const int i0 = __builtin_amdgcn_readfirstlane(c.i);
    const int i1 = __builtin_amdgcn_readlane(c.i, 15);
    const unsigned eoff = c.valid ? (unsigned)(li * D * 4) : kOob;
    store_row_w<D, kAuxNT>(rows_window(dpre3_out, base, ne, D), eoff, x, g);

    // ---------------- dm = g_m_aggr[i] (/deg) + W3^T dpre3   (z); xhat2 -> xh2 in flight
#pragma unroll
    for (int p = 0; p < T; ++p) z[p] = xh2[p] * gscale;
    load_row<D>(xh2, rowp(xr2, c.ec, D), g);
    if constexpr (HF) gemm_h2<D, true>(hW3t, sw3, 0, x, z, li, g);  // z += W3^T dpre3
    else gemm_wx<D, 2>(sW3t, x, z, li, g);
#pragma unroll
    for (int p = 0; p < T; ++p) {
      const f32x4 w = vec4<D>(sV, V_LN2W, p, g), b = vec4<D>(sV, V_LN2B, p, g);
#pragma unroll
      for (int q = 0; q < 4; ++q) z[p][q] *= act_df<ACT>(xh2[p][q] * w[q] + b[q]);  // dz2
    }
    accumulate_vec<D>([&](int s) { return slot<D>(z, s) * slot<D>(xh2, s); }, vacc[G_LN2W], li);
    accumulate_vec<D>([&](int s) { return slot<D>(z, s); }, vacc[G_LN2B], li);
#pragma unroll
    for (int p = 0; p < T; ++p) z[p] *= vec4<D>(sV, V_LN2W, p, g);
    ln_backward<D>(z, xh2, rstd2);  // z = dpre2
    if (AMAX) fold_max<D>(lmx, z, lane);
    store_row_w<D, kAuxNT>(rows_window(dpre2_out, base, ne, D), eoff, z, g);

    // ---------------- dy1 = W2^T dpre2 (x); xhat1 -> xh2 in flight
    load_row<D>(xh2, rowp(xr1, c.ec, D), g);
#pragma unroll
    for (int p = 0; p < T; ++p) x[p] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (HF) gemm_h2<D, true>(hW2t, sw2, 0, z, x, li, g);  // x = W2^T dpre2
    else gemm_wx<D, 2>(sW2t, z, x, li, g);
#pragma unroll
    for (int p = 0; p < T; ++p) {
      const f32x4 w = vec4<D>(sV, V_LN1W, p, g), b = vec4<D>(sV, V_LN1B, p, g);
#pragma unroll
      for (int q = 0; q < 4; ++q) x[p][q] *= act_df<ACT>(xh2[p][q] * w[q] + b[q]);  // dz1
    }
    accumulate_vec<D>([&](int s) { return slot<D>(x, s) * slot<D>(xh2, s); }, vacc[G_LN1W], li);
    accumulate_vec<D>([&](int s) { return slot<D>(x, s); }, vacc[G_LN1B], li);
#pragma unroll
    for (int p = 0; p < T; ++p) x[p] *= vec4<D>(sV, V_LN1W, p, g);
    ln_backward<D>(x, xh2, rstd1);  // x = dpre1
    store_row_w<D, kAuxNT>(rows_window(dpre1_out, base, ne, D), eoff, x, g);

    // dw1d += dpre1 * dist ; d(dist) = w1d . dpre1
    float dd = 0.f;
#pragma unroll
    for (int p = 0; p < T; ++p) {
      const f32x4 w = vec4<D>(sV, V_W1D, p, g);
      dd += w[0] * x[p][0] + w[1] * x[p][1] + w[2] * x[p][2] + w[3] * x[p][3];
    }
    dd = sum_groups(dd);
    const float dist = c.dist;
    accumulate_vec<D>([&](int s) { return slot<D>(x, s) * dist; }, vacc[G_W1D], li);

    const float rinv = (c.dist > 0.f) ? dd / c.dist : 0.f;
    float gd[3] = {gpx * s_e + rinv * c.rx, gpy * s_e + rinv * c.ry, gpz * s_e + rinv * c.rz};
    store3_w<kAuxNT>(rows_window(gdiff_out, base, ne, 3), (c.valid && g == 0) ? li * 12u : kOob,
                     gd[0], gd[1], gd[2]);

    // ---------------- receiver-side segmented sums: dA (dpre1), dpos_recv (gdiff)
    const int head = c.valid ? (int)((c.seg0 > base) ? (c.seg0 - base) : 0) : li;
    const bool is_end = c.valid && (c.e == c.seg1 - 1);
    const bool take = (li == 0) && c.valid && (c.i == carry_node);
    carry_apply<D>(cbuf, x, gd, take);
    seg_scan<T>(x, li, head);
    {
      f32x4 pw[1] = {{gd[0], gd[1], gd[2], 0.f}};
      seg_scan<1>(pw, li, head);
      gd[0] = pw[0][0]; gd[1] = pw[0][1]; gd[2] = pw[0][2];
    }
    {
      const int nn = max(i1 - i0 + 1, 0);  // (receiver-sorted: i0 <= i <= i1)
      store_row_w<D, 0>(rows_window(dA, i0, nn, D), is_end ? (unsigned)((c.i - i0) * D * 4) : kOob,
                        x, g);
      store3_w<0>(rows_window(dpos_recv, i0, nn, 3),
                  (is_end && g == 0) ? (unsigned)((c.i - i0) * 12) : kOob, gd[0], gd[1], gd[2]);
    }
    if (li == 15) carry_store<D>(cbuf, x, gd);
    carry_node = __builtin_amdgcn_readlane(c.i, 15);
  }

  // ---------------- workgroup reduction of the vector grads -> partials[blockIdx]
  __syncthreads();  // every wave is done with W2/W3: reuse that LDS as scratch
  if (AMAX && threadIdx.x == 0) {  // (invalid lanes held zeros: gscale / rstd = 0)
    atomicMax(&amax[0], lmx[0]);
    atomicMax(&amax[1], lmx[1]);
  }
  __syncthreads();
  float* red = smem;  // [wave][NVG*D + 1]
  constexpr int RW = NVG * D + 1;
  for (int t = lane; t < RW; t += 64) red[wid * RW + t] = 0.f;
  __syncthreads();
  if (acc_owner<D>(li)) {
#pragma unroll
    for (int v = 0; v < NVG; ++v)
#pragma unroll
      for (int k = 0; k < K; ++k) red[wid * RW + v * D + featq(acc_slot<D>(li, k), g)] = vacc[v][k];
  }
  float t4 = db4;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) t4 += __shfl_xor(t4, off);
  if (lane == 0) red[wid * RW + NVG * D] = t4;
  __syncthreads();
  for (int t = threadIdx.x; t < RW; t += blockDim.x) {
    float sacc = 0.f;
    for (int w = 0; w < kBwdWaves; ++w) sacc += red[w * RW + t];
    partials[(int64_t)blockIdx.x * RW + t] = sacc;
  }
}

int64_t n_waves_for(int64_t n_edges, int nwb) {
  int64_t w = ceil_div(n_edges, 128);  // >= 8 chunks per wave when the chip is full
  const int64_t cap = (int64_t)device_cu_count() * nwb;
  if (w > cap) w = cap;
  if (w < 1) w = 1;
  return ceil_div(w, nwb) * nwb;
}

template <int D, int ACT, bool MEAN>
int launch_fwd(int64_t N, int64_t E, const float* AB, const float* pos, const int64_t* rowptr,
               const int64_t* recv, const int64_t* send, const gmp_egnn_params& P, float eps,
               float* m_aggr, float* pos_aggr, float* xsave, int save_planes, float* rsave,
               hipStream_t s) {
  const bool hf = !egnn_f32();
  const int nwb = hf ? fwd_waves<true>() : fwd_waves<false>();
  const int64_t W = n_waves_for(E, nwb);
  const size_t smem = hf ? smem_total<D, fwd_waves<true>(), true>()
                         : smem_total<D, fwd_waves<false>(), false>();
  auto k = rsave ? (hf ? egnn_fwd_kernel<D, ACT, MEAN, true, true>
                       : egnn_fwd_kernel<D, ACT, MEAN, true, false>)
                 : (hf ? egnn_fwd_kernel<D, ACT, MEAN, false, true>
                       : egnn_fwd_kernel<D, ACT, MEAN, false, false>);
  int rc = prep_kernel(k, smem);
  if (rc) return rc;
  k<<<(unsigned)(W / nwb), nwb * 64, smem, s>>>(N, E, AB, pos, rowptr, recv, send, P,
                                                           eps, W, m_aggr, pos_aggr, xsave, rsave,
                                                           save_planes);
  return launch_status();
}

template <int D, int ACT, bool MEAN>
int launch_bwd(int64_t N, int64_t E, const float* pos, const int64_t* rowptr,
               const int64_t* recv, const int64_t* send, const gmp_egnn_params& P,
               const float* xsave, int save_planes, const float* rsave, const float* gm,
               const float* gp, float* dA, float* dpos_recv, float* dpre1, float* gdiff,
               float* dpre2, float* dpre3, float* partials, unsigned* amax, hipStream_t s) {
  const int64_t W = n_waves_for(E, kBwdWaves);
  const bool hf = !egnn_f32();
  const size_t smem = hf ? smem_total<D, kBwdWaves, true>() : smem_total<D, kBwdWaves, false>();
#define LAUNCH_BWD_K(RC)                                                  \
  (hf ? (amax ? egnn_bwd_kernel<D, ACT, MEAN, true, true, RC>          \
              : egnn_bwd_kernel<D, ACT, MEAN, true, false, RC>)        \
      : (amax ? egnn_bwd_kernel<D, ACT, MEAN, false, true, RC>         \
              : egnn_bwd_kernel<D, ACT, MEAN, false, false, RC>))
  auto k = save_planes == 3 ? LAUNCH_BWD_K(0) : LAUNCH_BWD_K(1);
#undef LAUNCH_BWD_K
  int rc = prep_kernel(k, smem);
  if (rc) return rc;
  k<<<(unsigned)(W / kBwdWaves), kBwdWaves * 64, smem, s>>>(N, E, pos, rowptr, recv, send, P, W,
                                                           xsave, rsave, gm, gp, dA, dpos_recv,
                                                           dpre1, gdiff, dpre2, dpre3, partials,
                                                           amax);
  return launch_status();
}

bool params_ok(const gmp_egnn_params* P) {
  return P && P->w1d && P->b1 && P->ln1_w && P->ln1_b && P->W2 && P->b2 && P->ln2_w &&
         P->ln2_b && P->W3 && P->b3 && P->ln3_w && P->ln3_b && P->w4 && P->b4;
}

}  // namespace

int prep_kernel_once(const void* k, size_t smem) {
  static std::mutex mu;
  static std::set<std::tuple<int, const void*, size_t>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return GMP_ERR_HIP;
  std::lock_guard<std::mutex> lk(mu);
  if (done.count({dev, k, smem})) return GMP_OK;
  const int rc = hip_check(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)smem));
  if (!rc) done.insert({dev, k, smem});
  return rc;
}

// 1: the f32-MFMA (exact fmaf chain) products instead of the HF path (gmp_egnn_set_f32_mfma)
int g_egnn_f32 = 0;

bool egnn_f32() { return g_egnn_f32 == 1; }

}  // namespace gmp

using namespace gmp;

#define LAUNCH_EGNN_DISPATCH(CALL)                                                                \
  do {                                                                                         \
    if (d == 128) {                                                                            \
      if (act == 0) { if (msg_mean) CALL(128, 0, true); else CALL(128, 0, false); }            \
      else          { if (msg_mean) CALL(128, 1, true); else CALL(128, 1, false); }            \
    } else if (d == 64) {                                                                      \
      if (act == 0) { if (msg_mean) CALL(64, 0, true); else CALL(64, 0, false); }              \
      else          { if (msg_mean) CALL(64, 1, true); else CALL(64, 1, false); }              \
    } else {                                                                                   \
      if (act == 0) { if (msg_mean) CALL(32, 0, true); else CALL(32, 0, false); }              \
      else          { if (msg_mean) CALL(32, 1, true); else CALL(32, 1, false); }              \
    }                                                                                          \
  } while (0)

extern "C" {

int gmp_egnn_set_f32_mfma(int on) {
  const int prev = egnn_f32() ? 1 : 0;
  g_egnn_f32 = on ? 1 : 0;
  return prev;
}

int gmp_egnn_edge_fwd_f32(int64_t n_nodes, int64_t n_edges, int64_t d, const float* AB,
                          const float* pos, const int64_t* rowptr, const int64_t* recv,
                          const int64_t* send, const gmp_egnn_params* params, int act,
                          int msg_mean, float ln_eps, float* m_aggr, float* pos_aggr,
                          float* save_xhat, int save_planes, float* save_rstd, void* stream) {
  if (!(d == 32 || d == 64 || d == 128)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(n_nodes >= 0 && n_edges >= 0 && (act == 0 || act == 1));
  GMP_CHECK_ARG(n_nodes < INT32_MAX && n_edges < INT32_MAX);  // 32-bit edge / node ids
  GMP_CHECK_ARG(params_ok(params) && m_aggr && pos_aggr && rowptr);
  // training: save_rstd and save_xhat together, 2 (x_hat1, x_hat2) or 3 planes
  GMP_CHECK_ARG((save_rstd == nullptr) == (save_xhat == nullptr));
  GMP_CHECK_ARG(save_xhat == nullptr || save_planes == 2 || save_planes == 3);
  hipStream_t s = as_stream(stream);
  if (n_nodes == 0) return GMP_OK;
  int rc = GMP_OK;
  if (n_edges == 0) {  // (otherwise the kernel writes every row: zero_isolated)
    rc = hip_check(hipMemsetAsync(m_aggr, 0, n_nodes * d * sizeof(float), s));
    if (!rc) rc = hip_check(hipMemsetAsync(pos_aggr, 0, n_nodes * 3 * sizeof(float), s));
    return rc;
  }
  GMP_CHECK_ARG(AB && pos && recv && send && aligned16(AB) && aligned16(m_aggr));
  GMP_CHECK_ARG(aligned16(params->W2) && aligned16(params->W3));
  GMP_CHECK_ARG(save_xhat == nullptr || aligned16(save_xhat));
#define LAUNCH_CALL_FWD(DD, AA, MM)                                                              \
  rc = launch_fwd<DD, AA, MM>(n_nodes, n_edges, AB, pos, rowptr, recv, send, *params, ln_eps, \
                              m_aggr, pos_aggr, save_xhat, save_planes, save_rstd, s)
  LAUNCH_EGNN_DISPATCH(LAUNCH_CALL_FWD);
#undef LAUNCH_CALL_FWD
  return rc;
}

int64_t gmp_egnn_edge_bwd_partials_rows(int64_t n_edges, int64_t d) {
  (void)d;
  return n_waves_for(n_edges, kBwdWaves) / kBwdWaves;
}

int gmp_egnn_edge_bwd_amax_f32(int64_t n_nodes, int64_t n_edges, int64_t d, const float* pos,
                               const int64_t* rowptr, const int64_t* recv, const int64_t* send,
                               const gmp_egnn_params* params, int act, int msg_mean,
                               const float* save_xhat, int save_planes, const float* save_rstd,
                               const float* g_m_aggr, const float* g_pos_aggr, float* dA,
                               float* dpos_recv, float* dpre1, float* gdiff, float* dpre2,
                               float* dpre3, float* vec_partials, uint32_t* amax, void* stream) {
  if (!(d == 32 || d == 64 || d == 128)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(n_nodes >= 0 && n_edges >= 0 && (act == 0 || act == 1));
  GMP_CHECK_ARG(n_nodes < INT32_MAX && n_edges < INT32_MAX);  // 32-bit edge / node ids
  GMP_CHECK_ARG(params_ok(params) && dA && dpos_recv && rowptr && vec_partials);
  GMP_CHECK_ARG(save_planes == 2 || save_planes == 3);
  hipStream_t s = as_stream(stream);
  int rc = GMP_OK;
  if (n_nodes > 0 && n_edges == 0) {  // (otherwise the kernel writes every row: zero_isolated)
    rc = hip_check(hipMemsetAsync(dA, 0, n_nodes * d * sizeof(float), s));
    if (!rc) rc = hip_check(hipMemsetAsync(dpos_recv, 0, n_nodes * 3 * sizeof(float), s));
  }
  if (rc) return rc;
  if (n_edges == 0 || n_nodes == 0) {
    return hip_check(hipMemsetAsync(
        vec_partials, 0,
        gmp_egnn_edge_bwd_partials_rows(n_edges, d) * (8 * d + 1) * sizeof(float), s));
  }
  GMP_CHECK_ARG(pos && recv && send && save_xhat && save_rstd && g_m_aggr && g_pos_aggr &&
                dpre1 && gdiff && dpre2 && dpre3);
  GMP_CHECK_ARG(aligned16(save_xhat) && aligned16(dA) && aligned16(g_m_aggr) &&
                aligned16(dpre1) && aligned16(dpre2) && aligned16(dpre3));
  GMP_CHECK_ARG(aligned16(params->W2) && aligned16(params->W3));
#define LAUNCH_CALL_BWD(DD, AA, MM)                                                              \
  rc = launch_bwd<DD, AA, MM>(n_nodes, n_edges, pos, rowptr, recv, send, *params, save_xhat,  \
                              save_planes, save_rstd, g_m_aggr, g_pos_aggr, dA, dpos_recv,    \
                              dpre1, gdiff, dpre2, dpre3, vec_partials, amax, s)
  LAUNCH_EGNN_DISPATCH(LAUNCH_CALL_BWD);
#undef LAUNCH_CALL_BWD
  return rc;
}

int gmp_egnn_edge_bwd_f32(int64_t n_nodes, int64_t n_edges, int64_t d, const float* pos,
                          const int64_t* rowptr, const int64_t* recv, const int64_t* send,
                          const gmp_egnn_params* params, int act, int msg_mean,
                          const float* save_xhat, int save_planes, const float* save_rstd,
                          const float* g_m_aggr, const float* g_pos_aggr, float* dA,
                          float* dpos_recv, float* dpre1, float* gdiff, float* dpre2, float* dpre3,
                          float* vec_partials, void* stream) {
  return gmp_egnn_edge_bwd_amax_f32(n_nodes, n_edges, d, pos, rowptr, recv, send, params, act,
                                    msg_mean, save_xhat, save_planes, save_rstd, g_m_aggr,
                                    g_pos_aggr, dA, dpos_recv, dpre1, gdiff, dpre2, dpre3,
                                    vec_partials, nullptr, stream);
}

}  // extern "C"
