// K1e: the GVP-GNN edge embedding W_e (models/gvpgnn.py:73-77, applied at :116) -- LayerNorm
// ((R, 1)) (gvp_layer.py:221-243) followed by GVP((R, 1), (SO, 1), activations (None, None),
// vector_gate) (gvp_layer.py:101-170, h_dim = 1) -- on the E edge rows (radial (E, R), unit
// (E, 3)), forward and the parameters' gradients in one pass each.  The module chain launches
// ~12 kernels per direction over 1M-row tensors, four of them library GEMMs with K or N = 1 that
// run at < 1 TB/s (r05 trace: ~0.6 ms forward, ~1.5 ms at the end of the backward); these
// kernels read R + 3 floats per edge and write SO + 3 (forward) or read SO + 3 more (backward).
//
// Lane mapping: half a wave per edge, lane o = lane & 31 owning output channel o (o >= SO idle);
// the LayerNorm, the vector norms and the vector gate are recomputed by every lane of the half
// (R + 3 inputs); the gate's dot product over the SO channels is a butterfly over the half.
//
// Backward: the edge rows only reach parameters (radial / unit carry no gradient on this path:
// positions without requires_grad).  Per channel o the lane accumulates over its edges
//   A[c] = sum ds2[o] xhat[c] (c < R), dbs = sum ds2[o], Bn = sum ds2[o] vn, Dg = sum dgate s2[o],
//   Cq = sum ds2[o] r    (r = (vh . v1) / vn where |vh|^2 >= 1e-8, else 0: the clamp's mask)
// and per edge the scalars dbsv = sum dgate, dwv = sum dv2 . vh, T1 = sum dv2 . v1; the
// parameter gradients are bilinear in these:
//   dWs[o][c] = gamma[c] A[o][c] + beta[c] dbs[o]   (s1 = xhat gamma + beta)
//   dWs[o][R] = Bn[o], dbs, dwsv[o] = Dg[o], dbsv, dwv,
//   dwh = wv T1 + sum_o Ws[o][R] Cq[o]               (dvh = wv dv2 + dvn vh / vn, dvn = Ws[:, R] . ds2)
//   dgamma[c] = sum_o Ws[o][c] A[o][c], dbeta[c] = sum_o Ws[o][c] dbs[o]   (ds1 = Ws[:, :R]^T ds2)
// Each workgroup writes one row of partial sums (lanes in edge order, the two halves and the
// four waves added in a fixed order); the finishing kernel adds the rows in row order and
// applies the bilinear forms: deterministic.
#include "gmp_common.h"

namespace gmp {
namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kEmbT = 256;                 // threads per workgroup (4 waves, 8 edges per step)
constexpr int kEmbR = 8;                   // radial features (num_bessel, gvpgnn.py:29)
constexpr int kEmbSO = 32;                 // lanes per edge: output scalar channels <= 32
constexpr int kEmbAcc = kEmbR + 4;         // per-channel accumulators A[R], dbs, Bn, Dg, Cq
constexpr int kEmbPart = kEmbSO * kEmbAcc + 3;  // + dbsv, dwv, T1
constexpr int kEmbStepsPerBlock = 16;      // forward: edge steps (8 edges each) per workgroup
constexpr int kEmbFinT = 1024;             // finishing kernel threads

struct EmbedW {
  const float *ln_w, *ln_b, *wh, *Ws, *bs, *wv, *wsv, *bsv;
  float eps;
};

__device__ __forceinline__ float half_sum(float x) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
  return x;
}

// forward state of one edge on one lane (channel o)
struct EmbedFwd {
  float xh[kEmbR], v1[3], vh[3], q, vn, s2, sg;
};

__device__ __forceinline__ EmbedFwd embed_fwd(const EmbedW& W, const float* __restrict__ radial,
                                              const float* __restrict__ unit, int64_t e, int o,
                                              bool on, const float (&wrow)[kEmbR + 1], float bo,
                                              float wso) {
  EmbedFwd F;
  const f32x4_t r0 = *reinterpret_cast<const f32x4_t*>(radial + e * kEmbR);
  const f32x4_t r1 = *reinterpret_cast<const f32x4_t*>(radial + e * kEmbR + 4);
  const float x[kEmbR] = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
  // LayerNorm (biased variance, two passes)
  float mean = 0.f;
#pragma unroll
  for (int c = 0; c < kEmbR; ++c) mean += x[c];
  mean *= 1.f / kEmbR;
  float var = 0.f;
#pragma unroll
  for (int c = 0; c < kEmbR; ++c) var += (x[c] - mean) * (x[c] - mean);
  var *= 1.f / kEmbR;
  const float rstd = 1.f / sqrtf(var + W.eps);
  float s1[kEmbR];
#pragma unroll
  for (int c = 0; c < kEmbR; ++c) {
    F.xh[c] = (x[c] - mean) * rstd;
    s1[c] = F.xh[c] * W.ln_w[c] + W.ln_b[c];
  }
  // vector LayerNorm of the single channel: v / sqrt(max(|v|^2, 1e-8))
  const float u0 = unit[3 * e], u1 = unit[3 * e + 1], u2 = unit[3 * e + 2];
  const float nv = sqrtf(fmaxf(u0 * u0 + u1 * u1 + u2 * u2, 1e-8f));
  F.v1[0] = u0 / nv;
  F.v1[1] = u1 / nv;
  F.v1[2] = u2 / nv;
  const float wh = W.wh[0];
#pragma unroll
  for (int k = 0; k < 3; ++k) F.vh[k] = F.v1[k] * wh;
  F.q = F.vh[0] * F.vh[0] + F.vh[1] * F.vh[1] + F.vh[2] * F.vh[2];
  F.vn = sqrtf(fmaxf(F.q, 1e-8f));
  // s2[o] = Ws[o] . [s1 | vn] + bs[o]
  float s2 = bo;
#pragma unroll
  for (int c = 0; c < kEmbR; ++c) s2 += wrow[c] * s1[c];
  s2 += wrow[kEmbR] * F.vn;
  F.s2 = on ? s2 : 0.f;
  const float gate = half_sum(wso * F.s2) + W.bsv[0];
  F.sg = 1.f / (1.f + expf(-gate));
  return F;
}

struct EmbedLane {
  float wrow[kEmbR + 1], bo, wso;
  bool on;
};
__device__ __forceinline__ EmbedLane embed_lane(const EmbedW& W, int o, int so) {
  EmbedLane L;
  L.on = o < so;
  const int oc = L.on ? o : 0;
#pragma unroll
  for (int c = 0; c <= kEmbR; ++c) L.wrow[c] = L.on ? W.Ws[oc * (kEmbR + 1) + c] : 0.f;
  L.bo = L.on ? W.bs[oc] : 0.f;
  L.wso = L.on ? W.wsv[oc] : 0.f;
  return L;
}

__global__ __launch_bounds__(kEmbT) void gvp_embed_fwd_kernel(int64_t E, int so, EmbedW W,
                                                              const float* __restrict__ radial,
                                                              const float* __restrict__ unit,
                                                              float* __restrict__ es,
                                                              float* __restrict__ ev) {
  const int lane = threadIdx.x & 63, o = lane & 31;
  const int slot = (threadIdx.x >> 6) * 2 + (lane >> 5);  // edge slot 0..7 of a step
  const EmbedLane L = embed_lane(W, o, so);
  const float wv = W.wv[0];
  const int64_t e0 = (int64_t)blockIdx.x * kEmbStepsPerBlock * 8;
  for (int st = 0; st < kEmbStepsPerBlock; ++st) {
    const int64_t e = e0 + 8 * st + slot;
    if (e0 + 8 * st >= E) break;  // workgroup-uniform
    const bool ok = e < E;
    const int64_t ec = ok ? e : E - 1;  // clamped (the half's shuffles stay converged)
    const EmbedFwd F = embed_fwd(W, radial, unit, ec, o, L.on, L.wrow, L.bo, L.wso);
    if (ok && L.on) es[e * so + o] = F.s2;
    const float vo = o == 0 ? F.vh[0] : (o == 1 ? F.vh[1] : F.vh[2]);
    if (ok && o < 3) ev[3 * e + o] = (wv * vo) * F.sg;
  }
}

// backward: one row of kEmbPart partial sums per workgroup over its contiguous edge range
__global__ __launch_bounds__(kEmbT) void gvp_embed_bwd_kernel(int64_t E, int so, int64_t per,
                                                              EmbedW W,
                                                              const float* __restrict__ radial,
                                                              const float* __restrict__ unit,
                                                              const float* __restrict__ des,
                                                              const float* __restrict__ dev,
                                                              float* __restrict__ part) {
  __shared__ float red[kEmbT / 64][kEmbPart];
  const int lane = threadIdx.x & 63, o = lane & 31, w = threadIdx.x >> 6;
  const int slot = w * 2 + (lane >> 5);
  const EmbedLane L = embed_lane(W, o, so);
  const float wv = W.wv[0];
  float acc[kEmbAcc];
#pragma unroll
  for (int k = 0; k < kEmbAcc; ++k) acc[k] = 0.f;
  float u_dbsv = 0.f, u_dwv = 0.f, u_t1 = 0.f;
  const int64_t k0 = (int64_t)blockIdx.x * per;
  const int64_t k1 = (k0 + per < E) ? k0 + per : E;
  for (int64_t b = k0; b < k1; b += 8) {
    const int64_t e = b + slot;
    const bool ok = e < k1;
    const int64_t ec = ok ? e : k1 - 1;
    const EmbedFwd F = embed_fwd(W, radial, unit, ec, o, L.on, L.wrow, L.bo, L.wso);
    const float d0 = dev[3 * ec], d1 = dev[3 * ec + 1], d2 = dev[3 * ec + 2];
    const float v20 = wv * F.vh[0], v21 = wv * F.vh[1], v22 = wv * F.vh[2];
    const float dsg = d0 * v20 + d1 * v21 + d2 * v22;
    const float dgate = ok ? dsg * F.sg * (1.f - F.sg) : 0.f;
    const float sgk = ok ? F.sg : 0.f;
    const float dv0 = d0 * sgk, dv1 = d1 * sgk, dv2 = d2 * sgk;
    const float ds2 = (ok && L.on) ? des[ec * so + o] + L.wso * dgate : 0.f;
    const float r = F.q >= 1e-8f
                        ? (F.vh[0] * F.v1[0] + F.vh[1] * F.v1[1] + F.vh[2] * F.v1[2]) / F.vn
                        : 0.f;
#pragma unroll
    for (int c = 0; c < kEmbR; ++c) acc[c] += ds2 * F.xh[c];
    acc[kEmbR] += ds2;
    acc[kEmbR + 1] += ds2 * F.vn;
    acc[kEmbR + 2] += dgate * F.s2;
    acc[kEmbR + 3] += ds2 * r;
    u_dbsv += dgate;
    u_dwv += dv0 * F.vh[0] + dv1 * F.vh[1] + dv2 * F.vh[2];
    u_t1 += dv0 * F.v1[0] + dv1 * F.v1[1] + dv2 * F.v1[2];
  }
  // the two halves of the wave (lanes o, o + 32), then the waves in order
#pragma unroll
  for (int k = 0; k < kEmbAcc; ++k) acc[k] += __shfl_xor(acc[k], 32, 64);
  u_dbsv += __shfl_xor(u_dbsv, 32, 64);
  u_dwv += __shfl_xor(u_dwv, 32, 64);
  u_t1 += __shfl_xor(u_t1, 32, 64);
  if (lane < 32) {
#pragma unroll
    for (int k = 0; k < kEmbAcc; ++k) red[w][o * kEmbAcc + k] = acc[k];
    if (lane == 0) {
      red[w][kEmbSO * kEmbAcc] = u_dbsv;
      red[w][kEmbSO * kEmbAcc + 1] = u_dwv;
      red[w][kEmbSO * kEmbAcc + 2] = u_t1;
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < kEmbPart; t += kEmbT) {
    float s = red[0][t];
#pragma unroll
    for (int q = 1; q < kEmbT / 64; ++q) s += red[q][t];
    part[(int64_t)blockIdx.x * kEmbPart + t] = s;
  }
}

// packed gradient layout (gmp.h): [ln_w R | ln_b R | wh 1 | Ws SO x (R+1) | bs SO | wv 1 |
// wsv SO | bsv 1].  16 waves, wave w adding rows w, w + 16, .. (4 rows of loads in flight per
// lane, lane owning columns lane + 64 k), the waves' sums added in wave order: deterministic.
constexpr int kEmbFinW = kEmbFinT / 64;
constexpr int kEmbFinC = (kEmbPart + 63) / 64;  // columns per lane
__global__ __launch_bounds__(kEmbFinT) void gvp_embed_finish_kernel(int64_t G, int so, EmbedW W,
                                                                    const float* __restrict__ part,
                                                                    float* __restrict__ grad) {
  __shared__ float sl[kEmbFinW][kEmbFinC * 64];
  __shared__ float tot[kEmbFinC * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc[kEmbFinC];
#pragma unroll
  for (int k = 0; k < kEmbFinC; ++k) acc[k] = 0.f;
  for (int64_t g0 = w; g0 < G; g0 += 4 * kEmbFinW) {
    float v[4][kEmbFinC];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t g = g0 + (int64_t)u * kEmbFinW;
#pragma unroll
      for (int k = 0; k < kEmbFinC; ++k) {
        const int col = lane + 64 * k;
        v[u][k] = (g < G && col < kEmbPart) ? part[g * kEmbPart + col] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < kEmbFinC; ++k) acc[k] += v[u][k];
  }
#pragma unroll
  for (int k = 0; k < kEmbFinC; ++k) sl[w][lane + 64 * k] = acc[k];
  __syncthreads();
  for (int t = threadIdx.x; t < kEmbPart; t += kEmbFinT) {
    float s = sl[0][t];
#pragma unroll
    for (int k = 1; k < kEmbFinW; ++k) s += sl[k][t];
    tot[t] = s;
  }
  __syncthreads();
  constexpr int R = kEmbR;
  float* g_lnw = grad;
  float* g_lnb = grad + R;
  float* g_wh = grad + 2 * R;
  float* g_Ws = grad + 2 * R + 1;
  float* g_bs = g_Ws + so * (R + 1);
  float* g_wv = g_bs + so;
  float* g_wsv = g_wv + 1;
  float* g_bsv = g_wsv + so;
  const float* U = tot + kEmbSO * kEmbAcc;
  for (int t = threadIdx.x; t < so * (R + 1); t += kEmbFinT) {
    const int o = t / (R + 1), c = t - o * (R + 1);
    const float* a = tot + o * kEmbAcc;
    g_Ws[t] = c < R ? W.ln_w[c] * a[c] + W.ln_b[c] * a[R] : a[R + 1];
  }
  for (int o = threadIdx.x; o < so; o += kEmbFinT) {
    g_bs[o] = tot[o * kEmbAcc + R];
    g_wsv[o] = tot[o * kEmbAcc + R + 2];
  }
  if (threadIdx.x < R) {
    const int c = threadIdx.x;
    float gg = 0.f, gb = 0.f;
    for (int o = 0; o < so; ++o) {
      const float wc = W.Ws[o * (R + 1) + c];
      gg += wc * tot[o * kEmbAcc + c];
      gb += wc * tot[o * kEmbAcc + R];
    }
    g_lnw[c] = gg;
    g_lnb[c] = gb;
  }
  if (threadIdx.x == 0) {
    float cq = 0.f;
    for (int o = 0; o < so; ++o) cq += W.Ws[o * (R + 1) + R] * tot[o * kEmbAcc + R + 3];
    g_wh[0] = W.wv[0] * U[2] + cq;
    g_wv[0] = U[1];
    g_bsv[0] = U[0];
  }
}

int64_t embed_bwd_blocks(int64_t E) {
  // two 4-wave workgroups per CU (fewer partial rows for the finishing kernel); >= 64 edges each
  int64_t g = 2 * (int64_t)device_cu_count();
  if (g * 64 > E) g = ceil_div(E, 64);
  return g < 1 ? 1 : g;
}

bool embed_shape_ok(int64_t R, int64_t so) { return R == kEmbR && so >= 1 && so <= kEmbSO; }

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_gvp_edge_embed_fwd_f32(int64_t n_edges, int64_t radial_dim, int64_t so,
                               const float* radial, const float* unit, const float* ln_w,
                               const float* ln_b, const float* wh, const float* Ws,
                               const float* bs, const float* wv, const float* wsv,
                               const float* bsv, float eps, float* es, float* ev, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && radial_dim >= 1 && so >= 1);
  if (!embed_shape_ok(radial_dim, so)) return GMP_ERR_UNSUPPORTED;
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(radial && unit && ln_w && ln_b && wh && Ws && bs && wv && wsv && bsv && es && ev);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(radial) % 16 == 0);
  const EmbedW W{ln_w, ln_b, wh, Ws, bs, wv, wsv, bsv, eps};
  const int64_t blocks = ceil_div(n_edges, (int64_t)kEmbStepsPerBlock * 8);
  gvp_embed_fwd_kernel<<<(unsigned)blocks, kEmbT, 0, as_stream(stream)>>>(n_edges, (int)so, W,
                                                                           radial, unit, es, ev);
  return launch_status();
}

size_t gmp_gvp_edge_embed_bwd_workspace_size(int64_t n_edges) {
  return (size_t)embed_bwd_blocks(n_edges) * kEmbPart * sizeof(float);
}

int gmp_gvp_edge_embed_bwd_f32(int64_t n_edges, int64_t radial_dim, int64_t so,
                               const float* radial, const float* unit, const float* ln_w,
                               const float* ln_b, const float* wh, const float* Ws,
                               const float* bs, const float* wv, const float* wsv,
                               const float* bsv, float eps, const float* grad_es,
                               const float* grad_ev, float* grad_params, void* workspace,
                               size_t workspace_bytes, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && radial_dim >= 1 && so >= 1);
  if (!embed_shape_ok(radial_dim, so)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(ln_w && ln_b && wh && Ws && bs && wv && wsv && bsv && grad_params);
  hipStream_t s = as_stream(stream);
  const int64_t n_params = 2 * radial_dim + 1 + so * (radial_dim + 1) + so + 1 + so + 1;
  if (n_edges == 0)
    return hip_check(hipMemsetAsync(grad_params, 0, n_params * sizeof(float), s));
  GMP_CHECK_ARG(radial && unit && grad_es && grad_ev && workspace);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(radial) % 16 == 0);
  if (workspace_bytes < gmp_gvp_edge_embed_bwd_workspace_size(n_edges)) return GMP_ERR_WORKSPACE;
  const EmbedW W{ln_w, ln_b, wh, Ws, bs, wv, wsv, bsv, eps};
  const int64_t G = embed_bwd_blocks(n_edges);
  const int64_t per = ceil_div(ceil_div(n_edges, G), 8) * 8;
  const int64_t Gr = ceil_div(n_edges, per);
  float* part = reinterpret_cast<float*>(workspace);
  gvp_embed_bwd_kernel<<<(unsigned)Gr, kEmbT, 0, s>>>(n_edges, (int)so, per, W, radial, unit,
                                                      grad_es, grad_ev, part);
  int rc = launch_status();
  if (rc) return rc;
  gvp_embed_finish_kernel<<<1, kEmbFinT, 0, s>>>(Gr, (int)so, W, part, grad_params);
  return launch_status();
}

}  // extern "C"
