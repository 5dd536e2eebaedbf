// K1e: the GVP-GNN edge embedding W_e (models/gvpgnn.py:73-77, applied at :116) -- LayerNorm
// ((R, 1)) (gvp_layer.py:221-243) followed by GVP((R, 1), (SO, 1), activations (None, None),
// vector_gate) (gvp_layer.py:101-170, h_dim = 1) -- on the E edge rows (radial (E, R), unit
// (E, 3)), forward and the parameters' gradients in one pass each.  The module chain launches
// ~12 kernels per direction over 1M-row tensors, four of them library GEMMs with K or N = 1 that
// run at < 1 TB/s (r05 trace: ~0.6 ms forward, ~1.5 ms at the end of the backward); these
// kernels read R + 3 floats per edge and write SO + 3 (forward) or read SO + 3 more (backward).
//
// One lane per edge: the LayerNorm, the vector norms, s2 = Ws [s1 | vn] + bs (SO x (R + 1)
// FMAs against LDS-broadcast weights) and the vector gate in registers; the forward stores the
// edge's SO-float es row as float4s.
//
// Backward: the edge rows only reach parameters (radial / unit carry no gradient on this path:
// positions without requires_grad).  With ds2 = des + wsv dgate the gradients need, per edge,
// the features F = [xhat (R) | 1 | vn | r] (r = (vh . v1) / vn where |vh|^2 >= 1e-8, else 0:
// the clamp's mask) and the scalars dgate, dv2 . vh, dv2 . v1:
//   P[o][k] = sum_e des[e][o] F[e][k]                     (the only per-(edge, channel) sums)
//   DX[c] = sum dgate xhat[c], U0 = sum dgate, Dvn = sum dgate vn, Dr = sum dgate r,
//   U1 = sum dv2 . vh, T1 = sum dv2 . v1                   (per-edge scalars)
// and every parameter gradient is bilinear in these (the finishing kernel):
//   A[o][c] = P[o][c] + wsv[o] DX[c], dbs[o] = P[o][R] + wsv[o] U0,
//   dWs[o][c] = gamma[c] A[o][c] + beta[c] dbs[o], dWs[o][R] = P[o][R+1] + wsv[o] Dvn,
//   dwsv[o] = sum_c Ws[o][c] (gamma[c] DX[c] + beta[c] U0) + Ws[o][R] Dvn + bs[o] U0,
//   dbsv = U0, dwv = U1, dwh = wv T1 + sum_o Ws[o][R] (P[o][R+2] + wsv[o] Dr),
//   dgamma[c] = sum_o Ws[o][c] A[o][c], dbeta[c] = sum_o Ws[o][c] dbs[o].
// A wave computes F for 64 edges (lane = edge) into LDS, then P over them with lane = channel o
// (two edges per step, des rows read coalesced); per-workgroup partial rows (lanes in edge
// order, the wave halves and the waves in a fixed order), added in row order by the finishing
// kernel: deterministic.
#include "gmp_common.h"

namespace gmp {
namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kEmbT = 256;                 // threads per workgroup (4 waves)
constexpr int kEmbR = 8;                   // radial features (num_bessel, gvpgnn.py:29)
constexpr int kEmbSO = 32;                 // output scalar channels <= 32
constexpr int kEmbF = kEmbR + 3;           // per-edge features [xhat | 1 | vn | r]
constexpr int kEmbFLd = 12;                // LDS row of F (three float4)
constexpr int kEmbU = kEmbR + 5;           // per-edge scalar sums DX[R], U0, Dvn, Dr, U1, T1
constexpr int kEmbPart = kEmbSO * kEmbF + kEmbU;
constexpr int kEmbFinT = 1024;             // finishing kernel threads
// LDS parameter image: Ws rows padded to 12 floats (o >= so zero), bs, wsv, gamma, beta, wh,
// wv, bsv
constexpr int kPWs = 0, kPbs = kEmbSO * 12, kPwsv = kPbs + kEmbSO, kPg = kPwsv + kEmbSO;
constexpr int kPb = kPg + kEmbR, kPwh = kPb + kEmbR, kPwv = kPwh + 1, kPbsv = kPwv + 1;
constexpr int kPN = kPbsv + 4;

struct EmbedW {
  const float *ln_w, *ln_b, *wh, *Ws, *bs, *wv, *wsv, *bsv;
  float eps;
};

__device__ __forceinline__ void load_params(float* sp, const EmbedW& W, int so) {
  for (int t = threadIdx.x; t < kPN; t += blockDim.x) {
    float v = 0.f;
    if (t < kPbs) {
      const int o = t / 12, c = t - 12 * o;
      v = (o < so && c <= kEmbR) ? W.Ws[o * (kEmbR + 1) + c] : 0.f;
    } else if (t < kPwsv) {
      v = t - kPbs < so ? W.bs[t - kPbs] : 0.f;
    } else if (t < kPg) {
      v = t - kPwsv < so ? W.wsv[t - kPwsv] : 0.f;
    } else if (t < kPb) {
      v = W.ln_w[t - kPg];
    } else if (t < kPwh) {
      v = W.ln_b[t - kPb];
    } else if (t == kPwh) {
      v = W.wh[0];
    } else if (t == kPwv) {
      v = W.wv[0];
    } else if (t == kPbsv) {
      v = W.bsv[0];
    }
    sp[t] = v;
  }
}

// forward state of one edge (one lane)
struct EmbedFwd {
  float xh[kEmbR], v1[3], vh[3], q, vn, sg, s2[kEmbSO];
};

__device__ __forceinline__ EmbedFwd embed_fwd(const float* sp, float eps,
                                              const float* __restrict__ radial,
                                              const float* __restrict__ unit, int64_t e) {
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
  const float rstd = 1.f / sqrtf(var + eps);
  float u9[kEmbR + 1];
#pragma unroll
  for (int c = 0; c < kEmbR; ++c) {
    F.xh[c] = (x[c] - mean) * rstd;
    u9[c] = F.xh[c] * sp[kPg + c] + sp[kPb + c];
  }
  // vector LayerNorm of the single channel: v / sqrt(max(|v|^2, 1e-8))
  const float u0 = unit[3 * e], u1 = unit[3 * e + 1], u2 = unit[3 * e + 2];
  const float nv = sqrtf(fmaxf(u0 * u0 + u1 * u1 + u2 * u2, 1e-8f));
  F.v1[0] = u0 / nv;
  F.v1[1] = u1 / nv;
  F.v1[2] = u2 / nv;
  const float wh = sp[kPwh];
#pragma unroll
  for (int k = 0; k < 3; ++k) F.vh[k] = F.v1[k] * wh;
  F.q = F.vh[0] * F.vh[0] + F.vh[1] * F.vh[1] + F.vh[2] * F.vh[2];
  F.vn = sqrtf(fmaxf(F.q, 1e-8f));
  u9[kEmbR] = F.vn;
  // s2 = Ws [s1 | vn] + bs ; gate = wsv . s2 + bsv
  float gate = sp[kPbsv];
#pragma unroll
  for (int o = 0; o < kEmbSO; ++o) {
    const f32x4_t w0 = *reinterpret_cast<const f32x4_t*>(sp + kPWs + 12 * o);
    const f32x4_t w1 = *reinterpret_cast<const f32x4_t*>(sp + kPWs + 12 * o + 4);
    const float w8 = sp[kPWs + 12 * o + 8];
    float a = sp[kPbs + o];
    a += w0[0] * u9[0] + w0[1] * u9[1] + w0[2] * u9[2] + w0[3] * u9[3];
    a += w1[0] * u9[4] + w1[1] * u9[5] + w1[2] * u9[6] + w1[3] * u9[7];
    a += w8 * u9[8];
    F.s2[o] = a;
    gate += sp[kPwsv + o] * a;
  }
  F.sg = 1.f / (1.f + expf(-gate));
  return F;
}

__global__ __launch_bounds__(kEmbT) void gvp_embed_fwd_kernel(int64_t E, int so, EmbedW W,
                                                              const float* __restrict__ radial,
                                                              const float* __restrict__ unit,
                                                              float* __restrict__ es,
                                                              float* __restrict__ ev) {
  __shared__ __attribute__((aligned(16))) float sp[kPN];
  load_params(sp, W, so);
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * kEmbT + threadIdx.x;
  if (e >= E) return;
  const EmbedFwd F = embed_fwd(sp, W.eps, radial, unit, e);
  float* row = es + e * so;
  if (so == kEmbSO) {
#pragma unroll
    for (int k = 0; k < kEmbSO / 4; ++k)
      *reinterpret_cast<f32x4_t*>(row + 4 * k) =
          f32x4_t{F.s2[4 * k], F.s2[4 * k + 1], F.s2[4 * k + 2], F.s2[4 * k + 3]};
  } else {
#pragma unroll
    for (int o = 0; o < kEmbSO; ++o)
      if (o < so) row[o] = F.s2[o];
  }
  const float wv = sp[kPwv];
#pragma unroll
  for (int k = 0; k < 3; ++k) ev[3 * e + k] = (wv * F.vh[k]) * F.sg;
}

// backward: one row of kEmbPart partial sums per workgroup over its contiguous edge range
// (a multiple of 256 edges: 64 per wave per chunk)
__global__ __launch_bounds__(kEmbT) void gvp_embed_bwd_kernel(int64_t E, int so, int64_t per,
                                                              EmbedW W,
                                                              const float* __restrict__ radial,
                                                              const float* __restrict__ unit,
                                                              const float* __restrict__ des,
                                                              const float* __restrict__ dev,
                                                              float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float sp[kPN];
  __shared__ __attribute__((aligned(16))) float sF[kEmbT / 64][64 * kEmbFLd];
  __shared__ float red[kEmbT / 64][kEmbPart];
  load_params(sp, W, so);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int o = lane & 31, h = lane >> 5;
  float P[kEmbF];
#pragma unroll
  for (int k = 0; k < kEmbF; ++k) P[k] = 0.f;
  float U[kEmbU];
#pragma unroll
  for (int k = 0; k < kEmbU; ++k) U[k] = 0.f;
  const float wv = sp[kPwv];
  const int64_t k0 = (int64_t)blockIdx.x * per;
  const int64_t k1 = (k0 + per < E) ? k0 + per : E;
  float* fw = sF[w];
  for (int64_t bb = k0; bb < k1; bb += kEmbT) {  // block-uniform: barriers below
    const int64_t b = bb + 64 * w, e = b + lane;
    const bool ok = b < k1 && e < k1;
    const int64_t ec = ok ? e : k0;
    const EmbedFwd F = embed_fwd(sp, W.eps, radial, unit, ec);
    float dgate = 0.f, r = 0.f;
    if (ok) {
      const float d0 = dev[3 * e], d1 = dev[3 * e + 1], d2 = dev[3 * e + 2];
      const float dsg = wv * (d0 * F.vh[0] + d1 * F.vh[1] + d2 * F.vh[2]);
      dgate = dsg * F.sg * (1.f - F.sg);
      const float t0 = d0 * F.sg, t1 = d1 * F.sg, t2 = d2 * F.sg;
      U[kEmbR + 3] += t0 * F.vh[0] + t1 * F.vh[1] + t2 * F.vh[2];
      U[kEmbR + 4] += t0 * F.v1[0] + t1 * F.v1[1] + t2 * F.v1[2];
      r = F.q >= 1e-8f ? (F.vh[0] * F.v1[0] + F.vh[1] * F.v1[1] + F.vh[2] * F.v1[2]) / F.vn
                       : 0.f;
#pragma unroll
      for (int c = 0; c < kEmbR; ++c) U[c] += dgate * F.xh[c];
      U[kEmbR] += dgate;
      U[kEmbR + 1] += dgate * F.vn;
      U[kEmbR + 2] += dgate * r;
    }
    // F rows of the wave's 64 edges (invalid edges: zeros, so they add nothing below)
    float* fr = fw + lane * kEmbFLd;
    *reinterpret_cast<f32x4_t*>(fr) =
        ok ? f32x4_t{F.xh[0], F.xh[1], F.xh[2], F.xh[3]} : f32x4_t{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4_t*>(fr + 4) =
        ok ? f32x4_t{F.xh[4], F.xh[5], F.xh[6], F.xh[7]} : f32x4_t{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4_t*>(fr + 8) =
        ok ? f32x4_t{1.f, F.vn, r, 0.f} : f32x4_t{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    // P[o][k] += des[e][o] F[e][k]: lanes o of half h take edges 2 j + h
    const bool on = o < so;
#pragma unroll 4
    for (int j = 0; j < 32; ++j) {
      const int el = 2 * j + h;
      const int64_t e2 = b + el;
      const float d = (on && b < k1 && e2 < k1) ? des[e2 * so + o] : 0.f;
      const float* f = fw + el * kEmbFLd;
      const f32x4_t fa = *reinterpret_cast<const f32x4_t*>(f);
      const f32x4_t fb = *reinterpret_cast<const f32x4_t*>(f + 4);
      const f32x4_t fc = *reinterpret_cast<const f32x4_t*>(f + 8);
      P[0] += d * fa[0];
      P[1] += d * fa[1];
      P[2] += d * fa[2];
      P[3] += d * fa[3];
      P[4] += d * fb[0];
      P[5] += d * fb[1];
      P[6] += d * fb[2];
      P[7] += d * fb[3];
      P[8] += d * fc[0];
      P[9] += d * fc[1];
      P[10] += d * fc[2];
    }
    __syncthreads();
  }
  // P: the two halves (lanes o, o + 32); U: the 64 lanes in a fixed butterfly; then the waves
#pragma unroll
  for (int k = 0; k < kEmbF; ++k) P[k] += __shfl_xor(P[k], 32, 64);
#pragma unroll
  for (int k = 0; k < kEmbU; ++k)
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) U[k] += __shfl_xor(U[k], m, 64);
  if (lane < 32) {
#pragma unroll
    for (int k = 0; k < kEmbF; ++k) red[w][o * kEmbF + k] = P[k];
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < kEmbU; ++k) red[w][kEmbSO * kEmbF + k] = U[k];
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
  __shared__ float sA[kEmbSO][kEmbR + 1];  // A[o][c], dbs[o]
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
  const float* U = tot + kEmbSO * kEmbF;  // DX[R], U0, Dvn, Dr, U1, T1
  const float U0 = U[R], Dvn = U[R + 1], Dr = U[R + 2], U1 = U[R + 3], T1 = U[R + 4];
  float* g_lnw = grad;
  float* g_lnb = grad + R;
  float* g_wh = grad + 2 * R;
  float* g_Ws = grad + 2 * R + 1;
  float* g_bs = g_Ws + so * (R + 1);
  float* g_wv = g_bs + so;
  float* g_wsv = g_wv + 1;
  float* g_bsv = g_wsv + so;
  for (int t = threadIdx.x; t < so * (R + 1); t += kEmbFinT) {
    const int o = t / (R + 1), c = t - o * (R + 1);
    const float* p = tot + o * kEmbF;
    const float ws = W.wsv[o];
    const float dbs = p[R] + ws * U0;
    if (c < R) {
      const float a = p[c] + ws * U[c];
      sA[o][c] = a;
      g_Ws[t] = W.ln_w[c] * a + W.ln_b[c] * dbs;
    } else {
      sA[o][R] = dbs;
      g_Ws[t] = p[R + 1] + ws * Dvn;
    }
  }
  for (int o = threadIdx.x; o < so; o += kEmbFinT) {
    const float* p = tot + o * kEmbF;
    g_bs[o] = p[R] + W.wsv[o] * U0;
    float dg = W.bs[o] * U0 + W.Ws[o * (R + 1) + R] * Dvn;
    for (int c = 0; c < R; ++c) dg += W.Ws[o * (R + 1) + c] * (W.ln_w[c] * U[c] + W.ln_b[c] * U0);
    g_wsv[o] = dg;
  }
  __syncthreads();
  if (threadIdx.x < R) {
    const int c = threadIdx.x;
    float gg = 0.f, gb = 0.f;
    for (int o = 0; o < so; ++o) {
      const float wc = W.Ws[o * (R + 1) + c];
      gg += wc * sA[o][c];
      gb += wc * sA[o][R];
    }
    g_lnw[c] = gg;
    g_lnb[c] = gb;
  }
  if (threadIdx.x == 0) {
    float cq = 0.f;
    for (int o = 0; o < so; ++o)
      cq += W.Ws[o * (R + 1) + R] * (tot[o * kEmbF + R + 2] + W.wsv[o] * Dr);
    g_wh[0] = W.wv[0] * T1 + cq;
    g_wv[0] = U1;
    g_bsv[0] = U0;
  }
}

int64_t embed_bwd_blocks(int64_t E) {
  // two 4-wave workgroups per CU (few partial rows for the finishing kernel); >= 256 edges each
  int64_t g = 2 * (int64_t)device_cu_count();
  if (g * kEmbT > E) g = ceil_div(E, (int64_t)kEmbT);
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
  const int64_t blocks = ceil_div(n_edges, (int64_t)kEmbT);
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
  const int64_t per = ceil_div(ceil_div(n_edges, G), (int64_t)kEmbT) * kEmbT;
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
