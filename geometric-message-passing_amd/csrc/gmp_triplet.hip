// K11: triplet enumeration + angle / torsion featurisation (the "angles"
// of the north star's featurisation list).  Follows models/layers/spherenet_layer.py:496-564
// (`xyz_to_dat`) and the DimeNet forward models/dimenet.py:77-90:
//   edge e = (j -> i); its triplets are the in-edges kj = (k -> j) of j with k != i, in
//   ascending k (the row-major order of torch_sparse's adj_t = SparseTensor(row=i, col=j));
//   triplets of all edges are concatenated in edge order.
//   angle (SphereNet, vertex j): atan2(|(p_i - p_j) x (p_k - p_j)|, (p_i - p_j).(p_k - p_j))
//   angle (DimeNet,   vertex i): atan2(|(p_j - p_i) x (p_k - p_i)|, (p_j - p_i).(p_k - p_i))
//   torsion (SphereNet): min over the in-neighbours k_n != i of j of atan2(b, a) mapped to
//   (0, 2*pi], with plane1 = v_ji x v_jk, plane2 = v_ji x v_jkn, a = plane1.plane2,
//   b = (plane1 x plane2).v_ji / |v_ji|.
// The arithmetic reproduces the reference's torch CPU evaluation operation by operation:
// torch.cross is a_i*b_j - a_j*b_i contracted to fma(a_i, b_j, -(a_j*b_i)); `(x*y).sum(-1)`
// rounds each product then adds (((+0 + 0) + 1) + 2); `.norm(-1)` accumulates fma(x, x, acc);
// `.pow(2).sum(-1).sqrt()` is products, ((0 + 1) + 2), sqrt.  This matters beyond the last ulp:
// for k_n = k plane1 == plane2, and the sign of the contracted cross product's rounding
// residual decides whether that candidate's torsion is ~1e-9 or 2*pi — the reference's
// output depends on it, so the kernel follows it.
#include "gmp_common.h"

namespace gmp {
namespace {

constexpr float kTwoPi = 6.283185307179586f;

struct V3 {
  float x, y, z;
};

__device__ __forceinline__ V3 ld3(const float* __restrict__ p, int64_t a) {
  return V3{p[3 * a], p[3 * a + 1], p[3 * a + 2]};
}
__device__ __forceinline__ V3 sub3(V3 a, V3 b) {
  return V3{__fsub_rn(a.x, b.x), __fsub_rn(a.y, b.y), __fsub_rn(a.z, b.z)};
}
// torch.cross on CPU: fma(a_i, b_j, -(a_j * b_i))
__device__ __forceinline__ V3 cross3(V3 a, V3 b) {
  return V3{__fmaf_rn(a.y, b.z, -__fmul_rn(a.z, b.y)), __fmaf_rn(a.z, b.x, -__fmul_rn(a.x, b.z)),
            __fmaf_rn(a.x, b.y, -__fmul_rn(a.y, b.x))};
}
// (a * b).sum(-1): the reduction starts from +0, so an all-(-0) sum is +0 (atan2(0, +0) = 0,
// not pi, for a degenerate self-loop vector)
__device__ __forceinline__ float dot3(V3 a, V3 b) {
  return __fadd_rn(__fadd_rn(__fadd_rn(0.f, __fmul_rn(a.x, b.x)), __fmul_rn(a.y, b.y)),
                   __fmul_rn(a.z, b.z));
}
// a.norm(dim=-1)
__device__ __forceinline__ float norm3(V3 a) {
  float acc = __fmul_rn(a.x, a.x);
  acc = __fmaf_rn(a.y, a.y, acc);
  acc = __fmaf_rn(a.z, a.z, acc);
  return __fsqrt_rn(acc);
}
// a.pow(2).sum(-1).sqrt()
__device__ __forceinline__ float len3(V3 a) { return __fsqrt_rn(dot3(a, a)); }

// [p, q): entries of the (source-sorted) adjacency row [r0, r1) whose source equals s
__device__ __forceinline__ void equal_range(const int64_t* __restrict__ asrc, int64_t r0,
                                            int64_t r1, int64_t s, int64_t& p, int64_t& q) {
  int64_t lo = r0, hi = r1;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (asrc[m] < s) lo = m + 1;
    else hi = m;
  }
  p = lo;
  hi = r1;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (asrc[m] <= s) lo = m + 1;
    else hi = m;
  }
  q = lo;
}

__global__ void triplet_count_kernel(const float* __restrict__ pos,
                                     const int64_t* __restrict__ ei, int64_t E,
                                     const int64_t* __restrict__ arow,
                                     const int64_t* __restrict__ asrc,
                                     int64_t* __restrict__ counts, float* __restrict__ dist) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += stride) {
    const int64_t j = ei[e], i = ei[E + e];
    const int64_t r0 = arow[j], r1 = arow[j + 1];
    int64_t p, q;
    equal_range(asrc, r0, r1, i, p, q);
    counts[e] = (r1 - r0) - (q - p);
    if (dist) dist[e] = len3(sub3(ld3(pos, i), ld3(pos, j)));
  }
}

// One workgroup per block of kFB consecutive edges.  Phase 1: a thread per edge puts the
// edge's triplet offset, endpoints and adjacency window (row start, the [p, q) run of source i)
// into LDS.  Phase 2: the block's triplets are spread over all threads; each finds its edge by
// a binary search in LDS (no global-memory search per triplet).
// mode 0: SphereNet angle at j (+ optional torsion); mode 1: DimeNet angle at i
constexpr int kFB = 256;

__global__ __launch_bounds__(kFB) void triplet_fill_kernel(
    const float* __restrict__ pos, const int64_t* __restrict__ ei, int64_t E,
    const int64_t* __restrict__ arow, const int64_t* __restrict__ asrc,
    const int64_t* __restrict__ aeid, const int64_t* __restrict__ offs, int mode,
    int64_t* __restrict__ idx_kj, int64_t* __restrict__ idx_ji, float* __restrict__ angle,
    float* __restrict__ torsion, int64_t* __restrict__ torsion_kn) {
  __shared__ int64_t s_off[kFB + 1];
  __shared__ int64_t s_i[kFB], s_j[kFB], s_r0[kFB], s_r1[kFB], s_p[kFB], s_q[kFB];
  const int64_t e0 = (int64_t)blockIdx.x * kFB;
  const int nE = (int)(E - e0 < kFB ? E - e0 : kFB);
  const int tid = threadIdx.x;
  if (tid < nE) {
    const int64_t e = e0 + tid;
    const int64_t j = ei[e], i = ei[E + e];
    const int64_t r0 = arow[j], r1 = arow[j + 1];
    int64_t p, q;
    equal_range(asrc, r0, r1, i, p, q);
    s_off[tid] = offs[e];
    s_i[tid] = i;
    s_j[tid] = j;
    s_r0[tid] = r0;
    s_r1[tid] = r1;
    s_p[tid] = p;
    s_q[tid] = q;
  }
  if (tid == 0) s_off[nE] = offs[e0 + nE];
  __syncthreads();
  const int64_t t_begin = s_off[0], t_end = s_off[nE];
  for (int64_t t = t_begin + tid; t < t_end; t += kFB) {
    int lo = 0, hi = nE;  // largest local edge with s_off <= t
    while (hi - lo > 1) {
      const int m = (lo + hi) >> 1;
      if (s_off[m] <= t) lo = m;
      else hi = m;
    }
    const int64_t e = e0 + lo;
    const int64_t i = s_i[lo], j = s_j[lo], r0 = s_r0[lo], r1 = s_r1[lo];
    const int64_t p = s_p[lo], q = s_q[lo];
    const int64_t local = t - s_off[lo];
    const int64_t slot = r0 + local + (r0 + local >= p ? q - p : 0);
    const int64_t k = asrc[slot];
    idx_kj[t] = aeid[slot];
    idx_ji[t] = e;
    if (!angle && !torsion) continue;
    const V3 pi = ld3(pos, i), pj = ld3(pos, j), pk = ld3(pos, k);
    if (angle) {
      V3 u, v;
      if (mode == 0) {
        u = sub3(pi, pj);
        v = sub3(pk, pj);
      } else {
        u = sub3(pj, pi);
        v = sub3(pk, pi);
      }
      angle[t] = atan2f(norm3(cross3(u, v)), dot3(u, v));
    }
    if (torsion) {
      const V3 vji = sub3(pi, pj);
      const V3 vj0 = sub3(pk, pj);
      const float dji = len3(vji);
      const V3 plane1 = cross3(vji, vj0);
      float best = 3.402823466e38f;  // torch_scatter min: identity FLT_MAX, NaN never wins
      int64_t arg = -1;                // the winning candidate k_n (first among equal minima)
      for (int64_t m = r0; m < r1; ++m) {
        const int64_t kn = asrc[m];
        if (kn == i) continue;
        const V3 vjk = sub3(ld3(pos, kn), pj);
        const V3 plane2 = cross3(vji, vjk);
        const float a = dot3(plane1, plane2);
        const float b = __fdiv_rn(dot3(cross3(plane1, plane2), vji), dji);
        float t1 = atan2f(b, a);
        if (t1 <= 0.f) t1 = __fadd_rn(t1, kTwoPi);
        if (t1 < best) {
          best = t1;
          arg = kn;
        }
      }
      torsion[t] = best == 3.402823466e38f ? 0.f : best;
      if (torsion_kn) torsion_kn[t] = arg;
    }
  }
}

int grid_for(int64_t n) {
  int64_t g = ceil_div(n, 256);
  const int64_t cap = (int64_t)device_cu_count() * 16;
  return (int)(g > cap ? cap : (g < 1 ? 1 : g));
}

// Backward of dist and angle w.r.t. pos (dimenet.py:82-89 / spherenet_layer.py:509,531-535
// under autograd).  theta = atan2(b, a), a = u.v, b = |c|, c = u x v:
//   d theta = (a db - b da) / (a^2 + b^2);  da/du = v, da/dv = u;
//   db/du = v x c^, db/dv = c^ x u (c^ = c / b; 0 when b = 0, as torch's norm backward).
// Rows written (3 floats each): [0, T) vertex -(g_u + g_v), [T, 2T) u end g_u, [2T, 3T) v end
// g_v, [3T, 3T+E) g_d (p_i - p_j) / d at i, [3T+E, 3T+2E) its negative at j; node[] receives
// the row's node so one segmented sum over a CSR of node[] yields d pos deterministically.
__global__ void triplet_geom_bwd_kernel(const float* __restrict__ pos,
                                        const int64_t* __restrict__ ei, int64_t E,
                                        const int64_t* __restrict__ idx_kj,
                                        const int64_t* __restrict__ idx_ji, int64_t T, int mode,
                                        const float* __restrict__ g_dist,
                                        const float* __restrict__ g_angle,
                                        float* __restrict__ rows, int64_t* __restrict__ node) {
  const int64_t n = T + E;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    if (q < T) {
      const int64_t t = q, e = idx_ji[t];
      const int64_t j = ei[e], i = ei[E + e], k = ei[idx_kj[t]];
      const int64_t vtx = mode == 0 ? j : i, ue = mode == 0 ? i : j;
      const V3 pv = ld3(pos, vtx), u = sub3(ld3(pos, ue), pv), v = sub3(ld3(pos, k), pv);
      float gux = 0.f, guy = 0.f, guz = 0.f, gvx = 0.f, gvy = 0.f, gvz = 0.f;
      const float g = g_angle ? g_angle[t] : 0.f;
      if (g != 0.f) {
        const V3 c = cross3(u, v);
        const float b = norm3(c), a = dot3(u, v);
        const float den = a * a + b * b;
        const float ga = -g * b / den, gb = g * a / den;
        gux = ga * v.x; guy = ga * v.y; guz = ga * v.z;
        gvx = ga * u.x; gvy = ga * u.y; gvz = ga * u.z;
        if (b > 0.f) {
          const V3 ch{c.x / b, c.y / b, c.z / b};
          gux += gb * (v.y * ch.z - v.z * ch.y);
          guy += gb * (v.z * ch.x - v.x * ch.z);
          guz += gb * (v.x * ch.y - v.y * ch.x);
          gvx += gb * (ch.y * u.z - ch.z * u.y);
          gvy += gb * (ch.z * u.x - ch.x * u.z);
          gvz += gb * (ch.x * u.y - ch.y * u.x);
        }
      }
      float* r0 = rows + 3 * t;
      float* r1 = rows + 3 * (T + t);
      float* r2 = rows + 3 * (2 * T + t);
      r0[0] = -(gux + gvx); r0[1] = -(guy + gvy); r0[2] = -(guz + gvz);
      r1[0] = gux; r1[1] = guy; r1[2] = guz;
      r2[0] = gvx; r2[1] = gvy; r2[2] = gvz;
      node[t] = vtx;
      node[T + t] = ue;
      node[2 * T + t] = k;
    } else {
      const int64_t e = q - T;
      const int64_t j = ei[e], i = ei[E + e];
      const V3 d = sub3(ld3(pos, i), ld3(pos, j));
      const float len = len3(d);
      const float g = g_dist ? g_dist[e] : 0.f;
      const float s = (g != 0.f && len > 0.f) ? g / len : 0.f;
      float* r0 = rows + 3 * (3 * T + e);
      float* r1 = rows + 3 * (3 * T + E + e);
      r0[0] = s * d.x; r0[1] = s * d.y; r0[2] = s * d.z;
      r1[0] = -(s * d.x); r1[1] = -(s * d.y); r1[2] = -(s * d.z);
      node[3 * T + e] = i;
      node[3 * T + E + e] = j;
    }
  }
}

// Backward of the SphereNet torsion w.r.t. pos (spherenet_layer.py:535-559 under autograd): the
// scatter-min routes the gradient to the winning candidate k_n (torch_scatter's arg), whose
// torsion1 = atan2(b, a) with u = p_i - p_j, v = p_k - p_j, w = p_kn - p_j,
//   P = u x v, Q = u x w, a = P.Q, R = P x Q, c = R.u, L = |u|, b = c / L
// (the 2 pi shift of torsion1 <= 0 has unit derivative).  Reverse mode:
//   ga = -g b / (a^2 + b^2), gb = g a / (a^2 + b^2), gc = gb / L, gL = -gb c / L^2;
//   gu = gL u / L + gc R;  gR = gc u;  gP = Q x gR + ga Q;  gQ = gR x P + ga P;
//   gu += v x gP + w x gQ;  gv = gP x u;  gw = gQ x u;
// rows [0, T) at i (gu), [T, 2T) at j (-(gu + gv + gw)), [2T, 3T) at k (gv), [3T, 4T) at k_n (gw);
// triplets without a candidate (k_n < 0) write zero rows.
__device__ __forceinline__ V3 xf(V3 a, V3 b) {
  return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__global__ void triplet_torsion_bwd_kernel(const float* __restrict__ pos,
                                           const int64_t* __restrict__ ei, int64_t E,
                                           const int64_t* __restrict__ idx_kj,
                                           const int64_t* __restrict__ idx_ji,
                                           const int64_t* __restrict__ kn_of, int64_t T,
                                           const float* __restrict__ g_tor,
                                           float* __restrict__ rows, int64_t* __restrict__ node) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < T;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = idx_ji[t];
    const int64_t j = ei[e], i = ei[E + e], k = ei[idx_kj[t]], kn = kn_of[t];
    const float g = g_tor[t];
    V3 gu{0.f, 0.f, 0.f}, gv{0.f, 0.f, 0.f}, gw{0.f, 0.f, 0.f};
    if (kn >= 0 && g != 0.f) {
      const V3 pj = ld3(pos, j);
      const V3 u = sub3(ld3(pos, i), pj), v = sub3(ld3(pos, k), pj), w = sub3(ld3(pos, kn), pj);
      const V3 P = cross3(u, v), Q = cross3(u, w), R = cross3(P, Q);
      const float a = dot3(P, Q), c = dot3(R, u), L = len3(u);
      const float b = c / L;
      const float den = a * a + b * b;
      const float ga = -g * b / den, gb = g * a / den;
      const float gc = gb / L, gL = -gb * c / (L * L);
      gu = V3{gL * u.x / L + gc * R.x, gL * u.y / L + gc * R.y, gL * u.z / L + gc * R.z};
      const V3 gR{gc * u.x, gc * u.y, gc * u.z};
      V3 gP = xf(Q, gR), gQ = xf(gR, P);
      gP = V3{gP.x + ga * Q.x, gP.y + ga * Q.y, gP.z + ga * Q.z};
      gQ = V3{gQ.x + ga * P.x, gQ.y + ga * P.y, gQ.z + ga * P.z};
      const V3 a1 = xf(v, gP), a2 = xf(w, gQ);
      gu = V3{gu.x + a1.x + a2.x, gu.y + a1.y + a2.y, gu.z + a1.z + a2.z};
      gv = xf(gP, u);
      gw = xf(gQ, u);
    }
    float* r = rows + 3 * t;
    r[0] = gu.x; r[1] = gu.y; r[2] = gu.z;
    r = rows + 3 * (T + t);
    r[0] = -(gu.x + gv.x + gw.x); r[1] = -(gu.y + gv.y + gw.y); r[2] = -(gu.z + gv.z + gw.z);
    r = rows + 3 * (2 * T + t);
    r[0] = gv.x; r[1] = gv.y; r[2] = gv.z;
    r = rows + 3 * (3 * T + t);
    r[0] = gw.x; r[1] = gw.y; r[2] = gw.z;
    node[t] = i;
    node[T + t] = j;
    node[2 * T + t] = k;
    node[3 * T + t] = kn >= 0 ? kn : i;
  }
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_triplet_count(const float* pos, const int64_t* edge_index, int64_t n_edges,
                      int64_t n_nodes, const int64_t* adj_rowptr, const int64_t* adj_src,
                      int64_t* counts, float* dist, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(edge_index && adj_rowptr && adj_src && counts && (pos || !dist));
  triplet_count_kernel<<<grid_for(n_edges), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, adj_rowptr, adj_src, counts, dist);
  return launch_status();
}

int gmp_triplet_fill_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                         int64_t n_nodes, const int64_t* adj_rowptr, const int64_t* adj_src,
                         const int64_t* adj_eid, const int64_t* offsets, int64_t n_triplets,
                         int mode, int64_t* idx_kj, int64_t* idx_ji, float* angle,
                         float* torsion, int64_t* torsion_kn, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && n_triplets >= 0 && (mode == 0 || mode == 1));
  GMP_CHECK_ARG(mode == 0 || !torsion);
  GMP_CHECK_ARG(!torsion_kn || torsion);
  if (n_triplets == 0) return GMP_OK;
  GMP_CHECK_ARG(n_edges > 0 && edge_index && adj_rowptr && adj_src && adj_eid && offsets &&
                idx_kj && idx_ji && (pos || (!angle && !torsion)));
  triplet_fill_kernel<<<(unsigned)ceil_div(n_edges, kFB), kFB, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, adj_rowptr, adj_src, adj_eid, offsets, mode, idx_kj, idx_ji,
      angle, torsion, torsion_kn);
  return launch_status();
}

int gmp_triplet_geom_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                             const int64_t* idx_kj, const int64_t* idx_ji, int64_t n_triplets,
                             int mode, const float* grad_dist, const float* grad_angle,
                             float* rows, int64_t* node, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && n_triplets >= 0 && (mode == 0 || mode == 1));
  if (n_edges + n_triplets == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && edge_index && rows && node && (n_triplets == 0 || (idx_kj && idx_ji)));
  triplet_geom_bwd_kernel<<<grid_for(n_edges + n_triplets), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, idx_kj, idx_ji, n_triplets, mode, grad_dist, grad_angle, rows,
      node);
  return launch_status();
}

int gmp_triplet_torsion_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                                const int64_t* idx_kj, const int64_t* idx_ji,
                                const int64_t* torsion_kn, int64_t n_triplets,
                                const float* grad_torsion, float* rows, int64_t* node,
                                void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && n_triplets >= 0);
  if (n_triplets == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && edge_index && idx_kj && idx_ji && torsion_kn && grad_torsion && rows &&
                node);
  triplet_torsion_bwd_kernel<<<grid_for(n_triplets), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, idx_kj, idx_ji, torsion_kn, n_triplets, grad_torsion, rows, node);
  return launch_status();
}

}  // extern "C"
