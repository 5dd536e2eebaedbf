// K1: per-edge geometric featurisation (forward + backward), HBM-bound, one thread per edge.
//
// Reference: models/mace.py:170-174 and models/tfn.py:171-175 —
//   vectors = pos[ei[0]] - pos[ei[1]]; lengths = |vectors|;
//   edge_sh = e3nn SphericalHarmonics(l<=2, normalize=True, 'component')(vectors)   (9)
//   edge_feats = RadialEmbeddingBlock(lengths) = BesselBasis * PolynomialCutoff      (nb)
// (models/mace_modules/radial.py:44-46, 71-78; blocks.py:91-96).  Bessel weights and the
// prefactor are read from the module buffers so the fp32 values match the reference exactly.
// GVP-GNN (models/gvpgnn.py:106-112) takes the same radial block plus the unit vectors
// nan_to_num(vectors / lengths) (unit_out; zero for a zero-length edge).
// SchNet (models/schnet.py:66-68 over PyG 2.3.1 SchNet / GaussianSmearing / CFConv):
//   edge_weight = |pos[row] - pos[col]|, edge_attr[k] = exp(coeff (d - offset[k])^2) and the
//   CFConv cosine cutoff C = 0.5 (cos(d pi / cutoff) + 1), all from one read of pos per edge.
#include "gmp_common.h"

namespace gmp {
namespace {

constexpr int kMaxBessel = 32;

struct FeatConsts {
  float w[kMaxBessel];  // bessel_weights
  float prefactor, r_max, p;
};

__device__ __forceinline__ void sh_l2(float x, float y, float z, float* Y) {
  const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f, s15 = 3.872983346207417f;
  Y[0] = 1.f;
  Y[1] = s3 * x;
  Y[2] = s3 * y;
  Y[3] = s3 * z;
  Y[4] = s15 * x * z;
  Y[5] = s15 * x * y;
  Y[6] = s5 * (y * y - 0.5f * (x * x + z * z));
  Y[7] = s15 * y * z;
  Y[8] = s15 / 2.f * (z * z - x * x);
}

// l = 3 block of e3nn's SphericalHarmonics (normalization='component') at a unit vector: the
// e3nn recursion's polynomials (sh_3_m of e3nn/o3/_spherical_harmonics.py) times sqrt(7);
// pinned by equivariance under the oracle's D^3 and the CG recursion (tests/test_oracle_o3.py)
constexpr float kS3 = 1.7320508075688772f, kR7 = 2.6457513110645907f;
constexpr float kA3 = 0.9128709291752769f /* sqrt(5/6) */, kB3 = 2.23606797749979f /* sqrt 5 */,
                kC3 = 0.6123724356957945f /* sqrt(3/8) */;
__device__ __forceinline__ void sh_l3(float x, float y, float z, float* Y) {
  const float q = 4.f * y * y - (x * x + z * z);
  Y[0] = kR7 * kA3 * kS3 * (1.5f * x * z * z - 0.5f * x * x * x);
  Y[1] = kR7 * kB3 * kS3 * x * y * z;
  Y[2] = kR7 * kC3 * q * x;
  Y[3] = kR7 * 0.5f * y * (2.f * y * y - 3.f * (x * x + z * z));
  Y[4] = kR7 * kC3 * z * q;
  Y[5] = kR7 * kB3 * kS3 * 0.5f * (z * z - x * x) * y;
  Y[6] = kR7 * kA3 * kS3 * (0.5f * z * z * z - 1.5f * x * x * z);
}
// gradient of sum_m g[m] Y3_m w.r.t. the unit vector (x, y, z), added to (ux, uy, uz)
__device__ __forceinline__ void sh_l3_grad(float x, float y, float z, const float* g, float& ux,
                                           float& uy, float& uz) {
  const float k0 = kR7 * kA3 * kS3, k1 = kR7 * kB3 * kS3, k2 = kR7 * kC3, k3 = kR7 * 0.5f,
              k5 = kR7 * kB3 * kS3 * 0.5f;
  ux += g[0] * k0 * (1.5f * z * z - 1.5f * x * x) + g[1] * k1 * y * z +
        g[2] * k2 * (4.f * y * y - 3.f * x * x - z * z) + g[3] * k3 * (-6.f * x * y) +
        g[4] * k2 * (-2.f * x * z) + g[5] * k5 * (-2.f * x * y) + g[6] * k0 * (-3.f * x * z);
  uy += g[1] * k1 * x * z + g[2] * k2 * 8.f * x * y +
        g[3] * k3 * (6.f * y * y - 3.f * (x * x + z * z)) + g[4] * k2 * 8.f * y * z +
        g[5] * k5 * (z * z - x * x);
  uz += g[0] * k0 * 3.f * x * z + g[1] * k1 * x * y + g[2] * k2 * (-2.f * x * z) +
        g[3] * k3 * (-6.f * y * z) + g[4] * k2 * (4.f * y * y - x * x - 3.f * z * z) +
        g[5] * k5 * 2.f * z * y + g[6] * k0 * (1.5f * z * z - 1.5f * x * x);
}

__global__ void featurize_fwd_kernel(const float* __restrict__ pos, const int64_t* __restrict__ ei,
                                     int64_t E, int nb, FeatConsts c, float* __restrict__ vec_out,
                                     float* __restrict__ len_out, float* __restrict__ sh_out,
                                     float* __restrict__ rad_out, float* __restrict__ unit_out,
                                     int lmax) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = ei[e], b = ei[E + e];
    const float vx = pos[3 * a] - pos[3 * b], vy = pos[3 * a + 1] - pos[3 * b + 1],
                vz = pos[3 * a + 2] - pos[3 * b + 2];
    const float r = sqrtf(vx * vx + vy * vy + vz * vz);
    if (vec_out) {
      vec_out[3 * e] = vx; vec_out[3 * e + 1] = vy; vec_out[3 * e + 2] = vz;
    }
    if (len_out) len_out[e] = r;
    if (unit_out) {  // torch.nan_to_num(vectors / lengths): 0/0 -> 0
      const bool z = !(r > 0.f);
      unit_out[3 * e] = z ? 0.f : vx / r;
      unit_out[3 * e + 1] = z ? 0.f : vy / r;
      unit_out[3 * e + 2] = z ? 0.f : vz / r;
    }
    if (sh_out) {
      const float inv = 1.f / fmaxf(r, 1e-12f);  // F.normalize(eps=1e-12)
      float Y[16];
      sh_l2(vx * inv, vy * inv, vz * inv, Y);
      if (lmax >= 3) sh_l3(vx * inv, vy * inv, vz * inv, Y + 9);
      const int nsh = (lmax + 1) * (lmax + 1);
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < nsh) sh_out[(int64_t)nsh * e + k] = Y[k];
    }
    if (rad_out) {
      const float u = r / c.r_max;
      const float p = c.p;
      const float env = 1.f - ((p + 1.f) * (p + 2.f) / 2.f) * powf(u, p) +
                        p * (p + 2.f) * powf(u, p + 1.f) - (p * (p + 1.f) / 2.f) * powf(u, p + 2.f);
      const float cut = (r < c.r_max) ? env : 0.f;
      for (int n = 0; n < nb; ++n) rad_out[(int64_t)nb * e + n] = c.prefactor * (sinf(c.w[n] * r) / r) * cut;
    }
  }
}

// d/dvec of (sh, radial): g_vec = J_sh^T g_sh + (d rad / d r) . g_rad * vec / r
__global__ void featurize_bwd_kernel(const float* __restrict__ pos, const int64_t* __restrict__ ei,
                                     int64_t E, int nb, FeatConsts c,
                                     const float* __restrict__ g_sh, const float* __restrict__ g_rad,
                                     const float* __restrict__ g_unit, float* __restrict__ g_vec,
                                     int lmax) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = ei[e], b = ei[E + e];
    const float vx = pos[3 * a] - pos[3 * b], vy = pos[3 * a + 1] - pos[3 * b + 1],
                vz = pos[3 * a + 2] - pos[3 * b + 2];
    const float r = sqrtf(vx * vx + vy * vy + vz * vz);
    float gx = 0.f, gy = 0.f, gz = 0.f;
    if (g_sh && r > 1e-12f) {
      const float inv = 1.f / r;
      const float x = vx * inv, y = vy * inv, z = vz * inv;
      const float s3 = 1.7320508075688772f, s5 = 2.23606797749979f, s15 = 3.872983346207417f;
      const int nsh = (lmax + 1) * (lmax + 1);
      const float* g = g_sh + (int64_t)nsh * e;
      // gradient w.r.t. the unit vector u = (x, y, z) (components past lmax read as zero)
      float gl[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) gl[k] = k < nsh ? g[k] : 0.f;
      float ux = s3 * gl[1] + s15 * z * gl[4] + s15 * y * gl[5] - s5 * x * gl[6] - s15 * x * gl[8];
      float uy = s3 * gl[2] + s15 * x * gl[5] + 2.f * s5 * y * gl[6] + s15 * z * gl[7];
      float uz = s3 * gl[3] + s15 * x * gl[4] - s5 * z * gl[6] + s15 * y * gl[7] + s15 * z * gl[8];
      if (lmax >= 3) sh_l3_grad(x, y, z, g + 9, ux, uy, uz);
      // through u = v / |v|: dv = (du - u (u . du)) / |v|
      const float dot = ux * x + uy * y + uz * z;
      gx += (ux - x * dot) * inv;
      gy += (uy - y * dot) * inv;
      gz += (uz - z * dot) * inv;
    }
    if (g_unit && r > 0.f) {  // u = v / |v|: dv = (du - u (u . du)) / |v|
      const float x = vx / r, y = vy / r, z = vz / r;
      const float ux = g_unit[3 * e], uy = g_unit[3 * e + 1], uz = g_unit[3 * e + 2];
      const float dot = ux * x + uy * y + uz * z;
      gx += (ux - x * dot) / r;
      gy += (uy - y * dot) / r;
      gz += (uz - z * dot) / r;
    }
    if (g_rad && r > 0.f) {
      const float u = r / c.r_max, p = c.p;
      float env = 1.f - ((p + 1.f) * (p + 2.f) / 2.f) * powf(u, p) +
                  p * (p + 2.f) * powf(u, p + 1.f) - (p * (p + 1.f) / 2.f) * powf(u, p + 2.f);
      float denv = (-((p + 1.f) * (p + 2.f) / 2.f) * p * powf(u, p - 1.f) +
                    p * (p + 2.f) * (p + 1.f) * powf(u, p) -
                    (p * (p + 1.f) / 2.f) * (p + 2.f) * powf(u, p + 1.f)) / c.r_max;
      if (!(r < c.r_max)) { env = 0.f; denv = 0.f; }
      float dr = 0.f;
      for (int n = 0; n < nb; ++n) {
        const float s = sinf(c.w[n] * r), co = cosf(c.w[n] * r);
        const float bes = c.prefactor * s / r;
        const float dbes = c.prefactor * (c.w[n] * co / r - s / (r * r));
        dr += g_rad[(int64_t)nb * e + n] * (dbes * env + bes * denv);
      }
      gx += dr * vx / r;
      gy += dr * vy / r;
      gz += dr * vz / r;
    }
    g_vec[3 * e] = gx;
    g_vec[3 * e + 1] = gy;
    g_vec[3 * e + 2] = gz;
  }
}

constexpr float kPi = 3.14159265358979323846f;

// SchNet: dist, Gaussians (E, G) and the cosine cutoff per edge.  Offsets come from the
// module's `offset` buffer (device); G <= kMaxGauss (PyG's default is 50).
constexpr int kMaxGauss = 256;

__device__ __forceinline__ float edge_dist(const float* __restrict__ pos, int64_t a, int64_t b,
                                           float& vx, float& vy, float& vz) {
  vx = pos[3 * a] - pos[3 * b];
  vy = pos[3 * a + 1] - pos[3 * b + 1];
  vz = pos[3 * a + 2] - pos[3 * b + 2];
  return sqrtf(vx * vx + vy * vy + vz * vz);
}

// 256 threads = 4 waves; each wave takes 64 edges at a time: lane = edge for the scalars
// (distance, cutoff), then the wave writes the (64, G) Gaussian block as one contiguous float
// range (lane j: floats j, j + 64, ...; coalesced), reading the distances back from LDS.
__global__ void __launch_bounds__(256) schnet_featurize_fwd_kernel(
    const float* __restrict__ pos, const int64_t* __restrict__ ei, int64_t E, int G,
    const float* __restrict__ offsets, float coeff, float cutoff, float* __restrict__ dist_out,
    float* __restrict__ rbf_out, float* __restrict__ cut_out) {
  __shared__ float off[kMaxGauss];
  __shared__ float dsh[4][64];
  for (int k = threadIdx.x; k < G; k += blockDim.x) off[k] = offsets[k];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t e0 = wave * 64; e0 < E; e0 += n_waves * 64) {
    const int ne = (int)(E - e0 < 64 ? E - e0 : 64);
    const int64_t e = e0 + lane;
    if (lane < ne) {
      float vx, vy, vz;
      const float d = edge_dist(pos, ei[e], ei[E + e], vx, vy, vz);
      dsh[wv][lane] = d;
      if (dist_out) dist_out[e] = d;
      if (cut_out) cut_out[e] = 0.5f * (cosf(d * kPi / cutoff) + 1.f);  // C (CFConv)
    }
    if (rbf_out) {
      __builtin_amdgcn_wave_barrier();  // dsh[wv] is wave-private
      float* out = rbf_out + e0 * G;
      const int total = ne * G;
      for (int i = lane; i < total; i += 64) {
        const int el = i / G;
        const float t = dsh[wv][el] - off[i - el * G];
        out[i] = expf(coeff * (t * t));
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// g_d = g_dist + sum_k g_rbf[k] rbf[k] 2 coeff (d - off[k]) - g_cut 0.5 sin(d pi / c) pi / c
// (k ascending); g_vec = g_d v / d, zero for a zero-length edge (torch's norm backward).
// One thread per edge: the backward runs only when pos requires grad.
__global__ void schnet_featurize_bwd_kernel(const float* __restrict__ pos,
                                            const int64_t* __restrict__ ei, int64_t E, int G,
                                            const float* __restrict__ offsets, float coeff,
                                            float cutoff, const float* __restrict__ g_dist,
                                            const float* __restrict__ g_rbf,
                                            const float* __restrict__ g_cut,
                                            float* __restrict__ g_vec) {
  __shared__ float off[kMaxGauss];
  for (int k = threadIdx.x; k < G; k += blockDim.x) off[k] = offsets[k];
  __syncthreads();
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    float vx, vy, vz;
    const float d = edge_dist(pos, ei[e], ei[E + e], vx, vy, vz);
    float gd = g_dist ? g_dist[e] : 0.f;
    if (g_cut) gd -= g_cut[e] * 0.5f * sinf(d * kPi / cutoff) * (kPi / cutoff);
    if (g_rbf) {
      const float* g = g_rbf + e * G;
      for (int k = 0; k < G; ++k) {
        const float t = d - off[k];
        gd += g[k] * expf(coeff * (t * t)) * (2.f * coeff * t);
      }
    }
    const bool z = !(d > 0.f);
    g_vec[3 * e] = z ? 0.f : gd * vx / d;
    g_vec[3 * e + 1] = z ? 0.f : gd * vy / d;
    g_vec[3 * e + 2] = z ? 0.f : gd * vz / d;
  }
}

int grid_for_edges(int64_t E) {
  int64_t g = ceil_div(E, 256);
  const int64_t cap = (int64_t)device_cu_count() * 16;
  return (int)(g > cap ? cap : (g < 1 ? 1 : g));
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_edge_featurize_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                           int num_bessel, const float* bessel_weights, float prefactor,
                           float r_max, float p_cutoff, float* vec_out, float* len_out,
                           float* sh_out, float* radial_out, void* stream) {
  return gmp_edge_featurize_lmax_f32(pos, edge_index, n_edges, 2, num_bessel, bessel_weights,
                                     prefactor, r_max, p_cutoff, vec_out, len_out, sh_out,
                                     radial_out, stream);
}

int gmp_edge_featurize_lmax_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                                int lmax, int num_bessel, const float* bessel_weights,
                                float prefactor, float r_max, float p_cutoff, float* vec_out,
                                float* len_out, float* sh_out, float* radial_out, void* stream) {
  GMP_CHECK_ARG(lmax >= 0 && lmax <= 3);
  GMP_CHECK_ARG(n_edges >= 0 && num_bessel >= 0 && num_bessel <= kMaxBessel);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && edge_index && (radial_out == nullptr || bessel_weights));
  FeatConsts c{};
  // bessel weights are a small host array (copied by value into the kernel argument)
  for (int n = 0; n < num_bessel && bessel_weights; ++n) c.w[n] = bessel_weights[n];
  c.prefactor = prefactor;
  c.r_max = r_max;
  c.p = p_cutoff;
  featurize_fwd_kernel<<<grid_for_edges(n_edges), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, num_bessel, c, vec_out, len_out, sh_out, radial_out, nullptr,
      lmax);
  return launch_status();
}

int gmp_edge_featurize_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                               int num_bessel, const float* bessel_weights, float prefactor,
                               float r_max, float p_cutoff, const float* g_sh,
                               const float* g_radial, float* g_vec, void* stream) {
  return gmp_edge_featurize_lmax_bwd_f32(pos, edge_index, n_edges, 2, num_bessel,
                                         bessel_weights, prefactor, r_max, p_cutoff, g_sh,
                                         g_radial, g_vec, stream);
}

int gmp_edge_featurize_lmax_bwd_f32(const float* pos, const int64_t* edge_index,
                                    int64_t n_edges, int lmax, int num_bessel,
                                    const float* bessel_weights, float prefactor, float r_max,
                                    float p_cutoff, const float* g_sh, const float* g_radial,
                                    float* g_vec, void* stream) {
  GMP_CHECK_ARG(lmax >= 0 && lmax <= 3);
  GMP_CHECK_ARG(n_edges >= 0 && num_bessel >= 0 && num_bessel <= kMaxBessel);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && edge_index && g_vec && (g_radial == nullptr || bessel_weights));
  FeatConsts c{};
  for (int n = 0; n < num_bessel && bessel_weights; ++n) c.w[n] = bessel_weights[n];
  c.prefactor = prefactor;
  c.r_max = r_max;
  c.p = p_cutoff;
  featurize_bwd_kernel<<<grid_for_edges(n_edges), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, num_bessel, c, g_sh, g_radial, nullptr, g_vec, lmax);
  return launch_status();
}

int gmp_edge_featurize_gvp_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                               int num_bessel, const float* bessel_weights, float prefactor,
                               float r_max, float p_cutoff, float* len_out, float* radial_out,
                               float* unit_out, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && num_bessel >= 0 && num_bessel <= kMaxBessel);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && edge_index && (radial_out == nullptr || bessel_weights));
  FeatConsts c{};
  for (int n = 0; n < num_bessel && bessel_weights; ++n) c.w[n] = bessel_weights[n];
  c.prefactor = prefactor;
  c.r_max = r_max;
  c.p = p_cutoff;
  featurize_fwd_kernel<<<grid_for_edges(n_edges), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, num_bessel, c, nullptr, len_out, nullptr, radial_out, unit_out,
      2);
  return launch_status();
}

int gmp_edge_featurize_gvp_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                                   int num_bessel, const float* bessel_weights, float prefactor,
                                   float r_max, float p_cutoff, const float* g_radial,
                                   const float* g_unit, float* g_vec, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && num_bessel >= 0 && num_bessel <= kMaxBessel);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && edge_index && g_vec && (g_radial == nullptr || bessel_weights));
  FeatConsts c{};
  for (int n = 0; n < num_bessel && bessel_weights; ++n) c.w[n] = bessel_weights[n];
  c.prefactor = prefactor;
  c.r_max = r_max;
  c.p = p_cutoff;
  featurize_bwd_kernel<<<grid_for_edges(n_edges), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, num_bessel, c, nullptr, g_radial, g_unit, g_vec, 2);
  return launch_status();
}

int gmp_schnet_featurize_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                             int num_gaussians, const float* offsets, float coeff, float cutoff,
                             float* dist_out, float* rbf_out, float* cut_out, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && num_gaussians >= 0 && num_gaussians <= kMaxGauss);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && edge_index && (rbf_out == nullptr || (offsets && num_gaussians > 0)));
  schnet_featurize_fwd_kernel<<<grid_for_edges(n_edges), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, num_gaussians, offsets, coeff, cutoff, dist_out, rbf_out,
      cut_out);
  return launch_status();
}

int gmp_schnet_featurize_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                                 int num_gaussians, const float* offsets, float coeff,
                                 float cutoff, const float* g_dist, const float* g_rbf,
                                 const float* g_cut, float* g_vec, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && num_gaussians >= 0 && num_gaussians <= kMaxGauss);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && edge_index && g_vec && (g_rbf == nullptr || offsets));
  schnet_featurize_bwd_kernel<<<grid_for_edges(n_edges), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, num_gaussians, offsets, coeff, cutoff, g_dist, g_rbf, g_cut,
      g_vec);
  return launch_status();
}

}  // extern "C"
