// K1: per-edge geometric featurisation (forward + backward), HBM-bound, one thread per edge.
//
// Reference: models/mace.py:170-174 and models/tfn.py:171-175 —
//   vectors = pos[ei[0]] - pos[ei[1]]; lengths = |vectors|;
//   edge_sh = e3nn SphericalHarmonics(l<=2, normalize=True, 'component')(vectors)   (9)
//   edge_feats = RadialEmbeddingBlock(lengths) = BesselBasis * PolynomialCutoff      (nb)
// (models/mace_modules/radial.py:44-46, 71-78; blocks.py:91-96).  Bessel weights and the
// prefactor are read from the module buffers so the fp32 values match the reference exactly.
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

__global__ void featurize_fwd_kernel(const float* __restrict__ pos, const int64_t* __restrict__ ei,
                                     int64_t E, int nb, FeatConsts c, float* __restrict__ vec_out,
                                     float* __restrict__ len_out, float* __restrict__ sh_out,
                                     float* __restrict__ rad_out) {
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
    if (sh_out) {
      const float inv = 1.f / fmaxf(r, 1e-12f);  // F.normalize(eps=1e-12)
      float Y[9];
      sh_l2(vx * inv, vy * inv, vz * inv, Y);
#pragma unroll
      for (int k = 0; k < 9; ++k) sh_out[9 * e + k] = Y[k];
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
                                     float* __restrict__ g_vec) {
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
      const float* g = g_sh + 9 * e;
      // gradient w.r.t. the unit vector u = (x, y, z)
      float ux = s3 * g[1] + s15 * z * g[4] + s15 * y * g[5] - s5 * x * g[6] - s15 * x * g[8];
      float uy = s3 * g[2] + s15 * x * g[5] + 2.f * s5 * y * g[6] + s15 * z * g[7];
      float uz = s3 * g[3] + s15 * x * g[4] - s5 * z * g[6] + s15 * y * g[7] + s15 * z * g[8];
      // through u = v / |v|: dv = (du - u (u . du)) / |v|
      const float dot = ux * x + uy * y + uz * z;
      gx += (ux - x * dot) * inv;
      gy += (uy - y * dot) * inv;
      gz += (uz - z * dot) * inv;
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
      pos, edge_index, n_edges, num_bessel, c, vec_out, len_out, sh_out, radial_out);
  return launch_status();
}

int gmp_edge_featurize_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                               int num_bessel, const float* bessel_weights, float prefactor,
                               float r_max, float p_cutoff, const float* g_sh,
                               const float* g_radial, float* g_vec, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && num_bessel >= 0 && num_bessel <= kMaxBessel);
  if (n_edges == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && edge_index && g_vec && (g_radial == nullptr || bessel_weights));
  FeatConsts c{};
  for (int n = 0; n < num_bessel && bessel_weights; ++n) c.w[n] = bessel_weights[n];
  c.prefactor = prefactor;
  c.r_max = r_max;
  c.p = p_cutoff;
  featurize_bwd_kernel<<<grid_for_edges(n_edges), 256, 0, as_stream(stream)>>>(
      pos, edge_index, n_edges, num_bessel, c, g_sh, g_radial, g_vec);
  return launch_status();
}

}  // extern "C"
