// K17: the node feed-forward of GVPConvLayer (models/layers/gvp_layer.py:361-366, :433-434) --
// GVP((128, 16) -> (512, 32), relu) then GVP((512, 32) -> (128, 16), no activations), both with
// vector_gate = True, vector_act = None, h_dim = 32 (gvp_layer.py:101-170) -- as ONE kernel per
// direction over the node rows, in place of ~25 library GEMMs, norms, concatenations and
// elementwise launches each way.
//
// Layout (gmp_gvp_common.h): one wave per 16-node chunk, lane l = node i = l & 15, feature group
// g = l >> 4; every Linear is a chain of v_mfma_f32_16x16x4_f32 products with the weights as the
// A operand from LDS (exact f32 products: the node-level products are ~15 GFLOP per layer and
// direction, ~0.1 ms at the f32 MFMA peak).  The 512-wide hidden scalar row never exists in
// registers: the first GVP's scalar Linear is produced 64 features at a time and immediately
// consumed by the second GVP's scalar Linear (K split over the chunks) and by the first GVP's
// gate (gate1 = Wsv1 p1, accumulated over the chunks); per chunk the workgroup stages
// Ws1[chunk, :] (64 x 160), Wsv1[:, chunk] (32 x 64) and Ws2[:, chunk] (128 x 64) in LDS
// (86 KB), next to the resident small weights (44 KB).
//
// The weight gradients are four node outer sums C = A^T B over the N rows (the host's
// deterministic quadrant sums, one launch each), whose operands the kernels write side by side,
// zero-padded to 64-column multiples:
//   forward : B1 = [s | vn1 | 0] (N, 192), B2 = [s1 | vn2 | 0] (N, 576) with s1 = relu(p1),
//             B3 = [v | 0] (N, 64), B4 = [v1 | 0] (N, 128), and gate1 (N, 32);
//   backward: A1 = [dp1 | dgate1 | 0] (N, 576), A2 = [dp2 | dgate2 | 0] (N, 192),
//             A3 = [dvh1 | du1] (N, 192), A4 = [dvh2 | du2 | 0] (N, 192)
// (vectors in the (channel, xyz) layout; dp the gradient at a scalar Linear's output, du =
// grad_v * sigmoid(gate) the gradient at W_v vh, dvh the gradient at vh).  A1^T B1 holds dWs1 and
// dgate1^T [s | vn1] (-> dWsv1 through Ws1), A2^T B2 dWs2 and dgate2^T [s1 | vn2] (-> dWsv2
// through Ws2), A3^T B3 and A4^T B4 the xyz-diagonal blocks of dWh / dWv (gmp.h).  The backward
// reads s1 from B2 and takes p2 = s2 (the second GVP has no scalar activation).
#include "gmp_gvp_common.h"

namespace gmp {
namespace {

using namespace gvpk;

constexpr int kFT = 512;  // 8 waves; one workgroup per CU (LDS)
constexpr int FS = 128;   // node scalar channels
constexpr int FV = 16;    // node vector channels
constexpr int HS = 512;   // hidden scalar channels
constexpr int HV = 32;    // hidden vector channels (= h_dim of both GVPs)
constexpr int CH = 64;    // hidden scalar features per LDS chunk
constexpr int NCH = HS / CH;

// LDS row strides (floats)
constexpr int L16 = 20, L32 = 36, L64 = 68, L128 = 132, L160 = 164;

// resident weights
constexpr int oWh1 = 0;                 // Wh1 (32 x 16)
constexpr int oWv1 = oWh1 + HV * L16;   // Wv1 (32 x 32)
constexpr int oWh2 = oWv1 + HV * L32;   // Wh2 (32 x 32)
constexpr int oWv2 = oWh2 + HV * L32;   // Wv2 (16 x 32)
constexpr int oWsv2 = oWv2 + FV * L32;  // Wsv2 (16 x 128)
constexpr int oWs2v = oWsv2 + FV * L128;  // Ws2[:, 512:544] (128 x 32)
constexpr int ob1 = oWs2v + FS * L32;   // b1 (512)
constexpr int obsv1 = ob1 + HS;         // bsv1 (32)
constexpr int ob2 = obsv1 + HV;         // b2 (128)
constexpr int obsv2 = ob2 + FS;         // bsv2 (16)
constexpr int oChunk = obsv2 + FV;
// per-chunk weights
constexpr int oWs1c = oChunk;                // Ws1[chunk rows, 0:160] (64 x 160)
constexpr int oWsv1c = oWs1c + CH * L160;    // Wsv1[:, chunk cols] (32 x 64)
constexpr int oWs2c = oWsv1c + HV * L64;     // Ws2[:, chunk cols] (128 x 64)
constexpr int kFFSmem = oWs2c + FS * L64;    // floats
// row strides of the weight-sum operands
constexpr int kB1 = 192, kB2 = 576, kB3 = 64, kB4 = 128, kA1 = 576, kA2 = 192, kA3 = 192,
              kA4 = 192;

struct FFW {
  const float *Wh1, *Ws1, *b1, *Wv1, *Wsv1, *bsv1;  // GVP 1: (32,16) (512,160) (512) (32,32) (32,512) (32)
  const float *Wh2, *Ws2, *b2, *Wv2, *Wsv2, *bsv2;  // GVP 2: (32,32) (128,544) (128) (16,32) (16,128) (16)
};

__device__ void copy_mat(float* dst, int ld, const float* __restrict__ src, int rows, int cols,
                         int src_ld, int col0) {
  for (int x = threadIdx.x; x < rows * cols; x += blockDim.x) {
    const int r = x / cols, c = x - r * cols;
    dst[r * ld + c] = src[(int64_t)r * src_ld + col0 + c];
  }
}

__device__ void ff_resident_to_lds(float* sm, const FFW& P) {
  copy_mat(sm + oWh1, L16, P.Wh1, HV, FV, FV, 0);
  copy_mat(sm + oWv1, L32, P.Wv1, HV, HV, HV, 0);
  copy_mat(sm + oWh2, L32, P.Wh2, HV, HV, HV, 0);
  copy_mat(sm + oWv2, L32, P.Wv2, FV, HV, HV, 0);
  copy_mat(sm + oWsv2, L128, P.Wsv2, FV, FS, FS, 0);
  copy_mat(sm + oWs2v, L32, P.Ws2, FS, HV, HS + HV, HS);
  for (int x = threadIdx.x; x < HS; x += blockDim.x) sm[ob1 + x] = P.b1[x];
  for (int x = threadIdx.x; x < HV; x += blockDim.x) sm[obsv1 + x] = P.bsv1[x];
  for (int x = threadIdx.x; x < FS; x += blockDim.x) sm[ob2 + x] = P.b2[x];
  for (int x = threadIdx.x; x < FV; x += blockDim.x) sm[obsv2 + x] = P.bsv2[x];
}

// float4 tile copy global -> LDS: ROWS x COLS floats (COLS % 4 == 0) of a row-major source with
// row stride SLD starting at column col0; the loads of a thread are issued together (one L2 round
// trip per chunk instead of one per element)
template <int ROWS, int COLS, int SLD, int LD>
struct Tile4 {
  static constexpr int N4 = ROWS * COLS / 4, PER = (N4 + kFT - 1) / kFT;
  f32x4 r[PER];
  __device__ __forceinline__ void load(const float* __restrict__ src, int col0) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int x = threadIdx.x + k * kFT;
      const int row = x / (COLS / 4), c4 = x - row * (COLS / 4);
      if (x < N4) r[k] = *reinterpret_cast<const f32x4*>(src + row * SLD + col0 + 4 * c4);
    }
  }
  __device__ __forceinline__ void store(float* dst) const {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int x = threadIdx.x + k * kFT;
      const int row = x / (COLS / 4), c4 = x - row * (COLS / 4);
      if (x < N4) *reinterpret_cast<f32x4*>(dst + row * LD + 4 * c4) = r[k];
    }
  }
};

__device__ __forceinline__ void ff_chunk_to_lds(float* sm, const FFW& P, int c) {
  Tile4<CH, FS + HV, FS + HV, L160> a;
  Tile4<HV, CH, HS, L64> b;
  Tile4<FS, CH, HS + HV, L64> d;
  a.load(P.Ws1 + (int64_t)c * CH * (FS + HV), 0);
  a.store(sm + oWs1c);  // (two bursts: the backward kernel has no registers for all ten)
  b.load(P.Wsv1, c * CH);
  d.load(P.Ws2, c * CH);
  b.store(sm + oWsv1c);
  d.store(sm + oWs2c);
}

// node n of a 16-row chunk, clamped for the loads (stores are masked by `valid`)
struct Node {
  int64_t n;
  bool valid;
};
__device__ __forceinline__ Node chunk_node(int64_t c, int i, int64_t N) {
  Node k{16 * c + i, true};
  if (k.n >= N) {
    k.valid = false;
    k.n = N - 1;
  }
  return k;
}

// the vector path shared by both directions: vh1 = Wh1 v, vn1, u1 = Wv1 vh1, v1 = u1 sigmoid(gate1),
// vh2 = Wh2 v1, vn2, u2 = Wv2 vh2
struct VecPath {
  f32x4 vh1[3][2], vn1[2], sq1[2], u1[3][2], sg1[2], v1[3][2], vh2[3][2], vn2[2], sq2[2], u2[3][1];
};

__device__ __forceinline__ void vec_path_1(const float* sm, const f32x4 (&v)[3][1], VecPath& F,
                                           int i, int g) {
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    zero(F.vh1[x]);
    gemm_wx<2, 1>(sm + oWh1, L16, v[x], F.vh1[x], i, g);
  }
  vnorm<2>(F.vh1, F.vn1, F.sq1);
}

__device__ __forceinline__ void vec_path_2(const float* sm, VecPath& F, int i, int g) {
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    zero(F.u1[x]);
    gemm_wx<2, 2>(sm + oWv1, L32, F.vh1[x], F.u1[x], i, g);
#pragma unroll
    for (int p = 0; p < 2; ++p) F.v1[x][p] = F.u1[x][p] * F.sg1[p];
  }
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    zero(F.vh2[x]);
    gemm_wx<2, 2>(sm + oWh2, L32, F.v1[x], F.vh2[x], i, g);
  }
  vnorm<2>(F.vh2, F.vn2, F.sq2);
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    zero(F.u2[x]);
    gemm_wx<1, 2>(sm + oWv2, L32, F.vh2[x], F.u2[x], i, g);
  }
}

__global__ __launch_bounds__(kFT) void gvp_ff_fwd_kernel(int64_t N, const float* __restrict__ s_in,
                                                         const float* __restrict__ v_in, FFW P,
                                                         float* __restrict__ s_out,
                                                         float* __restrict__ v_out,
                                                         float* __restrict__ gate1_out,
                                                         float* __restrict__ B1,
                                                         float* __restrict__ B2,
                                                         float* __restrict__ B3,
                                                         float* __restrict__ B4) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  ff_resident_to_lds(sm, P);
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int64_t nchunks = (N + 15) / 16;
  const int64_t c0 = (int64_t)blockIdx.x * (kFT / 64);
  // every wave of the workgroup walks the LDS chunks together (barriers), so the workgroup's
  // node chunks are processed as one group of 8 per pass
  for (int64_t base = c0; base < nchunks; base += (int64_t)gridDim.x * (kFT / 64)) {
    const int64_t cc = base + (threadIdx.x >> 6);
    const Node k = chunk_node(cc < nchunks ? cc : nchunks - 1, i, N);
    const bool valid = k.valid && cc < nchunks;
    f32x4 s[FS / 16], v[3][1];
    ld_row<FS / 16>(s, s_in + k.n * FS, g);
    ld_vrow<1>(v, v_in + k.n * (3 * FV), g);
    __syncthreads();  // resident weights (first pass) / previous pass done with the chunk LDS
    VecPath F;
    vec_path_1(sm, v, F, i, g);
    if (valid) {  // B1 = [s | vn1 | 0], B3 = [v | 0]: stored now, their registers freed early
      f32x4 z2[2], z1[1];
      zero(z2);
      zero(z1);
      st_row<FS / 16>(B1 + k.n * kB1, s, g);
      st_row<2>(B1 + k.n * kB1 + FS, F.vn1, g);
      st_row<2>(B1 + k.n * kB1 + FS + HV, z2, g);
      st_vrow<1>(B3 + k.n * kB3, v, g);
      st_row<1>(B3 + k.n * kB3 + 3 * FV, z1, g);
    }
    f32x4 gate1[2], p2[FS / 16];
    ld_vec<2>(gate1, sm + obsv1, g);
    ld_vec<FS / 16>(p2, sm + ob2, g);
    for (int c = 0; c < NCH; ++c) {
      if (c) __syncthreads();
      ff_chunk_to_lds(sm, P, c);
      __syncthreads();
      f32x4 p1[CH / 16];
      ld_vec<CH / 16>(p1, sm + ob1 + c * CH, g);
      gemm_wx<CH / 16, FS / 16>(sm + oWs1c, L160, s, p1, i, g);
      gemm_wx<CH / 16, 2>(sm + oWs1c + FS, L160, F.vn1, p1, i, g);
      gemm_wx<2, CH / 16>(sm + oWsv1c, L64, p1, gate1, i, g);  // gate from the pre-activation
#pragma unroll
      for (int p = 0; p < CH / 16; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) p1[p][q] = fmaxf(p1[p][q], 0.f);
      if (valid) st_row<CH / 16>(B2 + k.n * kB2 + c * CH, p1, g);
      gemm_wx<FS / 16, CH / 16>(sm + oWs2c, L64, p1, p2, i, g);
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) F.sg1[p][q] = sigm(gate1[p][q]);
    vec_path_2(sm, F, i, g);
    gemm_wx<FS / 16, 2>(sm + oWs2v, L32, F.vn2, p2, i, g);
    f32x4 gate2[1];
    ld_vec<1>(gate2, sm + obsv2, g);
    gemm_wx<1, FS / 16>(sm + oWsv2, L128, p2, gate2, i, g);
    f32x4 v2[3][1];
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int q = 0; q < 4; ++q) v2[x][0][q] = F.u2[x][0][q] * sigm(gate2[0][q]);
    if (valid) {
      st_row<FS / 16>(s_out + k.n * FS, p2, g);
      st_vrow<1>(v_out + k.n * (3 * FV), v2, g);
      st_row<2>(gate1_out + k.n * HV, gate1, g);
      f32x4 z2[2];
      zero(z2);
      st_row<2>(B2 + k.n * kB2 + HS, F.vn2, g);
      st_row<2>(B2 + k.n * kB2 + HS + HV, z2, g);
      st_vrow<2>(B4 + k.n * kB4, F.v1, g);
      st_row<2>(B4 + k.n * kB4 + 3 * HV, z2, g);
    }
  }
}

struct FFGrads {
  float *ds, *dv, *A1, *A2, *A3, *A4;
};

// d|vh| -> dvh with the reference's clamp: zero gradient where sum x^2 < 1e-8
template <int T>
__device__ __forceinline__ void norm_bwd(f32x4 (&dvh)[3][T], const f32x4 (&vh)[3][T],
                                         const f32x4 (&vn)[T], const f32x4 (&sq)[T],
                                         const f32x4 (&dvn)[T]) {
#pragma unroll
  for (int p = 0; p < T; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float f = sq[p][q] >= 1e-8f ? dvn[p][q] / vn[p][q] : 0.f;
#pragma unroll
      for (int x = 0; x < 3; ++x) dvh[x][p][q] += f * vh[x][p][q];
    }
}

// Factors are stored as soon as they are final and the first GVP's vector state (vh1, |vh1|) is
// recomputed after the scalar chunks instead of being held across them (register budget).
__global__ __launch_bounds__(kFT) void gvp_ff_bwd_kernel(
    int64_t N, const float* __restrict__ B2, const float* __restrict__ gate1_in,
    const float* __restrict__ s2, const float* __restrict__ ds_out,
    const float* __restrict__ v_in, const float* __restrict__ dv_out, FFW P, FFGrads O) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  ff_resident_to_lds(sm, P);
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int64_t nchunks = (N + 15) / 16;
  const int64_t c0 = (int64_t)blockIdx.x * (kFT / 64);
  for (int64_t base = c0; base < nchunks; base += (int64_t)gridDim.x * (kFT / 64)) {
    const int64_t cc = base + (threadIdx.x >> 6);
    const Node k = chunk_node(cc < nchunks ? cc : nchunks - 1, i, N);
    const bool valid = k.valid && cc < nchunks;
    f32x4 v[3][1];
    ld_vrow<1>(v, v_in + k.n * (3 * FV), g);
    __syncthreads();
    // ---- forward vector path (recomputed), factors vn1, v1, vn2 stored on the way
    f32x4 u1[3][2], sg1[2], vh2[3][2], vn2[2], sq2[2];
    {
      f32x4 vh1[3][2], vn1[2], sq1[2], gt1[2];
      ld_row<2>(gt1, gate1_in + k.n * HV, g);
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        zero(vh1[x]);
        gemm_wx<2, 1>(sm + oWh1, L16, v[x], vh1[x], i, g);
      }
      vnorm<2>(vh1, vn1, sq1);
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) sg1[p][q] = sigm(gt1[p][q]);
      f32x4 v1[3][2];
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        zero(u1[x]);
        gemm_wx<2, 2>(sm + oWv1, L32, vh1[x], u1[x], i, g);
#pragma unroll
        for (int p = 0; p < 2; ++p) v1[x][p] = u1[x][p] * sg1[p];
      }
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        zero(vh2[x]);
        gemm_wx<2, 2>(sm + oWh2, L32, v1[x], vh2[x], i, g);
      }
    }
    vnorm<2>(vh2, vn2, sq2);
    // ---- GVP 2 backward: du2 = dv2 sg2, dgate2 = sum_x dv2 u2 sg2 (1 - sg2), dvh2 = Wv2^T du2,
    // dp2 = ds2 + Wsv2^T dgate2, dvn2 = Ws2[:, 512:]^T dp2
    f32x4 dp2[FS / 16], dvh2[3][2];
    {
      f32x4 gate2[1], u2[3][1], dv2[3][1], du2[3][1], dg2[1];
      {
        f32x4 p2[FS / 16];
        ld_row<FS / 16>(p2, s2 + k.n * FS, g);  // p2 = s2 (no scalar activation)
        ld_vec<1>(gate2, sm + obsv2, g);
        gemm_wx<1, FS / 16>(sm + oWsv2, L128, p2, gate2, i, g);
      }
      ld_vrow<1>(dv2, dv_out + k.n * (3 * FV), g);
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        zero(u2[x]);
        gemm_wx<1, 2>(sm + oWv2, L32, vh2[x], u2[x], i, g);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float sg = sigm(gate2[0][q]);
        float acc = 0.f;
#pragma unroll
        for (int x = 0; x < 3; ++x) {
          du2[x][0][q] = dv2[x][0][q] * sg;
          acc += dv2[x][0][q] * u2[x][0][q];
        }
        dg2[0][q] = acc * sg * (1.f - sg);
      }
      if (valid) {
        f32x4 z[3];
        zero(z);
        st_vrow<1>(O.A4 + k.n * kA4 + 3 * HV, du2, g);
        st_row<3>(O.A4 + k.n * kA4 + 3 * HV + 3 * FV, z, g);
        st_row<1>(O.A2 + k.n * kA2 + FS, dg2, g);
        st_row<3>(O.A2 + k.n * kA2 + FS + FV, z, g);
      }
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        zero(dvh2[x]);
        gemm_wtx<2, 1>(sm + oWv2, L32, du2[x], dvh2[x], i, g);
      }
      ld_row<FS / 16>(dp2, ds_out + k.n * FS, g);
      gemm_wtx<FS / 16, 1>(sm + oWsv2, L128, dg2, dp2, i, g);
    }
    {
      f32x4 dvn2[2];
      zero(dvn2);
      gemm_wtx<2, FS / 16>(sm + oWs2v, L32, dp2, dvn2, i, g);
      norm_bwd<2>(dvh2, vh2, vn2, sq2, dvn2);
    }
    if (valid) {
      st_vrow<2>(O.A4 + k.n * kA4, dvh2, g);
      st_row<FS / 16>(O.A2 + k.n * kA2, dp2, g);
    }
    // ---- GVP 1 vector backward: dv1 = Wh2^T dvh2, du1 = dv1 sg1, dgate1, dvh1 = Wv1^T du1
    f32x4 dg1[2], dvh1[3][2];
    {
      f32x4 dv1[3][2], du1[3][2];
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        zero(dv1[x]);
        gemm_wtx<2, 2>(sm + oWh2, L32, dvh2[x], dv1[x], i, g);
      }
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float sg = sg1[p][q];
          float acc = 0.f;
#pragma unroll
          for (int x = 0; x < 3; ++x) {
            du1[x][p][q] = dv1[x][p][q] * sg;
            acc += dv1[x][p][q] * u1[x][p][q];
          }
          dg1[p][q] = acc * sg * (1.f - sg);
        }
      if (valid) {
        f32x4 z[2];
        zero(z);
        st_vrow<2>(O.A3 + k.n * kA3 + 3 * HV, du1, g);
        st_row<2>(O.A1 + k.n * kA1 + HS, dg1, g);
        st_row<2>(O.A1 + k.n * kA1 + HS + HV, z, g);
      }
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        zero(dvh1[x]);
        gemm_wtx<2, 2>(sm + oWv1, L32, du1[x], dvh1[x], i, g);
      }
    }
    // ---- scalar chunks: ds1 = Ws2[:, chunk]^T dp2, dp1 = ds1 relu'(p1) + Wsv1[:, chunk]^T dgate1,
    // [ds | dvn1] += Ws1[chunk, :]^T dp1
    f32x4 ds[FS / 16], dvn1[2];
    zero(ds);
    zero(dvn1);
    for (int c = 0; c < NCH; ++c) {
      if (c) __syncthreads();
      ff_chunk_to_lds(sm, P, c);
      __syncthreads();
      f32x4 a1[CH / 16], dp1[CH / 16];
      ld_row<CH / 16>(a1, B2 + k.n * kB2 + c * CH, g);
      zero(dp1);
      gemm_wtx<CH / 16, FS / 16>(sm + oWs2c, L64, dp2, dp1, i, g);
#pragma unroll
      for (int p = 0; p < CH / 16; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) dp1[p][q] = a1[p][q] > 0.f ? dp1[p][q] : 0.f;
      gemm_wtx<CH / 16, 2>(sm + oWsv1c, L64, dg1, dp1, i, g);
      if (valid) st_row<CH / 16>(O.A1 + k.n * kA1 + c * CH, dp1, g);
      gemm_wtx<FS / 16, CH / 16>(sm + oWs1c, L160, dp1, ds, i, g);
      gemm_wtx<2, CH / 16>(sm + oWs1c + FS, L160, dp1, dvn1, i, g);
    }
    // ---- |vh1| backward (vh1 recomputed from v), dv = Wh1^T dvh1
    {
      f32x4 vh1[3][2], vn1[2], sq1[2];
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        zero(vh1[x]);
        gemm_wx<2, 1>(sm + oWh1, L16, v[x], vh1[x], i, g);
      }
      vnorm<2>(vh1, vn1, sq1);
      norm_bwd<2>(dvh1, vh1, vn1, sq1, dvn1);
    }
    f32x4 dv[3][1];
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      zero(dv[x]);
      gemm_wtx<1, 2>(sm + oWh1, L16, dvh1[x], dv[x], i, g);
    }
    if (valid) {
      st_row<FS / 16>(O.ds + k.n * FS, ds, g);
      st_vrow<1>(O.dv + k.n * (3 * FV), dv, g);
      st_vrow<2>(O.A3 + k.n * kA3, dvh1, g);
    }
  }
}

bool a16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

unsigned ff_grid(int64_t N) {
  const int64_t groups = ceil_div(ceil_div(N, 16), kFT / 64);
  const int64_t cap = (int64_t)device_cu_count();
  return (unsigned)(groups < cap ? groups : cap);
}

bool ffw_ok(const FFW& P) {
  return P.Wh1 && P.Ws1 && P.b1 && P.Wv1 && P.Wsv1 && P.bsv1 && P.Wh2 && P.Ws2 && P.b2 &&
         P.Wv2 && P.Wsv2 && P.bsv2;
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_gvp_ff_fwd_f32(int64_t n_nodes, const float* s_in, const float* v_in, const float* Wh1,
                       const float* Ws1, const float* b1, const float* Wv1, const float* Wsv1,
                       const float* bsv1, const float* Wh2, const float* Ws2, const float* b2,
                       const float* Wv2, const float* Wsv2, const float* bsv2, float* s_out,
                       float* v_out, float* gate1_out, float* B1, float* B2, float* B3, float* B4,
                       void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0);
  if (n_nodes == 0) return GMP_OK;
  const FFW P{Wh1, Ws1, b1, Wv1, Wsv1, bsv1, Wh2, Ws2, b2, Wv2, Wsv2, bsv2};
  GMP_CHECK_ARG(ffw_ok(P) && s_in && v_in && s_out && v_out && gate1_out && B1 && B2 && B3 && B4);
  GMP_CHECK_ARG(a16(Ws1) && a16(Wsv1) && a16(Ws2));  // float4 chunk staging
  GMP_CHECK_ARG(a16(s_in) && a16(v_in) && a16(s_out) && a16(v_out) && a16(gate1_out) &&
                a16(B1) && a16(B2) && a16(B3) && a16(B4));
  const size_t smem = (size_t)kFFSmem * sizeof(float);
  int rc = hip_check(hipFuncSetAttribute((const void*)gvp_ff_fwd_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  if (rc) return rc;
  gvp_ff_fwd_kernel<<<ff_grid(n_nodes), kFT, smem, as_stream(stream)>>>(
      n_nodes, s_in, v_in, P, s_out, v_out, gate1_out, B1, B2, B3, B4);
  return launch_status();
}

int gmp_gvp_ff_bwd_f32(int64_t n_nodes, const float* v_in, const float* gate1, const float* B2,
                       const float* s2, const float* ds_out, const float* dv_out,
                       const float* Wh1, const float* Ws1, const float* b1, const float* Wv1,
                       const float* Wsv1, const float* bsv1, const float* Wh2, const float* Ws2,
                       const float* b2, const float* Wv2, const float* Wsv2, const float* bsv2,
                       float* ds_in, float* dv_in, float* A1, float* A2, float* A3, float* A4,
                       void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0);
  if (n_nodes == 0) return GMP_OK;
  const FFW P{Wh1, Ws1, b1, Wv1, Wsv1, bsv1, Wh2, Ws2, b2, Wv2, Wsv2, bsv2};
  const FFGrads O{ds_in, dv_in, A1, A2, A3, A4};
  GMP_CHECK_ARG(ffw_ok(P) && v_in && gate1 && B2 && s2 && ds_out && dv_out);
  GMP_CHECK_ARG(ds_in && dv_in && A1 && A2 && A3 && A4);
  GMP_CHECK_ARG(a16(Ws1) && a16(Wsv1) && a16(Ws2));
  GMP_CHECK_ARG(a16(v_in) && a16(gate1) && a16(B2) && a16(s2) && a16(ds_out) && a16(dv_out) &&
                a16(ds_in) && a16(dv_in) && a16(A1) && a16(A2) && a16(A3) && a16(A4));
  const size_t smem = (size_t)kFFSmem * sizeof(float);
  int rc = hip_check(hipFuncSetAttribute((const void*)gvp_ff_bwd_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  if (rc) return rc;
  gvp_ff_bwd_kernel<<<ff_grid(n_nodes), kFT, smem, as_stream(stream)>>>(
      n_nodes, B2, gate1, s2, ds_out, v_in, dv_out, P, O);
  return launch_status();
}

}  // extern "C"
