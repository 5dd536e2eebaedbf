// PyTorch operator registration of the gmp C ABI (include/gmp.h): TORCH_LIBRARY(gmp, m).
//
// The reference's native boundary is torch_scatter's custom operators
// (`torch.ops.torch_scatter.scatter_sum/mean/max`, reached from `from torch_scatter import
// scatter` at models/layers/egnn_layer.py:4 and models/layers/tfn_layer.py:2).
// This file is the same kind of boundary for the MI355X kernels: one schema per C-ABI entry
// point, a CUDA(HIP)-key implementation that allocates outputs through the caching allocator,
// launches on the current stream and maps error codes to RuntimeError (TORCH_CHECK, as
// torch_scatter does), and a Meta implementation (shapes only) so torch.compile / FakeTensor
// tracing treats every op as one opaque node.  No GPU work happens here; no CPU fallback.
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/ATen.h>
#include <torch/library.h>

#include <string>
#include <vector>

#include "../../../include/gmp.h"

namespace {

using at::Tensor;
using c10::optional;

void* cur_stream() {
  return reinterpret_cast<void*>(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
}

void check_rc(int rc, const char* name) {
  TORCH_CHECK(rc == GMP_OK, name, " failed: ", gmp_error_string(rc), " (code ", rc,
              ", hip error ", gmp_last_hip_error(), ")");
}

void need(const Tensor& t, at::ScalarType st, const char* what) {
  TORCH_CHECK(t.is_cuda(), "gmp: ", what, " must be a HIP device tensor (no CPU fallback)");
  TORCH_CHECK(t.scalar_type() == st, "gmp: ", what, " has dtype ", t.scalar_type(), ", expected ",
              st);
  TORCH_CHECK(t.is_contiguous(), "gmp: ", what, " must be contiguous");
}
Tensor f32(const Tensor& t, const char* what) {
  need(t, at::kFloat, what);
  return t;
}
Tensor i64(const Tensor& t, const char* what) {
  need(t, at::kLong, what);
  return t;
}
float* fp(const Tensor& t) { return t.defined() && t.numel() ? t.data_ptr<float>() : nullptr; }
const float* cfp(const optional<Tensor>& t) {
  return t.has_value() && t->defined() && t->numel() ? t->data_ptr<float>() : nullptr;
}
int64_t* ip(const Tensor& t) { return t.defined() && t.numel() ? t.data_ptr<int64_t>() : nullptr; }
at::TensorOptions fopt(const Tensor& like) { return like.options().dtype(at::kFloat); }

int reduce_code(const std::string& r) {
  if (r == "sum" || r == "add") return GMP_REDUCE_SUM;
  if (r == "mean") return GMP_REDUCE_MEAN;
  if (r == "max") return GMP_REDUCE_MAX;
  TORCH_CHECK(false, "gmp: unsupported reduce '", r, "'");
}

// ------------------------------------------------------------------ index: CSR, gather, reduce
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> csr_build(const Tensor& index, int64_t n_seg,
                                                             const optional<Tensor>& payload) {
  i64(index, "index");
  const int64_t n = index.numel();
  auto o = index.options();
  Tensor perm = at::empty({n}, o), rowptr = at::empty({n_seg + 1}, o), sorted = at::empty({n}, o);
  Tensor pl = payload.has_value() ? i64(*payload, "payload") : Tensor();
  Tensor pls = at::empty({pl.defined() ? n : 0}, o);
  Tensor err = at::zeros({1}, o.dtype(at::kInt));
  const size_t ws_b = gmp_csr_workspace_size(n, n_seg);
  Tensor ws = at::empty({(int64_t)ws_b}, o.dtype(at::kByte));
  check_rc(gmp_csr_build(ip(index), n, n_seg, pl.defined() ? ip(pl) : nullptr, ip(perm),
                         ip(rowptr), ip(sorted), pl.defined() ? ip(pls) : nullptr,
                         err.data_ptr<int32_t>(), ws.data_ptr(), ws_b, cur_stream()),
           "gmp_csr_build");
  return {perm, rowptr, sorted, pls, err};
}

Tensor gather_rows(const Tensor& src, const Tensor& index) {
  f32(src, "src");
  i64(index, "index");
  TORCH_CHECK(src.dim() == 2, "gmp.gather_rows: src must be 2-D");
  Tensor out = at::empty({index.numel(), src.size(1)}, src.options());
  check_rc(gmp_gather_rows_f32(fp(src), src.size(0), src.size(1), ip(index), index.numel(),
                               fp(out), nullptr, cur_stream()),
           "gmp_gather_rows_f32");
  return out;
}

std::tuple<Tensor, Tensor> segment_reduce(const Tensor& src, const optional<Tensor>& perm,
                                          const Tensor& rowptr, int64_t n_seg,
                                          const std::string& reduce) {
  f32(src, "src");
  i64(rowptr, "rowptr");
  TORCH_CHECK(src.dim() == 2 && rowptr.numel() == n_seg + 1, "gmp.segment_reduce: shapes");
  const int red = reduce_code(reduce);
  const int64_t F = src.size(1);
  Tensor out = at::empty({n_seg, F}, src.options());
  Tensor argmax = at::empty({red == GMP_REDUCE_MAX ? n_seg : 0, F}, rowptr.options());
  const size_t ws_b = gmp_segment_reduce_workspace_size(src.size(0), n_seg, F, red);
  Tensor ws = at::empty({(int64_t)ws_b}, src.options().dtype(at::kByte));
  Tensor pm = perm.has_value() ? i64(*perm, "perm") : Tensor();
  check_rc(gmp_segment_reduce_f32(fp(src), src.size(0), F, pm.defined() ? ip(pm) : nullptr,
                                  ip(rowptr), n_seg, red, fp(out),
                                  red == GMP_REDUCE_MAX ? ip(argmax) : nullptr,
                                  ws_b ? ws.data_ptr() : nullptr, ws_b, cur_stream()),
           "gmp_segment_reduce_f32");
  return {out, argmax};
}

Tensor segment_reduce_bwd(const Tensor& grad_out, const Tensor& index, const Tensor& rowptr,
                          const std::string& reduce, const optional<Tensor>& argmax,
                          int64_t n_items) {
  f32(grad_out, "grad_out");
  i64(index, "index");
  i64(rowptr, "rowptr");
  const int red = reduce_code(reduce);
  Tensor am = argmax.has_value() ? i64(*argmax, "argmax") : Tensor();
  TORCH_CHECK(red != GMP_REDUCE_MAX || am.defined(), "gmp.segment_reduce_bwd: max needs argmax");
  Tensor g = at::empty({n_items, grad_out.size(1)}, grad_out.options());
  check_rc(gmp_segment_reduce_bwd_f32(fp(grad_out), grad_out.size(0), grad_out.size(1),
                                      ip(index), n_items, ip(rowptr), red,
                                      am.defined() ? ip(am) : nullptr, fp(g), cur_stream()),
           "gmp_segment_reduce_bwd_f32");
  return g;
}

// ------------------------------------------------------------------ EGNN fused edge kernels
gmp_egnn_params egnn_params(const std::vector<Tensor>& p) {
  TORCH_CHECK(p.size() == 14, "gmp.egnn: 14 parameter tensors expected");
  for (size_t k = 0; k < p.size(); ++k) f32(p[k], "egnn parameter");
  gmp_egnn_params P;
  P.w1d = fp(p[0]); P.b1 = fp(p[1]); P.ln1_w = fp(p[2]); P.ln1_b = fp(p[3]);
  P.W2 = fp(p[4]); P.b2 = fp(p[5]); P.ln2_w = fp(p[6]); P.ln2_b = fp(p[7]);
  P.W3 = fp(p[8]); P.b3 = fp(p[9]); P.ln3_w = fp(p[10]); P.ln3_b = fp(p[11]);
  P.w4 = fp(p[12]); P.b4 = fp(p[13]);
  return P;
}

std::tuple<Tensor, Tensor, Tensor, Tensor> egnn_edge_fwd(
    const Tensor& AB, const Tensor& pos, const Tensor& rowptr, const Tensor& recv,
    const Tensor& send, const std::vector<Tensor>& params, int64_t act, bool msg_mean, double eps,
    bool train) {
  f32(AB, "AB");
  f32(pos, "pos");
  i64(rowptr, "rowptr");
  i64(recv, "recv");
  i64(send, "send");
  const int64_t N = pos.size(0), E = recv.numel(), d = AB.size(1) / 2;
  gmp_egnn_params P = egnn_params(params);
  Tensor m = at::empty({N, d}, fopt(AB)), pa = at::empty({N, 3}, fopt(AB));
  Tensor xh = at::empty({train ? 3 : 0, E, d}, fopt(AB)), rs = at::empty({train ? E : 0, 3}, fopt(AB));
  check_rc(gmp_egnn_edge_fwd_f32(N, E, d, fp(AB), fp(pos), ip(rowptr), ip(recv), ip(send), &P,
                                 (int)act, msg_mean, (float)eps, fp(m), fp(pa),
                                 train ? fp(xh) : nullptr, train ? fp(rs) : nullptr, cur_stream()),
           "gmp_egnn_edge_fwd_f32");
  return {m, pa, xh, rs};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> egnn_edge_bwd(
    const Tensor& pos, const Tensor& rowptr, const Tensor& recv, const Tensor& send,
    const std::vector<Tensor>& params, int64_t act, bool msg_mean, const Tensor& xhat,
    const Tensor& rstd, const Tensor& g_m, const Tensor& g_p, const optional<Tensor>& amax) {
  f32(pos, "pos");
  f32(xhat, "xhat");
  f32(rstd, "rstd");
  f32(g_m, "g_m_aggr");
  f32(g_p, "g_pos_aggr");
  const int64_t N = pos.size(0), E = recv.numel(), d = xhat.size(2);
  gmp_egnn_params P = egnn_params(params);
  auto o = fopt(pos);
  Tensor dA = at::empty({N, d}, o), dpr = at::empty({N, 3}, o), dp1 = at::empty({E, d}, o);
  Tensor gd = at::empty({E, 3}, o), dp2 = at::empty({E, d}, o), dp3 = at::empty({E, d}, o);
  Tensor part = at::empty({gmp_egnn_edge_bwd_partials_rows(E, d), 8 * d + 1}, o);
  TORCH_CHECK(!amax.has_value() || amax->numel() >= 2, "gmp.egnn_edge_bwd: amax has 2 words");
  check_rc(gmp_egnn_edge_bwd_amax_f32(
               N, E, d, fp(pos), ip(rowptr), ip(recv), ip(send), &P, (int)act, msg_mean,
               fp(xhat), fp(rstd), fp(g_m), fp(g_p), fp(dA), fp(dpr), fp(dp1), fp(gd), fp(dp2),
               fp(dp3), fp(part),
               amax.has_value() ? reinterpret_cast<uint32_t*>(amax->data_ptr<int32_t>())
                                : nullptr,
               cur_stream()),
           "gmp_egnn_edge_bwd_amax_f32");
  return {dA, dpr, dp1, gd, dp2, dp3, part};
}

// ------------------------------------------------------------------ SchNet CFConv, SSP
Tensor cfconv_aggregate(const Tensor& x, const Tensor& xidx, const Tensor& w, const Tensor& perm,
                        const Tensor& rowptr, int64_t n_seg, const optional<Tensor>& escale) {
  f32(x, "x");
  f32(w, "w");
  i64(xidx, "xidx");
  Tensor out = at::empty({n_seg, x.size(1)}, x.options());
  Tensor err = at::zeros({1}, x.options().dtype(at::kInt));
  check_rc(gmp_cfconv_aggregate_scaled_f32(fp(x), x.size(0), ip(xidx), fp(w), cfp(escale),
                                           w.size(0), x.size(1), ip(perm), ip(rowptr), n_seg,
                                           fp(out), err.data_ptr<int32_t>(), cur_stream()),
           "gmp_cfconv_aggregate_scaled_f32");
  return out;
}

Tensor cfconv_wgrad(const Tensor& g, const Tensor& gidx, const Tensor& x, const Tensor& xidx,
                    const optional<Tensor>& escale) {
  f32(g, "g");
  f32(x, "x");
  Tensor dw = at::empty({gidx.numel(), x.size(1)}, x.options());
  Tensor err = at::zeros({1}, x.options().dtype(at::kInt));
  check_rc(gmp_cfconv_wgrad_scaled_f32(fp(g), g.size(0), ip(gidx), fp(x), x.size(0), ip(xidx),
                                       cfp(escale), gidx.numel(), x.size(1), fp(dw),
                                       err.data_ptr<int32_t>(), cur_stream()),
           "gmp_cfconv_wgrad_scaled_f32");
  return dw;
}

Tensor ssp_fwd(const Tensor& x, double shift) {
  f32(x, "x");
  Tensor y = at::empty_like(x);
  check_rc(gmp_ssp_fwd_f32(fp(x), x.numel(), (float)shift, fp(y), cur_stream()), "gmp_ssp_fwd_f32");
  return y;
}

Tensor ssp_bwd(const Tensor& x, const Tensor& gy) {
  f32(x, "x");
  f32(gy, "grad_y");
  Tensor gx = at::empty_like(x);
  check_rc(gmp_ssp_bwd_f32(fp(x), fp(gy), x.numel(), fp(gx), cur_stream()), "gmp_ssp_bwd_f32");
  return gx;
}

// ------------------------------------------------------------------ LayerNorm + activation rows
std::tuple<Tensor, Tensor, Tensor> ln_act_fwd(const Tensor& x, const Tensor& gamma,
                                              const Tensor& beta, double eps, int64_t act) {
  f32(x, "x");
  const int64_t d = x.size(-1), rows = x.numel() / d;
  Tensor y = at::empty_like(x), xh = at::empty_like(x), rs = at::empty({rows}, x.options());
  check_rc(gmp_ln_act_fwd_f32(rows, d, fp(x), fp(f32(gamma, "gamma")), fp(f32(beta, "beta")),
                              (float)eps, (int)act, fp(y), fp(xh), fp(rs), cur_stream()),
           "gmp_ln_act_fwd_f32");
  return {y, xh, rs};
}

std::tuple<Tensor, Tensor> ln_act_bwd(const Tensor& gy, const Tensor& xhat, const Tensor& rstd,
                                      const Tensor& gamma, const Tensor& beta, int64_t act) {
  f32(gy, "grad_y");
  f32(xhat, "xhat");
  const int64_t d = xhat.size(-1), rows = xhat.numel() / d;
  Tensor gx = at::empty_like(xhat), gb = at::empty({2 * d}, xhat.options());
  const size_t ws_b = gmp_ln_act_bwd_workspace_size(rows, d);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, xhat.options().dtype(at::kByte));
  check_rc(gmp_ln_act_bwd_f32(rows, d, fp(gy), fp(xhat), fp(f32(rstd, "rstd")), fp(gamma),
                              fp(beta), (int)act, fp(gx), fp(gb), ws.data_ptr(), ws_b,
                              cur_stream()),
           "gmp_ln_act_bwd_f32");
  return {gx, gb};
}

// ------------------------------------------------------------------ K1 featurisation
std::tuple<Tensor, Tensor> edge_featurize(const Tensor& pos, const Tensor& edge_index,
                                          at::ArrayRef<double> bessel_w, double prefactor,
                                          double r_max, double p) {
  f32(pos, "pos");
  i64(edge_index, "edge_index");
  const int64_t E = edge_index.size(1), nb = (int64_t)bessel_w.size();
  std::vector<float> w(bessel_w.begin(), bessel_w.end());
  Tensor sh = at::empty({E, 9}, pos.options()), rad = at::empty({E, nb}, pos.options());
  check_rc(gmp_edge_featurize_f32(fp(pos), ip(edge_index), E, (int)nb, w.data(), (float)prefactor,
                                  (float)r_max, (float)p, nullptr, nullptr, fp(sh), fp(rad),
                                  cur_stream()),
           "gmp_edge_featurize_f32");
  return {sh, rad};
}

Tensor edge_featurize_bwd(const Tensor& pos, const Tensor& edge_index,
                          at::ArrayRef<double> bessel_w, double prefactor, double r_max, double p,
                          const optional<Tensor>& g_sh, const optional<Tensor>& g_rad) {
  f32(pos, "pos");
  const int64_t E = edge_index.size(1), nb = (int64_t)bessel_w.size();
  std::vector<float> w(bessel_w.begin(), bessel_w.end());
  Tensor gv = at::empty({E, 3}, pos.options());
  check_rc(gmp_edge_featurize_bwd_f32(fp(pos), ip(edge_index), E, (int)nb, w.data(),
                                      (float)prefactor, (float)r_max, (float)p, cfp(g_sh),
                                      cfp(g_rad), fp(gv), cur_stream()),
           "gmp_edge_featurize_bwd_f32");
  return gv;
}

std::tuple<Tensor, Tensor> edge_featurize_gvp(const Tensor& pos, const Tensor& edge_index,
                                              at::ArrayRef<double> bessel_w, double prefactor,
                                              double r_max, double p) {
  f32(pos, "pos");
  i64(edge_index, "edge_index");
  const int64_t E = edge_index.size(1), nb = (int64_t)bessel_w.size();
  std::vector<float> w(bessel_w.begin(), bessel_w.end());
  Tensor rad = at::empty({E, nb}, pos.options()), unit = at::empty({E, 3}, pos.options());
  check_rc(gmp_edge_featurize_gvp_f32(fp(pos), ip(edge_index), E, (int)nb, w.data(),
                                      (float)prefactor, (float)r_max, (float)p, nullptr, fp(rad),
                                      fp(unit), cur_stream()),
           "gmp_edge_featurize_gvp_f32");
  return {rad, unit};
}

Tensor edge_featurize_gvp_bwd(const Tensor& pos, const Tensor& edge_index,
                              at::ArrayRef<double> bessel_w, double prefactor, double r_max,
                              double p, const optional<Tensor>& g_rad,
                              const optional<Tensor>& g_unit) {
  f32(pos, "pos");
  const int64_t E = edge_index.size(1), nb = (int64_t)bessel_w.size();
  std::vector<float> w(bessel_w.begin(), bessel_w.end());
  Tensor gv = at::empty({E, 3}, pos.options());
  check_rc(gmp_edge_featurize_gvp_bwd_f32(fp(pos), ip(edge_index), E, (int)nb, w.data(),
                                          (float)prefactor, (float)r_max, (float)p, cfp(g_rad),
                                          cfp(g_unit), fp(gv), cur_stream()),
           "gmp_edge_featurize_gvp_bwd_f32");
  return gv;
}

std::tuple<Tensor, Tensor, Tensor> schnet_featurize(const Tensor& pos, const Tensor& edge_index,
                                                    const Tensor& offsets, double coeff,
                                                    double cutoff) {
  f32(pos, "pos");
  i64(edge_index, "edge_index");
  f32(offsets, "offsets");
  const int64_t E = edge_index.size(1), G = offsets.numel();
  Tensor d = at::empty({E}, pos.options()), rbf = at::empty({E, G}, pos.options()),
         cut = at::empty({E}, pos.options());
  check_rc(gmp_schnet_featurize_f32(fp(pos), ip(edge_index), E, (int)G, fp(offsets),
                                    (float)coeff, (float)cutoff, fp(d), fp(rbf), fp(cut),
                                    cur_stream()),
           "gmp_schnet_featurize_f32");
  return {d, rbf, cut};
}

Tensor schnet_featurize_bwd(const Tensor& pos, const Tensor& edge_index, const Tensor& offsets,
                            double coeff, double cutoff, const optional<Tensor>& g_dist,
                            const optional<Tensor>& g_rbf, const optional<Tensor>& g_cut) {
  f32(pos, "pos");
  const int64_t E = edge_index.size(1), G = offsets.numel();
  Tensor gv = at::empty({E, 3}, pos.options());
  check_rc(gmp_schnet_featurize_bwd_f32(fp(pos), ip(edge_index), E, (int)G, fp(offsets),
                                        (float)coeff, (float)cutoff, cfp(g_dist), cfp(g_rbf),
                                        cfp(g_cut), fp(gv), cur_stream()),
           "gmp_schnet_featurize_bwd_f32");
  return gv;
}

// ------------------------------------------------------------------ K16 Gate / BatchNorm
Tensor gate_fwd(const Tensor& x, const Tensor& out_map, double c_act, double c_gate) {
  f32(x, "x");
  const int64_t B = x.size(0), c_in = x.size(1), c_out = out_map.size(0);
  Tensor y = at::empty({B, c_out}, x.options());
  check_rc(gmp_gate_fwd_f32(B, (int)c_in, (int)c_out, out_map.data_ptr<int32_t>(), (float)c_act,
                            (float)c_gate, fp(x), fp(y), cur_stream()),
           "gmp_gate_fwd_f32");
  return y;
}

Tensor gate_bwd(const Tensor& x, const Tensor& grad_y, const Tensor& in_map, double c_act,
                double c_gate) {
  f32(x, "x");
  f32(grad_y, "grad_y");
  const int64_t B = x.size(0), c_in = x.size(1), c_out = grad_y.size(1);
  Tensor gx = at::empty_like(x);
  check_rc(gmp_gate_bwd_f32(B, (int)c_in, (int)c_out, in_map.data_ptr<int32_t>(), (float)c_act,
                            (float)c_gate, fp(x), fp(grad_y), fp(gx), cur_stream()),
           "gmp_gate_bwd_f32");
  return gx;
}

std::tuple<Tensor, Tensor, Tensor> irreps_bn_fwd(const Tensor& x, const Tensor& col_chan,
                                                 const Tensor& chan_col, const Tensor& chan_info,
                                                 const Tensor& weight,
                                                 const optional<Tensor>& bias,
                                                 Tensor running_mean, Tensor running_var,
                                                 bool training, double momentum, double eps) {
  f32(x, "x");
  const int64_t B = x.size(0), C = x.size(1), nf = chan_col.size(0);
  Tensor y = at::empty_like(x), shift = at::empty({nf}, x.options()),
         invstd = at::empty({nf}, x.options());
  const size_t ws_b = gmp_irreps_bn_workspace_size(B, (int)C, (int)nf);
  Tensor ws = at::empty({(int64_t)ws_b}, x.options().dtype(at::kByte));
  check_rc(gmp_irreps_bn_fwd_f32(B, (int)C, (int)nf, col_chan.data_ptr<int32_t>(),
                                 chan_col.data_ptr<int32_t>(), chan_info.data_ptr<int32_t>(),
                                 fp(x), fp(weight), cfp(bias), fp(running_mean), fp(running_var),
                                 training ? 1 : 0, (float)momentum, (float)eps, fp(y), fp(shift),
                                 fp(invstd), ws.data_ptr(), ws_b, cur_stream()),
           "gmp_irreps_bn_fwd_f32");
  return {y, shift, invstd};
}

std::tuple<Tensor, Tensor, Tensor> irreps_bn_bwd(const Tensor& x, const Tensor& grad_y,
                                                 const Tensor& col_chan, const Tensor& chan_col,
                                                 const Tensor& chan_info, const Tensor& weight,
                                                 const Tensor& shift, const Tensor& invstd,
                                                 bool training, int64_t n_scalar) {
  f32(x, "x");
  f32(grad_y, "grad_y");
  const int64_t B = x.size(0), C = x.size(1), nf = chan_col.size(0);
  Tensor gx = at::empty_like(x), gw = at::empty({nf}, x.options()),
         gb = at::empty({n_scalar}, x.options());
  const size_t ws_b = gmp_irreps_bn_workspace_size(B, (int)C, (int)nf);
  Tensor ws = at::empty({(int64_t)ws_b}, x.options().dtype(at::kByte));
  check_rc(gmp_irreps_bn_bwd_f32(B, (int)C, (int)nf, col_chan.data_ptr<int32_t>(),
                                 chan_col.data_ptr<int32_t>(), chan_info.data_ptr<int32_t>(),
                                 fp(x), fp(grad_y), fp(weight), fp(shift), fp(invstd),
                                 training ? 1 : 0, fp(gx), fp(gw),
                                 n_scalar > 0 ? fp(gb) : nullptr, ws.data_ptr(), ws_b,
                                 cur_stream()),
           "gmp_irreps_bn_bwd_f32");
  return {gx, gw, gb};
}

// ------------------------------------------------------------------ K8 symmetric contraction
Tensor symmetric_contraction_fwd(const Tensor& x, int64_t corr, const Tensor& A1,
                                 const optional<Tensor>& A2, const optional<Tensor>& A3) {
  f32(x, "x");
  const int64_t N = x.size(0), C = x.size(1);
  Tensor out = at::empty({N, 9 * C}, x.options());
  check_rc(gmp_symmetric_contraction_fwd_f32(N, (int)C, (int)corr, fp(x), fp(A1), cfp(A2),
                                             cfp(A3), fp(out), cur_stream()),
           "gmp_symmetric_contraction_fwd_f32");
  return out;
}

std::tuple<Tensor, Tensor> symmetric_contraction_bwd(const Tensor& x, int64_t corr,
                                                     const Tensor& A1, const optional<Tensor>& A2,
                                                     const optional<Tensor>& A3,
                                                     const Tensor& gout) {
  f32(x, "x");
  f32(gout, "gout");
  const int64_t N = x.size(0), C = x.size(1);
  Tensor dx = at::empty_like(x);
  const int64_t nq = corr == 1 ? 9 : (corr == 2 ? 54 : 219);
  Tensor part = at::empty({gmp_sc_groups(N), C, 9, nq}, x.options());
  check_rc(gmp_symmetric_contraction_bwd_f32(N, (int)C, (int)corr, fp(x), fp(A1), cfp(A2),
                                             cfp(A3), fp(gout), fp(dx), fp(part), cur_stream()),
           "gmp_symmetric_contraction_bwd_f32");
  return {dx, part};
}

// ------------------------------------------------------------------ K7 node form
uint32_t* u32p(const optional<Tensor>& t) {
  return t.has_value() ? reinterpret_cast<uint32_t*>(t->data_ptr<int32_t>()) : nullptr;
}
const uint32_t* u32p(const Tensor& t) {
  return reinterpret_cast<const uint32_t*>(t.data_ptr<int32_t>());
}

std::tuple<Tensor, Tensor> tp_node_outer(const Tensor& eoff, const Tensor& Z, const Tensor& A,
                                         int64_t w, const optional<Tensor>& rmax) {
  const int64_t c = eoff.numel() - 1, H = A.size(1);
  Tensor S = at::empty({c, w, H}, A.options()), Sb = at::empty({c, w}, A.options());
  if (rmax.has_value()) {
    f32(*rmax, "rmax");
    TORCH_CHECK(rmax->numel() >= c * (w / 16), "gmp.tp_node_outer: rmax holds n_recv * w / 16");
  }
  check_rc(gmp_tp_node_outer_rmax_f32(c, w, H, ip(i64(eoff, "eoff")), fp(Z), fp(f32(A, "A")),
                                      fp(S), fp(Sb), rmax.has_value() ? fp(*rmax) : nullptr,
                                      cur_stream()),
           "gmp_tp_node_outer_rmax_f32");
  return {S, Sb};
}

void absmax(const Tensor& x, Tensor amax) {
  f32(x, "x");
  check_rc(gmp_absmax_f32(fp(x), x.numel(), reinterpret_cast<uint32_t*>(amax.data_ptr<int32_t>()),
                          cur_stream()),
           "gmp_absmax_f32");
}

Tensor tp_split_w2_h2(const Tensor& W2, const Tensor& b2, int64_t off, int64_t mul1, int64_t mo,
                      bool fwd, const Tensor& wmax) {
  f32(W2, "W2");
  f32(b2, "b2");
  const int64_t H = W2.size(1), K1 = mul1 * H;
  Tensor planes = at::empty({fwd ? 2 * mo * (K1 + mul1) : 2 * K1 * mo},
                            W2.options().dtype(at::kShort));
  check_rc(gmp_tp_split_w2_h2_f32(mul1, mo, H, fp(W2) + off * H, fp(b2) + off, u32p(wmax),
                                  fwd ? planes.data_ptr() : nullptr,
                                  fwd ? nullptr : planes.data_ptr(), cur_stream()),
           "gmp_tp_split_w2_h2_f32");
  return planes;
}

void tp_gemm_h2(const Tensor& A1, int64_t K1, const optional<Tensor>& A2, int64_t K2,
                const Tensor& Bp, int64_t ldb, int64_t N, Tensor C, int64_t c_offset,
                int64_t cgrp, int64_t cldg, int64_t cldr, int64_t cldn, bool accumulate,
                const Tensor& arow, const Tensor& wmax) {
  f32(A1, "A1");
  f32(arow, "arow");
  need(Bp, at::kShort, "B planes");
  TORCH_CHECK(C.is_cuda() && C.scalar_type() == at::kFloat, "gmp.tp_gemm_h2: C");
  const int64_t M = A1.size(0);
  TORCH_CHECK(M > 0 && arow.numel() % M == 0, "gmp.tp_gemm_h2: arow holds M * nparts words");
  check_rc(gmp_tp_gemm_h2_f32(M, N, K1, fp(A1), A1.size(1), K2, cfp(A2),
                              A2.has_value() ? A2->size(1) : 0, Bp.data_ptr(), ldb, N * ldb,
                              fp(arow), arow.numel() / M, u32p(wmax),
                              C.data_ptr<float>() + c_offset, cgrp, cldg, cldr, cldn, accumulate,
                              cur_stream()),
           "gmp_tp_gemm_h2_f32");
}

Tensor tp_gemm_h2_widen(const Tensor& A, const Tensor& Bp, int64_t N, const Tensor& amax,
                        const Tensor& wmax) {
  f32(A, "A");
  need(Bp, at::kShort, "B planes");
  const int64_t M = A.size(0), K = A.size(1);
  Tensor C = at::empty({M, N}, A.options());
  check_rc(gmp_tp_gemm_h2_widen_f32(M, N, K, fp(A), K, Bp.data_ptr(), K, N * K, u32p(amax),
                                    u32p(wmax), fp(C), N, cur_stream()),
           "gmp_tp_gemm_h2_widen_f32");
  return C;
}

void tp_node_apply(const Tensor& eoff, const Tensor& Z, const Tensor& A, const Tensor& T,
                   const Tensor& Tb, Tensor dA, Tensor dZ) {
  const int64_t c = eoff.numel() - 1, w = Z.size(1), H = A.size(1);
  TORCH_CHECK(dZ.sizes() == Z.sizes(), "gmp.tp_node_apply: dZ shape");
  check_rc(gmp_tp_node_apply_f32(c, w, H, ip(eoff), fp(Z), fp(A), fp(f32(T, "T")), fp(Tb),
                                 fp(f32(dZ, "dZ")), fp(f32(dA, "dA")), cur_stream()),
           "gmp_tp_node_apply_f32");
}

Tensor tp_split_w2(const Tensor& W2, const Tensor& b2, int64_t off, int64_t mul1, int64_t mo,
                   bool fwd) {
  f32(W2, "W2");
  f32(b2, "b2");
  const int64_t H = W2.size(1), K1 = mul1 * H;
  Tensor planes = at::empty({fwd ? 3 * mo * (K1 + mul1) : 3 * K1 * mo},
                            W2.options().dtype(at::kShort));
  check_rc(gmp_tp_split_w2_f32(mul1, mo, H, fp(W2) + off * H, fp(b2) + off,
                               fwd ? planes.data_ptr() : nullptr, fwd ? nullptr : planes.data_ptr(),
                               cur_stream()),
           "gmp_tp_split_w2_f32");
  return planes;
}

// C (+)= [A1 | A2] B^T with the grouped epilogue addressing of gmp_tp_gemm_x3_f32 (C mutated)
void tp_gemm_x3(const Tensor& A1, int64_t K1, const optional<Tensor>& A2, int64_t K2,
                const Tensor& Bp, int64_t ldb, int64_t N, Tensor C, int64_t c_offset,
                int64_t cgrp, int64_t cldg, int64_t cldr, int64_t cldn, bool accumulate) {
  f32(A1, "A1");
  need(Bp, at::kShort, "B planes");
  TORCH_CHECK(C.is_cuda() && C.scalar_type() == at::kFloat, "gmp.tp_gemm_x3: C");
  const int64_t M = A1.size(0);
  check_rc(gmp_tp_gemm_x3_f32(M, N, K1, fp(A1), A1.size(1), K2, cfp(A2),
                              A2.has_value() ? A2->size(1) : 0, Bp.data_ptr(), ldb, N * ldb,
                              C.data_ptr<float>() + c_offset, cgrp, cldg, cldr, cldn, accumulate,
                              cur_stream()),
           "gmp_tp_gemm_x3_f32");
}

Tensor tp_gemm_x3_widen(const Tensor& A, const Tensor& Bp, int64_t N) {
  f32(A, "A");
  need(Bp, at::kShort, "B planes");
  const int64_t M = A.size(0), K = A.size(1);
  Tensor C = at::empty({M, N}, A.options());
  check_rc(gmp_tp_gemm_x3_widen_f32(M, N, K, fp(A), K, Bp.data_ptr(), K, N * K, fp(C), N,
                                    cur_stream()),
           "gmp_tp_gemm_x3_widen_f32");
  return C;
}

Tensor outer_sum_cols(const Tensor& A, const Tensor& B) {
  f32(A, "A");
  f32(B, "B");
  const int64_t K = A.size(0), m = A.size(1), n = B.size(1);
  Tensor C = at::empty({m, n}, A.options());
  const size_t ws_b = gmp_outer_sum_cols_workspace_size(K, m, n);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, A.options().dtype(at::kByte));
  check_rc(gmp_outer_sum_cols_f32(K, m, n, fp(A), m, fp(B), n, fp(C), n, ws.data_ptr(), ws_b,
                                  cur_stream()),
           "gmp_outer_sum_cols_f32");
  return C;
}

// ------------------------------------------------------------------ edge outer sums (K5)
std::tuple<Tensor, Tensor> edge_outer_sum(const Tensor& A, const Tensor& B) {
  f32(A, "A");
  f32(B, "B");
  const int64_t K = A.size(0), m = A.size(1), n = B.size(1);
  Tensor C = at::empty({m, n}, A.options()), cs = at::empty({m}, A.options());
  const size_t ws_b = gmp_edge_outer_sum_ex_workspace_size(K, m, n);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, A.options().dtype(at::kByte));
  check_rc(gmp_edge_outer_sum_ex_f32(K, m, n, fp(A), m, fp(B), n, -1, nullptr, nullptr, fp(C), n,
                                     fp(cs), ws.data_ptr(), ws_b, cur_stream()),
           "gmp_edge_outer_sum_ex_f32");
  return {C, cs};
}

// ------------------------------------------------------------------ Meta (shape) kernels
namespace meta {
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> csr_build(const Tensor& index, int64_t n_seg,
                                                             const optional<Tensor>& payload) {
  auto o = index.options();
  const int64_t n = index.numel();
  return {at::empty({n}, o), at::empty({n_seg + 1}, o), at::empty({n}, o),
          at::empty({payload.has_value() ? n : 0}, o), at::empty({1}, o.dtype(at::kInt))};
}
Tensor gather_rows(const Tensor& src, const Tensor& index) {
  return at::empty({index.numel(), src.size(1)}, src.options());
}
std::tuple<Tensor, Tensor> segment_reduce(const Tensor& src, const optional<Tensor>&,
                                          const Tensor& rowptr, int64_t n_seg,
                                          const std::string& reduce) {
  const bool mx = reduce_code(reduce) == GMP_REDUCE_MAX;
  return {at::empty({n_seg, src.size(1)}, src.options()),
          at::empty({mx ? n_seg : 0, src.size(1)}, rowptr.options())};
}
Tensor segment_reduce_bwd(const Tensor& grad_out, const Tensor&, const Tensor&, const std::string&,
                          const optional<Tensor>&, int64_t n_items) {
  return at::empty({n_items, grad_out.size(1)}, grad_out.options());
}
std::tuple<Tensor, Tensor, Tensor, Tensor> egnn_edge_fwd(const Tensor& AB, const Tensor& pos,
                                                         const Tensor&, const Tensor& recv,
                                                         const Tensor&, const std::vector<Tensor>&,
                                                         int64_t, bool, double, bool train) {
  const int64_t N = pos.size(0), E = recv.numel(), d = AB.size(1) / 2;
  auto o = AB.options();
  return {at::empty({N, d}, o), at::empty({N, 3}, o), at::empty({train ? 3 : 0, E, d}, o),
          at::empty({train ? E : 0, 3}, o)};
}
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> egnn_edge_bwd(
    const Tensor& pos, const Tensor&, const Tensor& recv, const Tensor&,
    const std::vector<Tensor>&, int64_t, bool, const Tensor& xhat, const Tensor&, const Tensor&,
    const Tensor&, const optional<Tensor>&) {
  const int64_t N = pos.size(0), E = recv.numel(), d = xhat.size(2);
  auto o = pos.options();
  return {at::empty({N, d}, o), at::empty({N, 3}, o), at::empty({E, d}, o), at::empty({E, 3}, o),
          at::empty({E, d}, o), at::empty({E, d}, o),
          at::empty({gmp_egnn_edge_bwd_partials_rows(E, d), 8 * d + 1}, o)};
}
Tensor cfconv_aggregate(const Tensor& x, const Tensor&, const Tensor&, const Tensor&,
                        const Tensor&, int64_t n_seg, const optional<Tensor>&) {
  return at::empty({n_seg, x.size(1)}, x.options());
}
Tensor cfconv_wgrad(const Tensor&, const Tensor& gidx, const Tensor& x, const Tensor&,
                    const optional<Tensor>&) {
  return at::empty({gidx.numel(), x.size(1)}, x.options());
}
Tensor ssp_fwd(const Tensor& x, double) { return at::empty_like(x); }
Tensor ssp_bwd(const Tensor& x, const Tensor&) { return at::empty_like(x); }
std::tuple<Tensor, Tensor, Tensor> ln_act_fwd(const Tensor& x, const Tensor&, const Tensor&, double,
                                              int64_t) {
  return {at::empty_like(x), at::empty_like(x), at::empty({x.numel() / x.size(-1)}, x.options())};
}
std::tuple<Tensor, Tensor> ln_act_bwd(const Tensor&, const Tensor& xhat, const Tensor&,
                                      const Tensor&, const Tensor&, int64_t) {
  return {at::empty_like(xhat), at::empty({2 * xhat.size(-1)}, xhat.options())};
}
std::tuple<Tensor, Tensor> edge_featurize(const Tensor& pos, const Tensor& ei,
                                          at::ArrayRef<double> w, double, double, double) {
  return {at::empty({ei.size(1), 9}, pos.options()),
          at::empty({ei.size(1), (int64_t)w.size()}, pos.options())};
}
Tensor edge_featurize_bwd(const Tensor& pos, const Tensor& ei, at::ArrayRef<double>, double,
                          double, double, const optional<Tensor>&, const optional<Tensor>&) {
  return at::empty({ei.size(1), 3}, pos.options());
}
std::tuple<Tensor, Tensor> edge_featurize_gvp(const Tensor& pos, const Tensor& ei,
                                              at::ArrayRef<double> w, double, double, double) {
  return {at::empty({ei.size(1), (int64_t)w.size()}, pos.options()),
          at::empty({ei.size(1), 3}, pos.options())};
}
Tensor edge_featurize_gvp_bwd(const Tensor& pos, const Tensor& ei, at::ArrayRef<double>, double,
                              double, double, const optional<Tensor>&, const optional<Tensor>&) {
  return at::empty({ei.size(1), 3}, pos.options());
}
std::tuple<Tensor, Tensor, Tensor> schnet_featurize(const Tensor& pos, const Tensor& ei,
                                                    const Tensor& offsets, double, double) {
  const int64_t E = ei.size(1);
  return {at::empty({E}, pos.options()), at::empty({E, offsets.numel()}, pos.options()),
          at::empty({E}, pos.options())};
}
Tensor schnet_featurize_bwd(const Tensor& pos, const Tensor& ei, const Tensor&, double, double,
                            const optional<Tensor>&, const optional<Tensor>&,
                            const optional<Tensor>&) {
  return at::empty({ei.size(1), 3}, pos.options());
}
Tensor gate_fwd(const Tensor& x, const Tensor& out_map, double, double) {
  return at::empty({x.size(0), out_map.size(0)}, x.options());
}
Tensor gate_bwd(const Tensor& x, const Tensor&, const Tensor&, double, double) {
  return at::empty_like(x);
}
std::tuple<Tensor, Tensor, Tensor> irreps_bn_fwd(const Tensor& x, const Tensor&,
                                                 const Tensor& chan_col, const Tensor&,
                                                 const Tensor&, const optional<Tensor>&, Tensor,
                                                 Tensor, bool, double, double) {
  const int64_t nf = chan_col.size(0);
  return {at::empty_like(x), at::empty({nf}, x.options()), at::empty({nf}, x.options())};
}
std::tuple<Tensor, Tensor, Tensor> irreps_bn_bwd(const Tensor& x, const Tensor&, const Tensor&,
                                                 const Tensor& chan_col, const Tensor&,
                                                 const Tensor&, const Tensor&, const Tensor&,
                                                 bool, int64_t n_scalar) {
  return {at::empty_like(x), at::empty({chan_col.size(0)}, x.options()),
          at::empty({n_scalar}, x.options())};
}
Tensor symmetric_contraction_fwd(const Tensor& x, int64_t, const Tensor&, const optional<Tensor>&,
                                 const optional<Tensor>&) {
  return at::empty({x.size(0), 9 * x.size(1)}, x.options());
}
std::tuple<Tensor, Tensor> symmetric_contraction_bwd(const Tensor& x, int64_t corr,
                                                     const Tensor&, const optional<Tensor>&,
                                                     const optional<Tensor>&, const Tensor&) {
  const int64_t nq = corr == 1 ? 9 : (corr == 2 ? 54 : 219);
  return {at::empty_like(x), at::empty({gmp_sc_groups(x.size(0)), x.size(1), 9, nq},
                                       x.options())};
}
std::tuple<Tensor, Tensor> tp_node_outer(const Tensor& eoff, const Tensor&, const Tensor& A,
                                         int64_t w, const optional<Tensor>&) {
  const int64_t c = eoff.numel() - 1;
  return {at::empty({c, w, A.size(1)}, A.options()), at::empty({c, w}, A.options())};
}
void absmax(const Tensor&, Tensor) {}
Tensor tp_split_w2_h2(const Tensor& W2, const Tensor&, int64_t, int64_t mul1, int64_t mo,
                      bool fwd, const Tensor&) {
  const int64_t K1 = mul1 * W2.size(1);
  return at::empty({fwd ? 2 * mo * (K1 + mul1) : 2 * K1 * mo}, W2.options().dtype(at::kShort));
}
void tp_gemm_h2(const Tensor&, int64_t, const optional<Tensor>&, int64_t, const Tensor&, int64_t,
                int64_t, Tensor, int64_t, int64_t, int64_t, int64_t, int64_t, bool,
                const Tensor&, const Tensor&) {}
Tensor tp_gemm_h2_widen(const Tensor& A, const Tensor&, int64_t N, const Tensor&,
                        const Tensor&) {
  return at::empty({A.size(0), N}, A.options());
}
void tp_node_apply(const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                   Tensor, Tensor) {}
Tensor tp_split_w2(const Tensor& W2, const Tensor&, int64_t, int64_t mul1, int64_t mo, bool fwd) {
  const int64_t K1 = mul1 * W2.size(1);
  return at::empty({fwd ? 3 * mo * (K1 + mul1) : 3 * K1 * mo}, W2.options().dtype(at::kShort));
}
void tp_gemm_x3(const Tensor&, int64_t, const optional<Tensor>&, int64_t, const Tensor&, int64_t,
                int64_t, Tensor, int64_t, int64_t, int64_t, int64_t, int64_t, bool) {}
Tensor tp_gemm_x3_widen(const Tensor& A, const Tensor&, int64_t N) {
  return at::empty({A.size(0), N}, A.options());
}
Tensor outer_sum_cols(const Tensor& A, const Tensor& B) {
  return at::empty({A.size(1), B.size(1)}, A.options());
}
std::tuple<Tensor, Tensor> edge_outer_sum(const Tensor& A, const Tensor& B) {
  return {at::empty({A.size(1), B.size(1)}, A.options()), at::empty({A.size(1)}, A.options())};
}
}  // namespace meta

}  // namespace

TORCH_LIBRARY(gmp, m) {
  m.def("csr_build(Tensor index, int n_seg, Tensor? payload=None) -> "
        "(Tensor perm, Tensor rowptr, Tensor sorted, Tensor payload_sorted, Tensor err)");
  m.def("gather_rows(Tensor src, Tensor index) -> Tensor");
  m.def("segment_reduce(Tensor src, Tensor? perm, Tensor rowptr, int n_seg, str reduce) -> "
        "(Tensor out, Tensor argmax)");
  m.def("segment_reduce_bwd(Tensor grad_out, Tensor index, Tensor rowptr, str reduce, "
        "Tensor? argmax, int n_items) -> Tensor");
  m.def("egnn_edge_fwd(Tensor AB, Tensor pos, Tensor rowptr, Tensor recv, Tensor send, "
        "Tensor[] params, int act, bool msg_mean, float eps, bool train) -> "
        "(Tensor m_aggr, Tensor pos_aggr, Tensor xhat, Tensor rstd)");
  m.def("egnn_edge_bwd(Tensor pos, Tensor rowptr, Tensor recv, Tensor send, Tensor[] params, "
        "int act, bool msg_mean, Tensor xhat, Tensor rstd, Tensor g_m_aggr, Tensor g_pos_aggr, "
        "Tensor(a!)? amax=None) -> (Tensor dA, Tensor dpos_recv, Tensor dpre1, Tensor gdiff, "
        "Tensor dpre2, Tensor dpre3, Tensor partials)");
  m.def("cfconv_aggregate(Tensor x, Tensor xidx, Tensor w, Tensor perm, Tensor rowptr, "
        "int n_seg, Tensor? escale=None) -> Tensor");
  m.def("cfconv_wgrad(Tensor g, Tensor gidx, Tensor x, Tensor xidx, Tensor? escale=None) -> "
        "Tensor");
  m.def("ssp_fwd(Tensor x, float shift) -> Tensor");
  m.def("ssp_bwd(Tensor x, Tensor grad_y) -> Tensor");
  m.def("ln_act_fwd(Tensor x, Tensor gamma, Tensor beta, float eps, int act) -> "
        "(Tensor y, Tensor xhat, Tensor rstd)");
  m.def("ln_act_bwd(Tensor grad_y, Tensor xhat, Tensor rstd, Tensor gamma, Tensor beta, "
        "int act) -> (Tensor grad_x, Tensor grad_gamma_beta)");
  m.def("edge_featurize(Tensor pos, Tensor edge_index, float[] bessel_weights, float prefactor, "
        "float r_max, float p) -> (Tensor sh, Tensor radial)");
  m.def("edge_featurize_bwd(Tensor pos, Tensor edge_index, float[] bessel_weights, "
        "float prefactor, float r_max, float p, Tensor? g_sh, Tensor? g_radial) -> Tensor");
  m.def("edge_featurize_gvp(Tensor pos, Tensor edge_index, float[] bessel_weights, "
        "float prefactor, float r_max, float p) -> (Tensor radial, Tensor unit)");
  m.def("edge_featurize_gvp_bwd(Tensor pos, Tensor edge_index, float[] bessel_weights, "
        "float prefactor, float r_max, float p, Tensor? g_radial, Tensor? g_unit) -> Tensor");
  m.def("schnet_featurize(Tensor pos, Tensor edge_index, Tensor offsets, float coeff, "
        "float cutoff) -> (Tensor dist, Tensor rbf, Tensor cut)");
  m.def("schnet_featurize_bwd(Tensor pos, Tensor edge_index, Tensor offsets, float coeff, "
        "float cutoff, Tensor? g_dist, Tensor? g_rbf, Tensor? g_cut) -> Tensor");
  m.def("gate_fwd(Tensor x, Tensor out_map, float c_act, float c_gate) -> Tensor");
  m.def("gate_bwd(Tensor x, Tensor grad_y, Tensor in_map, float c_act, float c_gate) -> Tensor");
  m.def("irreps_bn_fwd(Tensor x, Tensor col_chan, Tensor chan_col, Tensor chan_info, "
        "Tensor weight, Tensor? bias, Tensor(a!) running_mean, Tensor(b!) running_var, "
        "bool training, float momentum, float eps) -> (Tensor y, Tensor shift, Tensor invstd)");
  m.def("irreps_bn_bwd(Tensor x, Tensor grad_y, Tensor col_chan, Tensor chan_col, "
        "Tensor chan_info, Tensor weight, Tensor shift, Tensor invstd, bool training, "
        "int n_scalar) -> (Tensor grad_x, Tensor grad_weight, Tensor grad_bias)");
  m.def("symmetric_contraction_fwd(Tensor x, int correlation, Tensor A1, Tensor? A2, "
        "Tensor? A3) -> Tensor");
  m.def("symmetric_contraction_bwd(Tensor x, int correlation, Tensor A1, Tensor? A2, "
        "Tensor? A3, Tensor gout) -> (Tensor dx, Tensor dA_partials)");
  m.def("tp_node_outer(Tensor eoff, Tensor Z, Tensor A, int w, Tensor(a!)? rmax=None) -> "
        "(Tensor S, Tensor Sb)");
  m.def("absmax(Tensor x, Tensor(a!) amax) -> ()");
  m.def("tp_split_w2_h2(Tensor W2, Tensor b2, int off, int mul1, int mul_out, bool fwd, "
        "Tensor wmax) -> Tensor");
  m.def("tp_gemm_h2(Tensor A1, int K1, Tensor? A2, int K2, Tensor Bp, int ldb, int N, "
        "Tensor(a!) C, int c_offset, int cgrp, int cldg, int cldr, int cldn, bool accumulate, "
        "Tensor arow, Tensor wmax) -> ()");
  m.def("tp_gemm_h2_widen(Tensor A, Tensor Bp, int N, Tensor amax, Tensor wmax) -> Tensor");
  m.def("tp_node_apply(Tensor eoff, Tensor Z, Tensor A, Tensor T, Tensor Tb, Tensor(a!) dA, "
        "Tensor(b!) dZ) -> ()");
  m.def("tp_split_w2(Tensor W2, Tensor b2, int off, int mul1, int mul_out, bool fwd) -> Tensor");
  m.def("tp_gemm_x3(Tensor A1, int K1, Tensor? A2, int K2, Tensor Bp, int ldb, int N, "
        "Tensor(a!) C, int c_offset, int cgrp, int cldg, int cldr, int cldn, bool accumulate) "
        "-> ()");
  m.def("tp_gemm_x3_widen(Tensor A, Tensor Bp, int N) -> Tensor");
  m.def("outer_sum_cols(Tensor A, Tensor B) -> Tensor");
  m.def("edge_outer_sum(Tensor A, Tensor B) -> (Tensor C, Tensor colsum)");
}

#define GMP_IMPL(m, ns)                                                    \
  m.impl("csr_build", ns csr_build);                                      \
  m.impl("gather_rows", ns gather_rows);                                  \
  m.impl("segment_reduce", ns segment_reduce);                            \
  m.impl("segment_reduce_bwd", ns segment_reduce_bwd);                    \
  m.impl("egnn_edge_fwd", ns egnn_edge_fwd);                              \
  m.impl("egnn_edge_bwd", ns egnn_edge_bwd);                              \
  m.impl("cfconv_aggregate", ns cfconv_aggregate);                        \
  m.impl("cfconv_wgrad", ns cfconv_wgrad);                                \
  m.impl("ssp_fwd", ns ssp_fwd);                                          \
  m.impl("ssp_bwd", ns ssp_bwd);                                          \
  m.impl("ln_act_fwd", ns ln_act_fwd);                                    \
  m.impl("ln_act_bwd", ns ln_act_bwd);                                    \
  m.impl("edge_featurize", ns edge_featurize);                            \
  m.impl("edge_featurize_bwd", ns edge_featurize_bwd);                    \
  m.impl("edge_featurize_gvp", ns edge_featurize_gvp);                    \
  m.impl("edge_featurize_gvp_bwd", ns edge_featurize_gvp_bwd);            \
  m.impl("schnet_featurize", ns schnet_featurize);                        \
  m.impl("schnet_featurize_bwd", ns schnet_featurize_bwd);                \
  m.impl("gate_fwd", ns gate_fwd);                                        \
  m.impl("gate_bwd", ns gate_bwd);                                        \
  m.impl("irreps_bn_fwd", ns irreps_bn_fwd);                              \
  m.impl("irreps_bn_bwd", ns irreps_bn_bwd);                              \
  m.impl("symmetric_contraction_fwd", ns symmetric_contraction_fwd);      \
  m.impl("symmetric_contraction_bwd", ns symmetric_contraction_bwd);      \
  m.impl("tp_node_outer", ns tp_node_outer);                              \
  m.impl("absmax", ns absmax);                                            \
  m.impl("tp_split_w2_h2", ns tp_split_w2_h2);                            \
  m.impl("tp_gemm_h2", ns tp_gemm_h2);                                    \
  m.impl("tp_gemm_h2_widen", ns tp_gemm_h2_widen);                        \
  m.impl("tp_node_apply", ns tp_node_apply);                              \
  m.impl("tp_split_w2", ns tp_split_w2);                                  \
  m.impl("tp_gemm_x3", ns tp_gemm_x3);                                    \
  m.impl("tp_gemm_x3_widen", ns tp_gemm_x3_widen);                        \
  m.impl("outer_sum_cols", ns outer_sum_cols);                            \
  m.impl("edge_outer_sum", ns edge_outer_sum);

TORCH_LIBRARY_IMPL(gmp, CUDA, m) { GMP_IMPL(m, ) }
TORCH_LIBRARY_IMPL(gmp, Meta, m) { GMP_IMPL(m, meta::) }
