"""ctypes binding of libgmp.so (the C ABI declared in include/gmp.h).

The product path has no CPU fallback: if the library is missing or a CUDA/HIP device is not
available the ops raise.  Build with `python -c "import __graft_entry__ as g; g.build()"` or
`make -C geometric-message-passing_amd/csrc`.
"""
import ctypes
import os

# Import torch first: its bundled libamdhip64.so (SONAME libamdhip64.so.7) must be the HIP
# runtime that libgmp.so binds to, so both share one runtime, device context and streams.
import torch  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GMP_LIB", os.path.join(_HERE, "libgmp.so"))

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_vp = ctypes.c_void_p
c_f32 = ctypes.c_float
c_size = ctypes.c_size_t

GMP_OK, GMP_ERR_ARG, GMP_ERR_HIP, GMP_ERR_UNSUPPORTED, GMP_ERR_WORKSPACE = 0, -1, -2, -3, -4
REDUCE = {"sum": 0, "add": 0, "mean": 1, "max": 2}
ACT = {"relu": 0, "swish": 1, "silu": 1}


class GmpEgnnParams(ctypes.Structure):
    _fields_ = [(n, c_vp) for n in (
        "w1d", "b1", "ln1_w", "ln1_b", "W2", "b2", "ln2_w", "ln2_b", "W3", "b3", "ln3_w", "ln3_b",
        "w4", "b4")]


class GmpEgnnNodeParams(ctypes.Structure):
    _fields_ = [(n, c_vp) for n in ("W0", "b0", "ln1_w", "ln1_b", "W3", "b3", "ln2_w", "ln2_b",
                                     "W1n")] + [("ld1", ctypes.c_longlong)]


class TpPath(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("l1", "l2", "lo", "mul1", "mul_out", "x_off", "y_off", "io",
                                       "out_off", "z_off", "cg_off", "pad")] + [
        ("w_off", ctypes.c_longlong), ("alpha", c_f32), ("pad2", c_f32)]


class TpDesc(ctypes.Structure):
    _fields_ = [("n_paths", c_int), ("in_dim", c_int), ("out_dim", c_int), ("sh_dim", c_int),
                ("weight_numel", ctypes.c_longlong), ("z_size", c_int), ("n_blocks", c_int),
                ("blk_off", c_int * 8), ("blk_mul", c_int * 8), ("blk_l", c_int * 8)]


assert ctypes.sizeof(TpPath) == 64 and ctypes.sizeof(TpDesc) == 128

# name -> (restype, argtypes); must mirror include/gmp.h exactly
SIGNATURES = {
    "gmp_abi_version": (c_int, []),
    "gmp_error_string": (ctypes.c_char_p, [c_int]),
    "gmp_last_hip_error": (c_int, []),
    "gmp_csr_workspace_size": (c_size, [c_i64, c_i64]),
    "gmp_csr_build": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                              c_size, c_vp]),
    "gmp_gather_rows_f32": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "gmp_cfconv_aggregate_f32": (c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp,
                                         c_i64, c_vp, c_vp, c_vp]),
    "gmp_cfconv_wgrad_f32": (c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp,
                                     c_vp, c_vp]),
    "gmp_ssp_fwd_f32": (c_int, [c_vp, c_i64, c_f32, c_vp, c_vp]),
    "gmp_ssp_bwd_f32": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "gmp_segment_reduce_workspace_size": (c_size, [c_i64, c_i64, c_i64, c_int]),
    "gmp_segment_reduce_f32": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_int, c_vp, c_vp,
                                       c_vp, c_size, c_vp]),
    "gmp_segment_reduce_bwd_f32": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_int, c_vp,
                                           c_vp, c_vp]),
    "gmp_egnn_edge_fwd_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      ctypes.POINTER(GmpEgnnParams), c_int, c_int, c_f32, c_vp,
                                      c_vp, c_vp, c_int, c_vp, c_vp]),
    "gmp_egnn_edge_bwd_partials_rows": (c_i64, [c_i64, c_i64]),
    "gmp_egnn_set_f32_mfma": (c_int, [c_int]),
    "gmp_wgrad_set_f32_mfma": (c_int, [c_int]),
    "gmp_edge_outer_sum_workspace_size": (c_size, [c_i64, c_i64]),
    "gmp_edge_outer_sum_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    "gmp_edge_outer_sum_act_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_vp,
                                           c_vp, c_vp, c_size, c_vp]),
    "gmp_edge_featurize_f32": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_f32, c_f32, c_f32, c_vp,
                                       c_vp, c_vp, c_vp, c_vp]),
    "gmp_edge_featurize_bwd_f32": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_f32, c_f32, c_f32,
                                           c_vp, c_vp, c_vp, c_vp]),
    "gmp_edge_featurize_lmax_f32": (c_int, [c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_f32, c_f32,
                                            c_f32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_edge_featurize_lmax_bwd_f32": (c_int, [c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_f32,
                                                c_f32, c_f32, c_vp, c_vp, c_vp, c_vp]),
    "gmp_edge_featurize_gvp_f32": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_f32, c_f32, c_f32,
                                           c_vp, c_vp, c_vp, c_vp]),
    "gmp_edge_featurize_gvp_bwd_f32": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_f32, c_f32,
                                               c_f32, c_vp, c_vp, c_vp, c_vp]),
    "gmp_triplet_geom_bwd_f32": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_int, c_vp,
                                         c_vp, c_vp, c_vp, c_vp]),
    "gmp_cfconv_aggregate_scaled_f32": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64,
                                                c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "gmp_cfconv_wgrad_scaled_f32": (c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64,
                                            c_i64, c_vp, c_vp, c_vp]),
    "gmp_edge_outer_sum_act_hf_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_int,
                                              c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    "gmp_egnn_edge_bwd_amax_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                           c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp,
                                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_gate_fwd_f32": (c_int, [c_i64, c_int, c_int, c_vp, c_f32, c_f32, c_vp, c_vp, c_vp]),
    "gmp_gate_bwd_f32": (c_int, [c_i64, c_int, c_int, c_vp, c_f32, c_f32, c_vp, c_vp, c_vp,
                                 c_vp]),
    "gmp_irreps_bn_workspace_size": (c_size, [c_i64, c_int, c_int]),
    "gmp_irreps_bn_fwd_f32": (c_int, [c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp, c_vp, c_int, c_f32, c_f32, c_vp, c_vp, c_vp, c_vp,
                                      c_size, c_vp]),
    "gmp_irreps_bn_bwd_f32": (c_int, [c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_size,
                                      c_vp]),
    "gmp_schnet_featurize_f32": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_f32, c_f32, c_vp, c_vp,
                                         c_vp, c_vp]),
    "gmp_schnet_featurize_bwd_f32": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_f32, c_f32, c_vp,
                                             c_vp, c_vp, c_vp, c_vp]),
    "gmp_tp_conv_fwd_f32": (c_int, [c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_i64, c_i64, c_vp, c_vp]),
    "gmp_tp_conv_bwd_f32": (c_int, [c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                    c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_tp_edge_z_f32": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                  c_vp, c_vp]),
    "gmp_tp_edge_z_bwd_f32": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_i64,
                                      c_i64, c_vp, c_vp, c_vp, c_vp]),
    "gmp_tp_edge_z_lmax_f32": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp,
                                       c_i64, c_i64, c_vp, c_vp]),
    "gmp_tp_edge_z_bwd_lmax_f32": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp,
                                           c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "gmp_edge_outer_sum_ex2_f32": (c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64,
                                           c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_size, c_vp]),
    "gmp_edge_outer_sum_ex_workspace_size": (c_size, [c_i64, c_i64, c_i64]),
    "gmp_edge_outer_sum_ex_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_int,
                                          c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_size, c_vp]),
    "gmp_edge_outer_sum_rect_workspace_size": (c_size, [c_i64, c_i64, c_i64]),
    "gmp_edge_xyz_dot_workspace_size": (c_size, [c_i64]),
    "gmp_edge_xyz_dot_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    "gmp_edge_outer_sum_rect_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            c_size, c_vp]),
    "gmp_tp_node_outer_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_tp_node_apply_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp, c_vp]),
    "gmp_tp_apply_set_x3": (c_int, [c_int]),
    "gmp_tp_split_w2_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_tp_gemm_x3_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp,
                                   c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_int, c_vp]),
    "gmp_tp_gemm_x3_widen_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64,
                                         c_vp, c_i64, c_vp]),
    "gmp_outer_sum_cols_workspace_size": (c_size, [c_i64, c_i64, c_i64]),
    "gmp_outer_sum_cols_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp,
                                       c_i64, c_vp, c_size, c_vp]),
    "gmp_gvp_layer_fwd_f32": (c_int, [c_i64, c_int] + [c_vp] * 10 + [c_vp]),
    "gmp_gvp_layer_bwd_f32": (c_int, [c_i64, c_int] + [c_vp] * 19 + [c_vp]),
    "gmp_gvp_layer_bwd_agg_f32": (c_int, [c_i64, c_i64, c_int, c_vp, c_vp, c_int] + [c_vp] * 19
                                  + [c_vp]),
    "gmp_gvp_layer_fwd_agg_f32": (c_int, [c_i64, c_i64, c_int] + [c_vp] * 13 + [c_vp]),
    "gmp_gvp_msg0_bwd_agg_f32": (c_int, [c_i64, c_i64] + [c_vp] * 30 + [c_vp]),
    "gmp_gvp_msg0_fwd_f32": (c_int, [c_i64] + [c_vp] * 15 + [c_vp]),
    "gmp_gvp_ff_fwd_f32": (c_int, [c_i64] + [c_vp] * 21 + [c_vp]),
    "gmp_egnn_node_bwd_partial_rows": (c_i64, [c_i64]),
    "gmp_egnn_node_bwd_f32": (c_int, [c_i64, c_i64, c_int, c_int] + [c_vp] * 13 + [c_vp]),
    "gmp_gvp_ff_bwd_f32": (c_int, [c_i64] + [c_vp] * 25 + [c_vp]),
    "gmp_gvp_edge_embed_fwd_f32": (c_int, [c_i64, c_i64, c_i64] + [c_vp] * 10 + [c_f32, c_vp,
                                                                                 c_vp, c_vp]),
    "gmp_gvp_edge_embed_bwd_workspace_size": (c_size, [c_i64]),
    "gmp_gvp_edge_embed_bwd_f32": (c_int, [c_i64, c_i64, c_i64] + [c_vp] * 10 + [c_f32, c_vp,
                                                                                 c_vp, c_vp, c_vp,
                                                                                 c_size, c_vp]),
    "gmp_gvp_msg0_bwd_f32": (c_int, [c_i64] + [c_vp] * 24 + [c_vp]),
    "gmp_radius_cells_f32": (c_int, [c_vp, c_vp, c_i64, c_vp, c_f32, c_vp, c_vp, c_vp]),
    "gmp_radius_count_f32": (c_int, [c_vp, c_vp, c_i64, c_f32, c_i64, c_vp, c_f32, c_vp, c_vp,
                                     c_vp, c_vp, c_vp, c_vp]),
    "gmp_radius_fill_f32": (c_int, [c_vp, c_vp, c_i64, c_f32, c_i64, c_vp, c_f32, c_vp, c_vp,
                                    c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_batch_collate": (c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "gmp_triplet_count": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_triplet_fill_f32": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64,
                                     c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_triplet_torsion_bwd_f32": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp,
                                            c_vp, c_vp, c_vp]),
    "gmp_ln_act_fwd_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_f32, c_int, c_vp, c_vp,
                                   c_vp, c_vp]),
    "gmp_ln_act_bwd_workspace_size": (c_size, [c_i64, c_i64]),
    "gmp_ln_act_bwd_partial_rows": (c_i64, [c_i64]),
    "gmp_vec_norm_fwd_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp]),
    "gmp_vec_norm_bwd_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "gmp_xyz_norm_fwd_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp]),
    "gmp_xyz_norm_bwd_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "gmp_sum_rows_f32": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp]),
    "gmp_ln_act_bwd_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp,
                                   c_vp, c_size, c_vp]),
    "gmp_sc_groups": (c_int, [c_i64]),
    "gmp_symmetric_contraction_fwd_f32": (c_int, [c_i64, c_int, c_int, c_int, c_int, c_vp, c_vp,
                                                  c_vp, c_vp, c_vp]),
    "gmp_symmetric_contraction_bwd_f32": (c_int, [c_i64, c_int, c_int, c_int, c_int, c_vp, c_vp,
                                                  c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_egnn_node_image_bytes": (c_size, [c_i64]),
    "gmp_egnn_node_image_f32": (c_int, [c_i64, c_i64, ctypes.POINTER(GmpEgnnNodeParams), c_vp,
                                        c_vp]),
    "gmp_egnn_node_fwd_f32": (c_int, [c_i64, c_i64, c_vp, c_vp, ctypes.POINTER(GmpEgnnNodeParams),
                                      c_vp, c_int, c_int, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "gmp_egnn_edge_bwd_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp,
                                      ctypes.POINTER(GmpEgnnParams), c_int, c_int, c_vp, c_int]
                              + [c_vp] * 11),
}

# include/gmp.h GMP_ABI_VERSION (6: r06 — K17 gmp_gvp_ff_{fwd,bwd}_f32, K15b gmp_egnn_node_bwd_f32;
# 5: r05 — K7s / K7f, the row GEMM and the A/B setters removed;
# 4: r05 — gmp_egnn_node_fwd_f32;
# 3: r04 — K8 dim / A4 arguments; 2: r04 — EGNN save_planes
# arguments, the x_hat mode global and gmp_egnn_edge_bwd_ab_f32 removed)
ABI_VERSION = 6
_lib = None
TORCH_LIB_PATH = os.environ.get("GMP_TORCH_LIB", os.path.join(_HERE, "libgmp_torch.so"))
_torch_ops = None


class GmpError(RuntimeError):
    pass


def torch_ops():
    """torch.ops.gmp: the TORCH_LIBRARY(gmp) registration of the C ABI (csrc/torch/gmp_torch.cpp,
    libgmp_torch.so next to libgmp.so; the drop-in boundary of SURVEY §8(b), the same kind as
    torch_scatter's torch.ops.torch_scatter.*).  Raises if the library is missing."""
    global _torch_ops
    if _torch_ops is None:
        load()  # libgmp.so first: libgmp_torch.so binds to the already-loaded soname
        if not os.path.exists(TORCH_LIB_PATH):
            raise GmpError(f"libgmp_torch.so not found at {TORCH_LIB_PATH}: build it first "
                           "(python -c 'import __graft_entry__ as g; g.build()')")
        torch.ops.load_library(TORCH_LIB_PATH)
        _torch_ops = torch.ops.gmp
    return _torch_ops


def load(path=None):
    """Load libgmp.so and declare every C-ABI signature. Raises if anything is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise GmpError(f"libgmp.so not found at {p}: build it first "
                       "(python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the symbol is not exported
        fn.restype = res
        fn.argtypes = args
    if lib.gmp_abi_version() != ABI_VERSION:
        raise GmpError("libgmp ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def check(rc, what):
    if rc != GMP_OK:
        lib = load()
        msg = lib.gmp_error_string(rc).decode()
        hip = lib.gmp_last_hip_error() if rc == GMP_ERR_HIP else 0
        raise GmpError(f"{what} failed: {msg} (code {rc}, hip error {hip})")
