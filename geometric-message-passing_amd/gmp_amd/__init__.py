"""gmp_amd — MI355X-native geometric message-passing hot path (drop-in for the reference's
PyG MessagePassing / torch_scatter / EGNN / TFN / MACE layer APIs).

Native code: libgmp.so (HIP, gfx950) behind the C ABI in include/gmp.h, registered as PyTorch
operators torch.ops.gmp.* by libgmp_torch.so (TORCH_LIBRARY(gmp), csrc/torch/gmp_torch.cpp).
"""
from . import _lib, ops  # noqa: F401
from .scatter import (scatter, scatter_sum, scatter_add, scatter_mean, scatter_max,  # noqa: F401
                      scatter_min, global_add_pool, global_mean_pool)
from .message_passing import MessagePassing  # noqa: F401
from .egnn import EGNNLayer, EGNNModel  # noqa: F401
from .graph import Batch, collate, radius_graph, create_kchains  # noqa: F401
from .equivariant import (TensorProductConvLayer, MACEModel, TFNModel,  # noqa: F401
                          RadialEmbeddingBlock, EquivariantProductBasisBlock,
                          SymmetricContraction, first_node_pooling)
from .gvp import GVP, GVPConv, GVPConvLayer, GVPGNNModel  # noqa: F401
from .schnet import SchNetModel, CFConv, InteractionBlock  # noqa: F401

__all__ = ["scatter", "scatter_sum", "scatter_add", "scatter_mean", "scatter_max", "scatter_min",
           "global_add_pool", "global_mean_pool", "MessagePassing", "EGNNLayer", "EGNNModel",
           "Batch", "collate", "radius_graph", "create_kchains", "TensorProductConvLayer",
           "MACEModel", "TFNModel", "RadialEmbeddingBlock", "EquivariantProductBasisBlock",
           "SymmetricContraction", "first_node_pooling", "GVP", "GVPConv", "GVPConvLayer",
           "GVPGNNModel", "SchNetModel", "CFConv", "InteractionBlock"]
