"""Generate golden input/output vectors by running the REFERENCE's own layer code
(/root/reference, loaded by path with plumbing stubs, see _ref_stubs.py) on small seeded inputs.

Run in the dev container only (the reference does not exist on the GPU box):
    python tests/golden/make_golden.py
Writes tests/golden/*.pt (plain dicts of tensors; load with torch.load(weights_only=True)).

Modules exercised (all pure-torch arithmetic in the reference):
  models/layers/egnn_layer.py   EGNNLayer (7-89)
  models/egnn.py                EGNNModel (66-87)
  models/mace_modules/radial.py BesselBasis (12-52), PolynomialCutoff (55-81)
  models/mace_modules/blocks.py RadialEmbeddingBlock (84-96)
  models/layers/gvp_layer.py    GVP / GVPConv / GVPConvLayer (101-438)
  models/gvpgnn.py              GVPGNNModel (103-127)
  models/layers/spherenet_layer.py xyz_to_dat (496-564)   [`python make_golden.py triplets`]
  models/mace_modules/{cg,symmetric_contraction}.py at correlation 4 and max_ell 3
                                                         [`python make_golden.py mace_widening`]
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _ref_stubs  # noqa: E402

REF = os.environ.get("REFERENCE_ROOT", "/root/reference")


def radius_graph_np(pos, r):
    """All ordered pairs a != b with |pos_a - pos_b| < r; every node gets >= 1 in-edge
    (nearest neighbour added both ways) so that max(index)+1 == N (egnn_layer.py:77)."""
    n = pos.shape[0]
    d = np.linalg.norm(pos[:, None, :] - pos[None, :, :], axis=-1)
    np.fill_diagonal(d, np.inf)
    src, dst = np.nonzero(d < r)
    pairs = set(zip(src.tolist(), dst.tolist()))
    nn = np.argmin(d, axis=1)
    for a in range(n):
        pairs.add((a, int(nn[a])))
        pairs.add((int(nn[a]), a))
    e = np.array(sorted(pairs), dtype=np.int64).T
    return e


def make_graph(seed, n, box, r, shuffle=True):
    rng = np.random.default_rng(seed)
    pos = rng.uniform(0, box, size=(n, 3)).astype(np.float32)
    ei = radius_graph_np(pos.astype(np.float64), r)
    if shuffle:
        perm = rng.permutation(ei.shape[1])
        ei = ei[:, perm]
    return torch.from_numpy(pos), torch.from_numpy(np.ascontiguousarray(ei))


def batch_graphs(graphs):
    pos, ei, batch, off = [], [], [], 0
    for b, (p, e) in enumerate(graphs):
        pos.append(p)
        ei.append(e + off)
        batch.append(torch.full((p.shape[0],), b, dtype=torch.long))
        off += p.shape[0]
    return torch.cat(pos), torch.cat(ei, 1), torch.cat(batch)


def perturb_params(module, seed, scale=0.1):
    """Make LayerNorm affine params / biases non-trivial so their grads are exercised."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            if p.dim() == 1 and p.numel() > 0:
                p.add_(scale * torch.randn(p.shape, generator=g))


def grads_dict(module):
    return {f"grad.{k}": (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p))
            for k, p in module.named_parameters() if p.numel() > 0}


class Batch:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def create_kchains(k):
    """Restatement of experiments/kchains.ipynb:71 create_kchains (C1 input), batched."""
    graphs = []
    for sign in (-1, 1):
        pos = torch.tensor([[4.0 * sign, -3.0, 0.0]] + [[0.0, 5.0 * i, 0.0] for i in range(k)]
                           + [[4.0, 5.0 * (k - 1) + 3.0, 0.0]])
        pos = pos - pos.mean(0)
        a = torch.arange(k + 1)
        ei = torch.stack([a, a + 1])
        ei = torch.cat([ei, ei.flip(0)], 1)  # to_undirected
        order = torch.argsort(ei[0] * (k + 2) + ei[1])  # PyG to_undirected sorts by (row, col)
        graphs.append((pos, ei[:, order]))
    return graphs


def make_triplets(mods):
    """Reference xyz_to_dat (spherenet_layer.py:496-564) with and without torsion on seeded
    random radius graphs (one with self loops), a batched pair and the k-chains."""
    import warnings
    sp = mods["models.layers.spherenet_layer"]
    d = {}
    cases = []
    for seed, n, box, r in [(30, 40, 4.0, 1.6), (31, 64, 5.0, 1.8), (32, 25, 3.0, 1.5)]:
        cases.append(make_graph(seed, n, box, r))
    p, e, _ = batch_graphs([make_graph(33, 30, 4.0, 1.7), make_graph(34, 22, 3.5, 1.7)])
    cases.append((p, e))
    p, e, _ = batch_graphs(create_kchains(4))
    cases.append((p.float(), e))
    # self loops (dist 0: NaN torsion candidates, which torch_scatter's min never takes)
    p, e = make_graph(35, 20, 3.0, 1.6)
    loops = torch.arange(0, 20, 4)
    cases.append((p, torch.cat([e, torch.stack([loops, loops])], 1)))
    for c, (pos, ei) in enumerate(cases):
        n = pos.shape[0]
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            full = sp.xyz_to_dat(pos, ei, n, use_torsion=True)
            short = sp.xyz_to_dat(pos, ei, n, use_torsion=False)
        d[f"{c}.pos"], d[f"{c}.edge_index"] = pos, ei
        for name, v in zip(["dist", "angle", "torsion", "i", "j", "idx_kj", "idx_ji"], full):
            d[f"{c}.{name}"] = v
        for name, v in zip(["dist", "angle", "i", "j", "idx_kj", "idx_ji"], short):
            assert torch.equal(v, d[f"{c}.{name}"])
    d["n_cases"] = torch.tensor(len(cases))
    torch.save(d, os.path.join(HERE, "triplets.pt"))
    return "triplets.pt"


def make_mace_widening():
    """Symmetric contractions beyond config C4 (r04 widening), reference cg.py +
    symmetric_contraction.py: correlation 4 (cg.py's natural-parity coupling filter) on
    0e+1o+2e and correlation 3 at max_ell 3 (0e+1o+2e+3o)."""
    mm = _ref_stubs.load_mace_contraction(REF)
    o3l = sys.modules["e3nn.o3"]
    out = []
    cases = [("mace_symmetric_contraction_c4.pt", "4x0e+4x1o+4x2e", 4, 21),
             ("mace_symmetric_contraction_l3.pt", "4x0e+4x1o+4x2e+4x3o", 3, 22),
             # r05: both parities (incompleteness.ipynb:530-538's irreps; correlation 3 -- at 4
             # the reference raises, recorded below), max_ell 5 at correlation 2
             # (rotsym.ipynb:247-257), correlation 4 at max_ell 3
             ("mace_symmetric_contraction_bp3.pt", "4x0e+4x0o+4x1e+4x1o+4x2e+4x2o", 3, 23),
             ("mace_symmetric_contraction_l5.pt", "4x0e+4x1o+4x2e+4x3o+4x4e+4x5o", 2, 24),
             ("mace_symmetric_contraction_l3c4.pt", "2x0e+2x1o+2x2e+2x3o", 4, 25)]
    if os.environ.get("GOLDEN_CASES"):
        keep = set(os.environ["GOLDEN_CASES"].split(","))
        cases = [c for c in cases if c[0] in keep]
    for name, irr, corr, seed in cases:
        torch.manual_seed(seed)
        irreps = o3l.Irreps(irr)
        SC = mm["models.mace_modules.symmetric_contraction"].SymmetricContraction(
            irreps_in=irreps, irreps_out=irreps, correlation=corr, element_dependent=False,
            num_elements=1)
        D = sum(2 * ir.l + 1 for _, ir in irreps)
        C = int(irr.split("x")[0])
        x = torch.randn(23, C, D, requires_grad=True)
        y = SC(x, None)
        gy = torch.randn_like(y)
        (y * gy).sum().backward()
        d = {"x": x.detach(), "out": y.detach(), "g_out": gy, "grad_x": x.grad}
        # weights only: the U_matrix buffers (up to 9^4 x 9 x K floats) are rebuilt by the
        # module under test, and the outputs pin them
        d.update({f"param.{k}": v.detach().clone() for k, v in SC.state_dict().items()
                  if "U_matrix" not in k})
        d.update(grads_dict(SC))
        torch.save(d, os.path.join(HERE, name))
        out.append(name)
    # the incompleteness notebook's MACE line (correlation 4 on both parities): the reference's
    # U_matrix_real has no coupling path to 0o under its natural-parity filter and raises
    irreps = o3l.Irreps("4x0e+4x0o+4x1e+4x1o+4x2e+4x2o")
    try:
        mm["models.mace_modules.symmetric_contraction"].SymmetricContraction(
            irreps_in=irreps, irreps_out=irreps, correlation=4, element_dependent=False,
            num_elements=1)
        rec = {"raised": None}
    except Exception as e:  # noqa: BLE001 - the reference's own failure is the fixture
        rec = {"raised": type(e).__name__, "message": str(e)}
    rec.update(irreps=str(irreps), correlation=4)
    import json
    with open(os.path.join(HERE, "mace_symmetric_contraction_bp4_error.json"), "w") as fh:
        json.dump(rec, fh, indent=1)
    out.append("mace_symmetric_contraction_bp4_error.json")
    return out


def main(only=None):
    if only == "mace_widening":
        for f in make_mace_widening():
            print(f, os.path.getsize(os.path.join(HERE, f)))
        return
    mods = _ref_stubs.load_reference(REF)
    if only == "triplets":
        f = make_triplets(mods)
        print(f, os.path.getsize(os.path.join(HERE, f)))
        return
    torch.set_default_dtype(torch.float32)
    out_files = []

    # ---------------------------------------------------------------- EGNN layer, d=128
    torch.manual_seed(0)
    pos, ei = make_graph(1, 48, 6.0, 2.2)
    layer = mods["models.layers.egnn_layer"].EGNNLayer(128, "relu", "layer", "sum")
    perturb_params(layer, 1)
    h = torch.randn(48, 128, requires_grad=True)
    p = pos.clone().requires_grad_(True)
    h_out, p_out = layer(h, p, ei)
    gh = torch.randn_like(h_out)
    gp = torch.randn_like(p_out)
    (h_out * gh).sum().add_((p_out * gp).sum()).backward()
    d = {"h": h.detach(), "pos": pos, "edge_index": ei, "g_h": gh, "g_pos": gp,
         "out_h": h_out.detach(), "out_pos": p_out.detach(), "grad_h": h.grad, "grad_pos": p.grad}
    d.update({f"param.{k}": v.detach().clone() for k, v in layer.state_dict().items()})
    d.update(grads_dict(layer))
    torch.save(d, os.path.join(HERE, "egnn_layer_d128.pt"))
    out_files.append("egnn_layer_d128.pt")

    # ---------------------------------------------------------------- EGNN model, 3 layers, d=32, B=2
    torch.manual_seed(2)
    pos, ei, batch = batch_graphs([make_graph(3, 40, 5.0, 2.0), make_graph(4, 33, 5.0, 2.0)])
    atoms = torch.randint(0, 3, (pos.shape[0],))
    model = mods["models.egnn"].EGNNModel(num_layers=3, emb_dim=32, in_dim=3, out_dim=2)
    perturb_params(model, 5)
    p = pos.clone().requires_grad_(True)
    y = model(Batch(atoms=atoms, pos=p, edge_index=ei, batch=batch))
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    d = {"atoms": atoms, "pos": pos, "edge_index": ei, "batch": batch, "g_out": gy,
         "out": y.detach(), "grad_pos": p.grad}
    d.update({f"param.{k}": v.detach().clone() for k, v in model.state_dict().items()})
    d.update(grads_dict(model))
    torch.save(d, os.path.join(HERE, "egnn_model_d32.pt"))
    out_files.append("egnn_model_d32.pt")

    # ---------------------------------------------------------------- EGNN model on k-chains (C1 input)
    torch.manual_seed(6)
    pos, ei, batch = batch_graphs(create_kchains(4))
    atoms = torch.zeros(pos.shape[0], dtype=torch.long)
    model = mods["models.egnn"].EGNNModel(num_layers=4, emb_dim=16, in_dim=1, out_dim=2)
    perturb_params(model, 7)
    y = model(Batch(atoms=atoms, pos=pos, edge_index=ei, batch=batch))
    (y.sum()).backward()
    d = {"atoms": atoms, "pos": pos, "edge_index": ei, "batch": batch, "out": y.detach()}
    d.update({f"param.{k}": v.detach().clone() for k, v in model.state_dict().items()})
    d.update(grads_dict(model))
    torch.save(d, os.path.join(HERE, "egnn_kchains.pt"))
    out_files.append("egnn_kchains.pt")

    # ---------------------------------------------------------------- radial basis (a2-a4)
    rad = mods["models.mace_modules.blocks"].RadialEmbeddingBlock(r_max=10.0, num_bessel=8,
                                                                  num_polynomial_cutoff=5)
    lengths = torch.cat([torch.tensor([1e-3, 0.05, 0.5, 1.0, 2.5, 5.0, 7.5, 9.0, 9.5, 9.9, 9.99,
                                       9.999, 10.0, 10.5, 12.0]),
                         torch.rand(200, generator=torch.Generator().manual_seed(8)) * 11.0 + 0.01])
    lengths = lengths.unsqueeze(-1).requires_grad_(True)
    bessel = rad.bessel_fn(lengths)
    cutoff = rad.cutoff_fn(lengths)
    emb = rad(lengths)
    g = torch.randn_like(emb)
    (emb * g).sum().backward()
    torch.save({"lengths": lengths.detach(), "bessel": bessel.detach(), "cutoff": cutoff.detach(),
                "emb": emb.detach(), "g_emb": g, "grad_lengths": lengths.grad},
               os.path.join(HERE, "radial.pt"))
    out_files.append("radial.pt")

    # ---------------------------------------------------------------- GVP conv layer (eval: no dropout)
    gvp = mods["models.layers.gvp_layer"]
    torch.manual_seed(9)
    pos, ei = make_graph(10, 40, 5.0, 2.0)
    n, e = pos.shape[0], ei.shape[1]
    layer = gvp.GVPConvLayer((32, 4), (8, 1), activations=(torch.nn.functional.relu, None),
                             vector_gate=True)
    perturb_params(layer, 11)
    layer.eval()
    s = torch.randn(n, 32, requires_grad=True)
    v = torch.randn(n, 4, 3, requires_grad=True)
    es = torch.randn(e, 8, requires_grad=True)
    ev = torch.randn(e, 1, 3, requires_grad=True)
    so, vo = layer((s, v), ei, (es, ev))
    gs, gv = torch.randn_like(so), torch.randn_like(vo)
    ((so * gs).sum() + (vo * gv).sum()).backward()
    d = {"s": s.detach(), "v": v.detach(), "es": es.detach(), "ev": ev.detach(), "edge_index": ei,
         "g_s": gs, "g_v": gv, "out_s": so.detach(), "out_v": vo.detach(), "grad_s": s.grad,
         "grad_v": v.grad, "grad_es": es.grad, "grad_ev": ev.grad}
    d.update({f"param.{k}": t.detach().clone() for k, t in layer.state_dict().items()})
    d.update(grads_dict(layer))
    torch.save(d, os.path.join(HERE, "gvp_layer.pt"))
    out_files.append("gvp_layer.pt")

    # ---------------------------------------------------------------- GVP-GNN model (eval)
    torch.manual_seed(12)
    pos, ei, batch = batch_graphs([make_graph(13, 30, 5.0, 2.0), make_graph(14, 26, 5.0, 2.0)])
    atoms = torch.randint(0, 2, (pos.shape[0],))
    model = mods["models.gvpgnn"].GVPGNNModel(num_layers=2, in_dim=2, out_dim=1, s_dim=32,
                                              v_dim=4, s_dim_edge=8, v_dim_edge=1)
    perturb_params(model, 15)
    model.eval()
    p = pos.clone().requires_grad_(True)
    y = model(Batch(atoms=atoms, pos=p, edge_index=ei, batch=batch))
    y.sum().backward()
    d = {"atoms": atoms, "pos": pos, "edge_index": ei, "batch": batch, "out": y.detach(),
         "grad_pos": p.grad}
    d.update({f"param.{k}": t.detach().clone() for k, t in model.state_dict().items()})
    d.update(grads_dict(model))
    torch.save(d, os.path.join(HERE, "gvp_model.pt"))
    out_files.append("gvp_model.pt")

    # ---------------------------------------------------------------- MACE symmetric contraction
    # (reference cg.py + symmetric_contraction.py on e3nn-lite; wigner_3j restated)
    mm = _ref_stubs.load_mace_contraction(REF)
    o3l = sys.modules["e3nn.o3"]
    torch.manual_seed(16)
    C = 16
    irreps = o3l.Irreps(f"{C}x0e+{C}x1o+{C}x2e")
    SC = mm["models.mace_modules.symmetric_contraction"].SymmetricContraction(
        irreps_in=irreps, irreps_out=irreps, correlation=3, element_dependent=False,
        num_elements=1)
    x = torch.randn(37, C, 9, requires_grad=True)
    y = SC(x, None)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    d = {"x": x.detach(), "out": y.detach(), "g_out": gy, "grad_x": x.grad}
    d.update({f"param.{k}": v.detach().clone() for k, v in SC.state_dict().items()})
    d.update(grads_dict(SC))
    torch.save(d, os.path.join(HERE, "mace_symmetric_contraction.pt"))
    out_files.append("mace_symmetric_contraction.pt")

    for f in out_files:
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
