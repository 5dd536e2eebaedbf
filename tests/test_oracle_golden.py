"""Pin the CPU oracle against golden vectors produced by the reference's own code
(tests/golden/make_golden.py). CPU-only."""
import pytest
import torch

from oracle import egnn as oegnn
from oracle import radial as orad

ATOL = 1e-5


def _load_params(module, d):
    sd = {k[len("param."):]: v for k, v in d.items() if k.startswith("param.")}
    module.load_state_dict(sd, strict=True)


def _check_grads(module, d, atol=ATOL, rtol=1e-4):
    for k, p in module.named_parameters():
        if p.numel() == 0:
            continue
        ref = d[f"grad.{k}"]
        got = p.grad if p.grad is not None else torch.zeros_like(p)
        torch.testing.assert_close(got, ref, atol=atol, rtol=rtol, msg=lambda m: f"{k}: {m}")


class B:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def test_egnn_layer_golden(golden):
    d = golden("egnn_layer_d128.pt")
    layer = oegnn.EGNNLayer(128, "relu", "layer", "sum")
    _load_params(layer, d)
    h = d["h"].clone().requires_grad_(True)
    p = d["pos"].clone().requires_grad_(True)
    ho, po = layer(h, p, d["edge_index"])
    torch.testing.assert_close(ho, d["out_h"], atol=ATOL, rtol=1e-5)
    torch.testing.assert_close(po, d["out_pos"], atol=ATOL, rtol=1e-5)
    ((ho * d["g_h"]).sum() + (po * d["g_pos"]).sum()).backward()
    torch.testing.assert_close(h.grad, d["grad_h"], atol=ATOL, rtol=1e-4)
    torch.testing.assert_close(p.grad, d["grad_pos"], atol=ATOL, rtol=1e-4)
    _check_grads(layer, d, atol=1e-4)


@pytest.mark.parametrize("name,kw", [
    ("egnn_model_d32.pt", dict(num_layers=3, emb_dim=32, in_dim=3, out_dim=2)),
    ("egnn_kchains.pt", dict(num_layers=4, emb_dim=16, in_dim=1, out_dim=2)),
])
def test_egnn_model_golden(golden, name, kw):
    d = golden(name)
    model = oegnn.EGNNModel(**kw)
    _load_params(model, d)
    p = d["pos"].clone().requires_grad_(True)
    y = model(B(atoms=d["atoms"], pos=p, edge_index=d["edge_index"], batch=d["batch"]))
    torch.testing.assert_close(y, d["out"], atol=ATOL, rtol=1e-5)
    g = d.get("g_out", torch.ones_like(y))
    (y * g).sum().backward()
    if "grad_pos" in d:
        torch.testing.assert_close(p.grad, d["grad_pos"], atol=1e-4, rtol=1e-4)
    _check_grads(model, d, atol=1e-4)


def test_radial_golden(golden):
    d = golden("radial.pt")
    rad = orad.RadialEmbeddingBlock(10.0, 8, 5)
    r = d["lengths"].clone().requires_grad_(True)
    torch.testing.assert_close(rad.bessel_fn(r), d["bessel"], atol=ATOL, rtol=1e-6)
    torch.testing.assert_close(rad.cutoff_fn(r), d["cutoff"], atol=ATOL, rtol=1e-6)
    e = rad(r)
    torch.testing.assert_close(e, d["emb"], atol=ATOL, rtol=1e-6)
    (e * d["g_emb"]).sum().backward()
    torch.testing.assert_close(r.grad, d["grad_lengths"], atol=1e-4, rtol=1e-5)


def test_gvp_layer_golden(golden):
    from oracle import gvp as ogvp
    d = golden("gvp_layer.pt")
    layer = ogvp.GVPConvLayer((32, 4), (8, 1), activations=(torch.nn.functional.relu, None),
                              vector_gate=True)
    _load_params(layer, d)
    layer.eval()  # the fixture was made in eval mode (no dropout)
    xs = [d[k].clone().requires_grad_(True) for k in ("s", "v", "es", "ev")]
    so, vo = layer((xs[0], xs[1]), d["edge_index"], (xs[2], xs[3]))
    torch.testing.assert_close(so, d["out_s"], atol=ATOL, rtol=1e-5)
    torch.testing.assert_close(vo, d["out_v"], atol=ATOL, rtol=1e-5)
    ((so * d["g_s"]).sum() + (vo * d["g_v"]).sum()).backward()
    for t, k in zip(xs, ("grad_s", "grad_v", "grad_es", "grad_ev")):
        torch.testing.assert_close(t.grad, d[k], atol=1e-4, rtol=1e-4)
    _check_grads(layer, d, atol=1e-4)


def test_gvp_model_golden(golden):
    from oracle import gvp as ogvp
    d = golden("gvp_model.pt")
    model = ogvp.GVPGNNModel(num_layers=2, in_dim=2, out_dim=1, s_dim=32, v_dim=4, s_dim_edge=8,
                             v_dim_edge=1)
    _load_params(model, d)
    model.eval()
    p = d["pos"].clone().requires_grad_(True)
    y = model(B(atoms=d["atoms"], pos=p, edge_index=d["edge_index"], batch=d["batch"]))
    torch.testing.assert_close(y, d["out"], atol=ATOL, rtol=1e-5)
    y.sum().backward()
    torch.testing.assert_close(p.grad, d["grad_pos"], atol=1e-4, rtol=1e-4)
    _check_grads(model, d, atol=1e-4)
