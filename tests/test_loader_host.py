"""Host half of the batching pipeline (gmp_amd.loader.GraphCollator.stage):
the packed arrays and prefix sums it hands to K10 match PyG collation (oracle/batch.py)."""
import torch

from oracle.batch import collate


class G:
    def __init__(self, n, e, seed, y=True):
        g = torch.Generator().manual_seed(seed)
        self.pos = torch.randn(n, 3, generator=g)
        self.edge_index = torch.randint(0, max(n, 1), (2, e), generator=g)
        self.atoms = torch.randint(0, 5, (n,), generator=g)
        if y:
            self.y = torch.randn(1, generator=g)


def _graphs():
    return [G(5, 12, 0), G(0, 0, 1), G(17, 40, 2), G(1, 0, 3), G(9, 30, 4)]


def test_stage_packs_like_pyg():
    from gmp_amd.loader import GraphCollator
    gs = _graphs()
    st = GraphCollator("cpu").stage(gs)
    ref = collate(gs)
    h = st.host
    assert st.num_graphs == 5 and st.num_nodes == 32 and st.num_edges == 82
    assert torch.equal(h["ptrs"][0], ref["ptr"])
    assert torch.equal(h["ptrs"][1], torch.tensor([0, 12, 12, 52, 52, 82]))
    assert torch.equal(h["pos"], ref["pos"])
    assert torch.equal(h["atoms"], ref["atoms"])
    assert torch.equal(h["y"], ref["y"])
    # edge_index stays graph-local on the host; K10 adds node_ptr[graph] on the device
    local = torch.cat([g.edge_index for g in gs], 1)
    assert torch.equal(h["edge_index"], local)


def test_stage_reuses_slots():
    from gmp_amd.loader import GraphCollator
    col = GraphCollator("cpu", depth=2)
    a = col.stage(_graphs())
    b = col.stage(_graphs()[:2])
    c = col.stage(_graphs())
    assert a.slot == c.slot != b.slot
    assert c.host["pos"].data_ptr() == a.host["pos"].data_ptr()  # buffer reused, not regrown
