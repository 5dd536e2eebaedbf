"""GPU batching pipeline (K10 gmp_batch_collate + pinned async H2D) against
PyG collation restated in oracle/batch.py: edge_index, batch and ptr bit-exact."""
import pytest
import torch

from oracle.batch import collate

pytestmark = pytest.mark.gpu


class G:
    def __init__(self, n, e, seed):
        g = torch.Generator().manual_seed(seed)
        self.pos = torch.randn(n, 3, generator=g)
        self.edge_index = torch.randint(0, max(n, 1), (2, e), generator=g)
        self.atoms = torch.randint(0, 5, (n,), generator=g)
        self.y = torch.randn(1, generator=g)


def _check(b, gs):
    ref = collate(gs)
    assert torch.equal(b.edge_index.cpu(), ref["edge_index"])
    assert torch.equal(b.batch.cpu(), ref["batch"])
    assert torch.equal(b.ptr.cpu(), ref["ptr"])
    assert torch.equal(b.pos.cpu(), ref["pos"])
    assert torch.equal(b.atoms.cpu(), ref["atoms"])
    assert torch.equal(b.y.cpu(), ref["y"])
    assert b.num_graphs == len(gs)


@pytest.mark.parametrize("sizes", [[(5, 12)], [(5, 12), (0, 0), (17, 40), (1, 0), (9, 30)],
                                   [(300, 4000)] * 64, [(20_000, 400_000)] * 3])
def test_collate_matches_pyg(sizes):
    from gmp_amd.loader import GraphCollator, check_batch
    gs = [G(n, e, i) for i, (n, e) in enumerate(sizes)]
    b = GraphCollator()(gs)
    check_batch(b)
    _check(b, gs)


def test_collate_range_flag():
    from gmp_amd.loader import GraphCollator, check_batch
    gs = [G(5, 10, 0), G(4, 8, 1)]
    gs[1].edge_index[0, 3] = 4  # == n_g: out of range for graph 1
    with pytest.raises(IndexError):
        check_batch(GraphCollator()(gs))


def test_prefetcher_order_and_values():
    from gmp_amd.loader import Prefetcher
    batches = [[G(50 + 7 * k + j, 300 + k, 10 * k + j) for j in range(4)] for k in range(7)]
    seen = 0
    acc = torch.zeros((), device="cuda")
    for k, b in enumerate(Prefetcher(batches, depth=2)):
        acc += b.pos.sum()  # consume on the current stream while the next copy is in flight
        _check(b, batches[k])
        seen += 1
    assert seen == 7
