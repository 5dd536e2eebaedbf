"""PyG `Batch.from_data_list` on CPU (TEST INFRASTRUCTURE; see oracle/__init__.py) — SURVEY.md
§8(f) f2, as the reference's loaders produce batches (experiments/utils/train_utils.py:28,132;
PyG 2.3.1 collate, an external dependency restated from its documented behaviour): node-level
tensors concatenated, edge_index of graph g offset by the number of nodes in graphs < g,
`batch[a]` = graph of node a, `ptr` = node prefix sums.  Plain Python loop over graphs."""
import torch


def collate(graphs, fields=("atoms", "y")):
    pos, ei, bv, ptr, off = [], [], [], [0], 0
    extra = {f: [] for f in fields}
    for g, d in enumerate(graphs):
        n = d.pos.shape[0]
        pos.append(d.pos)
        ei.append(d.edge_index + off)
        bv.append(torch.full((n,), g, dtype=torch.long))
        off += n
        ptr.append(off)
        for f in fields:
            v = getattr(d, f, None)
            if v is not None:
                extra[f].append(v.reshape((-1,) + tuple(v.shape[1:])) if v.dim() else v[None])
    out = {
        "pos": torch.cat(pos) if pos else torch.zeros(0, 3),
        "edge_index": torch.cat(ei, 1) if ei else torch.zeros(2, 0, dtype=torch.long),
        "batch": torch.cat(bv) if bv else torch.zeros(0, dtype=torch.long),
        "ptr": torch.tensor(ptr, dtype=torch.long),
    }
    for f, parts in extra.items():
        if parts and len(parts) == len(graphs):
            out[f] = torch.cat(parts)
    return out
