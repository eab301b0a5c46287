"""graph_computation/transitive_closure.py entry logic."""
from __future__ import annotations

import torch

from dalgo.models.transitive_closure import DenseClosure, SparseClosure, compact_ids
from dalgo.parallel import runtime
from dalgo.utils.cli import common_parser, init_from_args

TOY_EDGES = [(1, 2), (1, 3), (2, 3), (3, 1)]   # transitive_closure.py:18


def main(argv=None):
    ap = common_parser("Linear transitive closure (MI355X-native)")
    ap.add_argument("--engine", choices=["auto", "dense", "sparse"], default="auto")
    ap.add_argument("--edges", default=None)
    ap.add_argument("--random", default=None, metavar="N,E", help="random graph with N vertices, E edges")
    a = ap.parse_args(argv)
    rt = init_from_args(a, "Transitive Closure")
    if a.random:
        n, e = (int(x) for x in a.random.split(","))
        g = torch.Generator().manual_seed(a.seed)
        src = torch.randint(0, n, (e,), generator=g)
        dst = torch.randint(0, n, (e,), generator=g)
    elif a.edges:
        from dalgo.apps.pagerank_app import load_edges
        src, dst = load_edges(a.edges)
    else:
        src = torch.tensor([x for x, _ in TOY_EDGES])
        dst = torch.tensor([y for _, y in TOY_EDGES])
    s, d, ids = compact_ids(src.long(), dst.long())
    n = len(ids)
    engine = a.engine if a.engine != "auto" else ("dense" if n <= 32768 else "sparse")
    if engine == "dense":
        tc = DenseClosure(s, d, n, rt.rank, rt.world_size, device=rt.device)
    else:
        tc = SparseClosure(s, d, rt.rank, rt.world_size, n=n, device=rt.device)
    res = tc.run()
    if not a.quiet:
        rt.log("path counts per round: %s" % res.counts)
    rt.log("The original graph has %i paths" % res.n_paths)   # transitive_closure.py:42 (sic)
    runtime.shutdown()
    return res
