"""PageRank multi-GPU partition statistics, computed in ONE process for W = 2, 4, 8
(no multi-GPU box needed): per-rank in-edge counts (load balance of the destination
partition) and per-iteration exchange volume of the ghost exchange against the full
all_gather, on the R-MAT graph of bench/pagerank_bench.py (default scale 26, 1.07B edges).
Both relabelings are reported: the round-1 contiguous degree order and the dealt one."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--worlds", default="2,4,8")
    a = ap.parse_args()
    from dalgo.apps.pagerank_app import deal_ids
    from dalgo.ops import graph as G
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    n = 1 << a.scale
    E = a.edge_factor * n
    chunk = 1 << 26
    deg = torch.zeros(n, dtype=torch.int64, device=dev)
    for off in range(0, E, chunk):
        s, _ = G.rmat_edges(min(chunk, E - off), a.scale, seed=2, e_off=off, device=dev)
        deg += torch.bincount(s.long(), minlength=n)
    order = torch.argsort(-deg * n - torch.arange(n, device=dev, dtype=torch.int64))
    out = {"scale": a.scale, "edges": E, "vertices": n,
           "vertices_with_out_edges": int((deg > 0).sum())}
    for W in (int(x) for x in a.worlds.split(",")):
        sl = G.vertex_slices(n, W)
        for name in ("contiguous", "dealt"):
            if name == "contiguous":
                nid = torch.empty_like(order)
                nid[order] = torch.arange(n, device=dev, dtype=torch.int64)
            else:
                nid = deal_ids(order, n, W)
            edges = torch.zeros(W, dtype=torch.int64, device=dev)
            need = [torch.zeros(n, dtype=torch.bool, device=dev) for _ in range(W)]
            for off in range(0, E, chunk):
                s, d = G.rmat_edges(min(chunk, E - off), a.scale, seed=2, e_off=off, device=dev)
                s = nid[s.long()]
                r = nid[d.long()] // sl
                edges += torch.bincount(r, minlength=W)
                for q in range(W):
                    need[q][s[r == q]] = True
            ghosts = []
            for q in range(W):
                lo, hi = q * sl, min(n, (q + 1) * sl)
                need[q][lo:hi] = False
                ghosts.append(int(need[q].sum()))
            del need
            e = edges.double()
            out[f"W{W}_{name}"] = {
                "max_over_mean_edges": float(e.max() / e.mean()),
                "ghost_floats_per_rank_mean": sum(ghosts) / W,
                "allgather_floats_per_rank": (W - 1) * sl,
                "ghost_over_allgather": sum(ghosts) / W / ((W - 1) * sl),
            }
            print(json.dumps({f"W{W}_{name}": out[f"W{W}_{name}"]}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
