#!/usr/bin/env python3
"""Per-rank share of the SHARDED PageRank build (BASELINE config #5 at W ranks), measured on
one MI355X: what rank r of W computes between the collectives of
dalgo.apps.pagerank_app.build_rmat_sharded --

  degree count of its E / W input edges (with the source partition) | [all_reduce of the
  degrees] | ranking + dealing | relabel + group by destination owner | [all_to_all] |
  native build over received edges

The collectives are left out (their inputs / outputs are computed untimed from the whole
stream, exactly what they would deliver) and reported as bytes per rank. Timed with HIP
events around each phase, best of --reps. Prints one JSON line."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="0,7")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--spmv-iters", type=int, default=0,
                    help="also time K4b (pb_spmv) over the rank's native layout, random c")
    ap.add_argument("--direct", action="store_true",
                    help="the direct shuffle (owner partition with random new_id gathers) instead "
                         "of build_rmat_sharded's source-bucketed path")
    a = ap.parse_args()
    from dalgo.apps.jobs import reserve_pool
    from dalgo.apps.pagerank_app import degree_new_id, edge_range, rmat_input
    from dalgo.ops import graph as G
    dev = torch.device("cuda")
    reserve_pool(dev, 120.0)
    N, W = 1 << a.scale, a.world
    E = a.edge_factor * N
    full, _ = rmat_input(a.scale, a.edge_factor, dev, 1)
    # what the degree all-reduce delivers: the whole stream's degrees
    deg_all = torch.zeros(N, dtype=torch.int32, device=dev)
    G.degree_sorted_(deg_all, torch.cat([s for s, _ in full]), a.scale)
    new_id = degree_new_id(deg_all, N, W)
    sl = G.vertex_slices(N, W)
    res = {"scale": a.scale, "world": W, "edges": E, "shuffle": "direct" if a.direct else "bucketed", "ranks": {}}
    for r in [int(x) for x in a.ranks.split(",")]:
        lo, hi = edge_range(E, r, W)
        s_own, d_own = G.rmat_edges(hi - lo, a.scale, seed=1, e_off=lo, device=dev)
        # what the all_to_all delivers to rank r: every input edge whose relabelled
        # destination r owns (built from the whole stream, untimed)
        recv = []
        for s, d in full:
            dn = new_id[d.long()]
            k = (dn >= r * sl) & (dn < min(N, (r + 1) * sl))
            recv.append(((new_id[s.long()][k].long() << 32) | dn[k].long()))
        recv = torch.cat(recv)
        rs, rd = G.unpack_edges(recv)
        del recv
        best = None
        for rep in range(a.reps + 1):                 # rep 0: warm-up
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
            torch.cuda.synchronize()
            ev[0].record()
            if a.direct:   # degree sort of the sources; relabel by random gathers
                deg = torch.zeros(N, dtype=torch.int32, device=dev)
                G.degree_sorted_(deg, s_own, a.scale)
                ev[1].record()
                nid = degree_new_id(deg_all, N, W)
                ev[2].record()
                packed, send = G.owner_partition(s_own, d_own, nid, N, W)
            else:          # build_rmat_sharded's bucketed path
                packed, deg = G.partition_edges([(s_own, d_own)], a.scale)
                ev[1].record()
                nid = degree_new_id(deg_all, N, W)
                ev[2].record()
                packed = G.relabel_partition_dst(packed, nid, a.scale)
                packed, send = G.owner_partition_packed(packed, nid, N, W)
            ev[3].record()
            G.build_marks = []
            G._mark("start")
            ng = G.build_native([(rs, rd)], N, r, W, None)
            ev[4].record()
            torch.cuda.synchronize()
            t = [ev[i].elapsed_time(ev[i + 1]) for i in range(4)]
            tot = sum(t)
            if rep > 0 and (best is None or tot < best["total_ms"]):
                best = {"total_ms": tot, "degree_count_ms": t[0], "rank_deal_ms": t[1],
                        "relabel_owner_partition_ms": t[2], "build_received_ms": t[3],
                        "input_edges": hi - lo, "received_edges": int(rs.numel()),
                        "edges_dedup": ng.n_edges, "ghosts": ng.n_ghost,
                        "all_to_all_send_bytes": 8 * (sum(send) - send[r]),
                        "degree_all_reduce_bytes": 4 * N,
                        "build_phases_ms": G.build_phase_spans()}
            G.build_marks = None
            if a.spmv_iters and rep == a.reps and best is not None:
                # K4b over this rank's layout (own slice + ghosts), random contributions
                lay = ng.layout
                c = torch.rand(ng.slice_size + ng.n_ghost, device=dev)
                acc = torch.empty(ng.n_local, device=dev)
                pres = torch.empty(ng.n_local, dtype=torch.int32, device=dev)
                for _ in range(3):
                    G.pb_spmv(lay, c, acc, pres)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.spmv_iters):
                    G.pb_spmv(lay, c, acc, pres)
                e1.record()
                torch.cuda.synchronize()
                best["k4b_ms_per_iter"] = e0.elapsed_time(e1) / a.spmv_iters
                best["k4b_work_items"] = int(lay.wi_bin.numel())
                best["k4b_split_bins"] = int(lay.split_bin.numel())
                del lay, c, acc, pres
            del packed, ng, deg, nid
        res["ranks"][r] = best
        print(f"rank {r}/{W}: {best}", file=sys.stderr, flush=True)
        del s_own, d_own, rs, rd
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
