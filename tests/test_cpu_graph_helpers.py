"""CPU checks of the PageRank build's host-side helpers (dalgo/ops/graph.py,
dalgo/apps/pagerank_app.py): the owner partition of source-relabelled packed edges, the
degree relabeling's dealing, the radix / run-sort bit split and the phase-2 work items.
Reference: graph_computation/pagerank.py:41 (distinct().groupByKey() over the edges)."""
import numpy as np
import pytest
import torch

from dalgo.apps.pagerank_app import deal_ids, degree_new_id, rank_by_degree
from dalgo.ops import graph as G


def _edges(n_vertices, n_edges, seed):
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(0, n_vertices, (n_edges,), generator=g, dtype=torch.int64)
    dst = torch.randint(0, n_vertices, (n_edges,), generator=g, dtype=torch.int64)
    return src, dst


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_owner_partition_packed_matches_owner_partition(world):
    """Packed (new_src << 32 | raw dst) words through owner_partition_packed == the raw
    (src, dst) edges through owner_partition: the same per-owner counts and, per owner,
    the same multiset of relabelled edges (both relabel through the same new_id)."""
    n = 1000
    src, dst = _edges(n, 20_000, seed=world)
    new_id = torch.randperm(n, generator=torch.Generator().manual_seed(7))
    ref, cref = G.owner_partition(src, dst, new_id, n, world)
    packed = (new_id[src] << 32) | dst
    got, cgot = G.owner_partition_packed(packed, new_id, n, world)
    assert cgot == cref and sum(cgot) == src.numel()
    o = 0
    for c in cref:
        a = torch.sort(ref[o:o + c]).values
        b = torch.sort(got[o:o + c]).values
        assert torch.equal(a, b)
        o += c
    sl = G.vertex_slices(n, world)
    d = got & 0xFFFFFFFF
    owners = torch.repeat_interleave(torch.arange(world), torch.tensor(cgot))
    assert torch.equal(d // sl, owners)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_degree_new_id_cpu_is_dealt_bijection(world):
    """degree_new_id on the CPU == deal_ids(rank_by_degree): a bijection; on one rank the
    rank-j vertex gets id j; on W ranks slice r holds ranks r, 2W - 1 - r, ... (snake)."""
    n = 1 << 10
    g = torch.Generator().manual_seed(world)
    deg = torch.randint(0, 50, (n,), generator=g, dtype=torch.int32)
    deg[torch.randint(0, n, (8,), generator=g)] = 10_000          # hubs
    nid = degree_new_id(deg, n, world).long()
    assert torch.equal(torch.sort(nid).values, torch.arange(n))
    order = rank_by_degree(deg)
    assert torch.equal(nid, deal_ids(order, n, world).long())
    # descending degree, ties by descending id
    d = deg.long()[order]
    assert bool((d[:-1] >= d[1:]).all())
    tie = d[:-1] == d[1:]
    assert bool((order[:-1][tie] > order[1:][tie]).all())
    sl = G.vertex_slices(n, world)
    for j in range(min(n, 4 * world)):
        p, r = j // world, j % world
        slot = r if p % 2 == 0 else world - 1 - r
        assert int(nid[order[j]]) == slot * sl + p


def test_sort_split_bits():
    """Whole 8-bit radix passes above the run sort's low bits (<= SRC_BITS of them)."""
    assert G.sort_split_bits(52) == 12            # scale 26: bits 12..51, 5 passes
    assert G.sort_split_bits(G.SRC_BITS) == 0
    for nbits in range(G.SRC_BITS + 1, 64):
        lo = G.sort_split_bits(nbits)
        assert 0 <= lo <= G.SRC_BITS and (nbits - lo) % 8 == 0


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_work_items_cover_every_bin(seed):
    """Phase-2 work items: per bin a contiguous cover of its bin-major entry range (one
    empty item for an empty bin), a split bin's pieces with consecutive slabs, the split
    tables consistent with the items."""
    rng = np.random.default_rng(seed)
    nb = 200
    cnt = rng.integers(0, 50, nb)
    cnt[rng.integers(0, nb, 6)] = rng.integers(2_000, 20_000, 6)     # hot bins
    cnt[:3] = 0
    bin_cnt = torch.tensor(cnt, dtype=torch.int64)
    bin_lo = torch.cumsum(bin_cnt, 0) - bin_cnt
    nent = int(bin_cnt.sum())
    (wb, wl, slab, sp_bin, sp_first, sp_cnt), nslab = G._work_items(bin_cnt, bin_lo, nent, 64, 256)
    wb, wl, slab = wb.tolist(), wl.tolist(), slab.tolist()
    assert wl[-1] == nent and len(wl) == len(wb) + 1
    assert wb == sorted(wb) and set(wb) == set(range(nb))
    cap = max(nent // 64, 256)
    for b in range(nb):
        items = [j for j, x in enumerate(wb) if x == b]
        lo, hi = int(bin_lo[b]), int(bin_lo[b] + bin_cnt[b])
        assert wl[items[0]] == lo and wl[items[-1] + 1] == hi
        assert all(wl[j] <= wl[j + 1] for j in items)
        assert all(wl[j + 1] - wl[j] <= cap for j in items)
        if len(items) > 1:
            s = [slab[j] for j in items]
            assert s == list(range(s[0], s[0] + len(s)))
        else:
            assert slab[items[0]] == -1
    assert nslab == sum(1 for s in slab if s >= 0)
    for b, f, c in zip(sp_bin.tolist(), sp_first.tolist(), sp_cnt.tolist()):
        items = [j for j, x in enumerate(wb) if x == b]
        assert c == len(items) > 1 and slab[items[0]] == f
