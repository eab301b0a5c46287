"""Distributed PageRank (graph_computation/pagerank.py).

Destination-partitioned formulation: rank r owns vertex slice r and its in-edges; per
iteration ONE collective exchange of contributions c[u] = r[u]/outdeg(u), then the SpMV
and the fused rank/contribution epilogue. The SpMV on GPUs is K4b by default
(csrc/kernels/pr_binned.hip: two-level propagation blocking, no random global access,
exact fixed-point sums; 5x the pull K4 at R-MAT scale 26: 2.1 vs 10.8 ms per iteration,
profiles/round4/r4_29); the pull K4 (segmented wave reduction over gathered c[src]) stays
selectable. The exchange is
either an all_gather of the full slices (half the bytes of an all-reduce of a full
vector) or, by default on several ranks, a ghost exchange: each rank receives only the
c[u] of the remote sources that actually have an edge into its slice (one uneven
all_to_all; on R-MAT scale 20 with W = 8 that is 25 % of the remote vertices), and its
edge list is relabeled once into the compact [own slice | ghosts] index space, which
also shrinks the gather footprint of the SpMV.

semantics="reference" reproduces the join/reduceByKey formulation bit-for-bit
in structure: N = #vertices with out-edges (pagerank.py:44),
r0 = 1/N on those (:47), vertices without incoming contributions drop out of the
ranks after the first iteration, dangling vertices never contribute.
semantics="standard" is textbook PageRank with uniform teleport over all
vertices and dangling mass redistributed.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from dalgo.ops import graph as Gops
from dalgo.parallel import comm
from dalgo.utils.obs import NULL_PHASE


@dataclass
class PageRankConfig:
    q: float = 0.15              # teleport probability (pagerank.py:19)
    n_iterations: int = 10       # pagerank.py:18
    semantics: str = "reference"  # "reference" | "standard"
    spmv: str = ""               # "blocked" | "pull" ("" = blocked (K4b) on GPUs, pull on
                                 # the CPU)
    bin_width: int = 16384       # blocked: destination vertices per LDS bin (8192 | 16384)
    chunk: int = 1 << 40         # blocked: ~edges per source chunk (<= 8192 sources; default:
                                 # no edge cut, the work units balance phase 1)
    tile: int = 16384            # blocked: ~edges per phase-1 wave tile
    exchange: str = "ghost"      # "ghost" | "allgather" (several ranks)
    overlap: str = "auto"        # ghost exchange under the SpMV: "auto" | "on" | "peer" | "off"
    fuse_update: bool = True     # K4b: rank / contribution update in the SpMV epilogue


class PageRank:
    timer = None   # dalgo.utils.obs.PhaseTimer (None = off)

    def __init__(self, cfg: PageRankConfig, shard, world: int = 1):
        """shard: a (dst, src)-sorted :class:`GraphShard`, or a :class:`NativeGraph` from
        ``Gops.build_native`` (blocked SpMV only: the K4b layout, out-degrees and ghost
        list come prebuilt)."""
        self.cfg = cfg
        self.g = shard
        self.world = world
        native = isinstance(shard, Gops.NativeGraph)
        self.native = native
        dev = shard.layout.srcl.device if native else shard.src.device
        self.dev = dev
        nl = shard.n_local
        sl = shard.slice_size
        # global out-degree (each rank holds the in-edges of its slice only)
        if native and world == 1 and shard.v_lo == 0 and shard.v_hi == shard.n_vertices and not shard.n_ghost:
            od_full = shard.outdeg_loc[:nl]        # one rank: the local out-degrees are global
        elif native:
            od_full = torch.zeros(shard.n_vertices, dtype=torch.int32, device=dev)
            od_full[shard.v_lo: shard.v_hi] += shard.outdeg_loc[:nl]
            if shard.ghosts is not None and shard.n_ghost:
                od_full.index_add_(0, shard.ghosts, shard.outdeg_loc[sl: sl + shard.n_ghost])
        else:
            od_full = Gops.local_outdeg(shard)
        comm.all_reduce_sum(od_full)
        self.outdeg = od_full[shard.v_lo: shard.v_hi].contiguous()
        self.mode = 0 if cfg.semantics == "reference" else 1
        self.spmv = cfg.spmv or ("blocked" if dev.type == "cuda" else "pull")
        if self.spmv not in ("blocked", "pull"):
            raise ValueError(f"spmv must be 'blocked' or 'pull' (got {self.spmv!r})")
        if native and self.spmv != "blocked":
            raise ValueError("a NativeGraph carries the blocked (K4b) layout only")
        if self.mode == 0:
            self.N = int((od_full > 0).sum().item())
        else:
            self.N = shard.n_vertices
        self.invN = 1.0 / max(self.N, 1)
        # f32 on the GPU kernels; the CPU reference path runs in f64 (the
        # reference's NumPy precision, so the toy ranks match digit for digit)
        fdt = torch.float32 if dev.type == "cuda" else torch.float64
        self.fdt = fdt
        self.acc = torch.zeros(nl, dtype=fdt, device=dev)
        self.pres = torch.zeros(nl, dtype=torch.int32, device=dev)
        self.r = torch.zeros(nl, dtype=fdt, device=dev)
        self.exchange = cfg.exchange if world > 1 else "allgather"
        if native and world > 1 and self.exchange != "ghost":
            raise ValueError("a NativeGraph uses the ghost exchange on several ranks")
        if self.exchange == "ghost":
            if native:
                self._native_ghosts()
            else:
                self._build_ghosts()
            # own slice first, then the ghosts: c_slice is a view, so the update kernel's
            # writes are already in place for the SpMV
            self.c_full = torch.zeros(sl + self.n_ghost, dtype=fdt, device=dev)
            self.c_slice = self.c_full[:sl]
        else:
            self.c_slice = torch.zeros(sl, dtype=fdt, device=dev)   # padded slice
            # one rank: the slice IS the full vector (no exchange copy)
            self.c_full = (self.c_slice if world == 1
                           else torch.zeros(sl * world, dtype=fdt, device=dev))
        # K4b: built over the edge list the SpMV reads (c_full index space)
        self.layout = None
        # fuse_update=False: K4b writes acc / pres and the separate update kernel runs
        self.fuse_update = cfg.fuse_update
        if native:
            self.layout = shard.layout
        elif self.spmv == "blocked":
            gsp = self.g_local if self.exchange == "ghost" else self.g
            # ghost index space: no chunk straddles the own slice's end or a peer's block,
            # so each peer's ghost chunks are one work-unit range (per-peer overlap)
            splits = None
            if self.exchange == "ghost":
                splits = [sl] + [sl + o for o in self.ghost_off[1:-1]]
            self.layout = Gops.build_blocked(gsp, cfg.bin_width, cfg.chunk, cfg.tile,
                                             src_split=sl if self.exchange == "ghost" else None,
                                             src_splits=splits)
        self.dang = torch.zeros(1, dtype=fdt, device=dev)
        self.dang_next = torch.zeros(1, dtype=fdt, device=dev)
        od = self.outdeg.to(fdt)
        if self.mode == 0:
            # (scalar where: one kernel each -- the full_like / clamp forms were ~1 ms of
            # small kernels in the scale-26 job, profiles/round6/r6_48)
            p = self.outdeg > 0
            self.r.copy_(torch.where(p, self.invN, -1.0))
            self.c_slice[:nl] = torch.where(p, self.invN / od, -1.0)
            self.c_slice[nl:] = -1.0
        else:
            self.r.fill_(self.invN)
            self.c_slice[:nl] = torch.where(self.outdeg > 0, self.invN / od.clamp_min(1),
                                            torch.zeros_like(od))
            self.dang.fill_(float(((self.outdeg == 0).float() * self.invN).sum().item()))
            comm.all_reduce_sum(self.dang)
        self.t = 0

    def _build_ghosts(self):
        """Relabel this rank's edge sources into [own slice (sl) | ghosts] and agree, with
        one exchange of request lists, which own c values every peer needs."""
        g, W, sl = self.g, self.world, self.g.slice_size
        rank = g.v_lo // sl if sl else 0
        E = g.n_edges
        src = g.src[:E].to(torch.int64)
        owner = src // sl
        remote = owner != rank
        ghosts = torch.unique(src[remote])                     # sorted: grouped by owner
        self.n_ghost = int(ghosts.numel())
        recv_counts = torch.bincount(ghosts // sl, minlength=W).to(torch.int64)
        local = torch.where(remote, sl + torch.searchsorted(ghosts, src), src - g.v_lo)
        src_local = torch.full_like(g.src, -1)
        src_local[:E] = local.to(torch.int32)
        if E:
            assert int(local.max()) < sl + self.n_ghost and int(local.min()) >= 0
        self.g_local = Gops.GraphShard(src_local, g.dstl, E, g.v_lo, g.v_hi, g.n_vertices, sl,
                                       g.new_id)
        # the same edges split by source: own slice (needs no exchange) and ghosts; each
        # keeps the (dst, src) order, so the ghost pass adds into rows the own pass wrote
        own = local < sl

        def _part(m):
            k = int(m.sum().item())
            kp = (k + 3) // 4 * 4
            s_ = torch.full((kp,), -1, dtype=torch.int32, device=src.device)
            d_ = torch.full((kp,), -1, dtype=torch.int32, device=src.device)
            s_[:k] = local[m].to(torch.int32)
            d_[:k] = g.dstl[:E][m]
            return Gops.GraphShard(s_, d_, k, g.v_lo, g.v_hi, g.n_vertices, sl, g.new_id)

        self.g_own, self.g_ghost = _part(own), _part(~own)
        self.own_share = self.g_own.n_edges / max(E, 1)
        # request lists: peer p asks for send_counts[p] of my vertices
        send_counts = torch.empty_like(recv_counts)
        comm.all_to_all_single(send_counts, recv_counts)
        self.recv_split = [int(x) for x in recv_counts.tolist()]
        self.send_split = [int(x) for x in send_counts.tolist()]
        # ghost block of peer p: [ghost_off[p], ghost_off[p + 1]) past the own slice
        self.ghost_off = [0]
        for c_ in self.recv_split:
            self.ghost_off.append(self.ghost_off[-1] + c_)
        req = torch.empty(sum(self.send_split), dtype=torch.int64, device=src.device)
        comm.all_to_all_single(req, ghosts, out_split=self.send_split, in_split=self.recv_split)
        self.send_idx = (req - g.v_lo).contiguous()
        assert bool(((self.send_idx >= 0) & (self.send_idx < g.n_local)).all())
        self.send_buf = None

    def _native_ghosts(self):
        """The ghost exchange plan from a NativeGraph's ghost list (sorted global ids,
        grouped by owner): who sends which own c values to whom."""
        g, W = self.g, self.world
        ghosts = g.ghosts if g.ghosts is not None else torch.zeros(0, dtype=torch.int64, device=self.dev)
        self.n_ghost = int(ghosts.numel())
        recv_counts = torch.tensor(g.recv_counts + [0] * (W - len(g.recv_counts)), dtype=torch.int64,
                                   device=self.dev)[:W]
        send_counts = torch.empty_like(recv_counts)
        comm.all_to_all_single(send_counts, recv_counts)
        self.recv_split = [int(x) for x in recv_counts.tolist()]
        self.send_split = [int(x) for x in send_counts.tolist()]
        self.ghost_off = [0]
        for c_ in self.recv_split:
            self.ghost_off.append(self.ghost_off[-1] + c_)
        req = torch.empty(sum(self.send_split), dtype=torch.int64, device=self.dev)
        comm.all_to_all_single(req, ghosts, out_split=self.send_split, in_split=self.recv_split)
        self.send_idx = (req - g.v_lo).contiguous()
        self.send_buf = None
        self.own_share = 0.0

    def _exchange(self):
        if self.exchange == "ghost":
            if self.send_buf is None:
                self.send_buf = torch.empty(self.send_idx.numel(), dtype=self.fdt, device=self.dev)
            torch.index_select(self.c_slice, 0, self.send_idx, out=self.send_buf)
            comm.all_to_all_single(self.c_full[self.g.slice_size:], self.send_buf,
                                   out_split=self.recv_split, in_split=self.send_split)
        elif self.world > 1:
            comm.all_gather_into(self.c_full, self.c_slice)

    def _spmv(self):
        if self.layout is not None:
            # K4b writes every destination and, with the update fused into its epilogue
            # (ranks + next contributions), needs no separate update launch
            Gops.pb_spmv(self.layout, self.c_full, self.acc, self.pres,
                         update=self._pb_update_args())
            return
        self.acc.zero_()
        self.pres.zero_()
        if self.exchange == "ghost":
            Gops.pr_spmv(self.g_local, self.c_full, self.acc, self.pres)
        else:
            Gops.pr_spmv(self.g, self.c_full, self.acc, self.pres)

    def _pb_update_args(self):
        nl = self.g.n_local
        if not self.fuse_update:
            return None
        if self.mode == 1:
            self.dang_next.zero_()
        return dict(outdeg=self.outdeg, q=self.cfg.q, invN=self.invN, mode=self.mode,
                    r=self.r, c=self.c_slice[:nl],
                    dangling_in=self.dang if self.mode == 1 else None,
                    dangling_out=self.dang_next if self.mode == 1 else None)

    def _update(self):
        nl = self.g.n_local
        if self.layout is not None and self.fuse_update:
            # the ranks / contributions were written by the K4b epilogue
            if self.mode == 1:
                comm.all_reduce_sum(self.dang_next)
                self.dang, self.dang_next = self.dang_next, self.dang
            return
        if self.mode == 1:
            self.dang_next.zero_()
        Gops.pr_update(self.acc, self.pres, self.outdeg, self.cfg.q, self.invN, self.mode, self.r,
                       self.c_slice[:nl], dangling_in=self.dang if self.mode == 1 else None,
                       dangling_out=self.dang_next if self.mode == 1 else None)
        if self.mode == 1:
            comm.all_reduce_sum(self.dang_next)
            self.dang, self.dang_next = self.dang_next, self.dang

    def _overlap_pb(self) -> str:
        """K4b with the ghost exchange: "whole" = phase 1 over the own-slice source chunks
        runs while the all_to_all of the ghost contributions is in flight, phase 1 over the
        ghost chunks after it; "peer" = the exchange is W - 1 grouped send/recv shifts and
        each peer's ghost chunks run as soon as that peer's shift lands (the own share
        alone is too short to hide a whole all_to_all at W >= 8); "" = no overlap.
        cfg.overlap: auto = whole while the own-slice units are >= 1/4 of all units, else
        peer; on = whole; peer; off."""
        if self.layout is None or self.exchange != "ghost":
            return ""
        ov = self.cfg.overlap
        if ov in ("on", "peer"):
            return "whole" if ov == "on" else "peer"
        if ov != "auto":
            return ""
        nwu = int(self.layout.wu_chunk.numel())
        if nwu == 0:
            return ""
        return "whole" if self.layout.n_wu_below >= 0.25 * nwu else "peer"

    def _overlap(self) -> bool:
        """Ghost exchange under the SpMV over own-slice sources: the all_to_all writes only
        the ghost part of c_full, the first pass reads only the own part, the second adds
        the ghost-source edges into the same rows. Splitting the SpMV costs ~10 % at the
        rank-0 share of R-MAT scale 26 (1.41 -> 1.54 ms at W = 8, 5.42 -> 5.80 ms at W = 2,
        profiles/round2/README.md), so by default (cfg.overlap = "auto") it is only used
        while the own-source pass is long enough to hide the exchange: at least a quarter
        of the edges (W <= 4 with the dealt relabeling). "on" / "off" force it."""
        if self.exchange != "ghost" or self.layout is not None:
            return False
        ov = self.cfg.overlap
        return ov == "on" or (ov == "auto" and self.own_share >= 0.25)

    def _ph(self, name: str):
        return self.timer.phase(name) if self.timer is not None else NULL_PHASE

    def _step_peer(self):
        """K4b with the per-peer overlapped exchange (see _overlap_pb)."""
        lay = self.layout
        sl = self.g.slice_size
        if self.send_buf is None:
            self.send_buf = torch.empty(self.send_idx.numel(), dtype=self.fdt, device=self.dev)
        with self._ph("exchange_issue"):
            torch.index_select(self.c_slice, 0, self.send_idx, out=self.send_buf)
            shifts = comm.exchange_by_shift(self.c_full[sl:], self.send_buf, self.recv_split,
                                            self.send_split)
        # work-unit range of every source block: own slice, then peer p's ghosts
        bounds = (0,) + tuple(lay.wu_bounds) + (1 << 31,)
        blk_of_peer = {}
        bi = 1                                   # block 0 = own slice
        for p in range(self.world):
            if self.ghost_off[p + 1] > self.ghost_off[p]:
                blk_of_peer[p] = bi
                bi += 1
        with self._ph("spmv_own"):
            Gops.pb_spmv(lay, self.c_full, self.acc, self.pres, wu_range=(0, bounds[1]),
                         phases=1)
        with self._ph("spmv_ghost"):
            for peer, h in shifts:
                h.wait()
                b = blk_of_peer.get(peer)
                if b is not None:
                    Gops.pb_spmv(lay, self.c_full, self.acc, self.pres,
                                 wu_range=(bounds[b], bounds[b + 1]), phases=1)
            Gops.pb_spmv(lay, self.c_full, self.acc, self.pres,
                         update=self._pb_update_args(), phases=2)

    def step(self):
        ovp = self._overlap_pb()
        if ovp == "peer":
            self._step_peer()
        elif ovp == "whole":
            lay = self.layout
            if self.send_buf is None:
                self.send_buf = torch.empty(self.send_idx.numel(), dtype=self.fdt, device=self.dev)
            with self._ph("exchange_issue"):
                torch.index_select(self.c_slice, 0, self.send_idx, out=self.send_buf)
                work = comm.all_to_all_single(self.c_full[self.g.slice_size:], self.send_buf,
                                              out_split=self.recv_split,
                                              in_split=self.send_split, async_op=True)
            with self._ph("spmv_own"):
                Gops.pb_spmv(lay, self.c_full, self.acc, self.pres, wu_range=(0, lay.n_wu_below),
                             phases=1)
            with self._ph("exchange_wait"):
                work.wait()
            with self._ph("spmv_ghost"):
                Gops.pb_spmv(lay, self.c_full, self.acc, self.pres,
                             wu_range=(lay.n_wu_below, 1 << 31), phases=1)
                Gops.pb_spmv(lay, self.c_full, self.acc, self.pres,
                             update=self._pb_update_args(), phases=2)
        elif self._overlap():
            if self.send_buf is None:
                self.send_buf = torch.empty(self.send_idx.numel(), dtype=self.fdt, device=self.dev)
            with self._ph("exchange_issue"):
                torch.index_select(self.c_slice, 0, self.send_idx, out=self.send_buf)
                work = comm.all_to_all_single(self.c_full[self.g.slice_size:], self.send_buf,
                                              out_split=self.recv_split,
                                              in_split=self.send_split, async_op=True)
            with self._ph("spmv_own"):
                self.acc.zero_()
                self.pres.zero_()
                Gops.pr_spmv(self.g_own, self.c_full, self.acc, self.pres)
            with self._ph("exchange_wait"):
                work.wait()
            with self._ph("spmv_ghost"):
                Gops.pr_spmv(self.g_ghost, self.c_full, self.acc, self.pres, accumulate=True)
        else:
            with self._ph("exchange"):
                self._exchange()      # contributions of the previous iteration
            with self._ph("spmv"):
                self._spmv()          # K4 pull SpMV over the local in-edges
        with self._ph("update"):
            self._update()        # ranks + next contributions (fused epilogue kernel)
        self.bytes_exchanged = getattr(self, "bytes_exchanged", 0) + \
            self.exchange_floats() * self.c_slice.element_size()
        self.t += 1

    def exchange_floats(self) -> int:
        """Contribution floats this rank receives per iteration."""
        if self.world == 1:
            return 0
        if self.exchange == "ghost":
            return self.n_ghost
        return self.g.slice_size * (self.world - 1)

    def fit(self, n_iterations: int | None = None):
        n = self.cfg.n_iterations if n_iterations is None else n_iterations
        for _ in range(n):
            self.step()
        comm.check_device_errors("end of PageRank fit")
        return self

    def state_dict(self) -> dict:
        """Per-rank state (this rank's destination slice) for checkpoint / resume."""
        return {"t": self.t, "r": self.r.cpu(), "c_slice": self.c_slice.cpu(),
                "dang": self.dang.cpu(), "v_lo": self.g.v_lo, "v_hi": self.g.v_hi}

    def load_state_dict(self, sd: dict):
        if (int(sd["v_lo"]), int(sd["v_hi"])) != (self.g.v_lo, self.g.v_hi):
            raise ValueError("checkpoint was written with a different vertex partition")
        self.t = int(sd["t"])
        self.r.copy_(sd["r"].to(self.dev))
        self.c_slice.copy_(sd["c_slice"].to(self.dev))
        self.dang.copy_(sd["dang"].to(self.dev))

    def ranks_local(self):
        """(vertex ids, ranks) of this rank's present vertices."""
        if self.mode == 0:
            present = self.r >= 0
        else:
            present = torch.ones_like(self.r, dtype=torch.bool)
        ids = torch.nonzero(present).flatten()
        return ids + self.g.v_lo, self.r[ids]

    def collect(self) -> dict:
        """``ranks.collect()``: {vertex: rank} of all present vertices (every rank)."""
        ids, vals = self.ranks_local()
        sl = self.g.slice_size
        full = torch.full((sl * self.world,), float("nan"), dtype=self.fdt, device=self.dev)
        loc = torch.full((sl,), float("nan"), dtype=self.fdt, device=self.dev)
        loc[ids - self.g.v_lo] = vals
        comm.all_gather_into(full, loc)
        full = full.cpu()
        keep = ~torch.isnan(full)
        return {int(v): float(full[v]) for v in torch.nonzero(keep).flatten().tolist()}
