"""graph_computation/transitive_closure.py entry logic."""
from __future__ import annotations

import hashlib
import time

import torch

from dalgo.models.transitive_closure import DenseClosure, SparseClosure, compact_ids
from dalgo.parallel import runtime
from dalgo.utils import checkpoint, obs
from dalgo.utils.cli import add_ckpt_args, common_parser, init_from_args

TOY_EDGES = [(1, 2), (1, 3), (2, 3), (3, 1)]   # transitive_closure.py:18


def main(argv=None):
    ap = common_parser("Linear transitive closure (MI355X-native)")
    ap.add_argument("--engine", choices=["auto", "dense", "sparse"], default="auto")
    ap.add_argument("--edges", default=None)
    ap.add_argument("--random", default=None, metavar="N,E", help="random graph with N vertices, E edges")
    ap.add_argument("--max-rounds", type=int, default=1 << 30,
                    help="stop after this many join rounds (resume later with --resume)")
    add_ckpt_args(ap)
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
    # per-rank state (each rank owns the paths of its target slice)
    name = f"closure_{engine}_w{rt.world_size}"
    # the input graph's identity travels with every per-rank checkpoint
    fp = hashlib.sha1(s.numpy().astype("int64").tobytes() + b"|" +
                      d.numpy().astype("int64").tobytes()).hexdigest() + f"/n={n}"
    if a.resume and a.ckpt_dir:
        sd = checkpoint.load_consistent(a.ckpt_dir, name, rt.rank, fingerprint=fp,
                                        progress=lambda st: len(st["counts"]))
        if sd is not None:
            tc.load_state_dict(sd)
            rt.log("resumed after %d rounds" % (len(tc.counts) - 1))

    def save(m):
        st = m.state_dict()
        st["fingerprint"] = fp
        checkpoint.save(st, a.ckpt_dir, name, rt.rank, per_rank=True)

    sink = obs.MetricsSink(a.metrics_out, rt.rank)
    if sink.enabled or obs.roctx_enabled():
        tc.timer = obs.PhaseTimer(rt.device)
    t_last = [time.time()]

    def cb(m):
        now = time.time()
        sink.log(phases=m.timer.take() if m.timer else None, round=len(m.counts) - 1,
                 paths=m.counts[-1], round_s=now - t_last[0], engine=engine,
                 bytes_allreduced=8 * (len(m.counts) - 1) if rt.world_size > 1 else 0,
                 world_size=rt.world_size)
        t_last[0] = now
        if a.ckpt_dir and a.ckpt_every and (len(m.counts) - 1) % a.ckpt_every == 0:
            save(m)

    res = tc.run(a.max_rounds, callback=cb)
    sink.close()
    if a.ckpt_dir:
        save(tc)
    if not a.quiet:
        rt.log("path counts per round: %s" % res.counts)
    if not tc.converged:
        rt.log("stopped after %d rounds before the fixpoint (--max-rounds); continue with --resume"
               % (len(res.counts) - 1))
    rt.log("The original graph has %i paths" % res.n_paths)   # transitive_closure.py:42 (sic)
    runtime.shutdown()
    return res
