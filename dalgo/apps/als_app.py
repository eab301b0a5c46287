"""matrix_computation/matrix_decomposition.py entry logic."""
from __future__ import annotations

from dalgo.models.als import ALS, ALSConfig
from dalgo.parallel import runtime
from dalgo.utils import checkpoint, obs
from dalgo.utils.cli import add_ckpt_args, common_parser, init_from_args


def main(argv=None):
    ap = common_parser("ALS matrix decomposition (MI355X-native)")
    ap.add_argument("--lam", type=float, default=0.01)
    ap.add_argument("--m", type=int, default=100)
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n-iterations", type=int, default=5)
    ap.add_argument("--n-slices", type=int, default=4)
    add_ckpt_args(ap)
    a = ap.parse_args(argv)
    rt = init_from_args(a, "Matrix Decomposition")
    cfg = ALSConfig(m=a.m, n=a.n, k=a.k, lam=a.lam, n_iterations=a.n_iterations,
                    n_workers=a.n_slices, seed=a.seed + 7)
    als = ALS(cfg, rt.rank, rt.world_size, device=rt.device)
    sink = obs.MetricsSink(a.metrics_out, rt.rank)
    if sink.enabled or obs.roctx_enabled():
        als.timer = obs.PhaseTimer(rt.device)

    if a.resume and a.ckpt_dir:
        sd = checkpoint.load(a.ckpt_dir, "als_state")
        if sd is not None:
            als.load_state_dict(sd)
            rt.log(f"Resumed from iteration {als.t}")

    def cb(m):
        rt.log("iterations: %d, rmse: %f" % (m.t - 1, m.history.rmse[-1]))   # :67
        sink.log(phases=m.timer.take() if m.timer else None, iteration=m.t,
                 rmse=m.history.rmse[-1], bytes_allgathered=m.bytes_gathered,
                 world_size=rt.world_size)
        if a.ckpt_dir and a.ckpt_every and m.t % a.ckpt_every == 0:
            checkpoint.save(m.state_dict(), a.ckpt_dir, "als_state", rt.rank)

    als.fit(max(0, a.n_iterations - als.t), callback=cb)
    if a.ckpt_dir:
        checkpoint.save(als.state_dict(), a.ckpt_dir, "als_state", rt.rank)
    sink.close()
    runtime.shutdown()
    return als.history.rmse
