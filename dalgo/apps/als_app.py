"""matrix_computation/matrix_decomposition.py entry logic."""
from __future__ import annotations

from dalgo.models.als import ALS, ALSConfig
from dalgo.parallel import runtime
from dalgo.utils import obs
from dalgo.utils.cli import common_parser, init_from_args


def main(argv=None):
    ap = common_parser("ALS matrix decomposition (MI355X-native)")
    ap.add_argument("--lam", type=float, default=0.01)
    ap.add_argument("--m", type=int, default=100)
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n-iterations", type=int, default=5)
    ap.add_argument("--n-slices", type=int, default=4)
    a = ap.parse_args(argv)
    rt = init_from_args(a, "Matrix Decomposition")
    cfg = ALSConfig(m=a.m, n=a.n, k=a.k, lam=a.lam, n_iterations=a.n_iterations,
                    n_workers=a.n_slices, seed=a.seed + 7)
    als = ALS(cfg, rt.rank, rt.world_size, device=rt.device)
    sink = obs.MetricsSink(a.metrics_out, rt.rank)

    def cb(m):
        rt.log("iterations: %d, rmse: %f" % (m.t - 1, m.history.rmse[-1]))   # :67
        sink.log(iteration=m.t, rmse=m.history.rmse[-1])

    als.fit(callback=cb)
    sink.close()
    runtime.shutdown()
    return als.history.rmse
