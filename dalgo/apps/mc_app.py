"""randomized_algorithm/monte_carlo.py entry logic."""
from __future__ import annotations

import time

from dalgo.models.monte_carlo import MonteCarloConfig, estimate_pi
from dalgo.parallel import runtime
from dalgo.utils import obs
from dalgo.utils.cli import common_parser, init_from_args


def main(argv=None):
    ap = common_parser("Monte-Carlo pi (MI355X-native)")
    ap.add_argument("--n-slices", type=int, default=4)
    ap.add_argument("--num-samples", type=int, default=None,
                    help="samples (default 100000 * n_slices, monte_carlo.py:15)")
    a = ap.parse_args(argv)
    rt = init_from_args(a, "monte_carlo")
    cfg = MonteCarloConfig(n_slices=a.n_slices, n=a.num_samples, seed=a.seed)
    sink = obs.MetricsSink(a.metrics_out, rt.rank)
    timer = obs.PhaseTimer(rt.device) if (sink.enabled or obs.roctx_enabled()) else None
    t0 = time.time()
    with (timer.phase("sample+count+allreduce") if timer else obs.NULL_PHASE):
        pi, total = estimate_pi(cfg, rt.rank, rt.world_size, device=rt.device)
    sink.log(phases=timer.take() if timer else None, samples=cfg.n_points, in_circle=total,
             pi=pi, elapsed_s=time.time() - t0, bytes_allreduced=8 if rt.world_size > 1 else 0,
             world_size=rt.world_size)
    sink.close()
    rt.log("Pi is roughly %f" % pi)   # monte_carlo.py:31
    runtime.shutdown()
    return pi
