"""randomized_algorithm/monte_carlo.py entry logic."""
from __future__ import annotations

from dalgo.models.monte_carlo import MonteCarloConfig, estimate_pi
from dalgo.parallel import runtime
from dalgo.utils.cli import common_parser, init_from_args


def main(argv=None):
    ap = common_parser("Monte-Carlo pi (MI355X-native)")
    ap.add_argument("--n-slices", type=int, default=4)
    ap.add_argument("--num-samples", type=int, default=None,
                    help="samples (default 100000 * n_slices, monte_carlo.py:15)")
    a = ap.parse_args(argv)
    rt = init_from_args(a, "monte_carlo")
    pi, _ = estimate_pi(MonteCarloConfig(n_slices=a.n_slices, n=a.num_samples, seed=a.seed),
                        rt.rank, rt.world_size, device=rt.device)
    rt.log("Pi is roughly %f" % pi)   # monte_carlo.py:31
    runtime.shutdown()
    return pi
