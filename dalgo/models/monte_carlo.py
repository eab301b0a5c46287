"""Monte-Carlo pi (randomized_algorithm/monte_carlo.py).

Reference (:15-31): n = 100000 * n_slices points, is_accept draws x, y ~ U[-1, 1)
with Python's unseeded random() per worker and counts x^2 + y^2 <= 1;
pi ~= 4 * count / n. Here point i of the global stream is a pure function of
(seed, i) (Philox, K6 csrc/kernels/random.hip); rank r evaluates the contiguous
index range [r*n/W, (r+1)*n/W) and one int64 all-reduce sums the counts, so the
estimate is identical for any number of ranks.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from dalgo.ops import random as drandom
from dalgo.parallel import comm


@dataclass
class MonteCarloConfig:
    n_slices: int = 4
    n: int | None = None          # default 100000 * n_slices (monte_carlo.py:15)
    seed: int = 0
    stream: int = 0

    @property
    def n_points(self) -> int:
        return self.n if self.n is not None else 100000 * self.n_slices


def estimate_pi(cfg: MonteCarloConfig, rank: int = 0, world: int = 1, device="cpu"):
    n = cfg.n_points
    # even split with offsets on Philox-block boundaries (a block serves 3 points)
    per = ((n // world) // 3) * 3
    lo = rank * per
    hi = n if rank == world - 1 else lo + per
    cnt = drandom.mc_pi_count(hi - lo, seed=cfg.seed, stream=cfg.stream, offset=lo, device=device)
    total = comm.all_reduce_count(cnt.to(torch.int64))
    return 4.0 * total / n, total
