"""Row partitioning: Spark-compatible slices and rank/logical-worker layout.

``sc.parallelize(matrix, n_slices)`` (ssgd.py:86) cuts a local list into
``n_slices`` partitions. PySpark first serialises the list in batches of
``max(1, min(len // n_slices, 1024))`` records and the JVM then slices the
batches evenly (ParallelCollectionRDD.slice) — which is why the reference's 398
breast-cancer training rows land as 99/99/99/101. The local-SGD
algorithms (MA/BMUF/EASGD) train one local model per partition, so reproducing
the partition boundaries reproduces the reference's per-worker data.

Logical workers (``n_slices`` = P) are mapped onto W ranks in contiguous blocks
(P % W == 0): rank r owns workers [r*P/W, (r+1)*P/W) and exactly their rows, so
a W-rank run computes the same thing as a 1-rank run with P logical workers.
"""
from __future__ import annotations

from dataclasses import dataclass


def spark_slices(n: int, n_slices: int, batch_cap: int = 1024) -> list[tuple[int, int]]:
    """Row ranges [lo, hi) of each partition of ``sc.parallelize(list_of_n, n_slices)``."""
    if n_slices <= 0:
        raise ValueError("n_slices must be positive")
    if n == 0:
        return [(0, 0)] * n_slices
    batch = max(1, min(n // n_slices, batch_cap))
    nb = (n + batch - 1) // batch
    out = []
    for i in range(n_slices):
        b0 = (i * nb) // n_slices
        b1 = ((i + 1) * nb) // n_slices
        out.append((min(n, b0 * batch), min(n, b1 * batch)))
    return out


def even_slices(n: int, parts: int) -> list[tuple[int, int]]:
    """Contiguous near-equal ranges (the layout used for synthetic / large data)."""
    return [((i * n) // parts, ((i + 1) * n) // parts) for i in range(parts)]


@dataclass
class ShardLayout:
    """Which rows and logical workers belong to this rank."""
    n_rows: int                 # global rows
    n_workers: int              # logical workers (P)
    world_size: int
    rank: int
    worker_rows: list           # global [lo, hi) per logical worker
    row_lo: int = 0             # this rank's global row range
    row_hi: int = 0
    worker_lo: int = 0          # this rank's worker range
    worker_hi: int = 0

    @property
    def local_workers(self) -> int:
        return self.worker_hi - self.worker_lo

    @property
    def local_rows(self) -> int:
        return self.row_hi - self.row_lo

    def local_segments(self) -> list[int]:
        """Local row bounds [b0, b1, ..., b_{P_local}] of this rank's workers."""
        b = [self.worker_rows[w][0] - self.row_lo for w in range(self.worker_lo, self.worker_hi)]
        b.append(self.worker_rows[self.worker_hi - 1][1] - self.row_lo)
        return b

    def rank_rows(self, r: int) -> tuple[int, int]:
        per = self.n_workers // self.world_size
        return self.worker_rows[r * per][0], self.worker_rows[(r + 1) * per - 1][1]


def make_layout(n_rows: int, n_workers: int, world_size: int, rank: int,
                spark_compatible: bool = True) -> ShardLayout:
    if n_workers % world_size != 0:
        raise ValueError(f"n_workers ({n_workers}) must be a multiple of world size ({world_size})")
    rows = spark_slices(n_rows, n_workers) if spark_compatible else even_slices(n_rows, n_workers)
    per = n_workers // world_size
    w0, w1 = rank * per, (rank + 1) * per
    return ShardLayout(n_rows=n_rows, n_workers=n_workers, world_size=world_size, rank=rank,
                       worker_rows=rows, row_lo=rows[w0][0], row_hi=rows[w1 - 1][1],
                       worker_lo=w0, worker_hi=w1)
