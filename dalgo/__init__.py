"""dalgo — MI355X-native distributed algorithms (gfx950 HIP kernels + RCCL over xGMI).

Same algorithm set and script entry points as the PySpark collection
*Distributed-Algorithm-PySpark*: parallel SGD (SSGD / MA / BMUF / EASGD),
logistic regression, K-means, PageRank, transitive closure, ALS matrix
decomposition and Monte-Carlo pi. See SURVEY.md for the design blueprint.

Layout:
  dalgo.ops       python wrappers of the HIP kernels (+ torch-CPU references)
  dalgo.parallel  runtime (process group), collectives, sharding, launcher
  dalgo.models    the algorithms (drivers of the reference scripts)
  dalgo.data      datasets and on-device synthetic generators
  dalgo.utils     Philox mirror, observability, config, checkpoints
"""
__version__ = "0.1.0"
