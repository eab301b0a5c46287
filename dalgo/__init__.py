"""dalgo — MI355X-native distributed algorithms (gfx950 HIP kernels + RCCL over xGMI).

Same algorithm set and script entry points as the PySpark collection
*Distributed-Algorithm-PySpark*: parallel SGD (SSGD / MA / BMUF / EASGD),
logistic regression, K-means, PageRank, transitive closure, ALS matrix
decomposition and Monte-Carlo pi. See SURVEY.md for the design blueprint.

Layout:
  dalgo.ops       python wrappers of the HIP kernels (+ torch-CPU references)
  dalgo.parallel  runtime (process group, device-sharing rule), collectives, K11, sharding
  dalgo.models    the algorithms (drivers of the reference scripts)
  dalgo.data      datasets and on-device synthetic generators
  dalgo.utils     Philox mirror, observability, config, checkpoints
"""
import os as _os

__version__ = "0.1.0"

# Kernel arguments in device memory (set before the HIP runtime initialises): the first
# scalar loads of every launch then hit HBM/L2 instead of host memory. Measured on the
# K1 gradient launch at the 8-GPU per-rank share (1.25M x 1024 bf16): first row load
# issued 9.2 -> 5.6 us after wave start, step 63.7 -> 56.3 us (profiles/round2/README.md).
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
