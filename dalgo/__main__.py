"""``python -m dalgo <algorithm> [args]`` — one launcher for every algorithm.

The reference ships one script per algorithm (README.md:17-31); the same scripts exist
here under the same paths. This dispatcher reaches the same application mains by name,
so ``torchrun --nproc-per-node 8 -m dalgo bmuf --synthetic 10000000,1024`` works without
knowing the script layout. ``python -m dalgo list`` prints the table.
"""
from __future__ import annotations

import sys

# name -> (module, callable name, fixed leading args, reference script)
ALGORITHMS = {
    "ssgd": ("dalgo.apps.lr_family", "main", ("ssgd",), "optimization/ssgd.py"),
    "ma": ("dalgo.apps.lr_family", "main", ("ma",), "optimization/ma.py"),
    "bmuf": ("dalgo.apps.lr_family", "main", ("bmuf",), "optimization/bmuf.py"),
    "easgd": ("dalgo.apps.lr_family", "main", ("easgd",), "optimization/easgd.py"),
    "logistic_regression": ("dalgo.apps.lr_family", "main", ("gd",),
                            "machine_learning/logistic_regression.py"),
    "kmeans": ("dalgo.apps.kmeans_app", "main", (), "machine_learning/k-means.py"),
    "pagerank": ("dalgo.apps.pagerank_app", "main", (), "graph_computation/pagerank.py"),
    "transitive_closure": ("dalgo.apps.closure_app", "main", (),
                           "graph_computation/transitive_closure.py"),
    "als": ("dalgo.apps.als_app", "main", (), "matrix_computation/matrix_decomposition.py"),
    "monte_carlo": ("dalgo.apps.mc_app", "main", (), "randomized_algorithm/monte_carlo.py"),
}
ALIASES = {"gd": "logistic_regression", "lr": "logistic_regression", "k-means": "kmeans",
           "closure": "transitive_closure", "matrix_decomposition": "als", "mc": "monte_carlo",
           "pi": "monte_carlo"}


def usage() -> str:
    rows = [f"  {name:<20} {spec[3]}" for name, spec in ALGORITHMS.items()]
    return ("usage: python -m dalgo <algorithm> [args ...]   (--help after the name for its flags)\n"
            "algorithms (and the reference script each one mirrors):\n" + "\n".join(rows))


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help", "list"):
        print(usage())
        return 0
    name = ALIASES.get(argv[0], argv[0])
    if name not in ALGORITHMS:
        print(f"unknown algorithm {argv[0]!r}\n" + usage(), file=sys.stderr)
        return 2
    mod_name, fn_name, lead, _ = ALGORITHMS[name]
    import importlib
    fn = getattr(importlib.import_module(mod_name), fn_name)
    fn(*lead, argv[1:])
    return 0


if __name__ == "__main__":
    sys.exit(main())
