#!/usr/bin/env python3
"""Entry point with the reference's path (graph_computation/pagerank.py).

python graph_computation/pagerank.py [--device cuda|cpu] ...   (one rank), or
torchrun --nproc-per-node N graph_computation/pagerank.py ...  (one rank per GPU)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalgo.apps.pagerank_app import main  # noqa: E402

if __name__ == "__main__":
    main()
