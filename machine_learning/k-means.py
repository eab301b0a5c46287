#!/usr/bin/env python3
"""Entry point with the reference's path (machine_learning/k-means.py).

python machine_learning/k-means.py [--device cuda|cpu] ...   (one rank), or
torchrun --nproc-per-node N machine_learning/k-means.py ...  (one rank per GPU)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalgo.apps.kmeans_app import main  # noqa: E402

if __name__ == "__main__":
    main()
