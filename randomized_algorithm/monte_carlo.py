#!/usr/bin/env python3
"""Entry point with the reference's path (randomized_algorithm/monte_carlo.py).

python randomized_algorithm/monte_carlo.py [--device cuda|cpu] ...   (one rank), or
torchrun --nproc-per-node N randomized_algorithm/monte_carlo.py ...  (one rank per GPU)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalgo.apps.mc_app import main  # noqa: E402

if __name__ == "__main__":
    main()
