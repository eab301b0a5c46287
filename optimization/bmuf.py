#!/usr/bin/env python3
"""Entry point with the reference's path (optimization/bmuf.py): bmuf logistic regression.

python optimization/bmuf.py [--device cuda|cpu] [--synthetic N,D] ...   (one rank), or
torchrun --nproc-per-node N optimization/bmuf.py ...                     (one rank per GPU)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalgo.apps.lr_family import main  # noqa: E402

if __name__ == "__main__":
    main("bmuf")
