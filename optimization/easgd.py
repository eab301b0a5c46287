#!/usr/bin/env python3
"""Entry point with the reference's path (optimization/easgd.py): easgd logistic regression.

python optimization/easgd.py [--device cuda|cpu] [--synthetic N,D] ...   (one rank), or
torchrun --nproc-per-node N optimization/easgd.py ...                     (one rank per GPU)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalgo.apps.lr_family import main  # noqa: E402

if __name__ == "__main__":
    main("easgd")
