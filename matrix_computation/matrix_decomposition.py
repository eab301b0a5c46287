#!/usr/bin/env python3
"""Entry point with the reference's path (matrix_computation/matrix_decomposition.py).

python matrix_computation/matrix_decomposition.py [--device cuda|cpu] ...   (one rank), or
torchrun --nproc-per-node N matrix_computation/matrix_decomposition.py ...  (one rank per GPU)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalgo.apps.als_app import main  # noqa: E402

if __name__ == "__main__":
    main()
