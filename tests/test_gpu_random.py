"""Philox fill + Monte-Carlo pi kernels vs the NumPy Philox mirror."""
import math

import numpy as np
import pytest
import torch

from dalgo.ops import random as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dist", [R.UNIFORM, R.NORMAL])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D,ld,row_offset", [(33, 40, 1000), (33, 40, 1001), (1, 1, 7),
                                             (64, 64, 3), (5, 8, 12345)])
def test_philox_fill_matches_numpy(cuda, dist, dtype, D, ld, row_offset):
    """4 elements per thread from one Philox block (groups straddle row ends for odd D
    and unaligned starts) == the NumPy mirror; padding columns zeroed."""
    a, b = (-1.0, 1.0) if dist == R.UNIFORM else (0.5, 2.0)
    out_c = torch.empty((37, ld), dtype=dtype)
    R.philox_fill_(out_c, D=D, row_offset=row_offset, seed=77, stream=5, dist=dist, a=a, b=b)
    out_d = torch.full((37, ld), 7.0, dtype=dtype, device=cuda)
    R.philox_fill_(out_d, D=D, row_offset=row_offset, seed=77, stream=5, dist=dist, a=a, b=b)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert torch.allclose(out_d.cpu().float(), out_c.float(), atol=tol * 4, rtol=tol)
    assert (out_d[:, D:] == 0).all()


def test_mc_pi_exact_count(cuda):
    n = 1_000_001                          # not a multiple of 3: partial last block
    c_ref = R.mc_pi_count(n, seed=3, stream=1, offset=12)
    c = R.mc_pi_count(n, seed=3, stream=1, offset=12, device=cuda)
    assert abs(int(c.item()) - int(c_ref.item())) <= 2   # float rounding at the circle edge
    pi = 4.0 * int(c.item()) / n
    assert abs(pi - math.pi) < 0.01
