"""Host-side native checks under AddressSanitizer + UBSan (sanitizers).

GPU sanitizers are not available on the MI355X pool, so the native layer's HOST
code is checked here: tests/native/host_checks.cpp is compiled by hipcc together
with kernel sources (device code for gfx950, host code instrumented via
``-Xarch_host -fsanitize=...``) and run on the CPU. It verifies the Philox stream
shared by every sampler against the NumPy mirror (dalgo/utils/philox.py) and the
launchers' argument validation, which must reject bad shapes before any HIP call.
"""
import os
import shutil
from pathlib import Path
import subprocess

import numpy as np
import pytest

from dalgo.utils import philox

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def host_binary(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("native") / "host_checks")
    srcs = ["tests/native/host_checks.cpp", "csrc/kernels/closure.hip",
            "csrc/kernels/xgmi_allreduce.hip", "csrc/kernels/lr_grad.hip"]
    cmd = [HIPCC, "--offload-arch=gfx950", "-O1", "-g",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined",
           f"-I{ROOT}/csrc/include", f"-I{ROOT}/csrc"]
    for s in srcs:
        cmd += ["-x", "hip", os.path.join(ROOT, s)]
    cmd += ["-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def test_native_host_checks_asan(host_binary):
    rng = np.random.default_rng(0)
    triples = [(0, 0, 0), (42, 7, 1), (2**64 - 1, 2**63, 2**40 + 3)]
    triples += [(int(rng.integers(0, 2**63)), int(rng.integers(0, 2**63)), int(rng.integers(0, 2**60)))
                for _ in range(20)]
    inp = "".join(f"{s} {t} {b}\n" for s, t, b in triples)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([host_binary], input=inp, capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "host checks passed" in r.stderr
    got = [tuple(int(v) for v in line.split()) for line in r.stdout.strip().splitlines()]
    assert len(got) == len(triples)
    for (s, t, b), g in zip(triples, got):
        # block b of stream t = indices 4b..4b+3 of the NumPy mirror
        exp = philox.draw_u32(s, t, np.uint64(4 * b) + np.arange(4, dtype=np.uint64))
        assert tuple(int(x) for x in exp) == g, (s, t, b)


def test_extension_loads_and_registers_ops():
    """The built extension loads in a fresh process on the CPU host (HIP runtime present,
    no GPU needed) and every operator schema parses: a schema error aborts the process
    at load time, which only a GPU box would otherwise reveal."""
    import subprocess
    import sys
    from dalgo.ops import _ext
    lib = _ext.lib_path() if hasattr(_ext, "lib_path") else _ext._LIB
    if not Path(lib).exists():
        pytest.skip("extension not built")
    code = ("import torch; torch.ops.load_library(%r); "
            "print(len([s for s in torch._C._jit_get_all_schemas() if s.name.startswith('dalgo::')]))"
            % str(lib))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert int(r.stdout.strip().splitlines()[-1]) >= 30
