"""Build an A/B variant of the extension: the given kernel sources recompiled with extra
preprocessor flags, linked with the other objects of the in-tree build into
``dalgo/_xp_<name>.so`` (load it with DALGO_EXT_LIB=...). Timing experiments only.

    python bench/probes/build_variant.py NAME kmeans -DKM_XP_FOO [...]

BV_SRC_<stem>=path compiles that file instead of csrc/kernels/<stem>.hip (e.g. an older
revision: git show HEAD~1:csrc/kernels/kmeans.hip > /tmp/old.hip).
"""
import os
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from dalgo import _build as B   # noqa: E402


def main():
    name, stems, flags = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
    B.build()
    objs = []
    for src in B.kernel_sources():
        if src.stem in stems:
            obj = B.BUILD / f"{src.stem}.xp_{name}.o"
            B._run([B._hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-fPIC", "-std=c++17",
                    f"-I{B.CSRC / 'include'}", f"-I{B.CSRC}", "-munsafe-fp-atomics", *flags,
                    "-c", os.environ.get(f"BV_SRC_{src.stem}", src), "-o", obj], False)
            objs.append(obj)
        else:
            objs.append(B.BUILD / f"{src.stem}.o")
    objs.append(B.BUILD / "bindings.o")
    tdir, tinc, tlib = B._torch_paths()
    out = B.ROOT / "dalgo" / f"_xp_{name}.so"
    B._run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-o", out,
            f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch",
            f"-Wl,-rpath,{tlib}", f"-L{B.ROCM / 'lib'}", "-lamdhip64", "-Wl,--no-undefined"], False)
    print(out)


if __name__ == "__main__":
    main()
