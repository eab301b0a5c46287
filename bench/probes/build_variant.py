"""Build an experiment copy of the extension with one kernel source patched, relinked as
``bench/variants/<name>.so``; a probe run with ``DALGO_EXT_LIB=bench/variants/<name>.so``
(dalgo/ops/_ext.py) loads it while the tree keeps one code path. Patches are literal
(old -> new) replacements that must match.

    python bench/probes/build_variant.py NAME csrc/kernels/X.hip 'old' 'new' ['old' 'new' ...]
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from dalgo import _build   # noqa: E402


def main(argv):
    name, src, pairs = argv[0], ROOT / argv[1], argv[2:]
    if len(pairs) % 2:
        raise SystemExit("patches come in (old, new) pairs")
    _build.build()
    text = src.read_text()
    for old, new in zip(pairs[::2], pairs[1::2]):
        if old not in text:
            raise SystemExit(f"patch does not match: {old[:60]!r}")
        text = text.replace(old, new, 1)
    out = ROOT / "bench" / "variants"
    out.mkdir(parents=True, exist_ok=True)
    vsrc = out / f"{name}_{src.name}"
    vsrc.write_text(text)
    obj = out / f"{name}_{src.stem}.o"
    hipcc = _build._hipcc()
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{_build.CSRC / 'include'}", f"-I{_build.CSRC}"]
    subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", *common, "-munsafe-fp-atomics", "-c", str(vsrc),
                    "-o", str(obj)], check=True)
    objs = [str(obj) if p.stem == src.stem else str(_build.BUILD / (p.stem + ".o"))
            for p in _build.kernel_sources()] + [str(_build.BUILD / "bindings.o")]
    _, _, tlib = _build._torch_paths()
    subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", *objs, "-o",
                    str(out / f"{name}.so"), f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip",
                    "-ltorch", f"-Wl,-rpath,{tlib}", f"-L{_build.ROCM / 'lib'}", "-lamdhip64",
                    "-Wl,--no-undefined"], check=True)
    vsrc.unlink()
    obj.unlink()
    print(f"[variant] {out / (name + '.so')}")


if __name__ == "__main__":
    main(sys.argv[1:])
