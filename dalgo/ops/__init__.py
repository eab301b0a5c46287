"""Kernel wrappers. GPU tensors -> gfx950 HIP kernels (fail loudly if the
extension is missing); CPU tensors -> torch reference implementations."""
from dalgo.ops._ext import NativeUnavailable, available  # noqa: F401
