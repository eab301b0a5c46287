"""Philox mirror, observability, config and checkpoint helpers."""
