"""Algorithms (the reference scripts' driver loops as SPMD trainers)."""
