"""Datasets and on-device synthetic generators."""
