"""Runtime, collectives, sharding and launch helpers."""
