"""Partitioning, communicators and process-level runtime."""
from .partition import Partition  # noqa: F401
from .runtime import Runtime, init_runtime, run_virtual_ranks  # noqa: F401
