"""I/O helpers, Graph500 metrics and validation utilities."""
from .metrics import harmonic_mean, gteps, summarize_runs  # noqa: F401
from .validate import check_levels_against_oracle, levels_are_consistent, parents_are_valid  # noqa: F401
