"""Utilities shared by the coordinator and the workers (no torch imports at module level)."""
from .ranks import RankSpecError, format_ranks, parse_ranks

__all__ = ["RankSpecError", "format_ranks", "parse_ranks"]
