"""Rank-spec parsing for ``%%rank``.

Reference: ``magic.py:1679-1715`` accepts ``[0,1,2]`` and ``[0-2]`` and silently returns ``[]``
for anything not bracketed.  This parser accepts the same forms plus mixtures (``[0-2,5]``),
bare forms (``0,1`` / ``0-3``), ``*``/``all``, and reports malformed specs instead of
swallowing them.
"""
from __future__ import annotations

from typing import List, Optional


class RankSpecError(ValueError):
    pass


def parse_ranks(spec: str, world_size: Optional[int] = None, strict: bool = False) -> List[int]:
    """Parse a rank spec into a sorted, de-duplicated list.

    Out-of-range ranks are dropped (as the reference does, magic.py:1715) unless ``strict``.
    """
    s = spec.strip()
    if s.startswith("[") and s.endswith("]"):
        s = s[1:-1]
    elif s.startswith("[") or s.endswith("]"):
        raise RankSpecError(f"unbalanced brackets in rank spec {spec!r}")
    s = s.strip()
    if not s:
        raise RankSpecError("empty rank spec")
    if s in ("*", "all"):
        if world_size is None:
            raise RankSpecError("'all' needs a known world size")
        return list(range(world_size))
    out = set()
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part[1:]:
            a, b = part.split("-", 1) if not part.startswith("-") else (part, "")
            try:
                lo, hi = int(a), int(b)
            except ValueError:
                raise RankSpecError(f"bad range {part!r} in rank spec {spec!r}") from None
            if hi < lo:
                raise RankSpecError(f"empty range {part!r}")
            out.update(range(lo, hi + 1))
        else:
            try:
                out.add(int(part))
            except ValueError:
                raise RankSpecError(f"bad rank {part!r} in rank spec {spec!r}") from None
    ranks = sorted(out)
    if world_size is not None:
        bad = [r for r in ranks if not 0 <= r < world_size]
        if bad and strict:
            raise RankSpecError(f"ranks {bad} out of range for world size {world_size}")
        ranks = [r for r in ranks if 0 <= r < world_size]
    return ranks


def format_ranks(ranks: List[int]) -> str:
    """Compact form: [0,1,2,5] -> '0-2,5'."""
    if not ranks:
        return ""
    rs = sorted(set(ranks))
    parts = []
    start = prev = rs[0]
    for r in rs[1:]:
        if r == prev + 1:
            prev = r
            continue
        parts.append(f"{start}-{prev}" if prev > start else str(start))
        start = prev = r
    parts.append(f"{start}-{prev}" if prev > start else str(start))
    return ",".join(parts)
