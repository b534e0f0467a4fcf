"""How a run of optimizer steps is cut into multi-step HIP graph replays.

Every graph-replay boundary costs an idle gap on MI355X (~9 us), so steps are replayed in
groups of up to ``max_group`` steps per graph.  A freshly captured graph is also slow on its first
launches (upload, cold instruction caches), so a timed region should only replay graphs that
were already replayed before it.  ``tile(steps, warmup)`` picks one group size S (and at most one
remainder graph) for the ``steps`` timed steps such that the ``warmup`` steps can replay every
graph the timed region uses, ending with an S-group right before the timed region.

Example: 20 timed / 5 warmup steps -> S = 5: warmup [5], timed [5, 5, 5, 5] (one graph, four
replays); 200 / 20 -> S = 8: warmup [4, 8, 8], timed [8] * 25.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple


@dataclass(frozen=True)
class Tiling:
    group: int               # S: steps per graph replay in the timed region
    timed: Tuple[int, ...]   # group sizes of the timed replays (sum = steps)
    warm: Tuple[int, ...]    # group sizes of the warmup replays (sum = warmup)
    covered: bool            # every timed graph was replayed during warmup

    @property
    def sizes(self) -> List[int]:
        return sorted(set(self.timed) | set(self.warm))


def tile(steps: int, warmup: int, max_group: int = 8, exact: bool = False) -> Tiling:
    """``exact``: use group size ``max_group`` (capped at ``steps``) whatever the warmup covers."""
    steps, warmup = int(steps), int(warmup)
    if steps < 1 or warmup < 0:
        raise ValueError(f"need steps >= 1 and warmup >= 0 (got {steps}, {warmup})")
    best = None
    lo = min(max_group, steps) if exact else 1
    for s in range(min(max_group, steps), lo - 1, -1):
        r = steps % s
        need = s + r  # one replay of each timed graph; the S-group last
        replays = steps // s + (1 if r else 0)
        ok = warmup >= need
        key = (not ok, replays, -s)  # covered first, then fewest replays, then the larger group
        if best is None or key < best[0]:
            best = (key, s, r, ok)
    _, s, r, ok = best
    timed = [s] * (steps // s) + ([r] if r else [])
    if ok:
        rest = warmup - s - r
        warm = ([rest % s] if rest % s else []) + [s] * (rest // s) + ([r] if r else []) + [s]
    else:  # too few warmup steps to replay every timed graph first: plain groups
        warm = ([warmup % s] if warmup % s else []) + [s] * (warmup // s)
    return Tiling(s, tuple(timed), tuple(warm), ok)


def chunks(steps: int, group: int) -> List[int]:
    """Untimed steps as groups of ``group`` plus one remainder."""
    steps = int(steps)
    return [group] * (steps // group) + ([steps % group] if steps % group else [])


def count_pattern(size: int, every: int = 8) -> Tuple[bool, ...]:
    """Feature-count sampling inside one replay: its first step, then every ``every`` steps."""
    return tuple(i % every == 0 for i in range(int(size)))
