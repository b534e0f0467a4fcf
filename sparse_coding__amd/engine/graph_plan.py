"""How a run of optimizer steps is cut into multi-step HIP graph replays.

Every graph-replay boundary costs an idle gap on MI355X (~9 us and more), so steps are replayed in
groups of up to ``max_group`` steps per graph and ``tile(steps, warmup)`` picks the group size S (and
at most one remainder graph) that needs the FEWEST replays for the ``steps`` timed steps; among equal
counts it prefers a tiling whose every graph the ``warmup`` steps can replay first (ending with an
S-group right before the timed region), then the larger group.  Round 4 preferred coverage first (a
freshly captured graph ran slow on its first launches); since every graph is uploaded right after
capture (``hipGraphUpload``), the driver's 20 / 5 command measured faster with two 10-step replays
(the timed graph not replayed in warmup) than with four covered 5-step replays: 0.3008 vs 0.3059
ms/step median of six interleaved runs, 0.2935 vs 0.2969 of three on another box
(profiles/r5/batch20/, batch6/).

Example: 20 timed / 5 warmup steps -> S = 10: warmup [5] (its own graph), timed [10, 10];
200 / 20 -> S = 10: warmup [10, 10], timed [10] * 20.
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


def tile(steps: int, warmup: int, max_group: int = 10, exact: bool = False) -> Tiling:
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
        key = (replays, not ok, -s)  # fewest replays, then covered, then the larger group
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
