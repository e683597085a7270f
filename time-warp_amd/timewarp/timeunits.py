"""Time units and time specifications of MonadTimed, in integer microseconds.

Mirrors src/Control/TimeWarp/Timed/MonadTimed.hs:
  * ``mcs, ms, sec, minute, hour :: Int -> Microsecond``      (:253-258)
  * primed ``mcs' .. hour' :: Double -> Microsecond`` use Haskell ``round``
    (banker's rounding, = Python ``round``)                    (:261-266)
  * ``for``/``after`` are relative (``(+)``), ``till``/``at`` absolute
    (``const``), ``now = id``                                   (:278-299, 355-365)
  * time accumulators: ``for 10 minute 34 sec 52 ms`` sums the parts (:351-376)
"""
from __future__ import annotations

from dataclasses import dataclass


def mcs(n: int) -> int:
    return int(n)


def ms(n: int) -> int:
    return int(n) * 1000


def sec(n: int) -> int:
    return int(n) * 1_000_000


def minute(n: int) -> int:
    return int(n) * 60_000_000


def hour(n: int) -> int:
    return int(n) * 3_600_000_000


def mcs_(x: float) -> int:
    return int(round(x))


def ms_(x: float) -> int:
    return int(round(x * 1000))


def sec_(x: float) -> int:
    return int(round(x * 1_000_000))


def minute_(x: float) -> int:
    return int(round(x * 60_000_000))


def hour_(x: float) -> int:
    return int(round(x * 3_600_000_000))


def interval(*parts) -> int:
    """``interval 1 sec`` / ``interval 10 minute 34 sec``: sum of (n, unit) parts."""
    return _accumulate(parts)


def _accumulate(parts) -> int:
    if len(parts) == 1 and not callable(parts[0]):
        return int(parts[0])
    if len(parts) % 2:
        raise ValueError("time accumulator expects (n, unit) pairs or a single microsecond value")
    total = 0
    for n, unit in zip(parts[0::2], parts[1::2]):
        total += unit(n)
    return total


@dataclass(frozen=True)
class TimeSpec:
    """A ``RelativeToNow`` (MonadTimed.hs:66): relative offset or absolute point."""

    relative: bool
    us: int

    def resolve(self, now: int) -> int:
        """``max cur (rel cur)`` as applied by TimedT's wait (TimedT.hs:349)."""
        t = now + self.us if self.relative else self.us
        return max(now, t)


def for_(*parts) -> TimeSpec:
    return TimeSpec(True, _accumulate(parts))


after = for_


def till(*parts) -> TimeSpec:
    return TimeSpec(False, _accumulate(parts))


at = till

now = TimeSpec(True, 0)
