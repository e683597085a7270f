"""timewarp — MI355X-native batched TimedT emulator (host side).

Lowers MonadTimed/MonadDialog scenarios to thread programs (program.py,
scenarios.py), draws link tables from random-1.1 StdGen (stdgen.py) and runs
them on the HIP engine through the C ABI of include/timewarp.h (engine.py).
"""
from . import isa, timeunits  # noqa: F401
from .program import Code, Image, Label, Program  # noqa: F401
from .scenario import Scenario, Topology  # noqa: F401
from .timeunits import after, at, for_, hour, interval, mcs, minute, ms, now, sec, till  # noqa: F401
