"""bench/Network measures from emulation traces.

The reference's network bench logs one line per measure event
(`logMeasure`, bench/Network/Common/Bench/Network/Commons.hs:121-171: PingSent
at the sender before `send`, PingReceived and PongSent at the receiver,
PongReceived at the sender) and its LogReader folds them into measures.csv
(bench/Network/LogReader/Main.hs:85-119): one row per message id with the
payload size and the four timestamps, "-" for a missing event, and no row for
an id with a repeated event.  Here the events are the hotspot scenario's
TRACE records (`Engine.trace`, or the oracle's trace log), with virtual time in
µs as the timestamp.
"""
from typing import Dict, Iterable, Tuple

from .scenarios import TAG_PING, TAG_PING_SENT, TAG_PONG, TAG_PONG_SENT

# MeasureEvent in declaration order (Commons.hs:121-127) and its Buildable
# rendering (:129-133), which is the csv header
EVENTS = ("PingSent", "PingReceived", "PongSent", "PongReceived")
EVENT_TEXT = {"PingSent": "• → ", "PingReceived": " → •",
              "PongSent": " ← •", "PongReceived": "• ← "}
TAG_EVENT = {TAG_PING_SENT: "PingSent", TAG_PING: "PingReceived", TAG_PONG_SENT: "PongSent",
             TAG_PONG: "PongReceived"}


def measures_from_trace(records: Iterable[Tuple[int, int, int, int]]) -> Dict[int, Dict[str, int]]:
    """records: (t, node, tag, val) in execution order, val = message id.
    Returns {msg_id: {event: t}}; an id with a repeated event maps to None
    (LogReader's `uniqMap` drops it)."""
    out: Dict[int, Dict[str, int]] = {}
    for t, _node, tag, val in records:
        ev = TAG_EVENT.get(int(tag))
        if ev is None:
            continue
        m = out.setdefault(int(val), {})
        if m is None:
            continue
        if ev in m:
            out[int(val)] = None
            continue
        m[ev] = int(t)
    return out


def format_measures_csv(measures: Dict[int, Dict[str, int]], size: int = 0) -> str:
    """measures.csv as LogReader prints it: rows sorted by id, each cell padded
    on the right to 7, 7, 18, 18, 18, 18 characters and joined with ","."""
    widths = (7, 7) + (18,) * len(EVENTS)

    def row(cells):
        return ",".join(c.ljust(w) for c, w in zip(cells, widths)) + "\n"

    lines = [row(["MsgId", "Size"] + [EVENT_TEXT[e] for e in EVENTS])]
    for mid in sorted(measures):
        m = measures[mid]
        if m is None:
            continue
        lines.append(row([str(mid), str(size)] + [str(m[e]) if e in m else "-" for e in EVENTS]))
    return "".join(lines)


def trace_tuples(recs) -> list:
    """Engine.trace records (TRACE_DTYPE) or oracle traces -> (t, node, tag, val) tuples."""
    if hasattr(recs, "dtype"):
        return [(int(r["t"]), int(r["node"]), int(r["tag"]), int(r["val"])) for r in recs]
    return [(int(t), int(n), int(k), int(v)) for t, n, k, v in recs]
