"""ctypes wrapper of the CPU TimedT restatement — TEST INFRASTRUCTURE ONLY.

May be imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the parity checker / CPU baseline.  The product package
(time-warp_amd/timewarp) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.join(os.path.dirname(_HERE), "time-warp_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from timewarp.abi import RESULT_DTYPE, RESULT_FIELDS, TwReplicaResult  # noqa: E402
from timewarp.scenario import Scenario  # noqa: E402

LIB_PATH = os.path.join(_HERE, "build", "libtw_oracle.so")

MODE_CANONICAL = 0
MODE_PQUEUE = 1
MODE_LIFO = 2        # canonical queue, equal timestamps in reverse insertion order (TW_TIE_LIFO)
MODE_SCRAMBLE = 3    # canonical queue, equal timestamps in scrambled order (TW_TIE_SCRAMBLE)
MODE_FORKFIRST = 5   # canonical queue, a forked child always the next pop (TW_TIE_FORKFIRST)


class TwoLiveDelays(C.Structure):
    _fields_ = [
        ("kind", C.c_void_p), ("lo", C.c_void_p), ("hi", C.c_void_p), ("seed", C.c_int64),
        ("record", C.c_void_p), ("record_depth", C.c_uint32), ("record_overflow", C.c_uint32),
    ]


class TwoTerm(C.Structure):
    _fields_ = [("t", C.c_int64), ("node", C.c_uint32), ("kind", C.c_uint32), ("val", C.c_int64)]


class TwoOpts(C.Structure):
    _fields_ = [
        ("mode", C.c_int), ("t_end", C.c_int64), ("max_events", C.c_uint64),
        ("live", C.POINTER(TwoLiveDelays)),
        ("terms", C.POINTER(TwoTerm)), ("terms_cap", C.c_size_t), ("terms_n", C.c_size_t),
        ("traces", C.POINTER(TwoTerm)), ("traces_cap", C.c_size_t), ("traces_n", C.c_size_t),
    ]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.two_run.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(TwoOpts), C.POINTER(TwReplicaResult),
                                 C.c_void_p]
        _lib.two_run_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_void_p,
                                       C.c_void_p]
        _lib.two_stdgen_draws.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_size_t]
        _lib.two_stdgen_next.argtypes = [C.c_int64, C.c_void_p, C.c_size_t, C.c_void_p]
        _lib.two_pqueue_order.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        _lib.two_pqueue_order.restype = C.c_size_t
    return _lib


@dataclass
class OracleRun:
    result: dict
    hashes: np.ndarray
    traces: List[tuple]
    terms: List[tuple]
    recorded_table: Optional[np.ndarray] = None


def run(scn: Scenario, replica: int = 0, mode: int = MODE_CANONICAL, live_seed: Optional[int] = None,
        record_depth: int = 0, t_end: int = (1 << 62), max_events: int = 0, trace_cap: int = 1 << 16,
        term_cap: int = 0) -> OracleRun:
    """Run one replica through the restatement; optionally with the live Delays RNG."""
    L = lib()
    d = scn.desc()
    o = TwoOpts()
    o.mode = mode
    o.t_end = t_end
    o.max_events = max_events
    traces = (TwoTerm * max(1, trace_cap))()
    o.traces = C.cast(traces, C.POINTER(TwoTerm))
    o.traces_cap = trace_cap
    terms = None
    if term_cap:
        terms = (TwoTerm * term_cap)()
        o.terms = C.cast(terms, C.POINTER(TwoTerm))
        o.terms_cap = term_cap
    live = None
    rec = None
    keep = []
    if live_seed is not None:
        live = TwoLiveDelays()
        for nm, arr, dt in (("kind", scn.live_kind, np.uint32), ("lo", scn.live_lo, np.int64),
                            ("hi", scn.live_hi, np.int64)):
            a = np.ascontiguousarray(arr, dtype=dt)
            keep.append(a)
            setattr(live, nm, a.ctypes.data)
        live.seed = live_seed
        if record_depth:
            rec = np.zeros((scn.topo.n_links, record_depth), np.uint32)
            live.record = rec.ctypes.data
            live.record_depth = record_depth
        o.live = C.pointer(live)
    res = TwReplicaResult()
    hashes = np.zeros(scn.n_nodes, np.uint64)
    rc = L.two_run(C.addressof(d), replica, C.byref(o), C.byref(res), hashes.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"two_run failed: {rc}")
    if live is not None and live.record_overflow:
        raise RuntimeError("record_depth too small for recorded link draws")
    tr = [(traces[i].t, traces[i].node, traces[i].kind, traces[i].val) for i in range(min(o.traces_n, trace_cap))]
    tm = []
    if terms is not None:
        tm = [(terms[i].t, terms[i].node, terms[i].kind, terms[i].val) for i in range(min(o.terms_n, term_cap))]
    result = {f: getattr(res, f) for f in RESULT_FIELDS}
    return OracleRun(result, hashes, tr, tm, rec)


def run_batch(scn: Scenario, r0: int = 0, r1: Optional[int] = None, mode: int = MODE_CANONICAL,
              threads: int = 1):
    """Replicas [r0, r1) on `threads` host threads; returns (results structured array, hashes)."""
    L = lib()
    r1 = scn.n_replicas if r1 is None else r1
    d = scn.desc()
    res = np.zeros(r1 - r0, RESULT_DTYPE)
    hashes = np.zeros((r1 - r0, scn.n_nodes), np.uint64)
    rc = L.two_run_batch(C.addressof(d), r0, r1, mode, threads, res.ctypes.data, hashes.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"two_run_batch failed: {rc}")
    return res, hashes


def stdgen_draws(seed: int, lo: int, hi: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.int64)
    lib().two_stdgen_draws(seed, lo, hi, out.ctypes.data, n)
    return out


def stdgen_next(seed: int, n: int):
    out = np.zeros(n, np.int32)
    s = np.zeros(2, np.int32)
    lib().two_stdgen_next(seed, out.ctypes.data, n, s.ctypes.data)
    return (int(s[0]), int(s[1])), out


def pqueue_order(ops) -> np.ndarray:
    """ops[i] >= 0: insert key ops[i] (payload i); -1: minView.  Returns popped payloads."""
    k = np.ascontiguousarray(ops, dtype=np.int64)
    out = np.zeros(len(k), np.int64)
    m = lib().two_pqueue_order(k.ctypes.data, len(k), out.ctypes.data)
    return out[:m]
