"""Host binding of libtimewarp.so (the HIP engine) — the product path.

``Engine`` mirrors the reference runner ``runTimedT`` (TimedT.hs:293-304) for a
batch of replicas: ``load`` = build the TimedT value + ``emptyScenario``,
``run`` = ``launchTimedT`` to quiescence, results = final virtual time,
counters and per-node trace hashes.  Calls go through the C ABI of
include/timewarp.h with plain pointers (ctypes); there is no CPU fallback —
if the library or a GPU is missing this raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .abi import RESULT_DTYPE, TwLpState, TwStats, TwTableDraw
from .scenario import Scenario

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG_ROOT, "lib", "libtimewarp.so")
UNLIMITED = (1 << 64) - 1
T_INF = (1 << 63) - 1

EXPORTS = ["tw_create", "tw_comm_id", "tw_create_rank", "tw_ctx_info", "tw_lp_run", "tw_set_tie_mode", "tw_load", "tw_reset", "tw_run", "tw_read_results", "tw_read_hashes", "tw_read_final",
           "tw_last_launch_ms", "tw_destroy", "tw_strerror", "tw_version",
           "tw_lp_load", "tw_lp_window", "tw_lp_take_outbox", "tw_lp_inject", "tw_lp_results",
           "tw_set_trace", "tw_read_trace", "tw_tie_audit", "tw_set_counter_base", "tw_geometry",
           "tw_set_stream", "tw_lp_exchange_setup", "tw_lp_loop_begin", "tw_lp_tick", "tw_lp_tick_import",
           "tw_lp_tick_end", "tw_lp_progress", "tw_lp_run_windows", "tw_lpb_load", "tw_lpb_windows",
           "tw_draw_link_table", "tw_lpb_batch"]
GEOMETRIES = ("dense", "sparse", "half", "wave", "lp", "narrow", "lpb", "compact")  # TW_GEO_* order

# tw_trace_rec (include/timewarp.h)
TRACE_DTYPE = np.dtype([("t", np.int64), ("val", np.int64), ("node", np.uint32), ("tag", np.uint32)])

# tw_lp_record (include/timewarp.h)
LP_RECORD_DTYPE = np.dtype([("t_arr", np.int64), ("payload", np.int64), ("link", np.uint32),
                            ("kind", np.uint32), ("src", np.uint32), ("dst", np.uint32)])


class EngineError(RuntimeError):
    pass


_lib = None


def load_library(path: Optional[str] = None):
    """dlopen libtimewarp.so and declare the C signatures (no device call)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # TW_LIB selects an alternative in-tree build of the same ABI (A/B runs of
    # kernel variants on one GPU box); default lib/libtimewarp.so
    p = path or os.environ.get("TW_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise EngineError(f"HIP engine library missing: {p} (run __graft_entry__.build())")
    # One HIP runtime per process: torch's wheel bundles libamdhip64.so.7 under
    # the same soname as /opt/rocm's.  Loading torch first makes this library
    # bind to that copy, so torch streams/tensors (tw_set_stream, the RCCL
    # exchange buffers) and the engine share one runtime; loading the engine
    # first would leave torch without a usable device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(p)
    lib.tw_create.argtypes = [C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_void_p)]
    lib.tw_comm_id.argtypes = [C.c_void_p]
    lib.tw_create_rank.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]
    lib.tw_ctx_info.argtypes = [C.c_void_p] + [C.POINTER(C.c_int)] * 4
    lib.tw_lp_run.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(TwLpState)]
    lib.tw_set_tie_mode.argtypes = [C.c_void_p, C.c_uint32]
    lib.tw_load.argtypes = [C.c_void_p, C.c_void_p]
    lib.tw_reset.argtypes = [C.c_void_p]
    lib.tw_run.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.POINTER(TwStats)]
    lib.tw_read_results.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    lib.tw_read_hashes.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    lib.tw_read_final.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.tw_last_launch_ms.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    lib.tw_destroy.argtypes = [C.c_void_p]
    lib.tw_strerror.argtypes = [C.c_int]
    lib.tw_strerror.restype = C.c_char_p
    lib.tw_version.restype = C.c_char_p
    lib.tw_lp_load.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int64, C.c_uint32, C.c_uint32]
    lib.tw_lp_window.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_uint64)]
    lib.tw_lp_take_outbox.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.tw_lp_inject.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_int64)]
    lib.tw_lp_results.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
    lib.tw_set_trace.argtypes = [C.c_void_p, C.c_uint32]
    lib.tw_read_trace.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64)]
    lib.tw_tie_audit.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint32, C.POINTER(TwStats)]
    lib.tw_set_counter_base.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
    lib.tw_geometry.argtypes = [C.c_void_p]
    lib.tw_set_stream.argtypes = [C.c_void_p, C.c_void_p]
    lib.tw_lp_exchange_setup.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_uint32, C.c_void_p]
    for name in ("tw_lp_loop_begin", "tw_lp_tick", "tw_lp_tick_import", "tw_lp_tick_end"):
        getattr(lib, name).argtypes = [C.c_void_p]
    lib.tw_lp_progress.argtypes = [C.c_void_p, C.POINTER(TwLpState)]
    lib.tw_lp_run_windows.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(TwLpState)]
    lib.tw_lpb_load.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_uint32, C.c_uint32]
    lib.tw_lpb_windows.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    lib.tw_lpb_batch.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    lib.tw_draw_link_table.argtypes = [C.c_int, C.POINTER(TwTableDraw), C.c_void_p]
    for name in ("tw_create", "tw_comm_id", "tw_create_rank", "tw_ctx_info", "tw_lp_run", "tw_set_tie_mode", "tw_load", "tw_reset", "tw_run", "tw_read_results", "tw_read_hashes", "tw_read_final",
                 "tw_last_launch_ms", "tw_lp_load", "tw_lp_window", "tw_lp_take_outbox", "tw_lp_inject",
                 "tw_lp_results", "tw_set_trace", "tw_read_trace", "tw_tie_audit", "tw_set_counter_base",
                 "tw_geometry", "tw_set_stream", "tw_lp_exchange_setup", "tw_lp_loop_begin", "tw_lp_tick",
                 "tw_lp_tick_import", "tw_lp_tick_end", "tw_lp_progress", "tw_lp_run_windows", "tw_lpb_load",
                 "tw_lpb_windows", "tw_draw_link_table", "tw_lpb_batch"):
        getattr(lib, name).restype = C.c_int
    if path is None:
        _lib = lib
    return lib


def draw_link_table(n_replicas: int, drawn, lo, hi, link_depth: int = 1, drop_log2: int = 0,
                    seed_base: int = 0, device: int = 0) -> np.ndarray:
    """The scenario builders' StdGen delay draws on the GPU (tw_draw_link_table):
    replica r's generator mkStdGen(seed_base + r) walks the links with
    drawn[l] in ascending order, link_depth entries each (a randomR(lo, hi)
    delay, then a drop coin when drop_log2 > 0); other links hold lo[l].
    Returns the [n_links][link_depth][n_replicas] uint32 table tw_load takes,
    entry for entry the host draw of timewarp/stdgen.py."""
    drawn = np.ascontiguousarray(drawn, dtype=np.uint8)
    lo = np.ascontiguousarray(lo, dtype=np.int64)
    hi = np.ascontiguousarray(hi, dtype=np.int64)
    L = drawn.shape[0]
    if lo.shape != (L,) or hi.shape != (L,):
        raise ValueError("drawn, lo and hi need one entry per link")
    out = np.empty((L, int(link_depth), int(n_replicas)), dtype=np.uint32)
    spec = TwTableDraw(n_links=L, link_depth=int(link_depth), n_replicas=int(n_replicas), drop_log2=int(drop_log2),
                       seed_base=int(seed_base), drawn=drawn.ctypes.data, lo=lo.ctypes.data, hi=hi.ctypes.data)
    _check(load_library().tw_draw_link_table(int(device), C.byref(spec), out.ctypes.data), "tw_draw_link_table")
    return out


def _check(rc: int, what: str):
    if rc < 0:
        msg = load_library().tw_strerror(rc).decode()
        raise EngineError(f"{what} failed: {rc} ({msg})")


@dataclass
class RunStats:
    events: int
    sends: int
    delivered: int
    dropped: int
    undeliverable: int
    max_final_t: int
    replicas_done: int
    replicas_error: int
    launches: int
    kernel_ms: float
    wall_ms: float


COMM_ID_BYTES = 128  # TW_COMM_ID_BYTES


def comm_id() -> bytes:
    """A fresh RCCL job id (tw_comm_id): made by rank 0, handed to every rank
    (e.g. torch.distributed.broadcast_object_list) for Engine(comm=...)."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    _check(load_library().tw_comm_id(buf), "tw_comm_id")
    return bytes(buf)


class Engine:
    """A tw_ctx holding one loaded scenario: on one GPU (`device`), on several
    GPUs of this process (`devices`: replicas split into contiguous blocks,
    statistics all-reduced over the library's RCCL communicators), or as one
    rank of a multi-process job (`comm=(nranks, rank, job_id)` from comm_id():
    the library's RCCL communicator over the ranks)."""

    def __init__(self, device: int = 0, devices=None, comm=None):
        self.lib = load_library()
        ctx = C.c_void_p()
        if comm is not None:
            nranks, rank, jid = comm
            idb = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(jid)
            _check(self.lib.tw_create_rank(int(device), int(nranks), int(rank), idb, C.byref(ctx)), "tw_create_rank")
        else:
            devs = list(devices) if devices is not None else [int(device)]
            arr = (C.c_int * len(devs))(*devs)
            _check(self.lib.tw_create(arr, len(devs), C.byref(ctx)), "tw_create")
        self.ctx = ctx
        self.scn: Optional[Scenario] = None

    def info(self):
        """(devices of this process, ranks of the job, global rank of the
        first device, transport: 0 none, 1 RCCL, 2 device copies)."""
        v = [C.c_int() for _ in range(4)]
        _check(self.lib.tw_ctx_info(self.ctx, *[C.byref(x) for x in v]), "tw_ctx_info")
        return tuple(x.value for x in v)

    def close(self):
        if self.ctx:
            self.lib.tw_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, scn: Scenario, geometry: Optional[str] = None) -> "Engine":
        """Upload the scenario.  `geometry` picks the kernel layout: "dense"
        (256 replicas per workgroup, 16-entry on-chip queue), "narrow" (the
        dense layout, one 64-replica wave per workgroup), "sparse" (16
        replicas per workgroup, 768-entry on-chip queue), "wave" (a
        wavefront per replica), "half" (the dense layout as two 32-lane waves
        per SIMD; an experiment), "lpb" (every (node, replica) a logical
        process: `load_lpb`) or None = the library's choice (wave for <=
        4096 replicas, narrow below 65536, else dense; env TW_GEOMETRY)."""
        if geometry == "lpb":
            return self.load_lpb(scn)
        d = scn.desc()
        old = os.environ.get("TW_GEOMETRY")
        if geometry is not None:
            if geometry not in ("dense", "sparse", "half", "wave", "narrow", "compact"):
                raise ValueError(f"geometry must be 'dense', 'sparse', 'half', 'wave', 'narrow' or 'compact', "
                                 f"not {geometry!r}")
            os.environ["TW_GEOMETRY"] = geometry
        try:
            _check(self.lib.tw_load(self.ctx, C.addressof(d)), "tw_load")
        finally:
            if geometry is not None:
                if old is None:
                    os.environ.pop("TW_GEOMETRY", None)
                else:
                    os.environ["TW_GEOMETRY"] = old
        self.scn = scn
        return self

    def load_lpb(self, scn: Scenario, lookahead_us: Optional[int] = None, node_inbox_cap=None,
                 outbox_cap: Optional[int] = None) -> "Engine":
        """Batched node-partitioned mode (tw_lpb_load): the replicas' nodes run
        as logical processes in conservative windows of `lookahead_us` (default:
        the smallest link delay of the table), so a replica's events run in
        parallel across its nodes.  Per-lane capacities come from the
        scenario's meta (lp_max_slots, lp_queue_capacity, lp_inbox_cap: one
        value or one per node, lp_outbox_cap), like `lp_scenario`."""
        import copy

        if scn.link_table is None:
            raise EngineError("load_lpb: the scenario needs a link table (its smallest delay is the lookahead)")
        if lookahead_us is None:
            lookahead_us = lpb_lookahead(scn)
        m = scn.meta
        s = copy.copy(scn)
        s.max_slots = int(m.get("lp_max_slots", 64))
        s.queue_capacity = int(m.get("lp_queue_capacity", 128))
        s.run_capacity = 0
        cap = node_inbox_cap if node_inbox_cap is not None else m.get("lp_inbox_cap", 32)
        caps = np.ascontiguousarray(np.broadcast_to(np.asarray(cap, np.uint32), (scn.n_nodes,)), dtype=np.uint32)
        if outbox_cap is None:
            outbox_cap = int(m.get("lp_outbox_cap", min(1 << 27, max(1 << 16, 8 * scn.n_nodes * scn.n_replicas))))
        d = s.desc()
        _check(self.lib.tw_lpb_load(self.ctx, C.addressof(d), int(lookahead_us), caps.ctypes.data, 32,
                                    int(outbox_cap)), "tw_lpb_load")
        self.scn = scn
        self.lookahead_us = int(lookahead_us)
        return self

    def lpb_windows(self):
        """(windows, ticks) of the last batched-LP run."""
        w, t = C.c_uint64(), C.c_uint64()
        _check(self.lib.tw_lpb_windows(self.ctx, C.byref(w), C.byref(t)), "tw_lpb_windows")
        return int(w.value), int(t.value)

    def lpb_batch(self):
        """(batched, due): batched-LP due records since the last reset that ran
        data-parallel in tw_lp_due, and all due records (tw_lpb_batch)."""
        b, d = C.c_uint64(), C.c_uint64()
        _check(self.lib.tw_lpb_batch(self.ctx, C.byref(b), C.byref(d)), "tw_lpb_batch")
        return int(b.value), int(d.value)

    def geometry(self) -> str:
        """The kernel geometry tw_load chose (GEOMETRIES)."""
        g = self.lib.tw_geometry(self.ctx)
        _check(g, "tw_geometry")
        return GEOMETRIES[g]

    def reset(self) -> "Engine":
        """Back to t=0 on the device-resident tables (no host upload)."""
        _check(self.lib.tw_reset(self.ctx), "tw_reset")
        return self

    def run(self, t_end: int = T_INF, max_events: int = UNLIMITED) -> RunStats:
        st = TwStats()
        _check(self.lib.tw_run(self.ctx, t_end, max_events, C.byref(st)), "tw_run")
        return RunStats(**{f: getattr(st, f) for f, _ in TwStats._fields_ if f != "reserved"})

    def tie_audit(self, probes: int = 2, t_end: int = T_INF, max_events: int = UNLIMITED) -> RunStats:
        """Run every replica under `probes` tie-order probes (reverse and
        scrambled order of equal-timestamp events) and then canonically;
        results()['tie_flags'] bit p marks replicas whose outputs differ under
        probe p (they depend on TimedT's pqueue tie order, TimedT.hs:100-104).
        The canonical run's results stay loaded."""
        st = TwStats()
        _check(self.lib.tw_tie_audit(self.ctx, int(t_end), int(max_events), int(probes), C.byref(st)),
               "tw_tie_audit")
        return RunStats(**{f: getattr(st, f) for f, _ in TwStats._fields_ if f != "reserved"})

    TIE_MODES = {"fifo": 0, "lifo": 1, "scramble": 2, "pqueue": 3, "forkfirst": 4}  # TW_TIE_*

    def set_tie_mode(self, mode: str) -> "Engine":
        """Equal-timestamp order of later runs: "fifo" (the engine's (t, seq)),
        the audit probes "lifo" / "scramble", or "pqueue": TimedT's own order
        (pqueue's MinQueue by timestamp only, TimedT.hs:100-104, with the
        throwTo rebuild of TimedT.hs:361-368), wave geometry only, or
        "forkfirst": fifo with a forked child always the next pop (pqueue's
        held-minimum rule; the replica kernels run it in place), lane-per-
        replica geometries only."""
        _check(self.lib.tw_set_tie_mode(self.ctx, self.TIE_MODES[mode]), "tw_set_tie_mode")
        return self

    def set_counter_base(self, seq0: int, tid0: int = 1) -> "Engine":
        """Testing hook: start the 32-bit insertion / thread counters at these
        values from the next reset on (TW_REP_ERR_COUNTER guard)."""
        _check(self.lib.tw_set_counter_base(self.ctx, int(seq0), int(tid0)), "tw_set_counter_base")
        return self

    def results(self) -> np.ndarray:
        out = np.zeros(self.scn.n_replicas, RESULT_DTYPE)
        _check(self.lib.tw_read_results(self.ctx, out.ctypes.data, out.shape[0]), "tw_read_results")
        return out

    def hashes(self) -> np.ndarray:
        out = np.zeros((self.scn.n_replicas, self.scn.n_nodes), np.uint64)
        _check(self.lib.tw_read_hashes(self.ctx, out.ctypes.data, out.size), "tw_read_hashes")
        return out

    def set_trace(self, cap: int) -> "Engine":
        """Record up to `cap` TRACE records per replica from the next reset on."""
        _check(self.lib.tw_set_trace(self.ctx, int(cap)), "tw_set_trace")
        self._trace_cap = int(cap)
        return self

    def trace(self, replica: int, cap: int = 1 << 20):
        """(records, n_emitted): a replica's TRACE records in execution order
        (TRACE_DTYPE), truncated at the trace capacity."""
        buf = np.zeros(cap, TRACE_DTYPE)
        n = C.c_uint64()
        _check(self.lib.tw_read_trace(self.ctx, int(replica), buf.ctypes.data, cap, C.byref(n)), "tw_read_trace")
        return buf[:min(int(n.value), cap, getattr(self, "_trace_cap", 0))].copy(), int(n.value)

    def launch_ms(self) -> np.ndarray:
        buf = np.zeros(1 << 16, np.float64)
        n = self.lib.tw_last_launch_ms(self.ctx, buf.ctypes.data, buf.shape[0])
        _check(n, "tw_last_launch_ms")
        return buf[:n].copy()


def lpb_lookahead(scn: Scenario) -> int:
    """The batched mode's window length: the smallest positive link delay over
    every replica and ordinal.  Links shorter than it (a 0 µs link into a sink,
    e.g. token ring's observer) make their destination a phase-1 node of every
    window; tw_lpb_load refuses a short link out of such a node."""
    if scn.link_table is None:
        raise EngineError("load_lpb: the scenario needs a link table (its smallest delay is the lookahead)")
    dmin = (scn.link_table & np.uint32(0x7FFFFFFF)).min(axis=(1, 2))
    pos = dmin[dmin > 0]
    if pos.size == 0:
        raise EngineError("load_lpb: no link with a positive delay (no lookahead)")
    return int(pos.min())


def lpb_short_link_destinations(scn: Scenario, lookahead_us: int) -> np.ndarray:
    """Nodes fed by a link shorter than the lookahead (the phase-1 nodes
    tw_lpb_load derives on the device side), for inspection and tests."""
    dmin = (scn.link_table & np.uint32(0x7FFFFFFF)).min(axis=(1, 2))
    return np.unique(scn.topo.dst[dmin < lookahead_us]).astype(np.int64)


def run_scenario(scn: Scenario, device: int = 0, t_end: int = T_INF, max_events: int = UNLIMITED,
                 geometry: Optional[str] = None):
    """Load + run to quiescence; returns (stats, results, hashes)."""
    with Engine(device) as e:
        e.load(scn, geometry=geometry)
        st = e.run(t_end, max_events)
        return st, e.results(), e.hashes()


class LPEngine(Engine):
    """One context of a node-partitioned run (config 4): owns nodes
    [lp_begin, lp_begin + lp_count) of a single scenario (split over
    `devices` when given; a rank's share of a job with `comm`)."""

    def __init__(self, scn: Scenario, lp_begin: int, lp_count: int, lookahead_us: int, device: int = 0,
                 inbox_cap: int = 16, outbox_cap: int = 1 << 22, devices=None, comm=None):
        super().__init__(device, devices=devices, comm=comm)
        d = scn.desc()
        _check(self.lib.tw_lp_load(self.ctx, C.addressof(d), lp_begin, lp_count, lookahead_us, inbox_cap,
                                   outbox_cap), "tw_lp_load")
        self.scn, self.lp_begin, self.lp_count = scn, lp_begin, lp_count
        self.outbox_cap = outbox_cap

    def window(self, t_end_excl: int):
        nt, nf = C.c_int64(), C.c_uint64()
        _check(self.lib.tw_lp_window(self.ctx, t_end_excl, C.byref(nt), C.byref(nf)), "tw_lp_window")
        return nt.value, nf.value

    def take_outbox(self) -> np.ndarray:
        n = C.c_size_t()
        buf = np.zeros(self.outbox_cap, LP_RECORD_DTYPE)
        _check(self.lib.tw_lp_take_outbox(self.ctx, buf.ctypes.data, buf.shape[0], C.byref(n)), "tw_lp_take_outbox")
        return buf[: n.value].copy()

    def inject(self, recs: np.ndarray) -> int:
        recs = np.ascontiguousarray(recs, dtype=LP_RECORD_DTYPE)
        nt = C.c_int64()
        _check(self.lib.tw_lp_inject(self.ctx, recs.ctypes.data if recs.size else None, recs.shape[0],
                                     C.byref(nt)), "tw_lp_inject")
        return nt.value

    # ---- device-driven windows (tw_lp_tick ...): no host round trip per window
    def set_stream(self, hip_stream: int):
        """Run every later kernel on the caller's HIP stream (0: the context's own)."""
        _check(self.lib.tw_set_stream(self.ctx, C.c_void_p(hip_stream or None)), "tw_set_stream")
        return self

    def exchange_setup(self, world: int, rank: int, starts, send_ptr: int = 0, recv_ptr: int = 0, cap: int = 0,
                       red_ptr: int = 0):
        """starts: world + 1 node boundaries; buffers are device pointers
        (world * (cap + 1) * 32 bytes each; red: 4 int64)."""
        st = np.ascontiguousarray(starts, dtype=np.uint32)
        _check(self.lib.tw_lp_exchange_setup(self.ctx, world, rank, st.ctypes.data, C.c_void_p(send_ptr or None),
                                             C.c_void_p(recv_ptr or None), cap, C.c_void_p(red_ptr or None)),
               "tw_lp_exchange_setup")
        return self

    def exchange_tensors(self, world: int, rank: int, starts, send, recv, cap: int, red):
        """exchange_setup over torch device tensors (the RCCL buffers); the
        engine then runs on torch's current stream, where the collectives go."""
        import torch

        cur = torch.cuda.current_stream(send.device).cuda_stream
        if not cur:
            # the legacy default stream: tw_set_stream(NULL) would mean the
            # context's own (non-blocking) stream, unordered with torch's work
            raise EngineError("exchange_tensors: run under a non-default torch stream (torch.cuda.stream(s))")
        self.set_stream(cur)
        self._ex_keep = (send, recv, red)  # the library holds raw pointers
        return self.exchange_setup(world, rank, starts, send.data_ptr(), recv.data_ptr(), cap, red.data_ptr())

    def loop_begin(self):
        _check(self.lib.tw_lp_loop_begin(self.ctx), "tw_lp_loop_begin")
        return self

    def tick(self):
        _check(self.lib.tw_lp_tick(self.ctx), "tw_lp_tick")

    def tick_import(self):
        _check(self.lib.tw_lp_tick_import(self.ctx), "tw_lp_tick_import")

    def tick_end(self):
        _check(self.lib.tw_lp_tick_end(self.ctx), "tw_lp_tick_end")

    def progress(self) -> TwLpState:
        st = TwLpState()
        _check(self.lib.tw_lp_progress(self.ctx, C.byref(st)), "tw_lp_progress")
        return st

    def run_lp(self, max_ticks: int = 1 << 22) -> TwLpState:
        """The whole window loop from t = 0 (after reset) over every device
        and rank of the context, the exchange owned by the library
        (tw_lp_run: RCCL send/recv of record blocks, all-reduce(min) of the
        window words)."""
        st = TwLpState()
        _check(self.lib.tw_lp_run(self.ctx, int(max_ticks), C.byref(st)), "tw_lp_run")
        return st

    def run_windows(self, max_ticks: int = 1 << 20) -> TwLpState:
        """Single context: the whole window loop on the device, one host
        synchronisation per 16 ticks."""
        st = TwLpState()
        _check(self.lib.tw_lp_run_windows(self.ctx, max_ticks, C.byref(st)), "tw_lp_run_windows")
        return st

    def lp_results(self):
        agg = np.zeros(1, RESULT_DTYPE)
        h = np.zeros(self.scn.n_nodes, np.uint64)
        _check(self.lib.tw_lp_results(self.ctx, agg.ctypes.data, h.ctypes.data, h.shape[0]), "tw_lp_results")
        return agg[0], h


def lp_scenario(scn: Scenario, max_slots: int = 32, queue_capacity: int = 64) -> Scenario:
    """Per-logical-process capacities (each lane holds one node's threads)."""
    import copy

    s = copy.copy(scn)
    s.max_slots, s.queue_capacity, s.run_capacity = max_slots, queue_capacity, 0
    return s


def _combine(engines, n_nodes: int):
    """Aggregate of the contexts' results: max times, summed counts, summed hashes."""
    agg, hashes = None, np.zeros(n_nodes, np.uint64)
    for e in engines:
        a, h = e.lp_results()
        hashes += h
        if agg is None:
            agg = a.copy()
        else:
            agg["final_t"] = max(agg["final_t"], a["final_t"])
            for f in ("events", "delivered", "dropped", "undeliverable", "threads"):
                agg[f] += a[f]
            agg["main_exc"] = max(agg["main_exc"], a["main_exc"])
            agg["status"] = max(agg["status"], a["status"])
    return agg, hashes


def run_partitioned(scn: Scenario, parts: int = 1, lookahead_us: Optional[int] = None, device: int = 0,
                    max_windows: int = 1 << 20):
    """Run one scenario node-partitioned over `parts` contexts in this process
    (records between contexts are routed on the host, exactly what the RCCL
    all-to-all does between GPUs).  Returns (aggregate result, node hashes,
    windows)."""
    L = int(lookahead_us if lookahead_us is not None else scn.meta["lookahead_us"])
    s = lp_scenario(scn)
    N = scn.n_nodes
    bounds = [(i * N // parts, (i + 1) * N // parts) for i in range(parts)]
    engines = [LPEngine(s, b0, b1 - b0, L, device) for b0, b1 in bounds]
    starts = np.array([b0 for b0, _ in bounds])
    try:
        T, windows = 0, 0
        while T < T_INF and windows < max_windows:
            nexts, outs = [], []
            for e in engines:
                nt, nf = e.window(T + L)
                nexts.append(nt)
                outs.append(e.take_outbox() if nf else None)
            allrec = [o for o in outs if o is not None and o.size]
            if allrec:
                recs = np.concatenate(allrec)
                owner = np.searchsorted(starts, recs["dst"], side="right") - 1
                for i, e in enumerate(engines):
                    mine = recs[owner == i]
                    if mine.size:
                        nexts[i] = min(nexts[i], e.inject(mine))
            T = min(nexts)
            windows += 1
        agg, hashes = _combine(engines, N)
        return agg, hashes, windows
    finally:
        for e in engines:
            e.close()


def run_partitioned_device(scn: Scenario, parts: int = 1, lookahead_us: Optional[int] = None, device: int = 0,
                           cap: int = 1 << 16, check_every: int = 16, max_ticks: int = 1 << 20):
    """The device-driven window loop (tw_lp_tick ...) over `parts` contexts of
    one process on one GPU.  Between the contexts' ticks, the block exchange an
    RCCL all-to-all does between GPUs is done with device copies, and the
    all-reduce(min) of the reduction words with a device min: everything stays
    on one stream, with one host synchronisation per `check_every` ticks.
    parts == 1 uses tw_lp_run_windows.  Returns (aggregate, node hashes,
    windows, ticks)."""
    import torch

    L = int(lookahead_us if lookahead_us is not None else scn.meta["lookahead_us"])
    s = lp_scenario(scn)
    N = scn.n_nodes
    bounds = [(i * N // parts, (i + 1) * N // parts) for i in range(parts)]
    starts = np.array([b0 for b0, _ in bounds] + [N], dtype=np.uint32)
    engines = [LPEngine(s, b0, b1 - b0, L, device) for b0, b1 in bounds]
    try:
        for e in engines:
            e.reset()
        if parts == 1:
            e = engines[0].loop_begin()
            st = e.run_windows(max_ticks)
            agg, hashes = _combine(engines, N)
            return agg, hashes, st.windows, st.ticks
        dev = torch.device("cuda", device)
        stream = torch.cuda.Stream(dev)  # not the legacy default stream (cuda_stream 0)
        ctx = torch.cuda.stream(stream)
        ctx.__enter__()
        blk = (cap + 1) * 32
        send = [torch.zeros(parts * blk, dtype=torch.uint8, device=dev) for _ in range(parts)]
        recv = [torch.zeros(parts * blk, dtype=torch.uint8, device=dev) for _ in range(parts)]
        red = [torch.zeros(4, dtype=torch.int64, device=dev) for _ in range(parts)]
        for g, e in enumerate(engines):
            e.set_stream(stream.cuda_stream)
            e.exchange_setup(parts, g, starts, send[g].data_ptr(), recv[g].data_ptr(), cap, red[g].data_ptr())
            e.loop_begin()
        ticks = 0
        while ticks < max_ticks:
            for _ in range(check_every):
                for e in engines:
                    e.tick()
                for g in range(parts):        # all-to-all: block g of src -> block src of g
                    for src in range(parts):
                        recv[g][src * blk:(src + 1) * blk].copy_(send[src][g * blk:(g + 1) * blk])
                for e in engines:
                    e.tick_import()
                m = torch.stack(red).min(dim=0).values   # all-reduce(min)
                for r in red:
                    r.copy_(m)
                for e in engines:
                    e.tick_end()
            ticks += check_every
            st = engines[0].progress()
            if st.err or any(e.progress().err for e in engines[1:]):
                raise EngineError(f"device window loop: overflow bits {st.err}")
            if st.done:
                break
        stream.synchronize()
        ctx.__exit__(None, None, None)
        agg, hashes = _combine(engines, N)
        return agg, hashes, st.windows, st.ticks
    finally:
        for e in engines:
            e.close()
