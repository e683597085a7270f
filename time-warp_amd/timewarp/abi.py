"""ctypes mirror of include/timewarp.h structs (no torch types cross the ABI)."""
from __future__ import annotations

import ctypes as C

from . import isa


class TwScenarioDesc(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32),
        ("n_replicas", C.c_uint32),
        ("n_nodes", C.c_uint32),
        ("n_insns", C.c_uint32),
        ("insns", C.c_void_p),
        ("n_consts", C.c_uint32),
        ("consts", C.c_void_p),
        ("main_pc", C.c_uint32),
        ("main_node", C.c_uint32),
        ("n_listener_sets", C.c_uint32),
        ("n_msg_kinds", C.c_uint32),
        ("listener_pc", C.c_void_p),
        ("n_links", C.c_uint32),
        ("out_off", C.c_void_p),
        ("link_dst", C.c_void_p),
        ("link_rev", C.c_void_p),
        ("link_depth", C.c_uint32),
        ("link_table", C.c_void_p),
        ("node_vars", C.c_void_p),
        ("main_regs", C.c_void_p),
        ("node_listen", C.c_void_p),
        ("max_slots", C.c_uint32),
        ("queue_capacity", C.c_uint32),
        ("near_horizon_us", C.c_int64),
        ("max_timeouts", C.c_uint32),
        ("run_capacity", C.c_uint32),
        ("max_frames", C.c_uint32),
        ("msg_bytes", C.c_void_p),
        ("link_bw", C.c_void_p),
    ]


class TwReplicaResult(C.Structure):
    _fields_ = [
        ("final_t", C.c_int64),
        ("events", C.c_uint64),
        ("delivered", C.c_uint64),
        ("dropped", C.c_uint64),
        ("undeliverable", C.c_uint64),
        ("status", C.c_uint32),
        ("main_exc", C.c_uint32),
        ("threads", C.c_uint64),
        ("tie_flags", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class TwStats(C.Structure):
    _fields_ = [
        ("events", C.c_uint64),
        ("sends", C.c_uint64),
        ("delivered", C.c_uint64),
        ("dropped", C.c_uint64),
        ("undeliverable", C.c_uint64),
        ("max_final_t", C.c_int64),
        ("replicas_done", C.c_uint32),
        ("replicas_error", C.c_uint32),
        ("launches", C.c_uint32),
        ("reserved", C.c_uint32),
        ("kernel_ms", C.c_double),
        ("wall_ms", C.c_double),
    ]


# the fields a run produces (tie_flags is set by tw_tie_audit only)
class TwLpState(C.Structure):
    """tw_lp_state: the device-driven window loop's progress."""
    _fields_ = [
        ("windows", C.c_uint64),
        ("ticks", C.c_uint64),
        ("t", C.c_int64),
        ("done", C.c_uint32),
        ("err", C.c_uint32),
    ]


class TwTableDraw(C.Structure):
    """tw_table_draw: a link-table draw on the GPU (tw_draw_link_table)."""
    _fields_ = [
        ("n_links", C.c_uint32),
        ("link_depth", C.c_uint32),
        ("n_replicas", C.c_uint32),
        ("drop_log2", C.c_int32),
        ("seed_base", C.c_int64),
        ("drawn", C.c_void_p),
        ("lo", C.c_void_p),
        ("hi", C.c_void_p),
    ]


RESULT_FIELDS = ["final_t", "events", "delivered", "dropped", "undeliverable", "status", "main_exc", "threads"]

# numpy dtype with the same layout as tw_replica_result (for bulk reads)
import numpy as _np  # noqa: E402

RESULT_DTYPE = _np.dtype([
    ("final_t", _np.int64), ("events", _np.uint64), ("delivered", _np.uint64),
    ("dropped", _np.uint64), ("undeliverable", _np.uint64), ("status", _np.uint32),
    ("main_exc", _np.uint32), ("threads", _np.uint64), ("tie_flags", _np.uint32), ("reserved", _np.uint32),
])
assert RESULT_DTYPE.itemsize == C.sizeof(TwReplicaResult)
assert isa.ABI_VERSION == 4
