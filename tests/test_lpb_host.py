"""Host logic of the batched node-partitioned mode (CPU): the lookahead a
scenario gets, its phase-1 nodes, and the capacity hints the scenario builders
give tw_lpb_load."""
import numpy as np
import pytest

from timewarp import scenarios
from timewarp.engine import EngineError, lpb_lookahead, lpb_short_link_destinations


def test_token_ring_lookahead_and_observer_phase():
    # ring links U[1 ms, 5 ms], observer links 0 µs (examples/token-ring/Main.hs:73-77)
    N = 16
    scn = scenarios.token_ring(n_nodes=N, n_replicas=8, launch_duration=5_000_000)
    L = lpb_lookahead(scn)
    assert 1000 <= L <= 5000
    assert L == int((scn.link_table[0::2] & 0x7FFFFFFF).min())
    # only the observer (node N) is fed by short links
    assert lpb_short_link_destinations(scn, L).tolist() == [N]


def test_hotspot_lookahead_and_caps():
    S = 32
    scn = scenarios.hotspot(n_senders=S, n_replicas=16, msg_num=10)
    L = lpb_lookahead(scn)
    assert L == int(scn.link_table.min()) and L >= 1000
    assert lpb_short_link_destinations(scn, L).size == 0
    caps = scn.meta["lp_inbox_cap"]
    assert caps.shape == (S + 2,)
    # senders light (<= 32: drained at the window start), the receiver heavy
    # (tw_lp_due) and able to hold every ping in flight
    assert (caps[:S] <= 32).all() and caps[S] > 32 and caps[S] <= 2048
    max_delay, send_delay = int(scn.link_table.max()), 1_000_000 // 1000
    assert caps[S] >= S * (max_delay // send_delay + 1)


def test_no_positive_delay_is_refused():
    scn = scenarios.ping_pong(n_replicas=4, round_trips=2)
    scn.link_table = np.zeros_like(scn.link_table)
    with pytest.raises(EngineError):
        lpb_lookahead(scn)


def test_bench_hotspot_defaults_to_lpb():
    import json
    import subprocess
    import sys
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--workload-key", "--config", "hotspot"],
                         check=True, capture_output=True, text=True).stdout
    assert json.loads(out)["bench_workload"].endswith(":geo=lpb")
