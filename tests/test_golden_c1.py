"""Config 1 (BASELINE.json): the 16-node token ring with live mkStdGen 0 Delays.

The fixture (tests/golden/make_golden.py) pins the oracle run; the recorded
per-link draws replayed as a link table must give the identical run
(record-replay = the reference's per-call draws)."""
import json
import os

import numpy as np

from timewarp import scenarios

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "token_ring_c1.json")))


def c1_table_scenario():
    scn = scenarios.token_ring(n_nodes=16, n_replicas=1, launch_duration=20_000_000,
                               link_depth=GOLD["record_depth"])
    tab = np.array(GOLD["recorded_table"], dtype=np.uint32)  # [link][depth]
    scn.link_table = np.ascontiguousarray(tab[:, :, None])
    return scn


def test_c1_live_matches_fixture(oracle_mod):
    scn = scenarios.token_ring(n_nodes=16, n_replicas=1, launch_duration=20_000_000)
    r = oracle_mod.run(scn, 0, live_seed=0, record_depth=GOLD["record_depth"])
    assert r.result == GOLD["result"]
    assert [f"{int(h):016x}" for h in r.hashes] == GOLD["hashes"]
    assert [list(t) for t in r.traces] == GOLD["traces"]


def test_c1_record_replay(oracle_mod):
    r = oracle_mod.run(c1_table_scenario(), 0)
    assert r.result == GOLD["result"]
    assert [f"{int(h):016x}" for h in r.hashes] == GOLD["hashes"]


def test_c1_semantics():
    """Token created at 1 s + 3 µs of start-up forks (Main.hs:132-135), passed
    every tokenPassingDelay + network delay, values strictly increasing by 1 at
    the observer (noteTokenMethod, :197-208), no 'wrong value' log."""
    tr = GOLD["traces"]
    assert tr[0][0] == 1_000_003 and tr[0][2] == scenarios.TAG_CREATE_TOKEN
    notes = [v for (t, node, tag, v) in tr if tag == scenarios.TAG_NOTE]
    assert notes == list(range(1, len(notes) + 1))
    assert not [1 for (_, _, tag, _) in tr if tag == scenarios.TAG_WRONG_VALUE]
    assert GOLD["result"]["final_t"] == 20_000_000 and GOLD["result"]["status"] == 1
