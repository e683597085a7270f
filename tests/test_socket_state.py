"""examples/socket-state on the oracle: ``userStateR`` (socket-state/Main.hs
:91-93) is per-connection state, so the server's request counter runs 1, 2, ...
separately for each client (:65-76).  Expected values follow from the drawn
round counts: client c sends at ~k s for k = 1..rounds_c, and the server stops
listening at 10 s, so min(rounds_c, 9) Pings are counted and the rest are
undeliverable.  CPU only; GPU parity is in tests/test_gpu_parity.py."""
import numpy as np

from timewarp import scenarios


def test_per_connection_counters(oracle_mod):
    scn = scenarios.socket_state(n_replicas=24, seed_base=100)
    rounds = scn.main_regs[:, 1:4]
    assert rounds.max() > 9 and (rounds == 0).any()  # both cut-offs are exercised
    for rep in range(scn.n_replicas):
        o = oracle_mod.run(scn, replica=rep, trace_cap=1 << 12)
        res = {k: int(o.result[k]) for k in ("delivered", "undeliverable", "dropped", "status")}
        got = np.minimum(rounds[rep], 9)
        assert res["status"] == 1
        assert res["delivered"] == int(got.sum())
        assert res["undeliverable"] == int(np.maximum(rounds[rep] - 9, 0).sum())
        recs = sorted(t for t in o.traces if t[2] in (scenarios.TAG_GOT_PING_NO, scenarios.TAG_FROM_CLIENT))
        # each delivery traces (reqNo, cid) at the same instant on the server
        per_client = {1: [], 2: [], 3: []}
        by_t = {}
        for t, node, tag, val in recs:
            assert node == 0
            by_t.setdefault(t, {})[tag] = val
        for t in sorted(by_t):
            d = by_t[t]
            per_client[d[scenarios.TAG_FROM_CLIENT]].append(d[scenarios.TAG_GOT_PING_NO])
        for cid in (1, 2, 3):
            assert per_client[cid] == list(range(1, int(got[cid - 1]) + 1)), (rep, cid)
