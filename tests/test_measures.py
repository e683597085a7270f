"""measures.csv (bench/Network/LogReader/Main.hs:85-119) from the hotspot
scenario's traces, on the oracle: every message has its four measure events in
causal order, and Ping/Pong latencies are exactly the per-link delays drawn for
that replica.  CPU only."""
import numpy as np

from timewarp import scenarios
from timewarp.measures import EVENTS, format_measures_csv, measures_from_trace, trace_tuples


def test_hotspot_measures_match_link_delays(oracle_mod):
    S, M = 4, 6
    scn = scenarios.hotspot(n_senders=S, n_replicas=3, msg_num=M)
    for rep in range(3):
        o = oracle_mod.run(scn, replica=rep, trace_cap=1 << 12)
        ms = measures_from_trace(trace_tuples(o.traces))
        assert sorted(ms) == list(range(1, S * M + 1))  # ids tid + k*threadNum (Sender/Main.hs:40)
        table = scn.link_table  # [link, depth, replica]; links i -> S (id i), S -> i (id S+i)
        for mid, m in ms.items():
            assert m is not None and set(m) == set(EVENTS)
            assert m["PingSent"] <= m["PingReceived"] == m["PongSent"] <= m["PongReceived"]
            sender = (mid - 1) % S
            d_ping = m["PingReceived"] - m["PingSent"]
            d_pong = m["PongReceived"] - m["PongSent"]
            assert 1000 <= d_ping <= 5000 and 1000 <= d_pong <= 5000
            assert d_ping == int(table[sender, 0, rep]) and d_pong == int(table[S + sender, 0, rep])


def test_measures_csv_format():
    recs = [(10, 0, scenarios.TAG_PING_SENT, 1), (1010, 4, scenarios.TAG_PING, 1),
            (1010, 4, scenarios.TAG_PONG_SENT, 1), (2020, 0, scenarios.TAG_PONG, 1),
            (20, 1, scenarios.TAG_PING_SENT, 2),
            (30, 2, scenarios.TAG_PING_SENT, 3), (31, 2, scenarios.TAG_PING_SENT, 3)]
    ms = measures_from_trace(recs)
    assert ms[3] is None  # repeated event: LogReader's uniqMap drops the row
    csv = format_measures_csv(ms).splitlines()
    assert csv[0].split(",")[0] == "MsgId  " and len(csv[0].split(",")) == 6
    assert csv[1] == ",".join(["1".ljust(7), "0".ljust(7), "10".ljust(18), "1010".ljust(18), "1010".ljust(18),
                               "2020".ljust(18)])
    assert csv[2].split(",")[3].strip() == "-" and len(csv) == 3
