"""BinaryP wire sizes (Message.hs:155-202) pinned by a direct Data.Binary-style
encoding, and the bandwidth-aware hotspot delays they feed.  CPU only."""
import pytest

from timewarp import scenarios, wire
from timewarp.measures import measures_from_trace, trace_tuples


@pytest.mark.parametrize("payload", [0, 1, 100, 4096])
def test_bench_message_size_matches_encoding(payload):
    for name in ("Ping", "Pong"):
        enc = wire.encode_binaryp(name, [12345, b"\x2a" * payload])  # Ping MsgId (Payload: 42s)
        assert len(enc) == wire.bench_message_size(name, payload) == 36 + payload


def test_size_pieces():
    assert wire.text_size("Ping") == 12
    assert wire.text_size("é") == 10  # UTF-8
    assert wire.binaryp_size("x", 0) == 8 + 9
    assert wire.transmission_us(125, 1_000_000) == 125
    assert wire.transmission_us(1, 3_000_000) == 1  # ceil
    with pytest.raises(ValueError):
        wire.transmission_us(1, 0)


def test_hotspot_bandwidth_delays(oracle_mod):
    S, M, P, BW = 3, 4, 2000, 1_000_000  # 2 kB payload at 1 MB/s: 2036 µs per message
    base = scenarios.hotspot(n_senders=S, n_replicas=2, msg_num=M)
    slow = scenarios.hotspot(n_senders=S, n_replicas=2, msg_num=M, payload_bytes=P, bandwidth_bytes_per_s=BW)
    tx = wire.transmission_us(wire.bench_message_size("Ping", P), BW)
    assert tx == 2036
    assert (slow.link_table[:2 * S].astype(int) - base.link_table[:2 * S].astype(int) == tx).all()
    o = oracle_mod.run(slow, replica=1, trace_cap=1 << 12)
    ms = measures_from_trace(trace_tuples(o.traces))
    for mid, m in ms.items():
        sender = (mid - 1) % S
        assert m["PingReceived"] - m["PingSent"] == int(base.link_table[sender, 0, 1]) + tx
