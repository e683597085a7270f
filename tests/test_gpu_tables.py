"""Link tables drawn on the GPU (tw_draw_link_table) against the host StdGen
draw (timewarp/stdgen.py, pinned to random-1.1 by tests/test_pqueue_stdgen.py):
entry for entry, for every scenario builder that takes a `drawer`, and at
C3's full shape (4,096-node rings x 65,536 replicas, drop coins) on sampled
replica columns."""
import time

import numpy as np
import pytest

from timewarp import isa, scenarios
from timewarp.engine import EngineError, draw_link_table

pytestmark = [pytest.mark.gpu, pytest.mark.one_geometry]


@pytest.mark.parametrize("build", [
    lambda d: scenarios.token_ring(n_nodes=16, n_replicas=1000, drop_log2=3, link_depth=3, seed_base=17, drawer=d),
    lambda d: scenarios.token_ring(n_nodes=5, n_replicas=1, drawer=d),
    lambda d: scenarios.ping_pong(n_replicas=777, seed_base=123456789, drawer=d),
    lambda d: scenarios.hotspot(n_senders=8, n_replicas=100, msg_num=4, seed_base=3, drawer=d),
    lambda d: scenarios.gatekeeper(n_clients=3, n_replicas=5, drawer=d),
])
def test_device_table_equals_host(build):
    dev, host = build(draw_link_table), build(None)
    assert dev.link_table.dtype == np.uint32 and dev.link_table.shape == host.link_table.shape
    assert np.array_equal(dev.link_table, host.link_table)


def test_constant_links_and_reversed_range():
    L, R = 6, 300
    drawn = np.array([0, 1, 0, 1, 1, 0], np.uint8)
    lo = np.array([7, 5000, 0, 1000, 9, 123456], np.int64)
    hi = np.array([0, 1000, 0, 5000, 9, 0], np.int64)  # link 1: reversed range (randomR swaps it)
    dev = draw_link_table(R, drawn, lo, hi, link_depth=2, drop_log2=1, seed_base=-5)
    host = scenarios.draw_table(L, R, np.nonzero(drawn)[0], lo, hi, link_depth=2, drop_log2=1, seed_base=-5)
    assert np.array_equal(dev, host)
    assert (dev[0] == 7).all() and (dev[5] == 123456).all()
    assert ((dev[4] & 0x7FFFFFFF) == 9).all() and (dev[4] & isa.LINK_DROP).any()


def test_rejects_multi_digit_ranges():
    with pytest.raises(EngineError):
        draw_link_table(4, np.ones(1, np.uint8), np.zeros(1, np.int64), np.full(1, 1 << 30, np.int64))
    with pytest.raises(EngineError):
        draw_link_table(4, np.ones(1, np.uint8), np.zeros(1, np.int64), np.ones(1, np.int64), drop_log2=22)


def test_c3_shape_sampled_columns():
    """C3's table (8,194 links x 65,536 replicas, drop 2^-10): the device draw
    against host draws of replica blocks at both ends and in the middle."""
    t0 = time.perf_counter()
    dev = scenarios.token_ring(n_nodes=4096, n_replicas=65536, drop_log2=10, drawer=draw_link_table).link_table
    dt = time.perf_counter() - t0
    for base in (0, 31_000, 65536 - 48):
        host = scenarios.token_ring(n_nodes=4096, n_replicas=48, drop_log2=10, seed_base=base).link_table
        assert np.array_equal(dev[:, :, base:base + 48], host), base
    assert (dev[1::2] == 0).all()  # the observer links: ConnectedIn 0
    dropped = (dev[0::2] & isa.LINK_DROP) != 0
    assert 0.5 / 1024 < dropped.mean() < 2.0 / 1024
    print(f"C3 table drawn on the GPU in {dt:.2f} s (scenario build included)")
