"""Link-table draws on the host (CPU): what the GPU draw (tw_draw_link_table,
tests/test_gpu_tables.py) and the replica sharding rely on.

- Replica independence: one StdGen per replica (mkStdGen(seed_base + r)), so
  a batch drawn at once equals its contiguous blocks drawn separately -- the
  rule by which ranks (dist.strong_block) and bench.py's 64-replica host check
  re-draw their share.
- Builder plumbing: every builder that takes `drawer=` hands it a spec
  (drawn links, lo, hi, depth, drop, seed) that reproduces its own host table."""
import numpy as np
import pytest

from timewarp import isa, scenarios


def test_blocks_equal_whole_batch():
    L = 7
    drawn = [0, 2, 3, 6]
    lo = np.array([1000, 0, 5, 2000, 0, 0, 1], np.int64)
    hi = np.array([5000, 0, 9, 1000, 0, 0, 1], np.int64)
    whole = scenarios.draw_table(L, 100, drawn, lo, hi, link_depth=2, drop_log2=2, seed_base=11)
    parts = [scenarios.draw_table(L, n, drawn, lo, hi, link_depth=2, drop_log2=2, seed_base=11 + b)
             for b, n in ((0, 37), (37, 63))]
    assert np.array_equal(whole, np.concatenate(parts, axis=2))
    assert (whole[1] == 0).all() and (whole[4] == 0).all()
    assert (whole[0] & isa.LINK_DROP).any()


def _host_drawer(n_replicas, drawn, lo, hi, link_depth=1, drop_log2=0, seed_base=0):
    return scenarios.draw_table(len(drawn), n_replicas, np.nonzero(drawn)[0], lo, hi, link_depth=link_depth,
                                drop_log2=drop_log2, seed_base=seed_base)


@pytest.mark.parametrize("build", [
    lambda d: scenarios.token_ring(n_nodes=12, n_replicas=9, drop_log2=4, link_depth=2, seed_base=5, drawer=d),
    lambda d: scenarios.ping_pong(n_replicas=10, seed_base=3, drawer=d),
    lambda d: scenarios.hotspot(n_senders=6, n_replicas=4, msg_num=3, drawer=d),
    lambda d: scenarios.gatekeeper(n_clients=3, n_replicas=2, drawer=d),
])
def test_builders_hand_the_drawer_their_table(build):
    assert np.array_equal(build(_host_drawer).link_table, build(None).link_table)
