"""Small host pushes on the C4 engine: the call sequence of the round-5 latency
probe whose run dumped core before its first push line (tools/lat_probe.py --workload c4 with
--compact / --reserve: the unpartitioned K_seq engine, sdh_engine_reserve_keys on an engine without
partitioned state, host pushes of 1, 64 and 4,096 events each followed by sdh_engine_poll or
sdh_engine_poll_compact_ex). The run did not reproduce at round 6 in any flag combination
(DESIGN.md §4); this pins the sequence: two engines take the same pushes, one polled as tuples and
one as compact rows, and their matches agree push by push."""
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("reserve", [False, True])
def test_c4_small_pushes_tuple_and_compact_polls(reserve):
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from siddhi_amd.workloads import txn_events
    P, _, K = bench.DEFAULTS["c4"]
    sh = bench.Shard("c4", "strong", P, 0, 1)
    a = bench.make_engine("c4", sh, K, 0, 0, 128)
    b = bench.make_engine("c4", sh, K, 0, 0, 128)
    if reserve:
        a.reserve_keys(K)
        b.reserve_keys(K)
    lo, total = 0, 0
    for bs, reps in ((1, 40), (64, 20), (4096, 4)):
        for _ in range(reps):
            ts, x, y, z = txn_events(lo, bs, K)
            lo += bs
            cols = [x, y.view(np.uint32), z]
            a.push_columns(0, ts, cols)
            b.push_columns(0, ts, cols)
            q, k, t, off, words, seq, tb = a.poll(with_seq=True)
            seq_base, rows, key, tbx, chain = b.poll_compact_ex()
            assert len(rows) == len(q)
            if len(q):  # the compact row's trigger seq and query are the tuple's
                assert np.array_equal(rows[:, 0], q) and np.array_equal(rows[:, 1] + seq_base, seq)
            total += len(q)
    assert total > 1000
    a.close()
    b.close()
