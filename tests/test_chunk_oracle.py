"""Chunk delivery on the CPU oracle (InputHandler.send(Event[]); include/siddhi_hip.h sdh_batch.chunk)
and the partition query order, on hand-checked cases.

No reference test sends an Event[] into a pattern query, so chunk order is parity-unpinned against
the reference's own suites: these cases pin the oracle's restatement of the delivery code it follows
(StreamJunction.sendEvent(Event[]):218-236, SingleProcessStreamReceiver.processAndClear:57-80,
PartitionStreamReceiver.receive(Event[]):192-239, InputHandler.send(Event[]):77-85), and the GPU
tests (test_gpu_chunk.py) hold the engine to the oracle."""
from harness import App
from siddhi_amd import chm
from siddhi_amd.planner import compile_app, java_string_hash

S = "define stream S (k int, v int);"


def _order(app):
    """(query name, event seqs of the match) in delivery order"""
    names = [q.name for q in app.ir.queries]
    return [(names[m[0]], tuple(s[0] for s in m[3] if s)) for m in app.matches]


def test_top_level_chunk_is_subscriber_major():
    src = S + ("@info(name='a') from every e1=S[v > 0] select e1.v as x insert into O; "
               "@info(name='b') from every e1=S[v > 1] select e1.v as x insert into O;")
    rows, ts = [[0, 1], [0, 2], [0, 3]], [10, 11, 12]
    one = App(src)
    one.send("S", rows, ts)              # three single-event sends
    assert _order(one) == [("a", (0,)), ("a", (1,)), ("b", (1,)), ("a", (2,)), ("b", (2,))]
    ch = App(src)
    ch.send("S", rows, ts, as_chunk=True)  # one Event[]: query a takes the whole chunk first
    assert _order(ch) == [("a", (0,)), ("a", (1,)), ("a", (2,)), ("b", (1,)), ("b", (2,))]


def test_partition_chunk_splits_same_key_runs():
    src = S + ("partition with (k of S) begin "
               "@info(name='a') from every e1=S[v > 0] select e1.v as x insert into O; "
               "@info(name='b') from every e1=S[v > 0] select e1.v as x insert into O; end;")
    rows = [[1, 1], [1, 2], [2, 3], [None, 9], [2, 4], [1, 5]]
    ch = App(src)
    ch.send("S", rows, list(range(6)), as_chunk=True)
    # names a, b hash into bins 1, 2: the key junctions hold clone a then clone b. Runs: key 1
    # [0, 1], key 2 [2, 4] (the null key 3 is skipped without ending the run), key 1 [5]
    assert _order(ch) == [("a", (0,)), ("a", (1,)), ("b", (0,)), ("b", (1,)),
                          ("a", (2,)), ("a", (4,)), ("b", (2,)), ("b", (4,)),
                          ("a", (5,)), ("b", (5,))]


def test_partition_clone_order_follows_query_name_map():
    # metaQueryRuntimeMap is a ConcurrentHashMap keyed by query name: 'q9' lands in bin 8 and
    # 'q10' in bin 4 of the 16-bin table, so q10's clone is ahead of q9's on every key junction
    h9, h10 = java_string_hash("q9"), java_string_hash("q10")
    assert chm.spread(h9) & 15 > chm.spread(h10) & 15
    src = S + ("partition with (k of S) begin "
               "@info(name='q9') from every e1=S[v > 0] select e1.v as x insert into O; "
               "@info(name='q10') from every e1=S[v > 0] select e1.v as x insert into O; end;")
    ir = compile_app(src)
    assert [ir.queries[i].name for i in ir.partitions[0].query_idx] == ["q10", "q9"]
    one = App(src)
    one.send("S", [[1, 1]], [0])
    assert _order(one) == [("q10", (0,)), ("q9", (0,))]


def test_chunk_timers_fire_once_before_the_chunk():
    # time moves once, to the chunk's last timestamp, before the chunk: e1 at t=0 waits 5 ms for
    # no S2; the chunk [S1 t=3, S1 t=20] first fires the due timer of the earlier e1 (at t=5 <= 20)
    src = ("@app:playback define stream S1 (v int); define stream S2 (v int); "
           "@info(name='a') from every e1=S1[v > 0] -> not S2[v > 0] for 5 milliseconds "
           "select e1.v as x insert into O;")
    one, ch = App(src), App(src)
    for a in (one, ch):
        a.start(0)
        a.send("S1", [[1]], [0])
    one.send("S1", [[2], [3]], [3, 20])
    ch.send("S1", [[2], [3]], [3, 20], as_chunk=True)
    # single events: e(0) fires at t=5 before the t=20 event; e(1) (t=3) fires at t=8, before it too
    assert [m[3][0] for m in one.matches] == [(0,), (1,)]
    # the chunk: only e(0)'s timer is queued when time jumps to 20; e(1)'s check is scheduled
    # inside the chunk (for t=8) and waits for the next time change
    assert [m[3][0] for m in ch.matches] == [(0,)]
    ch.advance_time(30)
    assert [m[3][0] for m in ch.matches] == [(0,), (1,), (2,)]


def test_chm_restatements_agree_with_the_planners():
    import numpy as np

    from harness import oracle_lib
    from test_chm_order import _c_positions, _colliding, jdk8_positions
    rng = np.random.default_rng(5)
    for hashes in (rng.integers(-2**31, 2**31, 300).tolist(), _colliding(90, rng, 6)):
        assert chm.positions(hashes) == jdk8_positions(hashes)
        assert chm.positions(hashes) == _c_positions(oracle_lib().oracle_chm_positions, hashes)
