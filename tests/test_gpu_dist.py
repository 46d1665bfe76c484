"""The multi-GPU device path under test: two ranks, each a fresh child process with
its own HIP engine on this box's one GPU (gloo between them, standing in for RCCL over xGMI), run
their shard of an app with unpartitioned queries (pattern-set shards), a partition (key shards) and
absent states in the partition (timer matches of several ranks before one event). Each rank's
R18-sorted matches leave HBM through sdh_engine_poll_device, are gathered to rank 0
(dist.gather_columns) and merged there (dist.merge_columns): the result must equal one unsharded
engine and the oracle, tuple for tuple, in order."""
import json
import os
import socket
import subprocess
import sys

import pytest

from dist_gpu_child import batches
from harness import App
from test_dist import events, full_src

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(app):
    evs = events()
    for stream, rows, ts in batches(evs):
        app.send(stream, rows, ts)
    app.advance_time(evs[-1][2] + 100)
    return json.loads(json.dumps(app.matches))


def test_two_ranks_gather_merge_equals_single_engine(tmp_path):
    world = 2
    out = str(tmp_path / "merged.json")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_gpu_child.py"), out],
                              env=dict(env, RANK=str(r), LOCAL_RANK="0")) for r in range(world)]
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world
    got = json.load(open(out))
    want = _run(App(full_src(absent=True)))
    from siddhi_amd.engine import HipEngine
    single = App(full_src(absent=True), engine_factory=lambda blob: None)
    single.engine = HipEngine(single.blob, stream_types=[s.attr_types for s in single.ir.streams])
    assert _run(single) == want
    assert len(want) > 50
    assert all(s > 0 for s in got["sizes"]) and sum(got["sizes"]) == len(want)
    assert got["timers"] > 10
    assert got["merged"] == want
