"""One rank of tests/test_gpu_dist.py (a child process; test infrastructure): the HIP engine on this
rank's shard of test_dist.full_src(absent=True) -- unpartitioned queries by pattern set, the
partition by key -- every rank pushing the whole event stream, then sdh_engine_poll_device ->
dist.columns_from_device -> dist.gather_columns (gloo) -> dist.merge_columns on rank 0, which writes
the merged match tuples as JSON to argv[1]."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def batches(evs, limit=20):
    i = 0
    while i < len(evs):
        j = i + 1
        while j < len(evs) and evs[j][0] == evs[i][0] and j - i < limit:
            j += 1
        yield evs[i][0], [r for _, r, _ in evs[i:j]], [t for _, _, t in evs[i:j]]
        i = j


def main(out_path):
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.init()  # (torch's HIP runtime first, as in the test sessions: conftest.py)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from harness import App
    from siddhi_amd import dist as sdist
    from siddhi_amd.engine import HipEngine
    from siddhi_amd.events import encode_rows
    from test_dist import events, full_src
    app = App(full_src(absent=True), engine_factory=lambda blob: None)
    ir = app.ir
    eng = HipEngine(app.blob, shard_rank=rank, shard_world=world, stream_types=[s.attr_types for s in ir.streams])
    log = sdist.StreamLog()
    evs = events()
    for stream, rows, ts in batches(evs):  # every rank sees the whole stream (the broadcast)
        si = ir.stream_index(stream)
        vals, nulls = encode_rows(rows, ir.streams[si].attr_types, app.dictionary)
        eng.send(si, ts, vals, nulls)
        log.push(si, len(ts))
    eng.advance_time(evs[-1][2] + 100)  # trailing timers fire (seq = one past the last event)
    cols = {k: v.cpu() for k, v in sdist.columns_from_device(eng, torch.device("cuda:0")).items()}
    per_rank = sdist.gather_columns(cols)
    if rank == 0:
        merged = sdist.columns_to_tuples(sdist.merge_columns(ir, per_rank, log))
        with open(out_path, "w") as f:
            json.dump({"merged": merged, "sizes": [int(c["q"].numel()) for c in per_rank],
                       "timers": sum(int((c["tb"] != sdist.TB_EVENT).sum()) for c in per_rank)}, f)
    dist.barrier()
    dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main(sys.argv[1])
