"""Which K_gen limit do the fuzz seeds that exceed the default pools hit? (GPU diagnostic)"""
import sys
sys.path.insert(0, "tests")
from test_gpu_gen import hip_app  # noqa: E402
from fuzz_apps import random_app, random_events  # noqa: E402
from harness import App  # noqa: E402
from siddhi_amd.engine import EngineError  # noqa: E402

for seed in (7, 11, 12, 14, 30):
    src = random_app(seed, partition=seed % 3 == 0)
    for kw in ({}, dict(gen_list_cap=512), dict(gen_pool_nodes=256), dict(gen_pool_nodes=256, gen_list_cap=512)):
        o = App(src)
        g = hip_app(src, **kw)
        try:
            for stream, row, t in random_events(seed):
                o.send(stream, [row], [t])
                g.send(stream, [row], [t])
            print(seed, kw, "ok", g.matches == o.matches, flush=True)
            break
        except EngineError as ex:
            print(seed, kw, "fail", ex, flush=True)
