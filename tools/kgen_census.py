"""Arena access census of the K_gen interpreter on the C3 shapes (test infrastructure, CPU only).

Builds tests/native/libkgen_prof.so (kgen.h with KG_PROFILE: every arena word access is counted by
field) and runs each C3 pattern kind over the C3 stream on the host. Prints accesses per
instance-event by field: the device's HBM traffic per instance-event follows these counts. The
hot words (flags / pending / newAndEvery counts, used-bitmasks) are counted per event here, but
the device loads them once per work item (LDS cache, kgen.h Ctx::h32/h64).

usage: python tools/kgen_census.py [keys] [events]
"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import kgen_host  # noqa: E402
from harness import App  # noqa: E402
from siddhi_amd.workloads import STOCK_STREAM, c3_query, stock_events  # noqa: E402

NAMES = ["flags", "pn", "nn", "plist", "nlist", "seslot", "ndnext", "ndnull", "init", "seused", "ndused",
         "sets", "ndseq", "ndts", "ndval", "gc"]


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    native = os.path.join(ROOT, "tests", "native")
    subprocess.check_call(["make", "-s", "-C", native, "libkgen_prof.so"])
    kgen_host.SO = os.path.join(native, "libkgen_prof.so")
    lib = kgen_host.lib()
    lib.kgh_prof.argtypes = [ctypes.c_void_p]
    for kind in range(3):
        app = App(f"{STOCK_STREAM} partition with (symbol of StockStream) begin {c3_query(kind)} end;")
        eng = kgen_host.KGenHostEngine(app.blob)
        ts, sym, price, vol = stock_events(0, N, K)
        vals = np.stack([sym.astype(np.int64), price.view(np.uint32).astype(np.int64), vol.astype(np.int64)], 1)
        lib.kgh_prof(np.zeros(16, np.int64).ctypes.data)
        t = time.time()
        eng.send(0, ts, vals, None)
        out = np.zeros(16, np.int64)
        lib.kgh_prof(out.ctypes.data)
        print(f"kind {kind}: {out.sum() / N:.1f} accesses/instance-event, "
              f"{lib.kgh_num_matches(eng.h) / N:.3f} matches/event ({time.time() - t:.1f} s)")
        print("    " + ", ".join(f"{NAMES[k]}={out[k] / N:.1f}" for k in range(16) if out[k]))


if __name__ == "__main__":
    main()
