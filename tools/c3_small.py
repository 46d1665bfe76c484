"""Small pushes on one workload's engine, timed per phase (the expansion leg's shape, bench.py
expansion / compact_leg): `python tools/c3_small.py [--workload c3] [--bs 65536] [--pushes 20]
[--mode compact|device|records]`. Keyed workloads reserve their keys first. Per push: the push call
(host time to return), the poll, and the library's last kernel time (sdh_engine_push_stats); run it
under `rocprofv3 --kernel-trace` for the kernel timeline between them."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--bs", type=int, default=1 << 16)
    ap.add_argument("--pushes", type=int, default=20)
    ap.add_argument("--mode", choices=("compact", "device", "records"), default="compact")
    args = ap.parse_args()
    print("cmd:", " ".join(sys.argv), flush=True)
    import torch
    import bench
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES
    P, _, K = bench.DEFAULTS[args.workload]
    sh = bench.Shard(args.workload, "strong", P, 0, 1)
    flags = SDH_FLAG_DEVICE_MATCHES if args.mode == "records" else 0
    eng = bench.make_engine(args.workload, sh, K, 0, flags, 128)
    if args.workload in ("c3", "c5"):
        eng.reserve_keys(K)
    dev = torch.device("cuda:0")
    E = args.bs
    bs = [bench.gen_batch(args.workload, i * E, E, K, dev) for i in range(args.pushes)]
    torch.cuda.synchronize()
    tot = [0.0, 0.0, 0.0]
    for i, cols in enumerate(bs):
        t0 = time.perf_counter()
        eng.push_device(0, E, cols[0].data_ptr(), [c.data_ptr() for c in cols[1:]])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if args.mode == "compact":
            n = eng.poll_compact_ex(device=True).n
        elif args.mode == "device":
            n = eng.poll_device().n
        else:
            n = eng.poll_records().n
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        kms = eng.push_stats()[0]
        print(f"push {i}: {n} matches, push {(t1 - t0) * 1e3:.3f} ms (kernels {kms:.3f}), "
              f"poll {(t2 - t1) * 1e3:.3f} ms", flush=True)
        if i >= 3:
            tot[0] += (t1 - t0) * 1e3
            tot[1] += (t2 - t1) * 1e3
            tot[2] += kms
    k = max(1, args.pushes - 3)
    print(f"mean over {k} pushes: push {tot[0] / k:.3f} ms, kernels {tot[2] / k:.3f} ms, poll {tot[1] / k:.3f} ms")
    eng.close()


if __name__ == "__main__":
    main()
