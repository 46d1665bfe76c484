#!/usr/bin/env python3
"""sha256 (16 hex digits) of the engine's sources -- every .hip / .h / .py / Makefile in this
directory except build_info.hip -- by name order. The library embeds it (build_info.hip,
sdh_build_info) and bench.py recomputes it from the tree: equal values show that the .so that ran
was built from these sources."""
import hashlib
import os
import sys


def src_hash(d):
    h = hashlib.sha256()
    for name in sorted(os.listdir(d)):
        if name == "build_info.hip" or not (name.endswith((".hip", ".h", ".py")) or name == "Makefile"):
            continue
        h.update(name.encode())
        with open(os.path.join(d, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(src_hash(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.abspath(__file__))))
