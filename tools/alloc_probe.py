"""Diagnostic: time hipMalloc / hipFree in the K_slab growth pattern (256 rings re-allocated at
1.3x their size, old ones freed after each batch of 32), to find where allocation stalls."""
import ctypes
import sys
import time

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemGetInfo.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
ring = int(float(sys.argv[1]) * 1e9) if len(sys.argv) > 1 else int(0.1e9)
keep = len(sys.argv) > 2 and sys.argv[2] == "keep"  # never free (is freeing what stalls?)
rings = [None] * 256
for gen in range(12):
    size = int(ring * (1.3 ** gen))
    worst, total = 0.0, 0.0
    for b in range(0, 256, 32):
        new = []
        for r in range(b, b + 32):
            p = ctypes.c_void_p()
            t = time.perf_counter()
            rc = hip.hipMalloc(ctypes.byref(p), size)
            dt = (time.perf_counter() - t) * 1e3
            worst, total = max(worst, dt), total + dt
            if rc != 0:
                print(f"gen {gen}: hipMalloc failed at ring {r}", flush=True)
                sys.exit(0)
            new.append(p)
        for r, p in zip(range(b, b + 32), new):
            if rings[r] is not None and not keep:
                hip.hipFree(rings[r])
            rings[r] = p
    fr, tot = ctypes.c_size_t(), ctypes.c_size_t()
    hip.hipMemGetInfo(ctypes.byref(fr), ctypes.byref(tot))
    print(f"gen {gen}: rings {size / 1e9:.2f} GB x 256 = {size * 256 / 1e9:.0f} GB, malloc total {total:.1f} ms, "
          f"worst {worst:.1f} ms, used {(tot.value - fr.value) / 1e9:.0f} GB", flush=True)
