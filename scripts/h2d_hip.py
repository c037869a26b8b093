"""One GB-sized H2D on the HIP runtime directly (hiprun.Hip): pinned staging by hipHostMalloc
flags (default / non-coherent), one synchronous hipMemcpy against chunked hipMemcpyAsync on
several streams.  Best of 3 ms.   python scripts/h2d_hip.py [MB]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from sam2consensus_amd.hiprun import Hip
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 1064
    n = mb << 20
    hip = Hip()
    hip.set_device(0)
    h = hip.h
    h.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    h.hipMemcpyAsync.restype = C.c_int
    h.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
    h.hipStreamSynchronize.argtypes = [C.c_void_p]
    d = hip.malloc(n)
    res = {"bytes": n}
    streams = []
    for _ in range(4):
        s = C.c_void_p()
        hip.check(h.hipStreamCreate(C.byref(s)), "hipStreamCreate")
        streams.append(s)
    for name, flags in (("default", 0), ("noncoherent", 0x80000000), ("portable", 0x1)):
        p = C.c_void_p()
        t0 = time.perf_counter()
        hip.check(h.hipHostMalloc(C.byref(p), n, flags), "hipHostMalloc")
        res[name + "_alloc_ms"] = (time.perf_counter() - t0) * 1e3
        C.memset(p.value, 1, n)
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            hip.memcpy(d, p.value, n, 1)
            best = min(best, time.perf_counter() - t0)
        res[name + "_sync_ms"] = best * 1e3
        for ns, chunk in ((1, 64 << 20), (4, 64 << 20), (4, 16 << 20)):
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter()
                for k, o in enumerate(range(0, n, chunk)):
                    hip.check(h.hipMemcpyAsync(C.c_void_p(d + o), C.c_void_p(p.value + o), min(chunk, n - o), 1,
                                               streams[k % ns]), "hipMemcpyAsync")
                for s in streams[:ns]:
                    h.hipStreamSynchronize(s)
                best = min(best, time.perf_counter() - t0)
            res["%s_async_%dx%dMB_ms" % (name, ns, chunk >> 20)] = best * 1e3
        hip.host_free(p.value)
    hip.free(d)
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
