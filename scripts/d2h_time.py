"""Device → host copy of a FASTA-body-sized buffer (65 MB, C5's bodies) by the ways a fetch can
take it: pinned (torch's caching host allocator: first and repeated allocation), pageable
`.cpu()`, into a numpy buffer, and the bytes / memoryview conversions after it.  Best of 3 ms.

    python scripts/d2h_time.py [MB]"""
import json
import sys
import time

import numpy as np
import torch


def best(f, n=3):
    r = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        r.append((time.perf_counter() - t0) * 1e3)
    return min(r), r


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 65.0
    n = int(mb * 1e6)
    dev = torch.device("cuda", 0)
    t = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    res = {"bytes": n}
    t0 = time.perf_counter()
    p0 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    res["pinned_alloc_first_ms"] = (time.perf_counter() - t0) * 1e3
    del p0

    def pinned_fresh():
        b = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        b.copy_(t, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return memoryview(b.numpy())
    res["pinned_cached_copy_ms"] = best(pinned_fresh)
    keep = torch.empty(n, dtype=torch.uint8, pin_memory=True)

    def pinned_kept():
        keep.copy_(t, non_blocking=True)
        torch.cuda.current_stream().synchronize()
    res["pinned_kept_copy_ms"] = best(pinned_kept)
    res["pinned_kept_tobytes_ms"] = best(lambda: keep.numpy().tobytes())
    res["pageable_cpu_ms"] = best(lambda: t.cpu())

    def into_numpy():
        a = np.empty(n, dtype=np.uint8)
        torch.from_numpy(a).copy_(t)
    res["into_fresh_numpy_ms"] = best(into_numpy)
    a = np.empty(n, dtype=np.uint8)
    a[:] = 1

    def into_touched_numpy():
        torch.from_numpy(a).copy_(t)
    res["into_touched_numpy_ms"] = best(into_touched_numpy)
    import mmap

    def into_mmap(flags, huge):
        def f():
            mm = mmap.mmap(-1, n, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS | flags)
            if huge:
                mm.madvise(mmap.MADV_HUGEPAGE)
            torch.from_numpy(np.frombuffer(mm, dtype=np.uint8)).copy_(t)
            return mm
        return f
    res["into_mmap_ms"] = best(into_mmap(0, False))
    res["into_mmap_populate_ms"] = best(into_mmap(mmap.MAP_POPULATE, False))
    res["into_mmap_huge_ms"] = best(into_mmap(0, True))
    res["cat8_device_ms"] = best(lambda: torch.cat([t[k * (n // 8):(k + 1) * (n // 8)] for k in range(8)]))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
