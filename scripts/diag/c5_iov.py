#!/usr/bin/env python3
"""Page-list (netcache block) end-to-end rate by gather mode: blocks of
16 KiB pages scattered over a pageable "page heap", hashed through a batcher
(H2D -> MD5 -> D2H).  HOST = memcpy into pinned staging (heap unregistered),
HOST_REG = same with the heap registered, DEVICE = gather kernel over PCIe from
the registered heap, DMA = one async copy per page.  Prints one JSON object."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402


def _arg(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    page, per_block = 16384, _arg("--pages", 16)
    slots, slice_mib = _arg("--slots", 0), _arg("--slice-mib", 0)     # 0 = library defaults
    heap_bytes = 2 << 30
    if "--huge" in sys.argv:
        # 2 MiB transparent huge pages behind the heap (fewer IOMMU/GPUVM
        # translations for the device and the DMA engine)
        import mmap
        mm = mmap.mmap(-1, heap_bytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        mm.madvise(mmap.MADV_HUGEPAGE)
        heap = np.frombuffer(mm, np.uint8)
    else:
        heap = np.empty(heap_bytes, np.uint8)
    heap[::4096] = 1                                   # touch every page
    rng = np.random.default_rng(7)
    npages = heap_bytes // page
    nblocks = npages // per_block
    # default: pages scattered at random over the heap; --contiguous: each
    # block's pages adjacent (one netcache bulk per block, bc_mgr.c:1269)
    perm = np.arange(npages) if "--contiguous" in sys.argv else rng.permutation(npages)
    blocks = [[heap[int(p) * page:(int(p) + 1) * page] for p in perm[b * per_block:(b + 1) * per_block]]
              for b in range(nblocks)]
    total = nblocks * per_block * page
    res = {"blocks": nblocks, "pages_per_block": per_block, "bytes": total,
           "layout": "contiguous" if "--contiguous" in sys.argv else "scattered",
           "coarse": os.environ.get("MD5HIP_REGISTER_COARSE", "default(1)"),
           "huge_pages": "--huge" in sys.argv}
    b = m.Batcher(device=0, slice_bytes=slice_mib << 20, nslots=slots)
    res.update(slots=slots, slice_mib=slice_mib)
    arr, fa, keep = b._iov(blocks)                     # build the segment list once
    out = np.empty((nblocks, 16), np.uint8)
    lib = m.lib()

    def run():
        rc = lib.md5_batch_submit_iov(b._h, arr, fa.ctypes.data, nblocks, out.ctypes.data)
        assert rc == 0, rc

    def timed(name, reps=3):
        run()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[len(ts) // 2]
        res[name] = {"s": round(t, 4), "GBps": round(total / t / 1e9, 2)}
        return out.copy()

    b.set_gather(b.GATHER_HOST)
    ref = timed("host")
    m.register_host(heap)
    try:
        timed("host_reg")
        for mode, name in ((b.GATHER_DEVICE, "device"), (b.GATHER_DMA, "dma"), (b.GATHER_AUTO, "auto")):
            b.set_gather(mode)
            got = timed(name)
            assert np.array_equal(got, ref), name
        if "--only-device" in sys.argv:
            b.set_gather(b.GATHER_DEVICE)
            got = timed("device_" + os.environ.get("MD5HIP_GATHER_UNROLL", "4"))
    finally:
        m.unregister_host(heap)
    # pinned H2D alone, for the roofline of this path
    src = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    dst = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    res["h2d_pinned_GBps"] = round(3 * (1 << 30) / (time.perf_counter() - t0) / 1e9, 2)
    b.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
