"""C5 (BASELINE config 5) as bench.py runs it: md5hip_batch_host_fixed over
page-locked host memory, which the batcher DMAs in place slot by slot
(md5_submit.c host_pinned -> fixed_submit) instead of copying it through its
staging.  Every digest of a > 1 GiB batch whose chunk count is not a
multiple of a slot's (64 MiB slices: 4,096 x 16 KiB, so 16 full slots and a
ragged 1,013) is checked against the oracle, for

  * a torch pin_memory buffer (hipHostMalloc -- what bench.py --config c5 uses),
  * a numpy buffer pinned by md5hip_host_register,
  * a numpy buffer pinned by someone else's hipHostRegister (not in the
    library's table: the runtime's RANGE attributes decide), and a
    sub-range of it,
  * the same through a two-device pool, whose parts start inside the pinned
    allocation (the RANGE check must accept a sub-range),
  * a numpy buffer whose first half only is registered: it starts pinned and
    runs on into pageable memory, so it must be staged, not DMA'd in place.

`bytes_staged` (the batcher's host bytes copied through staging) tells the
two branches apart: 0 for a source read in place, the batch for a staged one.
md5.c:169-215 semantics per chunk (one MD5Init/Update/Final each)."""
import numpy as np
import pytest
import torch

import gen
from sproxy_amd import md5 as m

pytestmark = pytest.mark.gpu

L = 16384
SLICE = 64 << 20
N = 65536 + 1000 + 13                 # 1.02 GiB; N % (SLICE // L) == 1013


@pytest.fixture(scope="module")
def batch():
    assert N % (SLICE // L) not in (0, N)
    host = gen.xorshift_array(N * L, seed=0xC5C5)
    return host, gen.oracle_digests_fixed(host, N, L)


def _run(b, arr):
    s0 = b.stats()["bytes_staged"]
    got = b.host_fixed(arr, N, L)
    return got, b.stats()["bytes_staged"] - s0


def test_torch_pinned_dma_in_place(cuda, batch):
    host, want = batch
    t = torch.empty(N * L, dtype=torch.uint8, pin_memory=True)
    t.numpy()[:] = host
    with m.Batcher(device=0, slice_bytes=SLICE, nslots=3) as b:
        got, staged = _run(b, t.numpy())
        assert staged == 0                      # the pinned branch: read in place
        assert np.array_equal(got, want)
        got2, _ = _run(b, t.numpy())            # slots reused, same answer
        assert np.array_equal(got2, want)


def test_registered_numpy_dma_in_place(cuda, batch):
    host, want = batch
    arr = host.copy()
    m.register_host(arr)
    try:
        with m.Batcher(device=0, slice_bytes=SLICE, nslots=3) as b:
            got, staged = _run(b, arr)
        assert staged == 0
        assert np.array_equal(got, want)
    finally:
        m.unregister_host(arr)


def test_pool_parts_of_a_pinned_buffer(cuda, batch):
    host, want = batch
    t = torch.empty(N * L, dtype=torch.uint8, pin_memory=True)
    t.numpy()[:] = host
    devs = tuple(range(torch.cuda.device_count()))[:4]
    devs = devs if len(devs) > 1 else (0, 0)
    with m.Pool(devs, slice_bytes=SLICE, nslots=3) as p:
        p.set_split(SLICE)                      # cut into parts that start mid-allocation
        got = p.host_fixed(t.numpy(), N, L)
        st = p.stats()
        staged = sum(p.device_stats(g)["bytes_staged"] for g in range(p.ndev))
    assert st["split"] >= 1
    assert staged == 0
    assert np.array_equal(got, want)


def test_partly_pinned_source_is_staged(cuda, batch):
    host, want = batch
    arr = host.copy()
    half = (N * L) // 2
    m.check("md5hip_host_register", m.lib().md5hip_host_register(arr.ctypes.data, half))
    try:
        with m.Batcher(device=0, slice_bytes=SLICE, nslots=3) as b:
            got, staged = _run(b, arr)
        assert staged == N * L                   # every slot through the pinned staging
        assert np.array_equal(got, want)
    finally:
        m.lib().md5hip_host_unregister(arr.ctypes.data)


def test_host_registered_outside_the_library_dma_in_place(cuda, batch):
    """A buffer page-locked by someone else's hipHostRegister (torch's
    cudaHostRegister binding here) -- not in the library's registration table,
    so host_pinned asks the runtime for both ends and the allocation's extent."""
    host, want = batch
    arr = host.copy()
    cudart = torch.cuda.cudart()
    assert int(cudart.cudaHostRegister(arr.ctypes.data, arr.nbytes, 0)) == 0
    try:
        with m.Batcher(device=0, slice_bytes=SLICE, nslots=3) as b:
            got, staged = _run(b, arr)
            assert np.array_equal(got, want)
            # a sub-range starting inside the registration is pinned too
            s0 = b.stats()["bytes_staged"]
            sub = b.host_fixed(arr[L * 5:], N - 5, L)
            assert b.stats()["bytes_staged"] == s0
        assert staged == 0
        assert np.array_equal(sub, want[5:])
    finally:
        cudart.cudaHostUnregister(arr.ctypes.data)
