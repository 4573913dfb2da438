"""Python host mirror of sproxy's MD5 interface (md5.h:31-51) plus the batched
device entries (include/md5hip.h).

Per-message API -- same names, argument order and behaviour as md5.c:153-265:
    ctx = MD5Context(); MD5Init(ctx); MD5Update(ctx, buf, len); MD5Final(digest, ctx)
(``MD5Final`` writes into ``digest`` -- a writable 16-byte buffer -- and also
returns the digest as ``bytes``; it zeroes ``ctx`` like md5.c:264.)

Batched device API (the hot path) -- torch CUDA tensors are only plumbing for
device memory and streams; every byte is hashed by the HIP kernels of
libmd5hip.so, and a CPU tensor is an error, never a fallback:
    digest_fixed(data, n, length, stride=None)      -> uint8 [n, 16] on device
    digest_desc(base, offsets, lens, order=None)     -> uint8 [n, 16] on device
    plan_order(lens)                                 -> longest-first lane order
Host-memory batches (the netcache block-checksum site, blk_io.c:354):
    with Batcher(device=0) as b: b.submit([buf, ...]); b.host_fixed(arr, n, len)
"""
import ctypes

import numpy as np

from ._lib import MD5Context, MD5HipBatcherStats, MD5HipError, MD5HipIov, MD5HipPoolStats, check, lib

try:
    import torch
except Exception:  # pragma: no cover
    torch = None

MD5_DIGEST_SIZE = 16

AUTO, DIRECT2, XDMA1NT = 0, 1, 10            # enum md5hip_variant (ABI 2: the shipped kernels)
VARIANTS = {"auto": AUTO, "direct2": DIRECT2, "xdma1nt": XDMA1NT}


# ---------------------------------------------------------------- per message
def _addr(buf):
    """(address, keepalive) of a bytes-like object."""
    if isinstance(buf, np.ndarray):
        a = np.ascontiguousarray(buf)
        return a.ctypes.data, a
    mv = memoryview(buf)
    if mv.readonly:
        b = ctypes.create_string_buffer(mv.tobytes(), max(mv.nbytes, 1))
        return ctypes.addressof(b), b
    c = (ctypes.c_char * max(mv.nbytes, 1)).from_buffer(mv) if mv.nbytes else ctypes.create_string_buffer(1)
    return ctypes.addressof(c), (c, mv)


def MD5Init(ctx: MD5Context) -> None:
    lib().MD5Init(ctypes.byref(ctx))


def MD5Update(ctx: MD5Context, buf, length: int = None) -> None:
    mv = memoryview(buf)
    n = mv.nbytes if length is None else int(length)
    if n < 0 or n > mv.nbytes or n > 0xFFFFFFFF:
        raise ValueError("length out of range (md5.h:47 takes an unsigned int)")
    addr, keep = _addr(buf)
    lib().MD5Update(ctypes.byref(ctx), addr, n)
    del keep


def MD5Final(digest, ctx: MD5Context) -> bytes:
    out = (ctypes.c_ubyte * 16)()
    lib().MD5Final(out, ctypes.byref(ctx))
    d = bytes(out)
    if digest is not None:
        memoryview(digest)[:16] = d
    return d


def md5(data) -> bytes:
    """One-shot convenience: Init/Update/Final over a bytes-like object."""
    ctx = MD5Context()
    MD5Init(ctx)
    mv = memoryview(data).cast("B")
    off = 0
    while off < mv.nbytes or off == 0:
        part = min(mv.nbytes - off, 1 << 30)
        MD5Update(ctx, mv[off:off + part])
        off += part
        if part == 0:
            break
    return MD5Final(None, ctx)


# ---------------------------------------------------------------- device batches
def _need_cuda(t, what):
    if torch is None or not isinstance(t, torch.Tensor):
        raise TypeError(f"{what} must be a torch tensor on a HIP device")
    if not t.is_cuda:
        raise ValueError(f"{what} is on {t.device}; the batched MD5 runs only on the GPU")
    if not t.is_contiguous():
        raise ValueError(f"{what} must be contiguous")


def _stream(stream):
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


def digest_fixed(data, n: int = None, length: int = None, stride: int = None, out=None,
                 stream=None, variant=AUTO):
    """digest[i] = MD5(data_bytes[i*stride : i*stride + length]).

    ``data`` is a contiguous uint8 CUDA tensor; with ``n``/``length`` omitted it
    must be 2-D [n, length]."""
    _need_cuda(data, "data")
    if data.dtype != torch.uint8:
        raise TypeError("data must be uint8")
    if n is None or length is None:
        if data.dim() != 2:
            raise ValueError("pass n and length, or a 2-D [n, length] tensor")
        n, length = data.shape
    stride = length if stride is None else stride
    if n and (n - 1) * stride + length > data.numel():
        raise ValueError("batch extends past the end of `data`")
    if out is None:
        out = torch.empty((n, 16), dtype=torch.uint8, device=data.device)
    _need_cuda(out, "out")
    if isinstance(variant, str):
        variant = VARIANTS[variant]
    rc = lib().md5hip_digest_fixed_variant(data.data_ptr(), n, length, stride, out.data_ptr(),
                                           _stream(stream), variant)
    check("md5hip_digest_fixed_variant", rc)
    return out


DESC_VARIANTS = {"auto": 0, "lane": 1, "hybrid": 3, "xdma": 4, "balanced": 5,
                 "fed": 6, "lines": 7}   # enum md5hip_desc_variant


def digest_desc(base, offsets, lens, order=None, out=None, stream=None, variant=0):
    """digest[i] = MD5(base_bytes[offsets[i] : offsets[i] + lens[i]])."""
    _need_cuda(base, "base")
    _need_cuda(offsets, "offsets")
    _need_cuda(lens, "lens")
    if offsets.dtype != torch.int64 or lens.dtype not in (torch.int32, torch.uint32):
        raise TypeError("offsets must be int64 and lens int32")
    n = offsets.numel()
    if lens.numel() != n:
        raise ValueError("offsets and lens differ in length")
    if order is not None:
        _need_cuda(order, "order")
        if order.numel() != n or order.dtype not in (torch.int32, torch.uint32):
            raise ValueError("order must be an int32 permutation of range(n)")
    if out is None:
        out = torch.empty((n, 16), dtype=torch.uint8, device=base.device)
    if isinstance(variant, str):
        variant = DESC_VARIANTS[variant]
    rc = lib().md5hip_digest_desc_variant(base.data_ptr(), offsets.data_ptr(), lens.data_ptr(),
                                          order.data_ptr() if order is not None else None, n,
                                          out.data_ptr(), _stream(stream), variant)
    check("md5hip_digest_desc_variant", rc)
    return out


def _ctx_tensor(ctxs):
    _need_cuda(ctxs, "ctxs")
    if ctxs.dtype != torch.uint8 or ctxs.dim() != 2 or ctxs.shape[1] != 88:
        raise ValueError("ctxs must be a uint8 [n, 88] device tensor (struct MD5Context, md5.h:33-38)")
    return ctxs.shape[0]


def init_ctx(ctxs, stream=None):
    """MD5Init on every context of a uint8 [n, 88] device tensor (in[] untouched)."""
    n = _ctx_tensor(ctxs)
    check("md5hip_init_ctx", lib().md5hip_init_ctx(ctxs.data_ptr(), n, _stream(stream)))
    return ctxs


def update_ctx(ctxs, ptrs, lens, stream=None):
    """MD5Update(ctx[i], ptrs[i], lens[i]) for every i: ptrs an int64 device
    tensor of device addresses, lens an int32 device tensor."""
    n = _ctx_tensor(ctxs)
    _need_cuda(ptrs, "ptrs")
    _need_cuda(lens, "lens")
    if ptrs.dtype != torch.int64 or lens.dtype not in (torch.int32, torch.uint32):
        raise TypeError("ptrs must be int64 and lens int32")
    if ptrs.numel() != n or lens.numel() != n:
        raise ValueError("one pointer and one length per context")
    check("md5hip_update_ctx", lib().md5hip_update_ctx(ctxs.data_ptr(), ptrs.data_ptr(), lens.data_ptr(),
                                                       n, _stream(stream)))
    return ctxs


def final_ctx(ctxs, out=None, stream=None):
    """MD5Final on every context: uint8 [n, 16] digests on the device; the
    contexts are zeroed (md5.c:264)."""
    n = _ctx_tensor(ctxs)
    if out is None:
        out = torch.empty((n, 16), dtype=torch.uint8, device=ctxs.device)
    _need_cuda(out, "out")
    check("md5hip_final_ctx", lib().md5hip_final_ctx(ctxs.data_ptr(), n, out.data_ptr(), _stream(stream)))
    return out


CRC_VARIANTS = {"auto": 0, "xdma16": 6, "split": 7}   # enum crc32hip_variant


def crc32_fixed(data, n: int = None, length: int = None, stride: int = None, fastcrc: int = 0,
                out=None, stream=None, variant=0):
    """crcs[i] = netcache block CRC-32 of chunk i (blk_make_crc semantics,
    blk_io.c:354-430; fastcrc > 0 -> head ^ tail).  uint32 [n] on device."""
    _need_cuda(data, "data")
    if n is None or length is None:
        if data.dim() != 2:
            raise ValueError("pass n and length, or a 2-D [n, length] tensor")
        n, length = data.shape
    stride = length if stride is None else stride
    if n and (n - 1) * stride + length > data.numel():
        raise ValueError("batch extends past the end of `data`")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=data.device)
    if isinstance(variant, str):
        variant = CRC_VARIANTS[variant]
    check("crc32hip_fixed_variant",
          lib().crc32hip_fixed_variant(data.data_ptr(), n, length, stride, fastcrc, out.data_ptr(),
                                       _stream(stream), variant))
    return out


def crc32_desc(base, offsets, lens, order=None, fastcrc: int = 0, out=None, stream=None, variant=0):
    _need_cuda(base, "base")
    _need_cuda(offsets, "offsets")
    _need_cuda(lens, "lens")
    n = offsets.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=base.device)
    if isinstance(variant, str):
        variant = CRC_VARIANTS[variant]
    check("crc32hip_desc_variant",
          lib().crc32hip_desc_variant(base.data_ptr(), offsets.data_ptr(), lens.data_ptr(),
                                      order.data_ptr() if order is not None else None, n,
                                      fastcrc, out.data_ptr(), _stream(stream), variant))
    return out


class _Arena:
    """Owner of one md5hip_arena_alloc block, exposed through
    __cuda_array_interface__ so torch can wrap it without a copy."""

    def __init__(self, nbytes: int, device: int):
        p = ctypes.c_void_p()
        check("md5hip_arena_alloc", lib().md5hip_arena_alloc(device, nbytes, ctypes.byref(p)))
        self.ptr, self.nbytes = p.value, nbytes
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                         "strides": None, "version": 2}

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().md5hip_arena_free(ctypes.c_void_p(self.ptr))
            self.ptr = None


def arena_empty(nbytes: int, device=None) -> torch.Tensor:
    """uint8 [nbytes] device tensor in a batch arena (md5hip_arena_alloc:
    1 GiB-aligned virtual range, large page-table fragments).  The arena is
    freed when the tensor is."""
    dev = torch.cuda.current_device() if device is None else int(device)
    owner = _Arena(int(nbytes), dev)
    with torch.cuda.device(dev):
        t = torch.as_tensor(owner, device=f"cuda:{dev}")
    t._md5hip_arena = owner            # keep the owner alive with the tensor
    return t


def plan_desc(lens):
    """(order, variant name): md5hip_plan_desc -- the longest-first order and
    the descriptor kernel the planner picks for this batch shape."""
    L = np.ascontiguousarray(lens, dtype=np.uint32)
    order = np.empty(max(L.size, 1), dtype=np.uint32)
    v = lib().md5hip_plan_desc(L.ctypes.data, L.size, order.ctypes.data)
    if v < 0:
        raise MD5HipError("md5hip_plan_desc", v)
    return order[:L.size], {x: k for k, x in DESC_VARIANTS.items()}[v]


def plan_desc_at(lens, addrs):
    """(order, variant name): md5hip_plan_desc_at -- as plan_desc, for chunks
    at the given device addresses (or offsets from a 128-B-aligned base):
    'lines' for an XDMA batch mostly of chunks off their 128-B lines."""
    L = np.ascontiguousarray(lens, dtype=np.uint32)
    A = np.ascontiguousarray(addrs, dtype=np.uint64)
    if A.size != L.size:
        raise ValueError("one address per length")
    order = np.empty(max(L.size, 1), dtype=np.uint32)
    v = lib().md5hip_plan_desc_at(L.ctypes.data, A.ctypes.data, L.size, order.ctypes.data)
    if v < 0:
        raise MD5HipError("md5hip_plan_desc_at", v)
    return order[:L.size], {x: k for k, x in DESC_VARIANTS.items()}[v]


def plan_order(lens) -> np.ndarray:
    """Longest-first lane order (md5hip_plan_order), host arrays."""
    L = np.ascontiguousarray(lens, dtype=np.uint32)
    order = np.empty(max(L.size, 1), dtype=np.uint32)
    check("md5hip_plan_order", lib().md5hip_plan_order(L.ctypes.data, L.size, order.ctypes.data))
    return order[:L.size]


def fill_synthetic(t, seed: int, stream=None):
    _need_cuda(t, "t")
    nbytes = t.numel() * t.element_size()
    check("md5hip_fill_synthetic",
          lib().md5hip_fill_synthetic(t.data_ptr(), nbytes, seed & (2**64 - 1), _stream(stream)))
    return t


def variant_name(v: int) -> str:
    return lib().md5hip_variant_name(v).decode()


def crc_variant_name(v=0) -> str:
    """Name (CRC_VARIANTS key) of the CRC-32 kernel variant v resolves to."""
    r = lib().crc32hip_resolve_variant(CRC_VARIANTS[v] if isinstance(v, str) else v)
    return {k: x for x, k in CRC_VARIANTS.items()}[r]


def crc_kernel_name(length: int, fastcrc: int = 0) -> str:
    """The kernel crc32hip_fixed launches for 16-B aligned chunks of `length`
    bytes (bench.py's roofline names it)."""
    if 0 < fastcrc < length:
        return "crc32_fast_pipe" if fastcrc in (64, 128) else "crc32_fast_xdma16"
    return "crc32_fixed_" + crc_variant_name(0)


def kernel_code_hash(kernel: str) -> str:
    """SHA-256 of one kernel's gfx950 machine code in libmd5hip.so (keys the
    PMC entries of profiles/traffic.json)."""
    from ._lib import kernel_code_hash as h
    return h(kernel)


def resolve_variant(v=AUTO) -> int:
    """The concrete kernel variant that `v` (AUTO by default) runs."""
    if isinstance(v, str):
        v = VARIANTS[v]
    return lib().md5hip_resolve_variant(v)


# ---------------------------------------------------------------- host batches
class Batcher:
    """The batcher (include/md5hip.h md5hip_batcher_*): a thread-safe,
    coalescing submission queue; tickets complete out of order."""

    MD5, CRC32 = 0, 1
    GATHER_HOST, GATHER_DEVICE, GATHER_DMA, GATHER_AUTO = 0, 1, 2, 3
    _fn = dict(set_digest="md5hip_batcher_set_digest", set_gather="md5hip_batcher_set_gather",
               destroy="md5hip_batcher_destroy",
               submit="md5_batch_submit", submit_iov="md5_batch_submit_iov",
               verify_iov="md5hip_batch_verify_iov", host_fixed="md5hip_batch_host_fixed",
               submit_async="md5_batch_submit_async", submit_iov_async="md5_batch_submit_iov_async",
               wait="md5_batch_wait", poll="md5_batch_poll", flush="md5_batch_flush",
               submit_device_async="md5_batch_submit_device_async",
               submit_device="md5_batch_submit_device", submit_device_on="md5_batch_submit_device_on",
               submit_device_after="md5_batch_submit_device_after",
               submit_device_fixed="md5_batch_submit_device_fixed",
               set_inflight="md5hip_batcher_set_inflight",
               set_linger="md5hip_batcher_set_linger", set_chain="md5hip_batcher_set_chain",
               stats="md5hip_batcher_get_stats", inject_fault="md5hip_batcher_inject_fault")

    def __init__(self, device: int = 0, slice_bytes: int = 0, nslots: int = 0,
                 kind: int = 0, fastcrc: int = 0):
        """slice_bytes / nslots 0 = the library defaults (128 MiB x 4)."""
        h = ctypes.c_void_p()
        check("md5hip_batcher_create", lib().md5hip_batcher_create(device, slice_bytes, nslots,
                                                                    ctypes.byref(h)))
        self._h = h
        self.device = device
        self.set_digest(kind, fastcrc)

    def _call(self, op, *args):
        name = self._fn[op]
        return name, getattr(lib(), name)(self._h, *args)

    def set_digest(self, kind: int, fastcrc: int = 0):
        """MD5 (16 B per chunk) or netcache CRC-32 (4 B, optional fastcrc window)."""
        check(*self._call("set_digest", kind, fastcrc))
        self.kind, self.dsz = kind, (16 if kind == self.MD5 else 4)

    def set_gather(self, mode: int):
        """HOST (memcpy into pinned staging), DEVICE (gather kernel over PCIe)
        or DMA (batched async copies); the last two apply to calls whose
        segments all lie in register_host()'ed memory."""
        check(*self._call("set_gather", mode))

    def _out(self, n):
        return np.empty((max(n, 1), self.dsz), dtype=np.uint8)

    def _ret(self, out, n):
        out = out[:n]
        return out if self.dsz == 16 else out.view("<u4").reshape(n)

    def close(self):
        if getattr(self, "_h", None):
            getattr(lib(), self._fn["destroy"])(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def submit(self, buffers) -> np.ndarray:
        """digests[i] = MD5(buffers[i]) for a list of bytes-like host buffers."""
        n = len(buffers)
        keep, ptrs = [], (ctypes.c_void_p * max(n, 1))()
        lens = np.empty(max(n, 1), dtype=np.uint32)
        for i, b in enumerate(buffers):
            a, k = _addr(b)
            keep.append(k)
            ptrs[i] = a
            lens[i] = memoryview(b).nbytes
        out = self._out(n)
        check(*self._call("submit", ptrs, lens.ctypes.data, n, out.ctypes.data))
        return self._ret(out, n)

    def _iov(self, chunks):
        segs, first, keep = [], [0], []
        for segl in chunks:
            for sgm in segl:
                a, k = _addr(sgm)
                keep.append(k)
                segs.append((a, memoryview(sgm).nbytes))
            first.append(len(segs))
        arr = (MD5HipIov * max(len(segs), 1))()
        for j, (a, L) in enumerate(segs):
            arr[j].base = a
            arr[j].len = L
        return arr, np.asarray(first, dtype=np.uint64), keep

    def submit_iov(self, chunks) -> np.ndarray:
        """digests[i] = digest(b"".join(chunks[i])) for a list of segment lists
        (a netcache block = its list of pages)."""
        arr, fa, keep = self._iov(chunks)
        n = len(chunks)
        out = self._out(n)
        check(*self._call("submit_iov", arr, fa.ctypes.data, n, out.ctypes.data))
        del keep
        return self._ret(out, n)

    class Pending:
        """An asynchronous submission: `ticket`, the output array, and the
        input references the device may still read (zero-copy modes)."""

        def __init__(self, batcher, ticket, out, n, keep, on_device=False):
            self.batcher, self.ticket, self._out, self.n, self._keep = batcher, ticket, out, n, keep
            self.on_device = on_device

        def poll(self) -> bool:
            name, rc = self.batcher._call("poll", ctypes.c_uint64(self.ticket))
            if rc < 0:
                check(name, rc)
            return rc == 1

        def wait(self):
            check(*self.batcher._call("wait", ctypes.c_uint64(self.ticket)))
            self._keep = None
            return self._out if self.on_device else self.batcher._ret(self._out, self.n)

    def submit_async(self, buffers) -> "Batcher.Pending":
        """md5_batch_submit_async: returns once the chunks are staged; the
        digests are valid after .wait() (or once .poll() is True)."""
        n = len(buffers)
        keep, ptrs = [], (ctypes.c_void_p * max(n, 1))()
        lens = np.empty(max(n, 1), dtype=np.uint32)
        for i, b in enumerate(buffers):
            a, k = _addr(b)
            keep.append(k)
            ptrs[i] = a
            lens[i] = memoryview(b).nbytes
        out = self._out(n)
        t = ctypes.c_uint64()
        check(*self._call("submit_async", ptrs, lens.ctypes.data, n, out.ctypes.data, ctypes.byref(t)))
        return Batcher.Pending(self, t.value, out, n, (keep, ptrs, lens))

    def submit_iov_async(self, chunks) -> "Batcher.Pending":
        arr, fa, keep = self._iov(chunks)
        n = len(chunks)
        out = self._out(n)
        t = ctypes.c_uint64()
        check(*self._call("submit_iov_async", arr, fa.ctypes.data, n, out.ctypes.data,
                          ctypes.byref(t)))
        return Batcher.Pending(self, t.value, out, n, (keep, arr, fa))

    def _dev_args(self, ptrs, lens, out):
        """(ptrs, lens, digest destination, on_device) for the device-input
        entries; `out` is a device tensor on the batcher's device (digests
        stay there), a C-contiguous uint8 numpy array, or None (a new host
        array).  Either must hold n digests of this batcher's kind."""
        P = np.ascontiguousarray(ptrs, dtype=np.uint64)
        L = np.ascontiguousarray(lens, dtype=np.uint32)
        if P.size != L.size:
            raise ValueError("ptrs and lens differ in length")
        o, on_dev = self._dev_out(P.size, out)
        return P, L, o, on_dev

    def _dev_out(self, n, out):
        """(digest destination, on_device) for n digests: a device tensor on
        the batcher's device, a C-contiguous uint8 numpy array, or None (a
        new host array)."""
        need = n * self.dsz
        if torch is not None and isinstance(out, torch.Tensor):
            if not out.is_cuda or not out.is_contiguous() or out.numel() * out.element_size() < need:
                raise ValueError(f"out must be a contiguous device tensor of >= n x {self.dsz} bytes")
            if out.device.index != self.device:
                raise ValueError(f"out is on cuda:{out.device.index}, the batcher on cuda:{self.device}")
            return out, 1
        if out is None:
            return self._out(n), 0
        if not (isinstance(out, np.ndarray) and out.dtype == np.uint8 and out.flags.c_contiguous
                and out.nbytes >= need):
            raise ValueError(f"out must be a C-contiguous uint8 array of >= n x {self.dsz} bytes")
        return out, 0

    def _producer(self, after):
        """(stream handle, order) for md5_batch_submit_device_after:
        'current' = torch's current stream on the batcher's device -- its
        handle is 0 (NULL) when that is the default stream, which the library
        then orders on as the null stream, never as "no ordering"; without
        torch, 'current' is the null stream of the batcher's device (what a
        raw-HIP producer enqueues on when it names no stream); None = no
        ordering."""
        if isinstance(after, str):
            if after != "current":
                raise ValueError("after: 'current', None or a stream")
            if torch is None:
                return None, 1
            return torch.cuda.current_stream(self.device).cuda_stream, 1
        if after is None:
            return None, 0
        return getattr(after, "cuda_stream", after), 1

    def submit_device_async(self, ptrs, lens, out=None, after="current") -> "Batcher.Pending":
        """md5_batch_submit_device_after: chunk i = (device address ptrs[i],
        lens[i]); digests into `out` -- a device tensor (digests stay on the
        device) or, by default, a host array returned by .wait().  The kernel
        runs after the work already enqueued on `after` (default: torch's
        current stream -- the stream that wrote the chunks); None = no
        ordering (the caller has synchronized)."""
        P, L, o, on_dev = self._dev_args(ptrs, lens, out)
        t = ctypes.c_uint64()
        dst = o.data_ptr() if on_dev else o.ctypes.data
        check(*self._call("submit_device_after", P.ctypes.data, L.ctypes.data, P.size, dst, on_dev,
                          *self._producer(after), ctypes.byref(t)))
        return Batcher.Pending(self, t.value, o, P.size, (P, L, o), on_dev)

    def submit_device(self, ptrs, lens, out=None, after="current"):
        P, L, o, on_dev = self._dev_args(ptrs, lens, out)
        dst = o.data_ptr() if on_dev else o.ctypes.data
        check(*self._call("submit_device_after", P.ctypes.data, L.ctypes.data, P.size, dst, on_dev,
                          *self._producer(after), None))
        return o if on_dev else self._ret(o, P.size)

    def submit_device_fixed_async(self, base, n: int, length: int, stride: int = None, out=None,
                                  after="current") -> "Batcher.Pending":
        """md5_batch_submit_device_fixed (ABI 4): digest i of (base + i*stride,
        length) for a device tensor (or device address) `base` on the
        batcher's device, read in place -- no per-chunk descriptor; digests in
        the batcher's kind into `out` (a device tensor, or by default a host
        array returned by .wait()); `after` as submit_device_async."""
        stride = length if stride is None else stride
        if n and length > stride:
            raise ValueError("length > stride")
        if torch is not None and isinstance(base, torch.Tensor):
            if not base.is_cuda or base.device.index != self.device:
                raise ValueError(f"base must be a device tensor on cuda:{self.device}")
            if n and base.numel() * base.element_size() < (n - 1) * stride + length:
                raise ValueError("base is smaller than n chunks of the stride")
            addr = base.data_ptr()
        else:
            addr = int(base)
        o, on_dev = self._dev_out(n, out)
        t = ctypes.c_uint64()
        dst = o.data_ptr() if on_dev else o.ctypes.data
        check(*self._call("submit_device_fixed", ctypes.c_void_p(addr), n, length, stride, dst, on_dev,
                          *self._producer(after), ctypes.byref(t)))
        return Batcher.Pending(self, t.value, o, n, (base, o), on_dev)

    def flush(self):
        check(*self._call("flush"))

    def health(self) -> int:
        """0 healthy, -ENODEV once the device failed (ABI 4, sticky)."""
        return lib().md5hip_batcher_health(self._h)

    def inject_fault(self, after: int = 1):
        """Test control (ABI 4): the after-th launch from now completes as a
        device fault (its tickets -EIO, the batcher failed from then on)."""
        check(*self._call("inject_fault", ctypes.c_uint64(after)))

    def set_inflight(self, target: int):
        """Launch the open slot at once while fewer than `target` slots run."""
        check(*self._call("set_inflight", target))

    def set_linger(self, max_us: int):
        """Idle pipeline: hold an async submission's slot up to
        min(max_us, 1/8 of recent launch time) for more work (0 = never)."""
        check(*self._call("set_linger", max_us))

    def set_chain(self, on):
        """Chained launches: 1 = the next slot's kernel queued behind the
        running launch's event just before it ends; 2 (the default) = the
        same without the device-side wait when both launches are BALANCED
        (the next one's workgroups take CUs as the running one's finish);
        0/False = off."""
        check(*self._call("set_chain", int(on)))

    def stats(self) -> dict:
        st = MD5HipBatcherStats()
        check(*self._call("stats", ctypes.byref(st)))
        return {n: int(getattr(st, n)) for n, _ in MD5HipBatcherStats._fields_}

    def verify_iov(self, chunks, expected):
        """(ok[i] bool array, mismatch count): digest(chunks[i]) == expected[i]."""
        arr, fa, keep = self._iov(chunks)
        n = len(chunks)
        exp = np.ascontiguousarray(expected)
        if exp.nbytes != n * self.dsz:
            raise ValueError("expected must hold one digest per chunk")
        ok = np.empty(max(n, 1), dtype=np.uint8)
        name, rc = self._call("verify_iov", arr, fa.ctypes.data, n, exp.ctypes.data, ok.ctypes.data)
        if rc < 0:
            check(name, rc)
        del keep
        return ok[:n].astype(bool), rc

    def host_fixed(self, arr: np.ndarray, n: int, length: int, stride: int = None) -> np.ndarray:
        stride = length if stride is None else stride
        a = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        if n and (n - 1) * stride + length > a.size:
            raise ValueError("batch extends past the end of the buffer")
        out = self._out(n)
        check(*self._call("host_fixed", a.ctypes.data, n, length, stride, out.ctypes.data))
        return self._ret(out, n)


class Queue(Batcher):
    """A batcher sized for device-resident chunks (md5hip_queue_create):
    `max_chunks` descriptors per launch, small host staging."""

    def __init__(self, device: int = 0, max_chunks: int = 0, nslots: int = 0, inflight: int = 0):
        h = ctypes.c_void_p()
        check("md5hip_queue_create", lib().md5hip_queue_create(device, max_chunks, nslots,
                                                                ctypes.byref(h)))
        self._h = h
        self.device = device
        self.kind, self.dsz = self.MD5, 16
        if inflight:
            self.set_inflight(inflight)

    def submit(self, *a, **k):           # host-memory chunks work too, through 16 MiB slices
        return Batcher.submit(self, *a, **k)


class Pool(Batcher):
    """Multi-GPU host pool (include/md5hip.h md5hip_pool_*): a router over one
    coalescing batcher per listed device.  A submission goes whole to the
    least-loaded device; only one heavier than the split threshold is cut
    over devices.  No collective.  Same methods and results as
    Batcher, including the asynchronous forms and their tickets."""

    _fn = dict(set_digest="md5hip_pool_set_digest", set_gather="md5hip_pool_set_gather",
               destroy="md5hip_pool_destroy",
               submit="md5hip_pool_submit", submit_iov="md5hip_pool_submit_iov",
               verify_iov="md5hip_pool_verify_iov", host_fixed="md5hip_pool_host_fixed",
               submit_async="md5hip_pool_submit_async", submit_iov_async="md5hip_pool_submit_iov_async",
               wait="md5hip_pool_wait", poll="md5hip_pool_poll", set_split="md5hip_pool_set_split")

    def __init__(self, devices=(0,), slice_bytes: int = 0, nslots: int = 0,
                 kind: int = 0, fastcrc: int = 0):
        devs = (ctypes.c_int * max(len(devices), 1))(*devices)
        h = ctypes.c_void_p()
        check("md5hip_pool_create", lib().md5hip_pool_create(devs, len(devices), slice_bytes,
                                                              nslots, ctypes.byref(h)))
        self._h = h
        self.devices = tuple(devices)
        self.set_digest(kind, fastcrc)

    @property
    def ndev(self) -> int:
        return lib().md5hip_pool_ndev(self._h)

    def set_split(self, nbytes: int):
        """Submissions heavier than `nbytes` are cut over devices (0 = one slice)."""
        check(*self._call("set_split", nbytes))

    def health(self) -> dict:
        """md5hip_pool_get_health (ABI 4): failed devices and failovers."""
        from ._lib import MD5HipPoolHealth
        h = MD5HipPoolHealth()
        check("md5hip_pool_get_health", lib().md5hip_pool_get_health(self._h, ctypes.byref(h)))
        return {"ndev": h.ndev, "nfailed": h.nfailed, "failed_mask": h.failed_mask, "failovers": h.failovers}

    def inject_fault(self, g: int, after: int = 1):
        check("md5hip_pool_inject_fault", lib().md5hip_pool_inject_fault(self._h, g, ctypes.c_uint64(after)))

    def stats(self) -> dict:
        """Routing counters: submissions, routed_whole, split, parts."""
        st = MD5HipPoolStats()
        check("md5hip_pool_get_stats", lib().md5hip_pool_get_stats(self._h, ctypes.byref(st)))
        return {n: int(getattr(st, n)) for n, _ in MD5HipPoolStats._fields_}

    def device_stats(self, g: int) -> dict:
        """Device g's batcher counters (as Batcher.stats())."""
        st = MD5HipBatcherStats()
        check("md5hip_pool_device_stats", lib().md5hip_pool_device_stats(self._h, g, ctypes.byref(st)))
        return {n: int(getattr(st, n)) for n, _ in MD5HipBatcherStats._fields_}

    def _unsupported(self, *a, **k):
        raise NotImplementedError("device-resident chunks belong to one device: use a Queue")

    submit_device = submit_device_async = submit_device_fixed_async = flush = set_inflight = set_linger = \
        _unsupported


def register_host(arr: np.ndarray):
    """md5hip_host_register over a numpy array's buffer (pin + device-map)."""
    check("md5hip_host_register", lib().md5hip_host_register(arr.ctypes.data, arr.nbytes))


def unregister_host(arr: np.ndarray):
    check("md5hip_host_unregister", lib().md5hip_host_unregister(arr.ctypes.data))


def pool_plan(lens, nparts: int) -> np.ndarray:
    """md5hip_pool_plan: first[0..nparts] of the pool's contiguous split
    (lens None: equal counts over `lens`=n given as an int)."""
    first = np.empty(nparts + 1, dtype=np.uint64)
    if isinstance(lens, int):
        check("md5hip_pool_plan", lib().md5hip_pool_plan(None, lens, nparts, first.ctypes.data))
    else:
        L = np.ascontiguousarray(lens, dtype=np.uint32)
        check("md5hip_pool_plan", lib().md5hip_pool_plan(L.ctypes.data if L.size else None, L.size,
                                                          nparts, first.ctypes.data))
    return first


__all__ = ["init_ctx", "update_ctx", "final_ctx", "MD5Context", "MD5Init", "MD5Update", "MD5Final", "MD5_DIGEST_SIZE", "MD5HipError", "arena_empty",
           "plan_desc", "plan_desc_at",
           "md5", "digest_fixed", "digest_desc", "crc32_fixed", "crc32_desc", "plan_order", "fill_synthetic", "Batcher",
           "Pool", "Queue", "pool_plan", "CRC_VARIANTS", "DESC_VARIANTS",
           "register_host", "unregister_host",
           "variant_name", "resolve_variant", "VARIANTS", "crc_variant_name"]
