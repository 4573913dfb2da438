"""Per-block digest array and header CRC of netcache's on-disk object header
(include/nc_digest.h; netcache.h:763-792, diskcache.c:1228-1420, :3149-3265,
:3660-3690).  Thin ctypes layer over libmd5hip.so -- no Python fallback."""
import ctypes

import numpy as np

from ._lib import MD5HipError, check, lib
from .md5 import _addr

NC_MAGIC_V30 = ord("0") << 24 | ord("3") << 16 | ord("B") << 8 | ord("S")   # netcache.h:740
HDR_MIN_SIZE = 20


def canned_digest_size(bitmaplen: int, dsz: int = 4) -> int:
    """Bytes of header chunk #5: align8(bitmaplen*dsz) (NC_CANNED_CRC_SIZE for dsz=4)."""
    return lib().nc_canned_digest_size(bitmaplen, dsz)


class DigestArray:
    """inode->blockcrc / crcsize (netcache.h:408-410) for `dsz`-byte digests."""

    def __init__(self, bitmaplen: int, dsz: int = 4, buf=None):
        self.dsz = dsz
        size = canned_digest_size(bitmaplen, dsz)
        self.buf = np.zeros(size, np.uint8) if buf is None else np.ascontiguousarray(buf, np.uint8)
        if self.buf.size < size:
            raise ValueError("buffer smaller than the canned digest size")

    def _d(self, d):
        a = np.ascontiguousarray(np.frombuffer(bytes(d), np.uint8) if isinstance(d, (bytes, bytearray))
                                 else np.asarray(d).view(np.uint8).reshape(-1))
        return a

    def update(self, blkno: int, digest, mapped: int) -> int:
        """dm_update_block_crc_nolock: 0, -ERANGE (blkno >= mapped), -E2BIG (past the array)."""
        d = self._d(digest)
        return lib().nc_digest_update(self.buf.ctypes.data, self.buf.size, self.dsz, mapped, blkno,
                                      d.ctypes.data)

    def verify(self, blkno: int, digest) -> int:
        """dm_verify_block_crc: 1 equal, 0 mismatch, -ERANGE past the array."""
        d = self._d(digest)
        return lib().nc_digest_verify(self.buf.ctypes.data, self.buf.size, self.dsz, blkno,
                                      d.ctypes.data)

    def scatter(self, blknos, digests, mapped: int) -> int:
        b = np.ascontiguousarray(blknos, np.uint64)
        d = np.ascontiguousarray(digests)
        rc = lib().nc_digest_scatter(self.buf.ctypes.data, self.buf.size, self.dsz, mapped,
                                     b.ctypes.data, b.size, d.ctypes.data)
        if rc < 0:
            check("nc_digest_scatter", rc)
        return rc

    def compare(self, blknos, digests):
        b = np.ascontiguousarray(blknos, np.uint64)
        d = np.ascontiguousarray(digests)
        ok = np.empty(max(b.size, 1), np.uint8)
        rc = lib().nc_digest_compare(self.buf.ctypes.data, self.buf.size, self.dsz, b.ctypes.data,
                                     b.size, d.ctypes.data, ok.ctypes.data)
        if rc < 0:
            check("nc_digest_compare", rc)
        return ok[:b.size].astype(bool), rc


def crc32(data) -> int:
    a, keep = _addr(data)
    return lib().nc_crc32(a, memoryview(data).nbytes)


def _hdr(header):
    """(address, keep-alive) of a header buffer that holds every byte the C
    entry reads: the 20-byte fixed part and header_size bytes (the C ABI,
    like dm_verify_header, takes no buffer size)."""
    nb = memoryview(header).nbytes
    if nb < HDR_MIN_SIZE:
        raise ValueError(f"header buffer of {nb} B: the fixed part is {HDR_MIN_SIZE} B")
    hs = int.from_bytes(bytes(memoryview(header).cast("B")[8:12]), "little", signed=True)
    if hs > nb:
        raise ValueError(f"header_size {hs} exceeds the {nb}-B buffer")
    return _addr(header)


def header_crc(header) -> int:
    """dm_verify_header's CRC: header_size bytes, disk_header_size / flag /
    crc read as zero wherever they fall inside them (0 for header_size < 0)."""
    a, keep = _hdr(header)
    return lib().nc_header_crc(a)


def header_seal(header: bytearray) -> None:
    """Write side (diskcache.c:1391-1393): header.crc := header_crc(header), in place."""
    a, keep = _hdr(header)
    check("nc_header_seal", lib().nc_header_seal(a))


def header_verify(header) -> bool:
    a, keep = _hdr(header)
    return lib().nc_header_verify(a) == 1


def verify_headers(batcher, headers):
    """dm_verify_header over a batch on the GPU: (ok bool array, failures)."""
    n = len(headers)
    keep, ptrs = [], (ctypes.c_void_p * max(n, 1))()
    for i, h in enumerate(headers):
        a, k = _hdr(h)
        keep.append(k)
        ptrs[i] = a
    ok = np.empty(max(n, 1), np.uint8)
    rc = lib().md5hip_batch_verify_headers(batcher._h, ptrs, n, ok.ctypes.data)
    if rc < 0:
        raise MD5HipError("md5hip_batch_verify_headers", rc)
    return ok[:n].astype(bool), rc


__all__ = ["NC_MAGIC_V30", "HDR_MIN_SIZE", "canned_digest_size", "DigestArray", "crc32", "header_crc",
           "header_seal", "header_verify", "verify_headers"]
