"""ctypes binding of libmd5hip.so (the C ABI declared in include/md5.h and
include/md5hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (make -C
sproxy_amd/csrc).  There is NO fallback: if the shared object is missing or a
call fails, the error surfaces -- the product never routes through the oracle
or a host-side hash.

torch is imported first when available so that libmd5hip.so binds to the same
libamdhip64.so.7 instance torch uses (both carry that SONAME), which makes torch
streams and torch-allocated device pointers valid handles for our entries.
"""
import ctypes
import errno
import os

try:  # share torch's HIP runtime (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is plumbing, not required for the C path
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libmd5hip.so")

_lib = None

c_u8p = ctypes.c_void_p


class MD5Context(ctypes.Structure):
    """struct MD5Context, md5.h:33-38 (88 bytes)."""
    _fields_ = [("buf", ctypes.c_uint32 * 4), ("bits", ctypes.c_uint32 * 2),
                ("in_", ctypes.c_ubyte * 64)]


class MD5HipIov(ctypes.Structure):
    """struct md5hip_iov (include/md5hip.h)."""
    _fields_ = [("base", ctypes.c_void_p), ("len", ctypes.c_uint32)]


class MD5HipBatcherStats(ctypes.Structure):
    """struct md5hip_batcher_stats (include/md5hip.h)."""
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "submissions", "launches", "coalesced_launches", "chunks", "bytes_staged",
        "max_chunks_per_launch", "max_tickets_per_launch", "inflight_target", "nslots",
        "max_chunks_per_slot")]


class MD5HipPoolStats(ctypes.Structure):
    """struct md5hip_pool_stats (include/md5hip.h)."""
    _fields_ = [(n, ctypes.c_uint64) for n in ("submissions", "routed_whole", "split", "parts")]


class MD5HipPoolHealth(ctypes.Structure):
    """struct md5hip_pool_health (include/md5hip.h, ABI 4)."""
    _fields_ = [("ndev", ctypes.c_uint32), ("nfailed", ctypes.c_uint32),
                ("failed_mask", ctypes.c_uint64), ("failovers", ctypes.c_uint64)]


class MD5HipError(RuntimeError):
    def __init__(self, fn, rc):
        name = errno.errorcode.get(-rc, str(rc))
        super().__init__(f"{fn} failed: {rc} ({name})")
        self.rc = rc


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    u64, u32, vp, i = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int
    sig = {
        "MD5Init": (None, [ctypes.POINTER(MD5Context)]),
        "MD5Update": (None, [ctypes.POINTER(MD5Context), vp, ctypes.c_uint]),
        "MD5Final": (None, [vp, ctypes.POINTER(MD5Context)]),
        "md5hip_abi_version": (i, []),
        "md5hip_variant_name": (ctypes.c_char_p, [i]),
        "md5hip_resolve_variant": (i, [i]),
        "crc32hip_resolve_variant": (i, [i]),
        "md5hip_digest_fixed": (i, [vp, u64, u32, u64, vp, vp]),
        "md5hip_digest_fixed_variant": (i, [vp, u64, u32, u64, vp, vp, i]),
        "md5hip_digest_desc": (i, [vp, vp, vp, vp, u64, vp, vp]),
        "md5hip_digest_desc_variant": (i, [vp, vp, vp, vp, u64, vp, vp, i]),
        "md5hip_plan_order": (i, [vp, u64, vp]),
        "md5hip_plan_desc": (i, [vp, u64, vp]),
        "md5hip_plan_desc_at": (i, [vp, vp, u64, vp]),
        "md5hip_arena_alloc": (i, [i, u64, vp]),
        "md5hip_arena_free": (i, [vp]),
        "crc32hip_fixed": (i, [vp, u64, u32, u64, u32, vp, vp]),
        "crc32hip_desc": (i, [vp, vp, vp, vp, u64, u32, vp, vp]),
        "crc32hip_desc_variant": (i, [vp, vp, vp, vp, u64, u32, vp, vp, i]),
        "crc32hip_fixed_variant": (i, [vp, u64, u32, u64, u32, vp, vp, i]),
        "md5hip_fill_synthetic": (i, [vp, u64, u64, vp]),
        "md5hip_batcher_create": (i, [i, u64, u32, ctypes.POINTER(vp)]),
        "md5hip_queue_create": (i, [i, u64, u32, ctypes.POINTER(vp)]),
        "md5hip_batcher_set_inflight": (i, [vp, u32]),
        "md5hip_batcher_set_linger": (i, [vp, u32]),
        "md5hip_batcher_set_chain": (i, [vp, i]),
        "md5hip_plan_hist": (i, [vp, u32, u64, vp]),
        "md5hip_order_device": (i, [vp, u64, u32, vp, vp, vp]),
        "md5hip_order_stable_scratch": (u64, [u64, u32]),
        "md5hip_order_device_stable": (i, [vp, u64, u32, vp, u64, vp, vp]),
        "md5hip_batcher_get_stats": (i, [vp, ctypes.POINTER(MD5HipBatcherStats)]),
        "md5_batch_submit_device_async": (i, [vp, vp, vp, u64, vp, i, vp]),
        "md5_batch_submit_device": (i, [vp, vp, vp, u64, vp, i]),
        "md5_batch_flush": (i, [vp]),
        "md5hip_init_ctx": (i, [vp, u64, vp]),
        "md5hip_update_ctx": (i, [vp, vp, vp, u64, vp]),
        "md5hip_final_ctx": (i, [vp, u64, vp, vp]),
        "md5hip_batcher_destroy": (None, [vp]),
        "md5_batch_submit": (i, [vp, vp, vp, u64, vp]),
        "md5_batch_submit_iov": (i, [vp, vp, vp, u64, vp]),
        "md5_batch_submit_async": (i, [vp, vp, vp, u64, vp, vp]),
        "md5_batch_submit_iov_async": (i, [vp, vp, vp, u64, vp, vp]),
        "md5_batch_wait": (i, [vp, u64]),
        "md5_batch_poll": (i, [vp, u64]),
        "md5hip_batcher_set_digest": (i, [vp, i, u32]),
        "md5hip_batch_verify_iov": (i, [vp, vp, vp, u64, vp, vp]),
        "md5hip_batch_host_fixed": (i, [vp, vp, u64, u32, u64, vp]),
        "md5hip_pool_create": (i, [vp, u32, u64, u32, ctypes.POINTER(vp)]),
        "md5hip_pool_destroy": (None, [vp]),
        "md5hip_pool_ndev": (i, [vp]),
        "md5hip_pool_set_digest": (i, [vp, i, u32]),
        "md5hip_pool_submit": (i, [vp, vp, vp, u64, vp]),
        "md5hip_pool_submit_iov": (i, [vp, vp, vp, u64, vp]),
        "md5hip_pool_verify_iov": (i, [vp, vp, vp, u64, vp, vp]),
        "md5hip_pool_host_fixed": (i, [vp, vp, u64, u32, u64, vp]),
        "md5hip_pool_plan": (i, [vp, u64, u32, vp]),
        "md5hip_batcher_get_digest": (i, [vp, vp, vp]),
        "md5hip_host_register": (i, [vp, u64]),
        "md5hip_host_unregister": (i, [vp]),
        "md5hip_batcher_set_gather": (i, [vp, i]),
        "md5hip_pool_set_gather": (i, [vp, i]),
        "md5hip_pool_set_split": (i, [vp, u64]),
        "md5hip_pool_submit_async": (i, [vp, vp, vp, u64, vp, vp]),
        "md5hip_pool_submit_iov_async": (i, [vp, vp, vp, u64, vp, vp]),
        "md5hip_pool_wait": (i, [vp, u64]),
        "md5hip_pool_poll": (i, [vp, u64]),
        "md5hip_pool_get_stats": (i, [vp, ctypes.POINTER(MD5HipPoolStats)]),
        "md5hip_pool_device_stats": (i, [vp, u32, ctypes.POINTER(MD5HipBatcherStats)]),
        "md5_batch_submit_device_on": (i, [vp, vp, vp, u64, vp, i, vp, vp]),
        "md5_batch_submit_device_after": (i, [vp, vp, vp, u64, vp, i, vp, i, vp]),
        "nc_canned_digest_size": (u64, [u32, u32]),
        "nc_digest_update": (i, [vp, u64, u32, u64, u64, vp]),
        "nc_digest_verify": (i, [vp, u64, u32, u64, vp]),
        "nc_digest_scatter": (i, [vp, u64, u32, u64, vp, u64, vp]),
        "nc_digest_compare": (i, [vp, u64, u32, vp, u64, vp, vp]),
        "nc_crc32": (u32, [vp, u64]),
        "nc_header_crc": (u32, [vp]),
        "nc_header_seal": (i, [vp]),
        "nc_header_verify": (i, [vp]),
        "md5hip_batch_verify_headers": (i, [vp, vp, u64, vp]),
        "md5hip_batcher_health": (i, [vp]),
        "md5hip_batcher_inject_fault": (i, [vp, u64]),
        "md5hip_pool_get_health": (i, [vp, ctypes.POINTER(MD5HipPoolHealth)]),
        "md5hip_pool_device_health": (i, [vp, u32]),
        "md5hip_pool_inject_fault": (i, [vp, u32, u64]),
        "md5_batch_submit_device_fixed": (i, [vp, vp, u64, u32, u64, vp, i, vp, i, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


# Every symbol include/*.h declares (checked by tests/test_abi.py).
EXPORTS = ["MD5Init", "MD5Update", "MD5Final", "nc_MD5Init", "nc_MD5Update", "nc_MD5Final", "md5hip_abi_version", "md5hip_variant_name",
           "md5hip_resolve_variant", "crc32hip_resolve_variant",
           "md5hip_digest_fixed", "md5hip_digest_fixed_variant", "md5hip_digest_desc",
           "md5hip_digest_desc_variant",
           "md5hip_plan_order", "md5hip_plan_desc", "md5hip_arena_alloc", "md5hip_arena_free",
           "md5hip_fill_synthetic", "md5hip_batcher_create",
           "crc32hip_fixed", "crc32hip_desc", "crc32hip_desc_variant", "crc32hip_fixed_variant",
           "md5hip_batcher_destroy", "md5_batch_submit", "md5_batch_submit_iov",
           "md5_batch_submit_async", "md5_batch_submit_iov_async", "md5_batch_wait", "md5_batch_poll",
           "md5hip_batcher_set_digest", "md5hip_batch_verify_iov",
           "md5hip_batch_host_fixed", "md5hip_pool_create", "md5hip_pool_destroy",
           "md5hip_pool_ndev", "md5hip_pool_set_digest", "md5hip_pool_submit",
           "md5hip_pool_submit_iov", "md5hip_pool_verify_iov", "md5hip_pool_host_fixed",
           "md5hip_pool_plan", "md5hip_batcher_get_digest", "nc_canned_digest_size",
           "nc_digest_update", "nc_digest_verify", "nc_digest_scatter", "nc_digest_compare",
           "nc_crc32", "nc_header_crc", "nc_header_seal", "nc_header_verify",
           "md5hip_batch_verify_headers", "md5hip_host_register", "md5hip_host_unregister",
           "md5hip_batcher_set_gather", "md5hip_pool_set_gather", "md5hip_queue_create",
           "md5hip_batcher_set_inflight", "md5hip_batcher_set_linger", "md5hip_plan_hist", "md5hip_order_device",
           "md5hip_order_stable_scratch", "md5hip_order_device_stable",
           "md5hip_batcher_get_stats", "md5_batch_submit_device_async",
           "md5_batch_submit_device", "md5_batch_flush", "md5hip_init_ctx", "md5hip_update_ctx",
           "md5hip_final_ctx", "md5hip_pool_set_split", "md5hip_pool_submit_async",
           "md5hip_pool_submit_iov_async", "md5hip_pool_wait", "md5hip_pool_poll",
           "md5hip_pool_get_stats", "md5hip_pool_device_stats", "md5_batch_submit_device_on",
           "md5_batch_submit_device_after", "md5hip_plan_desc_at", "md5hip_batcher_set_chain",
           "md5hip_batcher_health", "md5hip_batcher_inject_fault", "md5hip_pool_get_health",
           "md5hip_pool_device_health", "md5hip_pool_inject_fault", "md5_batch_submit_device_fixed"]


def check(fn, rc):
    if rc != 0:
        raise MD5HipError(fn, rc)


def _elf_sections(elf: bytes):
    import struct
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError("not an ELF64 object")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + k * shentsize) for k in range(shnum)]
    stroff = secs[shstrndx][4]
    out = {}
    for sec in secs:
        name = elf[stroff + sec[0]:elf.index(b"\0", stroff + sec[0])].decode()
        out[name] = sec           # (name, type, flags, addr, offset, size, link, info, align, entsize)
    return out


def _device_elf(path: str = LIB_PATH) -> bytes:
    """The gfx950 code object inside the library's offload bundle."""
    import struct
    with open(path, "rb") as f:
        elf = f.read()
    sec = _elf_sections(elf)[".hip_fatbin"]
    fb = elf[sec[4]:sec[4] + sec[5]]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    if not fb.startswith(magic):
        raise ValueError(f"{path}: unsupported offload bundle")
    nent, = struct.unpack_from("<Q", fb, len(magic))
    pos = len(magic) + 8
    for _ in range(nent):
        off, size, tlen = struct.unpack_from("<QQQ", fb, pos)
        triple = fb[pos + 24:pos + 24 + tlen].decode()
        pos += 24 + tlen
        if "gfx950" in triple:
            return fb[off:off + size]
    raise ValueError(f"{path}: no gfx950 code object")


OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def kernel_code_hash(kernel: str, path: str = LIB_PATH) -> str:
    """SHA-256 of one kernel's gfx950 machine code in the library, position
    independent: the kernel (`kernel` = the rocprof short name, e.g.
    md5_fixed_xdma1nt) is disassembled from the library's code object and its
    text hashed with the PC-relative literals after s_getpc_b64 (addresses of
    constants, which move whenever another kernel changes size) masked.
    profiles/traffic.json records it beside each PMC measurement, so counter
    bytes stay attached to the code they measured."""
    import hashlib
    import re
    import struct
    import subprocess
    import tempfile
    co = _device_elf(path)
    secs = _elf_sections(co)
    symtab, strtab = secs[".symtab"], secs[".strtab"]
    ent = symtab[9] or 24
    tag = f"{len(kernel)}{kernel}".encode()
    names = set()
    for k in range(symtab[5] // ent):
        st_name, st_info, _, _, _, st_size = struct.unpack_from("<IBBHQQ", co, symtab[4] + k * ent)
        name = co[strtab[4] + st_name:co.index(b"\0", strtab[4] + st_name)]
        if tag in name and st_size > 64 and (st_info & 0xF) == 2:      # STT_FUNC
            names.add(name.decode())
    if not names:
        raise KeyError(f"kernel {kernel} not in {path}")
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        text = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--no-leading-addr",
                               "--disassemble-symbols=" + ",".join(sorted(names)), f.name],
                              capture_output=True, text=True, check=True).stdout
    h = hashlib.sha256()
    pcrel = 0
    for line in text.splitlines():
        ins = line.split("//")[0].strip()
        if not ins or ins.endswith("file format elf64-amdgpu") or ins.startswith("Disassembly of"):
            continue
        if pcrel and re.match(r"s_addc?_u32 ", ins):
            ins = re.sub(r",[^,]*$", ", PCREL", ins)
            pcrel -= 1
        else:
            pcrel = 2 if ins.startswith("s_getpc_b64") else 0
        h.update(ins.encode() + b"\n")
    return h.hexdigest()


def code_object_hash(path: str = LIB_PATH) -> str:
    """SHA-256 of the library's device code (its .hip_fatbin ELF section):
    counter evidence (profiles/traffic.json) is keyed by it, so numbers taken
    from other kernel code never read as current."""
    import hashlib
    import struct
    with open(path, "rb") as f:
        elf = f.read()
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError(f"{path}: not an ELF64 object")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + k * shentsize) for k in range(shnum)]
    stroff = secs[shstrndx][4]
    for name, _, _, _, off, size, *_ in secs:
        end = elf.index(b"\0", stroff + name)
        if elf[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(elf[off:off + size]).hexdigest()
    raise ValueError(f"{path}: no .hip_fatbin section")
