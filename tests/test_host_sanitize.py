"""The host-side C entries (MD5 streaming, nc_MD5, CRC-32, header CRC, digest
array, pool split) built from source with AddressSanitizer + UBSan and driven
from plain C (tests/c/host_abi_check.c); results checked against the oracle and
the golden vectors.  Host code only: no HIP call is linked
(-ffunction-sections + --gc-sections drop the device entries)."""
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import gen

sys.path.insert(0, os.path.join(gen.REPO, "oracle"))
import nc_md5_oracle  # noqa: E402

CSRC = os.path.join(gen.REPO, "sproxy_amd", "csrc")
INC = os.path.join(gen.REPO, "include")
SRCS = ["md5_stream.c", "nc_md5.c", "nc_digest.c", "md5_pool.c"]


@pytest.fixture(scope="module")
def asan_run():
    if not shutil.which("gcc"):
        pytest.skip("gcc absent")
    exe = os.path.join(gen.REPO, "build", "host_abi_check_asan")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    cmd = ["gcc", "-O1", "-g", "-std=gnu11", "-Wall", "-Werror", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-ffunction-sections", "-fdata-sections", "-Wl,--gc-sections",
           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", INC,
           os.path.join(gen.REPO, "tests", "c", "host_abi_check.c")] + \
          [os.path.join(CSRC, s) for s in SRCS] + ["-lpthread", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    # verify_asan_link_order=0: the environment may preload other libraries
    # ahead of the ASan runtime; the environment itself is passed unchanged
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    out = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    return [ln.split() for ln in out.stdout.splitlines()]


def test_host_entries_under_asan(asan_run, golden):
    rows = asan_run
    big = gen.mul_pattern(1 << 16)
    crc_gold = json.load(open(os.path.join(gen.REPO, "tests", "golden", "crc32_golden.json")))
    crc_edge = dict(zip(crc_gold["edge"]["lengths"], crc_gold["edge"]["crc"]))
    seen = set()
    for r in rows:
        if r[0] == "md5":
            L = int(r[1])
            want = gen.oracle_digests(np.frombuffer(big + b"\0", np.uint8), [0], [L])[0]
            assert r[2] == bytes(want).hex(), L
            seen.add("md5")
        elif r[0] == "crc":
            L = int(r[1])
            if L in crc_edge:
                assert r[2] == crc_edge[L], L
            seen.add("crc")
        elif r[0] == "hdr":
            assert r[2] == "1"
            seen.add("hdr")
        elif r[0] == "hdrbad":
            assert r[1] == "0"
        elif r[0] == "plan":
            f = [int(x) for x in r[2:]]
            assert f[0] == 0 and f[-1] == 100 and f == sorted(f)
            seen.add("plan")
        elif r[0] == "arr":
            assert r[1:] == ["0", "-34", "-7", "1", "0"]      # ok, ERANGE, E2BIG, equal, differs
            seen.add("arr")
    assert seen == {"md5", "crc", "hdr", "plan", "arr"}
    ctx_rows = [r for r in rows if r[0] == "ctx"]
    assert len(ctx_rows) == 240
    ref = os.path.join(gen.REPO, "oracle", "_ref", "libmd5_ref.so")
    if os.path.exists(ref):                  # replay through the reference md5.c
        import ctypes
        R = ctypes.CDLL(ref)
        R.MD5Init.argtypes = [ctypes.c_void_p]
        R.MD5Update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        src = np.frombuffer(big, np.uint8)
        ctx = np.zeros(88, np.uint8)
        for r in ctx_rows:
            seq, off, n = int(r[1]), int(r[2]), int(r[3])
            if r is ctx_rows[0] or seq != prev:
                R.MD5Init(ctx.ctypes.data)
                ctx[24:] = 0x5A
            prev = seq
            R.MD5Update(ctx.ctypes.data, src.ctypes.data + off, n)
            assert ctx.tobytes().hex() == r[4], (seq, off, n)
    ncm = {int(r[1]): r[2] for r in rows if r[0] == "ncmd5"}
    assert len(ncm) == 16
    for L, hx in ncm.items():
        if L <= 16385:
            assert nc_md5_oracle.nc_md5(big[:L]).hex() == hx, L
