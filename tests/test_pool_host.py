"""The multi-GPU pool's host logic (sproxy_amd/csrc/md5_pool.c) with no
device: tests/c/pool_check.c links md5_pool.c against a fake batcher that
hashes on the CPU (the library's host MD5 / CRC-32) and completes tickets
only after a few polls, failing some on purpose.  Routing, whole and split
submissions, digest placement, split-ticket bookkeeping, per-ticket errors,
stats, lost devices (a synchronous split part moved off the failed device,
the device never routed to again, an asynchronous ticket keeping -EIO,
-ENODEV once every device failed) and 8 concurrent submitting threads -- under ASan+UBSan, and under
ThreadSanitizer for the lock-free routing and the ticket table."""
import os
import shutil
import subprocess

import pytest

import gen

CSRC = os.path.join(gen.REPO, "sproxy_amd", "csrc")
INC = os.path.join(gen.REPO, "include")
SRCS = [os.path.join(gen.REPO, "tests", "c", "pool_check.c")] + \
       [os.path.join(CSRC, s) for s in ("md5_pool.c", "md5_stream.c", "nc_digest.c")]


def _build_and_run(name, san, env_extra):
    if not shutil.which("gcc"):
        pytest.skip("gcc absent")
    exe = os.path.join(gen.REPO, "build", name)
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    cmd = ["gcc", "-O1", "-g", "-std=gnu11", "-Wall", "-Werror", f"-fsanitize={san}",
           "-fno-sanitize-recover=all", "-ffunction-sections", "-fdata-sections", "-Wl,--gc-sections",
           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", INC, *SRCS, "-lpthread", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, **env_extra)
    out = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert out.stdout.strip().endswith("pool ok")


def test_pool_logic_under_asan():
    _build_and_run("pool_check_asan", "address,undefined",
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1:verify_asan_link_order=0"})


def test_pool_logic_under_tsan():
    _build_and_run("pool_check_tsan", "thread", {"TSAN_OPTIONS": "halt_on_error=1"})
