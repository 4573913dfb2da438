"""The whole batcher with no device: tests/c/batcher_check.c links
md5_submit.c (batcher, device queue), md5_pool.c (router) and the host
MD5/CRC-32 against tests/c/fake_hip.c, a fake HIP runtime whose streams run
copies and "kernels" (the library's host MD5/CRC-32) at enqueue and whose
events stay NotReady for a few queries, so slots are in flight, coalesce and
complete out of order.  10 threads submit at random (sync/async pointer and
page lists, verify, host_fixed, device-resident with host or device digests
and a producer stream, pool whole and split, CRC-32, netcache header
verification on the shared MD5 batcher, explicit flush) while one thread
changes the knobs and another registers, uses and unregisters a private
page range; a failing launch is injected once; the pool spans three devices
and every copy or kernel must be enqueued from its stream's device (waits
and polls on another device's ticket included).  First, 64 blocked callers
wait on one slot for 12 rounds, every other round with the watcher's spin
ending on NotReady just as the launch completes (the round-3 lost wake-up,
which hangs that phase).  Then the device-failure policy: a device lost
after launch K (its completion event reports the fault, or the launch itself
fails, or md5hip_batcher_inject_fault) gives the failing ticket -EIO, the
ticket coalescing behind it and every later call -ENODEV, with nothing
enqueued again and no digest written; a 2-device pool moves a synchronous
part off the failed device, never routes to it again, returns -ENODEV once
every device failed, and 8 threads keep getting correct digests while a
device dies under them.  Then large device-resident vectors (md5_submit.c
reserve_device), three coalesced in one slot with their device digests
scattered in pieces; the fake planner rejects a histogram that misses a
chunk.  Then host_fixed over a source pinned only in part (first half,
two adjacent pinned blocks, an extent the runtime will not tell): staged,
never DMA'd from past a page-locked range; wholly pinned: read in place.
Runs under ASan+UBSan and under ThreadSanitizer
(which found the unlocked gather-mode read in submit(), now atomic)."""
import os
import shutil
import subprocess

import pytest

import gen

CSRC = os.path.join(gen.REPO, "sproxy_amd", "csrc")
INC = os.path.join(gen.REPO, "include")
SRCS = [os.path.join(gen.REPO, "tests", "c", s) for s in ("batcher_check.c", "fake_hip.c")] + \
       [os.path.join(CSRC, s) for s in ("md5_submit.c", "md5_pool.c", "md5_stream.c", "nc_digest.c")]


def _build_and_run(name, san, env_extra, secs):
    if not shutil.which("gcc") or not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("gcc or the HIP headers absent")
    exe = os.path.join(gen.REPO, "build", name)
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    cmd = ["gcc", "-O1", "-g", "-std=gnu11", "-Wall", "-Werror", f"-fsanitize={san}",
           "-fno-sanitize-recover=all", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", INC,
           *SRCS, "-lpthread", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, **env_extra)
    out = subprocess.run([exe, str(secs)], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert out.stdout.strip().endswith("batcher ok")
    assert "blocked callers: 12 rounds x 64 waiters on one slot ok" in out.stdout
    assert "large device submissions ok" in out.stdout
    assert "device lost: -EIO / -ENODEV / failover ok" in out.stdout
    assert "host_fixed: partly pinned, split, extent-unknown and pageable sources staged" in out.stdout


def test_batcher_under_asan():
    _build_and_run("batcher_check_asan", "address,undefined",
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1:verify_asan_link_order=0"}, 3)


def test_batcher_under_tsan():
    _build_and_run("batcher_check_tsan", "thread", {"TSAN_OPTIONS": "halt_on_error=1"}, 3)
