"""The netcache call site of INTEGRATION.md §2 as a plain-C program
(tests/c/netcache_site.c) linked against libmd5hip.so: page-list blocks, MD5,
CRC-32 / fastcrc, batched verify with one corrupted block, asynchronous
submit, zero-copy gather modes, the multi-device pool and MD5Init/Update/Final,
each block checked against the oracle; then the failure policy of
INTEGRATION.md §2j with a device fault injected under a vector (-EIO, no
checksum stored, -ENODEV after, host fallback, no inode reset from a device
error, pool failover).  No Python or torch between the caller
and the library.  Built by __graft_entry__.build() (tests/c/Makefile)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "build", "c", "netcache_site")


def _run(timeout):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} missing: run __graft_entry__.build() (make -C tests/c)")
    return subprocess.run([EXE], capture_output=True, text=True, timeout=timeout)


def test_c_site_without_device_fails_loudly():
    """No HIP device: the batched entries return -ENODEV (exit 77), no host fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is visible; the -m gpu test covers this box")
    out = _run(120)
    assert out.returncode == 77, out.stdout + out.stderr
    assert "md5hip_batcher_create = -19" in out.stdout


@pytest.mark.gpu
def test_c_site_on_gpu(cuda):
    out = _run(120)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    assert "netcache_site ok" in out.stdout
    assert "failure policy ok" in out.stdout
