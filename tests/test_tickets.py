"""The batcher's ticket table (sproxy_amd/csrc/md5_tickets.h, included by
md5_submit.c) on the host under AddressSanitizer + UBSan: a ticket that fails
and leaves the ring does not turn later tickets' results into its error
(ADVICE r2, high), out-of-order completion over a grown ring, first error
kept, bounded memory for old failures (tests/c/tickets_check.c)."""
import os
import shutil
import subprocess

import pytest

import gen


def test_ticket_table_under_asan():
    if not shutil.which("gcc"):
        pytest.skip("gcc absent")
    exe = os.path.join(gen.REPO, "build", "tickets_check_asan")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-Wall", "-Werror",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    os.path.join(gen.REPO, "tests", "c", "tickets_check.c"), "-o", exe],
                   check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    out = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr[-2000:]
    assert out.stdout.strip().endswith("tickets ok")
