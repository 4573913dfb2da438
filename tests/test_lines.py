"""MD5HIP_DESC_LINES (md5_desc_lines, md5_kernels.h desc_xpose_group kShift):
the descriptor loader for chunks that start 16-B but not 128-B aligned.  It
loads whole 128-B lines once each and forms every 128-B window from two lines
with a per-lane rotation, where XDMA's chunk-relative stages straddle two
lines (1.29x the payload from HBM on 16-B-packed blocks).

Bit-exact against the oracle on every shift a lane can have (0-7 x 16 B),
mixed shifts inside one wave, tails, empty chunks, chunks shorter than a
stage, rows whose line count differs from their wave's longest, and through
the batcher's device-resident path (which picks LINES for such batches);
the planner's choice is checked on the host."""
import numpy as np
import pytest

import gen
import sproxy_amd.md5 as m


def _pack(lens, align, shift_of=None):
    """offsets packed at `align`, plus per-chunk extra 16-B shifts"""
    offs, at = [], 128
    for i, L in enumerate(lens):
        s = shift_of(i) if shift_of else 0
        at = (at + align - 1) // align * align
        offs.append(at + 16 * s)
        at = offs[-1] + L
    return offs, at + 256


def test_plan_desc_at_picks_lines_for_unlined_batches():
    n = 256 * 64 * 3                                  # past the small-batch planners
    lens = np.full(n, 16384, np.uint32)
    lens[::8] = 9000
    offs16, _ = _pack(lens, 16)
    offs128, _ = _pack(lens, 128)
    assert m.plan_desc(lens)[1] == "xdma"
    assert m.plan_desc_at(lens, np.asarray(offs16, np.uint64))[1] == "lines"
    assert m.plan_desc_at(lens, np.asarray(offs128, np.uint64))[1] == "xdma"
    with pytest.raises(ValueError):
        m.plan_desc_at(lens, np.zeros(3, np.uint64))


def test_plan_desc_at_boundary_is_more_than_half_the_bytes():
    """md5hip_lines_choice: LINES once 2 x unlined bytes > the batch's bytes.
    Groups of 8 chunks (one of 9,000 B, seven of 16 KiB) are all 128-B
    aligned, or all shifted 16 B off the line; half of the groups shifted is
    exactly half the bytes (XDMA stays), and one lined chunk 16 B shorter
    tips it over (LINES)."""
    n = 256 * 64 * 3
    lens = np.full(n, 16384, np.uint32)
    lens[::8] = 9000
    offs = np.arange(n, dtype=np.uint64) * np.uint64(16384 + 256) + np.uint64(128)
    unlined = (np.arange(n) // 8) % 2 == 1                # every other group of 8
    addrs = offs + np.where(unlined, 16, 0).astype(np.uint64)
    assert 2 * int(lens[unlined].sum()) == int(lens.sum())
    assert m.plan_desc(lens)[1] == "xdma"
    assert m.plan_desc_at(lens, addrs)[1] == "xdma"       # exactly half: stays
    shorter = lens.copy()
    shorter[np.flatnonzero(~unlined)[-1]] -= 16
    assert 2 * int(shorter[unlined].sum()) == int(shorter.sum()) + 16
    assert m.plan_desc_at(shorter, addrs)[1] == "lines"   # just over half


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["every_shift", "mixed_lengths", "short_and_empty", "packed16"])
def test_lines_kernel_matches_oracle(cuda, case):
    import torch
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    if case == "every_shift":
        lens = [16384 - 16 * (i % 5) for i in range(64 * 40)]
        offs, total = _pack(lens, 128, lambda i: i % 8)
    elif case == "mixed_lengths":
        lens = [int(x) for x in rng.integers(0, 70000, 64 * 30)]
        offs, total = _pack(lens, 16)
    elif case == "short_and_empty":
        lens = [int(x) for x in rng.choice([0, 1, 15, 16, 63, 64, 65, 127, 128, 129, 255, 256, 257, 4096],
                                           64 * 20)]
        offs, total = _pack(lens, 16)
    else:
        lens = [16384] * (64 * 300)
        for i in range(0, len(lens), 8):
            lens[i] = int(rng.integers(1, 16384))
        offs, total = _pack(lens, 16)
    buf = gen.xorshift_array(total, seed=1234 + len(lens))
    want = gen.oracle_digests(buf, offs, lens)
    d = torch.from_numpy(buf).to(cuda)
    dO = torch.tensor(offs, dtype=torch.int64, device=cuda)
    dL = torch.tensor(lens, dtype=torch.int32, device=cuda)
    order = m.plan_order(np.asarray(lens, np.uint32))
    dR = torch.from_numpy(order.astype(np.int32)).to(cuda)
    for ordered in (True, False):
        got = m.digest_desc(d, dO, dL, dR if ordered else None, variant="lines")
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), want), (case, ordered)


@pytest.mark.gpu
def test_queue_device_submit_packed16_matches_oracle(cuda):
    """Device-resident netcache blocks packed at 16 B through the queue: the
    slot's plan takes LINES (md5hip_lines_choice); digests equal the oracle.
    (768 groups: past the small-batch planners' two groups per CU.)"""
    import torch
    n = 256 * 64 * 3
    lens = [16384] * n
    rng = np.random.default_rng(7)
    for i in range(0, n, 8):
        lens[i] = int(rng.integers(1, 16384))
    offs, total = _pack(lens, 16)
    buf = gen.xorshift_array(total, seed=99)
    want = gen.oracle_digests(buf, offs, lens)
    d = torch.from_numpy(buf).to(cuda)
    torch.cuda.synchronize()
    ptrs = np.asarray(offs, np.uint64) + np.uint64(d.data_ptr())
    assert m.plan_desc_at(np.asarray(lens, np.uint32), ptrs)[1] == "lines"
    with m.Queue(device=0, max_chunks=n) as q:
        got = q.submit_device(ptrs, np.asarray(lens, np.uint32), after=None)
    assert np.array_equal(got, want)
