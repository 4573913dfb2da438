"""bench.py's CPU-side helpers (no GPU): the list-schedule model of one
BALANCED launch (lpt_schedule) and the C5 parity sample
(c5_sample: first, last, both sides of every slot boundary, distinct random
chunks, re-digested by the host reference)."""
import numpy as np

import gen
import bench


def test_lpt_schedule_small_cases():
    # 64 chunks of one length: one group, one SIMD busy -> util 1/simds
    s = bench.lpt_schedule(np.full(64, 4096), simds=4)
    assert s["groups"] == 1 and s["makespan_compressions"] == 65 and abs(s["util"] - 0.25) < 1e-9
    # one long chain beside short groups: the chain sets the makespan
    lens = np.concatenate([np.full(64, 1 << 20), np.full(64 * 6, 16384)])
    s = bench.lpt_schedule(lens, simds=4)
    assert s["groups"] == 7 and s["makespan_compressions"] == 16385
    assert abs(s["mean_compressions"] - (16385 + 6 * 257) / 4) <= 0.05 + 1e-9     # rounded to 0.1
    # enough short work: load-bound, util near 1
    s = bench.lpt_schedule(np.full(64 * 400, 16384), simds=4)
    assert s["makespan_compressions"] == 100 * 257 and s["util"] == 1.0
    # a group costs its longest chunk; lengths past a block boundary add one
    s = bench.lpt_schedule([55, 56, 63, 64], simds=1)
    assert s["groups"] == 1 and s["makespan_compressions"] == (64 + 8) // 64 + 1


def test_lpt_sizes_the_coalesced_c3_launch():
    """The rule bench.py's coalesced leg uses: 3 of its C3 batches leave a
    quarter of SIMD-time idle (one 1 MiB chain is the makespan), 4 do not."""
    lk = [bench.c3_lens(16 << 30, 1000)] + [bench.c3_lens(16 << 30, 2000 + 17 * j) for j in (1, 2, 3)]
    u3 = bench.lpt_schedule(np.concatenate(lk[:3]))
    u4 = bench.lpt_schedule(np.concatenate(lk))
    assert u3["makespan_compressions"] == 16385 and 0.70 < u3["util"] < 0.80
    assert u4["util"] >= 0.95


def test_c5_sample_covers_slot_boundaries():
    n, L, per = 1000, 256, 64
    arr = gen.xorshift_array(n * L, seed=5)
    dig = gen.oracle_digests_fixed(arr, n, L)
    par = bench.c5_sample(arr, dig, n, L, per, 100, seed=1)
    bounds = list(range(per, n, per))
    assert par["ok"] and par["mismatches"] == 0
    assert par["checked"] >= 100 + 2 and par["checked"] <= 100 + 2 + 2 * len(bounds)
    assert f"{len(bounds)} slot boundaries" in par["sample"]
    bad = dig.copy()
    bad[per - 1, 0] ^= 1                     # the last chunk before a boundary
    bad[n - 1, 3] ^= 1                       # and the very last one
    par = bench.c5_sample(arr, bad, n, L, per, 10, seed=2)
    assert par["ok"] is False and par["mismatches"] == 2
