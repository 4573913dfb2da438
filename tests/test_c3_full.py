"""Full-scale C3 parity: the bench's exact C3
batch -- 16 GiB of mixed 4 KiB-1 MiB chunks with 1-in-8 ragged tails, seed
1000 (rank 0), in a batch arena, lanes and kernel from md5hip_plan_desc
(HYBRID) -- hashed on the GPU, and then checked against the oracle on
  - every 1 MiB chunk (all of them sit in the first wave per CU, the
    lane-direct chains of HYBRID),
  - >= 4,096 seeded-random chunks, the first and last in lane order,
  - 8 chunks of every length class and 64 of each ragged residue
    len % 64 in {1, 55, 56, 63, 0} (tails of 1/55/56/63/64 bytes),
with the chunk bytes copied back from the device (the device fill itself is
pinned by test_fill_synthetic_matches_numpy_mirror)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

import gen
import sproxy_amd.md5 as m

sys.path.insert(0, gen.REPO)
import bench  # noqa: E402  (c3_lens / c3_offsets / c3_sample: the bench's own batch)

pytestmark = pytest.mark.gpu


def _oracle_chunks(data, offs, lens, idx, got):
    """oracle digests of chunks idx (device bytes copied back in ~1 GiB
    pieces, hashed on host threads) compared with got[idx]."""
    bad = 0
    idx = np.asarray(idx, dtype=np.int64)
    pos = 0
    while pos < idx.size:
        take, acc = [], 0
        while pos < idx.size and (acc < (1 << 30) or not take):
            take.append(int(idx[pos]))
            acc += int(lens[idx[pos]])
            pos += 1
        flat = torch.cat([data[int(offs[j]):int(offs[j]) + int(lens[j])] for j in take]).cpu().numpy()
        l_s = lens[take].astype(np.int64)
        o_s = np.concatenate([[0], np.cumsum(l_s)[:-1]])
        parts = np.array_split(np.arange(len(take)), 16)
        with ThreadPoolExecutor(16) as ex:
            outs = list(ex.map(lambda p: gen.oracle_digests(flat, o_s[p], l_s[p]), parts))
        want = np.concatenate(outs)
        bad += int((want != got[take]).any(axis=1).sum())
    return bad


def test_c3_full_batch_hybrid_vs_oracle(cuda):
    lens = bench.c3_lens(16 << 30, 1000)
    offs, total = bench.c3_offsets(lens)
    assert lens.size == 79462 and int(lens.sum()) >= 16 << 30
    data = m.arena_empty((total + 15) // 16 * 16)
    m.fill_synthetic(data, seed=0xC3)
    order, dvar = m.plan_desc(lens.astype(np.uint32))
    assert dvar == "hybrid"
    out = m.digest_desc(data, torch.from_numpy(offs).to(cuda),
                        torch.from_numpy(lens.astype(np.int32)).to(cuda),
                        torch.from_numpy(order.astype(np.int32)).to(cuda), variant=dvar)
    got = out.cpu().numpy()
    # every chunk in the first wave per CU (lane-direct chains) that is 1 MiB
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    first_waves = order[: 64 * cus]
    long_idx = first_waves[lens[first_waves] == (1 << 20)]
    assert long_idx.size == int((lens == (1 << 20)).sum())
    sample = bench.c3_sample(lens, order, 4096, seed=91)
    assert sample.size >= 4096
    idx = np.unique(np.concatenate([long_idx, sample]))
    assert _oracle_chunks(data, offs, lens, idx, got) == 0
    # the other descriptor kernels produce the identical digest array
    for v in ("xdma", "lane", "balanced", "fed"):
        assert np.array_equal(m.digest_desc(data, torch.from_numpy(offs).to(cuda),
                                            torch.from_numpy(lens.astype(np.int32)).to(cuda),
                                            torch.from_numpy(order.astype(np.int32)).to(cuda),
                                            variant=v).cpu().numpy(), got), v
    del data
    torch.cuda.empty_cache()
