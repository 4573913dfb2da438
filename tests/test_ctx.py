"""Batched MD5Init / MD5Update / MD5Final on caller-owned contexts
(md5hip_init_ctx / md5hip_update_ctx / md5hip_final_ctx) against the
reference md5.c itself (oracle/_ref/libmd5_ref.so, compiled in place from
/root/reference) driven call by call on the same 88-byte contexts: every
context byte after every update, then the digests and the zeroed contexts.
Without the reference build the restatement (oracle/md5_oracle.c) checks the
state md5.c defines -- buf, bits and the pending bytes in[0 .. count)."""
import ctypes
import os

import numpy as np
import pytest
import torch

import gen
import sproxy_amd.md5 as m

pytestmark = pytest.mark.gpu

REF = os.path.join(gen.REPO, "oracle", "_ref", "libmd5_ref.so")


class HostRef:
    """Sequential MD5Update/MD5Final on host copies of the contexts."""

    def __init__(self):
        if os.path.exists(REF):
            self.lib, self.exact = ctypes.CDLL(REF), True
            self.upd, self.fin = self.lib.MD5Update, self.lib.MD5Final
        else:
            self.lib, self.exact = gen.oracle_lib(), False
            self.upd, self.fin = self.lib.oracle_md5_update, self.lib.oracle_md5_final
        self.upd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        self.fin.argtypes = [ctypes.c_void_p, ctypes.c_void_p]

    def update(self, ctxs: np.ndarray, data: np.ndarray, offs, lens):
        for i in range(ctxs.shape[0]):
            self.upd(ctxs[i].ctypes.data, data.ctypes.data + int(offs[i]), int(lens[i]))

    def final(self, ctxs: np.ndarray) -> np.ndarray:
        out = np.empty((ctxs.shape[0], 16), np.uint8)
        for i in range(ctxs.shape[0]):
            self.fin(out[i].ctypes.data, ctxs[i].ctypes.data)
        return out

    def same(self, got: np.ndarray, want: np.ndarray) -> bool:
        if self.exact:
            return np.array_equal(got, want)
        cnt = (want[:, 16:20].view("<u4")[:, 0] >> 3) & 63
        ok = np.array_equal(got[:, :24], want[:, :24])
        for i in range(got.shape[0]):
            ok &= np.array_equal(got[i, 24:24 + cnt[i]], want[i, 24:24 + cnt[i]])
        return bool(ok)


def _dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def _update(ctx_d, base_d, offs, lens, cuda):
    ptrs = torch.tensor(np.asarray(offs, np.int64) + base_d.data_ptr(), dtype=torch.int64, device=cuda)
    m.update_ctx(ctx_d, ptrs, torch.tensor(np.asarray(lens, np.int64), dtype=torch.int32, device=cuda))


def test_golden_random_lengths_two_updates(golden, cuda):
    """tests/golden random_lengths (from the reference md5.c): MD5Update of
    data[:split] then data[split:len], then MD5Final, all contexts at once."""
    g = golden["random_lengths"]
    lens, splits = np.array(g["lengths"]), np.array(g["splits"])
    data = gen.xorshift_array(int(lens.max()) + 64, seed=0x243F6A8885A308D3)
    d = _dev(data, cuda)
    n = lens.size
    ctx = torch.zeros((n, 88), dtype=torch.uint8, device=cuda)
    m.init_ctx(ctx)
    _update(ctx, d, np.zeros(n), splits, cuda)
    _update(ctx, d, splits, lens - splits, cuda)
    got = m.final_ctx(ctx).cpu().numpy()
    want = np.array([np.frombuffer(bytes.fromhex(h), np.uint8) for h in g["md5"]])
    assert np.array_equal(got, want)
    assert not ctx.any().item()                            # md5.c:264


def test_random_update_sequences_match_reference(cuda):
    """512 contexts, 7 rounds of one update each (0-byte, sub-block,
    block-straddling and multi-block lengths at any alignment, from shared
    data): every context byte equals the reference after every round."""
    ref = HostRef()
    rng = np.random.default_rng(1321)
    n, rounds = 512, 7
    data = gen.xorshift_array(4 << 20, seed=77)
    d = _dev(data, cuda)
    ctx_h = np.zeros((n, 88), np.uint8)
    ctx_h[:, 24:] = rng.integers(0, 256, (n, 64), dtype=np.uint8)     # stale in[] bytes
    ctx = _dev(ctx_h, cuda)
    m.init_ctx(ctx)
    for i in range(n):
        ctx_h[i, :16] = np.frombuffer(bytes.fromhex("0123456789abcdeffedcba9876543210"), np.uint8)
        ctx_h[i, 16:24] = 0
    assert np.array_equal(ctx.cpu().numpy(), ctx_h)           # MD5Init leaves in[] alone
    for r in range(rounds):
        kind = rng.integers(0, 5, n)
        lens = np.where(kind == 0, 0,
               np.where(kind == 1, rng.integers(1, 64, n),
               np.where(kind == 2, rng.integers(64, 200, n),
               np.where(kind == 3, rng.integers(1000, 70000, n), rng.integers(0, 300000, n)))))
        offs = rng.integers(0, data.size - 300000, n)
        _update(ctx, d, offs, lens, cuda)
        ref.update(ctx_h, data, offs, lens)
        assert ref.same(ctx.cpu().numpy(), ctx_h), r
    got = m.final_ctx(ctx).cpu().numpy()
    assert np.array_equal(got, ref.final(ctx_h))
    assert not ctx.any().item()


def test_bit_count_carry_and_high_word(cuda):
    """Contexts whose bit count sits just below 2^32 (carry into bits[1],
    md5.c:180-181), one update of 2^29 + 5 bytes (len >> 29 into bits[1],
    md5.c:182), pending bytes of every residue."""
    ref = HostRef()
    rng = np.random.default_rng(29)
    n = 64
    big = (1 << 29) + 5
    data = gen.xorshift_array(big + 4096, seed=5)
    d = _dev(data, cuda)
    ctx_h = rng.integers(0, 256, (n, 88), dtype=np.uint8)
    bits = ctx_h[:, 16:24].view("<u4")
    # 0xFFFFFE00 + pending bytes * 8: every residue, and +len<<3 wraps
    bits[:, 0] = (np.uint64(0xFFFFFE00) + (np.arange(n, dtype=np.uint64) % 64) * 8).astype(np.uint32)
    bits[:, 1] = rng.integers(0, 1 << 31, n).astype(np.uint32)
    ctx = _dev(ctx_h, cuda)
    lens = rng.integers(0, 9000, n)
    lens[0] = big
    offs = rng.integers(0, 4000, n)
    offs[0] = 3                                                # unaligned 512 MiB chunk
    _update(ctx, d, offs, lens, cuda)
    ref.update(ctx_h, data, offs, lens)
    assert ref.same(ctx.cpu().numpy(), ctx_h)
    assert np.array_equal(m.final_ctx(ctx).cpu().numpy(), ref.final(ctx_h))


@pytest.mark.parametrize("groups", [24, 300])
def test_lds_dma_waves_and_pending_blocks(cuda, groups):
    """Waves whose update data is 16-B (and 128-B) aligned take the LDS-DMA
    loader (md5_update_ctx -> desc_xpose_group); contexts with a pending
    partial block shift the bulk by 64 - t bytes, so neighbouring waves mix
    the DMA and lane-direct paths.  24 groups (at most one per CU) run as fed
    pairs (md5_update_ctx_fed) where a group's bulk is 16-B aligned, on the
    loader otherwise; 300 groups always take the loader.  Three rounds,
    every context byte against the reference after each."""
    ref = HostRef()
    rng = np.random.default_rng(4242 + groups)
    n = 64 * groups
    data = gen.xorshift_array(12 << 20, seed=91)
    d = _dev(data, cuda)
    ctx_h = np.zeros((n, 88), np.uint8)
    ctx = _dev(ctx_h, cuda)
    m.init_ctx(ctx)
    ctx_h = ctx.cpu().numpy()
    wave = np.arange(n) // 64
    for r in range(3):
        lens = rng.integers(1, 200, n) * 64 + np.where(wave % 3 == 0, 0, rng.integers(0, 64, n))
        offs = rng.integers(0, (data.size - 20000) // 128, n) * 128
        offs = np.where(wave % 4 == 1, offs + 16 * rng.integers(1, 8, n), offs)   # 16-B, off the line
        offs = np.where(wave % 4 == 2, offs + rng.integers(1, 16, n), offs)       # unaligned waves
        _update(ctx, d, offs, lens, cuda)
        ref.update(ctx_h, data, offs, lens)
        assert ref.same(ctx.cpu().numpy(), ctx_h), r
    assert np.array_equal(m.final_ctx(ctx).cpu().numpy(), ref.final(ctx_h))
