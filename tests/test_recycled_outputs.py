"""CPU: the recycling of solve()'s page-locked output blocks
(ffddp.solver._RecycledPinned) with a stand-in allocator in place of
ffddp_host_alloc / ffddp_host_free (no GPU needed): fresh arrays while the
caller holds earlier ones, the block reused once they are gone, the
page-locked cap, and the frees at close."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from ffddp import solver as S


class _FakeLib:
    def __init__(self):
        self.live = {}
        self.allocs = 0
        self.frees = 0

    def ffddp_host_alloc(self, n, pp):
        buf = C.create_string_buffer(int(n))
        self.live[C.addressof(buf)] = buf
        pp._obj.value = C.addressof(buf)
        self.allocs += 1
        return 0

    def ffddp_host_free(self, p):
        self.live.pop(p.value)
        self.frees += 1
        return 0


@pytest.fixture
def fake(monkeypatch):
    lib = _FakeLib()
    monkeypatch.setattr(S._abi, "load", lambda: lib)
    return lib


SPECS = dict(xs=((4, 3, 2), np.float64), it=((4,), np.int32), ok=((4,), np.uint8))


def test_fresh_while_held_and_reused_after_release(fake):
    pool = S._RecycledPinned(cap=10 ** 6)
    a = pool.arrays(SPECS)
    a["xs"][...] = 1.0
    b = pool.arrays(SPECS)  # a is still held: another block
    assert not np.shares_memory(a["xs"], b["xs"]) and fake.allocs == 2
    addr = a["xs"].ctypes.data
    del a
    c = pool.arrays(SPECS)  # a's block comes back, no new allocation
    assert c["xs"].ctypes.data == addr and fake.allocs == 2
    assert c["xs"].shape == (4, 3, 2) and c["it"].dtype == np.int32 and c["ok"].dtype == np.uint8
    pool.close()
    assert fake.frees == 0  # both blocks are still viewed by b and c
    del b, c
    assert fake.frees == 2 and not fake.live


def test_cap_falls_back(fake):
    pool = S._RecycledPinned(cap=256)  # one block of these specs (3 fields x 256 B) does not fit
    assert pool.arrays(SPECS) is None and fake.allocs == 0
    pool = S._RecycledPinned(cap=768)
    first = pool.arrays(SPECS)
    assert first is not None
    assert pool.arrays(SPECS) is None  # the second would exceed the cap
    pool.close()
    del first
    assert fake.frees == 1 and not fake.live


def test_views_keep_the_block(fake):
    pool = S._RecycledPinned(cap=10 ** 6)
    a = pool.arrays(SPECS)
    view = a["xs"][1:]
    addr = a["xs"].ctypes.data
    del a
    b = pool.arrays(SPECS)  # the view still holds the first block
    assert b["xs"].ctypes.data != addr
    del view
    c = pool.arrays(SPECS)
    assert c["xs"].ctypes.data == addr
    pool.close()
