"""A subscribe's commit never allocates (the first subscribe of every bench
run stalled 5-8 ms).  The engine's host code on the fake HIP runtime (tests/host_harness), whose
hipMalloc / hipHostMalloc / hipFree are counted: after the index's first commit, the writing
node's hooks (emqxgm_route_dests_batch / emqxgm_subscribers_batch with EMQXGM_SET_COMMIT, each
with a filter string the registry has never seen, so the string pool, offsets and verify
records grow) are delta commits that make no device or pinned allocation and free nothing (a
hipFree synchronises the device).  The reference's subscriber waits on this path before SUBACK
(emqx_broker.erl:163-168, 484-486)."""
import ctypes as C
import random

import pytest

from emqx_amd.engine import Engine, load_library
from tests.test_route_mirror import build_fake_lib


@pytest.fixture(scope="module")
def fakelib():
    return load_library(build_fake_lib(), allow_missing=True)


def _counts(lib):
    f = C.CDLL(lib._name)
    f.fakehip_allocs.restype = C.c_ulonglong
    f.fakehip_frees.restype = C.c_ulonglong
    return lambda: (int(f.fakehip_allocs()), int(f.fakehip_frees()))


@pytest.mark.parametrize("n0", [3000, 20000])
def test_hooks_after_the_first_commit_do_not_allocate(fakelib, n0):
    counts = _counts(fakelib)
    rng = random.Random(n0)
    eng = Engine(library=fakelib)
    eng.tune("bg_build", 0)  # (a full build, when one is due, blocks: none may be due here)
    eng.set_local_node(0)
    items = [(b"site/%d/device/%d/+" % (i % 97, i), [(rng.randint(0, 3), 0xFFFFFFFF)])
             for i in range(n0)]
    eng.route_dests_batch(items, commit=False)
    eng.subscribers_batch([(t, [i]) for i, (t, _) in enumerate(items[:n0 // 4])], commit=False)
    eng.commit()  # the first (full) commit sizes everything with headroom
    d0 = eng.stats()["delta_commits"]
    f0 = eng.stats()["full_commits"]
    a0 = counts()
    hooks = 600
    for k in range(hooks):
        f = b"site/%d/device/%d/bench%d/+" % (k % 97, k, k)
        if k % 3 == 2:
            eng.subscribers_batch([(f, [100000 + k])], commit=True)
        else:
            eng.route_dests_batch([(f, [(k % 4, 0xFFFFFFFF)])], commit=True)
        if k % 5 == 4:  # an unsubscribe of an earlier one
            eng.route_dests_batch([(b"site/%d/device/%d/bench%d/+" % ((k - 4) % 97, k - 4, k - 4), [])],
                                  commit=True)
    st = eng.stats()
    assert st["full_commits"] == f0, "a hook fell back to a full build"
    assert st["delta_commits"] - d0 >= hooks
    assert counts() == a0, f"hooks allocated / freed: {a0} -> {counts()}"
    assert eng.route_member(b"site/1/device/1/bench1/+")
    # the mirror's own commit path regrows ahead of need (off the hook): later hooks still fit
    eng.commit()
    a1 = counts()
    for k in range(hooks, hooks + 100):
        eng.route_dests_batch([(b"x/%d/+" % k, [(1, 0xFFFFFFFF)])], commit=True)
    assert counts() == a1
