"""ctypes wrapper of oracle/ref_trie.cpp -- TEST INFRASTRUCTURE ONLY (checker + CPU baseline).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module."""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libemqx_ref.so")
_V = C.c_void_p


def _lib():
    lib = C.CDLL(_SO)
    lib.ref_create.restype = _V
    lib.ref_create.argtypes = [C.c_int]
    lib.ref_destroy.argtypes = [_V]
    lib.ref_add_many.argtypes = [_V, _V, _V, C.c_uint64, _V]
    lib.ref_trie_delete.argtypes = [_V, C.c_char_p, C.c_uint32]
    lib.ref_route_delete.argtypes = [_V, C.c_char_p, C.c_uint32]
    lib.ref_trie_empty.argtypes = [_V]
    lib.ref_n_ids.restype = C.c_uint64
    lib.ref_n_ids.argtypes = [_V]
    lib.ref_match_batch.argtypes = [_V, _V, _V, C.c_uint64, C.c_int, _V,
                                    C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_uint64), _V]
    lib.ref_match_count.restype = C.c_uint64
    lib.ref_match_count.argtypes = [_V, _V, _V, C.c_uint64, C.c_int]
    lib.ref_bruteforce.argtypes = [_V, _V, _V, C.c_uint64, _V, C.POINTER(C.POINTER(C.c_uint32)),
                                   C.POINTER(C.c_uint64)]
    lib.ref_states.argtypes = [_V, _V, _V, C.c_uint64, _V, C.c_int]
    lib.ref_free.argtypes = [_V]
    return lib


def _p(a):
    return a.ctypes.data_as(_V) if a.size else _V(0)


class RefIndex:
    """The reference's trie + route-key set (emqx_trie / emqx_route) on the CPU."""

    def __init__(self, compact: bool = True):
        self.lib = _lib()
        self.h = self.lib.ref_create(1 if compact else 0)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.ref_destroy(self.h)
            self.h = None

    def add_many(self, fbytes, foff, kind):
        """kind bit 1 = trie insert, bit 2 = route key (ids = first-registration order)."""
        fbytes = np.ascontiguousarray(fbytes, np.uint8)
        foff = np.ascontiguousarray(foff, np.uint64)
        kind = np.ascontiguousarray(kind, np.uint8)
        self.lib.ref_add_many(self.h, _p(fbytes), _p(foff), len(kind), _p(kind))

    def trie_delete(self, f: bytes):
        self.lib.ref_trie_delete(self.h, f, len(f))

    def route_delete(self, f: bytes):
        self.lib.ref_route_delete(self.h, f, len(f))

    def match(self, tbytes, toff, threads: int = 1):
        tbytes = np.ascontiguousarray(tbytes, np.uint8)
        toff = np.ascontiguousarray(toff, np.uint32)
        n = len(toff) - 1
        row = np.zeros(n + 1, np.uint64)
        ex = np.zeros(n, np.uint32)
        ids = C.POINTER(C.c_uint32)()
        nid = C.c_uint64()
        self.lib.ref_match_batch(self.h, _p(tbytes), _p(toff), n, threads, _p(row), C.byref(ids),
                                 C.byref(nid), _p(ex))
        out = np.ctypeslib.as_array(ids, shape=(max(nid.value, 1),))[:nid.value].copy()
        self.lib.ref_free(ids)
        return row, out, ex

    def bruteforce(self, tbytes, toff):
        tbytes = np.ascontiguousarray(tbytes, np.uint8)
        toff = np.ascontiguousarray(toff, np.uint32)
        n = len(toff) - 1
        row = np.zeros(n + 1, np.uint64)
        ids = C.POINTER(C.c_uint32)()
        nid = C.c_uint64()
        self.lib.ref_bruteforce(self.h, _p(tbytes), _p(toff), n, _p(row), C.byref(ids),
                                C.byref(nid))
        out = np.ctypeslib.as_array(ids, shape=(max(nid.value, 1),))[:nid.value].copy()
        self.lib.ref_free(ids)
        return row, out

    def states(self, tbytes, toff, threads: int = 1):
        tbytes = np.ascontiguousarray(tbytes, np.uint8)
        toff = np.ascontiguousarray(toff, np.uint32)
        s = np.zeros(len(toff) - 1, np.uint32)
        self.lib.ref_states(self.h, _p(tbytes), _p(toff), len(s), _p(s), threads)
        return s

    def time_match(self, tbytes, toff, threads: int):
        """Wall time of matching every topic once with `threads` threads (CPU baseline)."""
        tbytes = np.ascontiguousarray(tbytes, np.uint8)
        toff = np.ascontiguousarray(toff, np.uint32)
        t0 = time.perf_counter()
        found = self.lib.ref_match_count(self.h, _p(tbytes), _p(toff), len(toff) - 1, threads)
        return time.perf_counter() - t0, found
