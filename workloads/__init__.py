"""Deterministic synthetic workloads, generated natively by
``workloads/gen.cpp``.  Shared by the parity tests and bench.py; not part of the engine."""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libemqx_workload.so")


class _Set(C.Structure):
    _fields_ = [("fbytes", C.POINTER(C.c_uint8)), ("foff", C.POINTER(C.c_uint64)),
                ("fwild", C.POINTER(C.c_uint8)), ("nf", C.c_uint64),
                ("tbytes", C.POINTER(C.c_uint8)), ("toff", C.POINTER(C.c_uint32)),
                ("nt", C.c_uint64), ("fbytes_len", C.c_uint64), ("tbytes_len", C.c_uint64)]


# (n_filters, n_topics, seed_filters, seed_topics) per SURVEY 8d
DEFAULTS = {1: (10_000, 100_000, 1, 2), 2: (1_000_000, 1_000_000, 11, 12),
            3: (10_000_000, 2_000_000, 21, 22), 4: (101_000_000, 1_000_000, 31, 32)}


@dataclass
class Workload:
    cfg: int
    fbytes: np.ndarray   # u8
    foff: np.ndarray     # u64 [nf+1]
    fwild: np.ndarray    # u8 [nf]  1 = wildcard filter (trie + route key), 0 = exact route key
    tbytes: np.ndarray   # u8
    toff: np.ndarray     # u32 [nt+1]

    @property
    def nf(self):
        return len(self.fwild)

    @property
    def nt(self):
        return len(self.toff) - 1

    def filter(self, i):
        return self.fbytes[self.foff[i]:self.foff[i + 1]].tobytes()

    def topic(self, i):
        return self.tbytes[self.toff[i]:self.toff[i + 1]].tobytes()


def generate(cfg: int, n_filters: int = None, n_topics: int = None, seed_f: int = None,
             seed_t: int = None, topics_only: bool = False) -> Workload:
    """The cfg's filters and a topic batch; topics_only=True draws the same topics without the
    filters (empty filter arrays), for further batches against an index already built."""
    d = DEFAULTS[cfg]
    nf = d[0] if n_filters is None else n_filters
    nt = d[1] if n_topics is None else n_topics
    sf = d[2] if seed_f is None else seed_f
    st = d[3] if seed_t is None else seed_t
    lib = C.CDLL(_SO)
    lib.wl_generate.restype = C.c_int
    lib.wl_generate.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                C.POINTER(_Set)]
    lib.wl_generate_topics.restype = C.c_int
    lib.wl_generate_topics.argtypes = lib.wl_generate.argtypes
    lib.wl_free.argtypes = [C.POINTER(_Set)]
    s = _Set()
    rc = (lib.wl_generate_topics if topics_only else lib.wl_generate)(cfg, nf, nt, sf, st, C.byref(s))
    if rc != 0:
        raise RuntimeError(f"wl_generate({cfg}) failed: {rc}")
    try:
        def arr(p, n, dt):
            return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True) if n else np.zeros(0, dt)
        w = Workload(cfg, arr(s.fbytes, s.fbytes_len, np.uint8), arr(s.foff, s.nf + 1, np.uint64),
                     arr(s.fwild, s.nf, np.uint8), arr(s.tbytes, s.tbytes_len, np.uint8),
                     arr(s.toff, s.nt + 1, np.uint32))
    finally:
        lib.wl_free(C.byref(s))
    return w
