"""Publisher threads on the engine's concurrent entry (tests/host_harness/async_load.cpp, built
into tests/host_harness/lib/libasync_load.so by emqx_amd.build) -- test and bench
infrastructure.

T threads stand for T BEAM schedulers, each running P publisher processes: one
``emqxgm_async_match`` call per topic, at most P outstanding per thread, each call ending when
the engine's callback reports it (emqx_broker.erl:218-232 -> emqx_trie:match/1 in every
publisher process).  ``run`` returns throughput and call -> result latency percentiles, and
optionally per call: topic index, trie filter count, an order-independent hash of the filters'
bytes and the exact-hit flag, which ``row_hashes`` computes the same way for a reference CSR.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOAD_SO = os.path.join(ROOT, "tests", "host_harness", "lib", "libasync_load.so")

_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LOAD_SO):
            raise ImportError(f"{LOAD_SO} is missing: python -m emqx_amd.build")
        lib = C.CDLL(LOAD_SO)
        lib.async_load_run.restype = C.c_int
        lib.async_load_run.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_uint32]
        _lib = lib
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


def run(engines, tbytes, toff, threads: int, procs: int, calls_per_thread: int,
        window_topics: int, window_us: int = 50, max_levels: int = 0, record: bool = False,
        deliver_threads: int = 0, report_ns: int = 0, eager: bool = False):
    """One load run over the engines (one AsyncMatcher-equivalent layer inside the harness).
    Returns a dict of stats, plus 'topic', 'count', 'hash', 'exact' arrays when record.
    deliver_threads: the layer's report pool (emqxgm_async_cfg); report_ns: a busy wait per
    reported call standing for the NIF's per-call work (terms, enif_send); eager: windows sealed as
    soon as a pipe is free (EMQXGM_ASYNC_EAGER)."""
    from emqx_amd.engine import _AsyncCfg, ASYNC_EAGER
    lib = _load()
    tbytes = np.ascontiguousarray(tbytes, np.uint8)
    toff = np.ascontiguousarray(toff, np.uint64)
    n_topics = len(toff) - 1
    total = threads * calls_per_thread
    arr = (C.c_void_p * len(engines))(*[e._h for e in engines])
    cfg = _AsyncCfg(window_topics, 64 * window_topics, window_us, max_levels, 0,
                    ASYNC_EAGER if eager else 0, deliver_threads)
    topic = count = hsh = exact = None
    if record:
        topic = np.zeros(total, np.uint32)
        count = np.zeros(total, np.uint32)
        hsh = np.zeros(total, np.uint64)
        exact = np.zeros(total, np.uint8)
    st = np.zeros(10, np.float64)
    rc = lib.async_load_run(arr, len(engines), C.byref(cfg), _p(tbytes), _p(toff), n_topics,
                            threads, procs, calls_per_thread, _p(topic), _p(count), _p(hsh),
                            _p(exact), _p(st), report_ns)
    if rc:
        raise RuntimeError(f"async_load_run failed: {rc}")
    out = {"seconds": float(st[0]), "calls": int(st[1]), "topics_per_s": float(st[1] / st[0]),
           "latency_us_p50": float(st[2]), "latency_us_p99": float(st[3]),
           "latency_us_p999": float(st[4]), "latency_us_max": float(st[9]),
           "windows": int(st[5]), "calls_per_window": float(st[8]),
           "busy_retries": int(st[6]), "failed": int(st[7])}
    if record:
        out.update(topic=topic, count=count, hash=hsh, exact=exact)
    return out


_M1, _M2 = np.uint64(0xff51afd7ed558ccd), np.uint64(0xc4ceb9fe1a85ec53)


def _mix64(x):
    x = x ^ (x >> np.uint64(33))
    x = x * _M1
    x = x ^ (x >> np.uint64(33))
    x = x * _M2
    return x ^ (x >> np.uint64(33))


def string_hashes(fbytes, foff) -> np.ndarray:
    """mix64(fnv1a64(s)) of every packed string s (vectorised over byte positions)."""
    foff = np.asarray(foff, np.int64)
    lens = np.diff(foff)
    h = np.full(len(lens), 0xcbf29ce484222325, np.uint64)
    fb = np.asarray(fbytes, np.uint8)
    with np.errstate(over="ignore"):
        for k in range(int(lens.max(initial=0))):
            live = lens > k
            idx = np.nonzero(live)[0]
            b = fb[foff[idx] + k].astype(np.uint64)
            h[idx] = (h[idx] ^ b) * np.uint64(0x100000001b3)
        return _mix64(h)


def row_hashes(row_ptr, ids, id_hash) -> np.ndarray:
    """Per CSR row: the sum (mod 2^64) of id_hash over its ids -- the harness's row hash."""
    row_ptr = np.asarray(row_ptr, np.int64)
    vals = id_hash[np.asarray(ids, np.int64)] if len(ids) else np.zeros(0, np.uint64)
    csum = np.zeros(len(vals) + 1, np.uint64)
    with np.errstate(over="ignore"):
        np.cumsum(vals, out=csum[1:])
        return csum[row_ptr[1:]] - csum[row_ptr[:-1]]
