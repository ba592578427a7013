"""ctypes binding of the engine's C-ABI (include/emqx_gpumatch.h).

This is the only way the Python host code reaches the device: there is no CPU fallback.  If the
in-tree ``libemqx_gpumatch.so`` (built by ``emqx_amd.build``) is missing, importing this module
raises; if the engine cannot be created on the device, ``Engine()`` raises ``EngineError``.
"""
from __future__ import annotations

import ctypes as C
import errno
import os
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libemqx_gpumatch.so")
NONE = 0xFFFFFFFF
ABI_VERSION = 5  # include/emqx_gpumatch.h EMQXGM_ABI_VERSION
SET_COMMIT = 1  # EMQXGM_SET_COMMIT
TAG_CANCELLED = 0xFFFFFFFFFFFFFFFF  # EMQXGM_TAG_CANCELLED


class EngineError(RuntimeError):
    pass


class _Cfg(C.Structure):
    _fields_ = [("device", C.c_int32), ("word_hash_bits", C.c_uint32),
                ("full_hash_bits", C.c_uint32), ("batch_max", C.c_uint32),
                ("walk_wg_per_cu", C.c_uint32), ("reject_cap", C.c_uint32),
                ("reserved", C.c_uint32 * 2)]


class _Out(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_pairs", C.c_uint64),
                ("row_ptr", C.POINTER(C.c_uint64)), ("filter_id", C.POINTER(C.c_uint32)),
                ("exact_id", C.POINTER(C.c_uint32))]


class _DevOut(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_pairs", C.c_uint32), ("row_ptr", C.c_void_p),
                ("filter_id", C.c_void_p), ("exact_id", C.c_void_p), ("n_words", C.c_void_p)]


class _PubOut(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_routes", C.c_uint64), ("n_deliveries", C.c_uint64),
                ("route_ptr", C.POINTER(C.c_uint64)), ("route_filter", C.POINTER(C.c_uint32)),
                ("route_dest", C.POINTER(C.c_uint32)), ("deliver_ptr", C.POINTER(C.c_uint64)),
                ("deliver_filter", C.POINTER(C.c_uint32)),
                ("deliver_sub", C.POINTER(C.c_uint32))]


class _BatchOut(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_pairs", C.c_uint32), ("row_ptr", C.POINTER(C.c_uint32)),
                ("filter_id", C.POINTER(C.c_uint32)), ("exact_id", C.POINTER(C.c_uint32))]


class _BatcherCfg(C.Structure):
    _fields_ = [("window_topics", C.c_uint32), ("window_bytes", C.c_uint32),
                ("window_us", C.c_uint32), ("reserved", C.c_uint32)]


class _WindowOut(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_pairs", C.c_uint32), ("tag", C.POINTER(C.c_uint64)),
                ("row", C.POINTER(C.c_uint32)), ("filter_id", C.POINTER(C.c_uint32)),
                ("foff", C.POINTER(C.c_uint32)), ("fbytes", C.POINTER(C.c_uint8)),
                ("exact_id", C.POINTER(C.c_uint32)), ("flush_ns", C.c_uint64),
                ("done_ns", C.c_uint64)]


class _AsyncCfg(C.Structure):
    _fields_ = [("window_topics", C.c_uint32), ("window_bytes", C.c_uint32),
                ("window_us", C.c_uint32), ("max_levels", C.c_uint32),
                ("queued_windows", C.c_uint32), ("flags", C.c_uint32),
                ("deliver_threads", C.c_uint32), ("fail_threshold", C.c_uint32)]


class _Health(C.Structure):  # emqxgm_health_t
    _fields_ = [("stale", C.c_uint32), ("last_error", C.c_int32), ("marks", C.c_uint64),
                ("repairs", C.c_uint64), ("refused", C.c_uint64)]


STALE_COMMIT = 1  # EMQXGM_STALE_COMMIT
STALE_RESYNC = 2  # EMQXGM_STALE_RESYNC


ASYNC_PUBLISH = 1  # EMQXGM_ASYNC_PUBLISH
ASYNC_EAGER = 2    # EMQXGM_ASYNC_EAGER


class _AsyncWindow(C.Structure):
    _fields_ = [("status", C.c_int), ("n", C.c_uint32), ("n_pairs", C.c_uint32),
                ("device_index", C.c_uint32), ("tag", C.POINTER(C.c_uint64)),
                ("owner", C.POINTER(C.c_uint64)), ("row", C.POINTER(C.c_uint32)),
                ("filter_id", C.POINTER(C.c_uint32)), ("foff", C.POINTER(C.c_uint32)),
                ("fbytes", C.POINTER(C.c_uint8)), ("exact_id", C.POINTER(C.c_uint32)),
                ("first_ns", C.c_uint64), ("flush_ns", C.c_uint64), ("done_ns", C.c_uint64),
                ("n_routes", C.c_uint64), ("n_deliveries", C.c_uint64),
                ("route_ptr", C.POINTER(C.c_uint64)), ("route_filter", C.POINTER(C.c_uint32)),
                ("route_dest", C.POINTER(C.c_uint32)), ("deliver_ptr", C.POINTER(C.c_uint64)),
                ("deliver_filter", C.POINTER(C.c_uint32)), ("deliver_sub", C.POINTER(C.c_uint32)),
                ("rfoff", C.POINTER(C.c_uint64)), ("rfbytes", C.POINTER(C.c_uint8))]


ASYNC_CB = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(_AsyncWindow))


class _RetOut(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_ids", C.c_uint64), ("ptr", C.POINTER(C.c_uint64)),
                ("id", C.POINTER(C.c_uint32))]


class _Stats(C.Structure):
    _fields_ = [("epoch", C.c_uint64), ("n_filters", C.c_uint64), ("n_trie_filters", C.c_uint64),
                ("n_route_keys", C.c_uint64), ("n_nodes", C.c_uint64), ("n_edges", C.c_uint64),
                ("edge_slots", C.c_uint64), ("exact_slots", C.c_uint64),
                ("device_bytes", C.c_uint64), ("max_depth", C.c_uint32),
                ("legacy_batches", C.c_uint32), ("batches", C.c_uint64),
                ("topics", C.c_uint64), ("pairs", C.c_uint64), ("rejected_pairs", C.c_uint64),
                ("reruns", C.c_uint64), ("walk_ms", C.c_double), ("walk_launches", C.c_uint64),
                ("total_ms", C.c_double), ("full_commits", C.c_uint64),
                ("delta_commits", C.c_uint64), ("last_commit_ms", C.c_double),
                ("tok_ms", C.c_double), ("tok_launches", C.c_uint64),
                ("exact_ms", C.c_double), ("keyed_nodes", C.c_uint64),
                ("buffer_grows", C.c_uint64), ("sync_gathers", C.c_uint64),
                ("bg_builds", C.c_uint64), ("bg_waits", C.c_uint64),
                ("last_build_ms", C.c_double), ("catchup_changes", C.c_uint64)]


# name -> (restype, argtypes): exactly the entry points declared in include/emqx_gpumatch.h
_P = C.c_void_p
_U8P = C.POINTER(C.c_uint8)
_U32P = C.POINTER(C.c_uint32)
_U64P = C.POINTER(C.c_uint64)
SYMBOLS = {
    "emqxgm_abi_version": (C.c_int, []),
    "emqxgm_device_pipes": (C.c_int, []),
    "emqxgm_create": (C.c_int, [C.POINTER(_Cfg), C.POINTER(_P)]),
    "emqxgm_destroy": (None, [_P]),
    "emqxgm_trie_insert": (C.c_int, [_P, C.c_char_p, C.c_uint32, _U32P]),
    "emqxgm_trie_delete": (C.c_int, [_P, C.c_char_p, C.c_uint32]),
    "emqxgm_route_ref": (C.c_int, [_P, C.c_char_p, C.c_uint32, _U32P]),
    "emqxgm_route_unref": (C.c_int, [_P, C.c_char_p, C.c_uint32]),
    "emqxgm_trie_insert_many": (C.c_int, [_P, _P, _P, C.c_uint64, _P]),
    "emqxgm_route_ref_many": (C.c_int, [_P, _P, _P, C.c_uint64, _P]),
    "emqxgm_route_set": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.c_int]),
    "emqxgm_route_set_many": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_int]),
    "emqxgm_route_set_batch": (C.c_int, [_P, _P, _P, _P, C.c_uint64, C.c_uint32, _U64P]),
    "emqxgm_route_dests_batch": (C.c_int, [_P, _P, _P, C.c_uint64, _P, _P, _P, C.c_uint32, _U64P]),
    "emqxgm_subscribers_batch": (C.c_int, [_P, _P, _P, C.c_uint64, _P, _P, C.c_uint32, _U64P]),
    "emqxgm_route_sync_begin": (C.c_int, [_P, _U32P]),
    "emqxgm_route_sync_end": (C.c_int, [_P, C.c_uint32, _U64P]),
    "emqxgm_route_member": (C.c_int, [_P, C.c_char_p, C.c_uint32]),
    "emqxgm_commit": (C.c_int, [_P, _U64P]),
    "emqxgm_get_health": (C.c_int, [_P, C.POINTER(_Health)]),
    "emqxgm_mark_stale": (C.c_int, [_P, C.c_int]),
    "emqxgm_trie_empty": (C.c_int, [_P]),
    "emqxgm_snapshot_save": (C.c_int, [_P, C.c_char_p]),
    "emqxgm_snapshot_load": (C.c_int, [_P, C.c_char_p]),
    "emqxgm_trie_member": (C.c_int, [_P, C.c_char_p, C.c_uint32]),
    "emqxgm_lookup_id": (C.c_int, [_P, C.c_char_p, C.c_uint32, _U32P]),
    "emqxgm_filter_bytes": (C.c_int, [_P, C.c_uint32, C.POINTER(_U8P), _U32P]),
    "emqxgm_filter_copy": (C.c_int, [_P, C.c_uint32, _P, C.c_uint32, _U32P]),
    "emqxgm_filters_copy": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint64, _P]),
    "emqxgm_match_batch": (C.c_int, [_P, _P, _P, C.c_uint32, C.POINTER(_Out)]),
    "emqxgm_match_device": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint64, C.POINTER(_DevOut)]),
    "emqxgm_match_device_submit": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint64, _U64P]),
    "emqxgm_host_alloc": (C.c_void_p, [_P, C.c_uint64]),
    "emqxgm_host_free": (None, [_P, C.c_void_p]),
    "emqxgm_match_device_wait": (C.c_int, [_P, C.c_uint64, C.POINTER(_DevOut)]),
    "emqxgm_match_batch_submit": (C.c_int, [_P, _P, _P, C.c_uint32, _U64P]),
    "emqxgm_match_batch_submit_filters": (C.c_int, [_P, _P, _P, C.c_uint32, _U64P]),
    "emqxgm_match_batch_wait": (C.c_int, [_P, C.c_uint64, C.POINTER(_BatchOut)]),
    "emqxgm_match_batch_wait_filters": (C.c_int, [_P, C.c_uint64, C.POINTER(_BatchOut),
                                                  C.POINTER(_U32P), C.POINTER(_U8P)]),
    "emqxgm_walk_census": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint64, _U64P]),
    "emqxgm_walk_census_levels": (C.c_int, [_P, _U64P, C.c_uint32]),
    "emqxgm_key_owners": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint32, _P]),
    "emqxgm_exact_owned_device": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint32, C.c_uint32, _P]),
    "emqxgm_export": (C.c_int, [_P, C.POINTER(_DevOut), _P, _P, _P, _P]),
    "emqxgm_merge": (C.c_int, [_P, C.c_uint32, _P, _P, _P, C.c_uint32, _P, _P, _P, _U32P]),
    "emqxgm_export_wire": (C.c_int, [_P, C.POINTER(_DevOut), _P, C.c_uint32, _P, _P, _P, _P,
                                     _U32P]),
    "emqxgm_merge_wire": (C.c_int, [_P, C.c_uint32, _P, _P, _P, _P, _P, _P, _P, _P, C.c_uint32,
                                    _P, _P, _P, _U32P]),
    "emqxgm_route_add": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32]),
    "emqxgm_route_delete": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32]),
    "emqxgm_set_local_node": (C.c_int, [_P, C.c_uint32]),
    "emqxgm_subscriber_add": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.c_uint32]),
    "emqxgm_subscriber_delete": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.c_uint32]),
    "emqxgm_publish_batch": (C.c_int, [_P, _P, _P, C.c_uint32, C.POINTER(_PubOut)]),
    "emqxgm_match_rules": (C.c_int, [_P, _P, _P, C.c_uint32, _P, _P, _P, C.c_uint32, _P]),
    "emqxgm_retain_create": (C.c_int, [C.c_int32, C.POINTER(_P)]),
    "emqxgm_retain_destroy": (None, [_P]),
    "emqxgm_retain_store": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.c_uint64, _U32P]),
    "emqxgm_retain_delete": (C.c_int, [_P, C.c_char_p, C.c_uint32]),
    "emqxgm_retain_clean": (C.c_int, [_P]),
    "emqxgm_retain_commit": (C.c_int, [_P]),
    "emqxgm_retain_size": (C.c_int, [_P, _U64P]),
    "emqxgm_retain_tune": (C.c_int, [_P, C.c_char_p, C.c_int64]),
    "emqxgm_retain_stats": (C.c_int, [_P, _U64P]),
    "emqxgm_retain_set_indices": (C.c_int, [_P, _P, _P, C.c_uint32]),
    "emqxgm_retain_read": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.c_uint64, _U32P]),
    "emqxgm_retain_topic": (C.c_int, [_P, C.c_uint32, C.POINTER(_U8P), _U32P]),
    "emqxgm_retain_match": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint64, C.POINTER(_RetOut)]),
    "emqxgm_batcher_create": (C.c_int, [_P, C.POINTER(_BatcherCfg), C.POINTER(_P)]),
    "emqxgm_batcher_destroy": (None, [_P]),
    "emqxgm_batcher_add": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.c_uint64, _U32P]),
    "emqxgm_batcher_due": (C.c_int, [_P, C.c_uint64]),
    "emqxgm_batcher_add_many": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint64]),
    "emqxgm_batcher_flush": (C.c_int, [_P, _U64P]),
    "emqxgm_batcher_collect": (C.c_int, [_P, C.c_uint64, C.POINTER(_WindowOut)]),
    "emqxgm_async_create": (C.c_int, [_P, C.c_uint32, C.POINTER(_AsyncCfg), ASYNC_CB, _P,
                                      C.POINTER(_P)]),
    "emqxgm_async_destroy": (None, [_P]),
    "emqxgm_async_match": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.c_uint64, C.c_uint64]),
    "emqxgm_async_cancel": (C.c_int, [_P, C.c_uint64, C.c_uint64]),
    "emqxgm_async_stats": (C.c_int, [_P, _U64P]),
    "emqxgm_async_health": (C.c_int, [_P, _U64P]),
    "emqxgm_handles_create": (C.c_int, [_P, C.c_uint32, C.POINTER(_P)]),
    "emqxgm_handles_destroy": (None, [_P]),
    "emqxgm_handles_alloc": (C.c_int, [_P, C.c_uint32, _U32P]),
    "emqxgm_handles_release": (C.c_int, [_P, C.c_uint32, C.c_uint32]),
    "emqxgm_handles_reset": (C.c_int, [_P]),
    "emqxgm_handles_stats": (C.c_int, [_P, C.c_uint32, _U64P]),
    "emqxgm_set_profiling": (C.c_int, [_P, C.c_int]),
    "emqxgm_tune": (C.c_int, [_P, C.c_char_p, C.c_int64]),
    "emqxgm_get_stats": (C.c_int, [_P, C.POINTER(_Stats)]),
    "emqxgm_last_error": (C.c_char_p, [_P]),
}


def load_library(path: str = LIB_PATH, allow_missing: bool = False) -> C.CDLL:
    """The engine library with every SYMBOLS signature set.  allow_missing: skip entry points
    the library lacks (tests/host_harness's CPU build of the host code has no retainer)."""
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build the HIP engine first (python -m emqx_amd.build); "
            "there is no CPU fallback")
    lib = C.CDLL(path)
    for name, (res, args) in SYMBOLS.items():
        if allow_missing and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.emqxgm_abi_version() != ABI_VERSION:
        raise ImportError("emqx_gpumatch ABI mismatch")
    return lib


_lib: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = load_library()
    return _lib


def pack(items: Sequence[bytes], off_dtype=np.uint64) -> Tuple[np.ndarray, np.ndarray]:
    """Pack byte strings into (bytes u8, offsets[n+1])."""
    lens = np.fromiter((len(x) for x in items), dtype=np.uint64, count=len(items))
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    buf = np.frombuffer(b"".join(items), dtype=np.uint8) if items else np.zeros(0, np.uint8)
    return buf, off.astype(off_dtype)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a.size else C.c_void_p(0)


DEST_GROUP = 0x80000000
RULE_EQ = 1     # include/emqx_gpumatch.h EMQXGM_RULE_EQ
RULE_WORDS = 2  # EMQXGM_RULE_WORDS


@dataclass
class PublishResult:
    """Host-resident result of publish_batch (emqx_broker:publish/1 over a batch): per topic
    the aggre/1 entries (filter id, dest handle; DEST_GROUP bit = shared group) and the local
    dispatches (filter id, subscriber handle)."""
    route_ptr: np.ndarray      # uint64 [n+1]
    route_filter: np.ndarray   # uint32
    route_dest: np.ndarray     # uint32
    deliver_ptr: np.ndarray    # uint64 [n+1]
    deliver_filter: np.ndarray
    deliver_sub: np.ndarray

    def routes(self, i: int):
        a, b = int(self.route_ptr[i]), int(self.route_ptr[i + 1])
        return list(zip(self.route_filter[a:b].tolist(), self.route_dest[a:b].tolist()))

    def deliveries(self, i: int):
        a, b = int(self.deliver_ptr[i]), int(self.deliver_ptr[i + 1])
        return list(zip(self.deliver_filter[a:b].tolist(), self.deliver_sub[a:b].tolist()))


@dataclass
class MatchResult:
    """Host-resident result of a batch: CSR rows of trie filter ids + exact route key ids."""
    row_ptr: np.ndarray    # uint64 [n+1]
    filter_id: np.ndarray  # uint32 [n_pairs]
    exact_id: np.ndarray   # uint32 [n]  (NONE = no route key equal to the topic)

    def row(self, i: int) -> np.ndarray:
        return self.filter_id[self.row_ptr[i]:self.row_ptr[i + 1]]


@dataclass
class DeviceResult:
    n: int
    n_pairs: int
    row_ptr: int    # device pointers (valid until the next match on the engine)
    filter_id: int
    exact_id: int
    n_words: int


class Engine:
    """One engine instance = one device index (one emqx_trie + route-key set) on one GPU."""

    def __init__(self, device: int = 0, word_hash_bits: int = 0, full_hash_bits: int = 64,
                 batch_max: int = 0, walk_wg_per_cu: int = 0, reject_cap: int = 0,
                 library: Optional[C.CDLL] = None):
        # library: another build of the C-ABI (tests: the host code on a fake HIP runtime)
        self._lib = library or lib()
        self.device = device
        cfg = _Cfg(device, word_hash_bits, full_hash_bits, batch_max, walk_wg_per_cu, reject_cap)
        h = C.c_void_p()
        rc = self._lib.emqxgm_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise EngineError(f"emqxgm_create failed ({rc}): no usable HIP device {device}")
        self._h = h
        self._pinned = []
        self.PIPES = int(self._lib.emqxgm_device_pipes())  # EMQXGM_PIPES of this build

    def close(self):
        if getattr(self, "_h", None):
            for p in getattr(self, "_pinned", []):
                self._lib.emqxgm_host_free(self._h, p)
            self._pinned = []
            self._lib.emqxgm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc < 0:
            msg = self._lib.emqxgm_last_error(self._h) or b""
            raise EngineError(f"{what}: {errno.errorcode.get(-rc, rc)} {msg.decode(errors='replace')}")
        return rc

    # ---- index mutation ----
    def trie_insert(self, f: bytes) -> int:
        i = C.c_uint32()
        self._check(self._lib.emqxgm_trie_insert(self._h, f, len(f), C.byref(i)), "trie_insert")
        return i.value

    def trie_delete(self, f: bytes) -> None:
        self._check(self._lib.emqxgm_trie_delete(self._h, f, len(f)), "trie_delete")

    def route_ref(self, f: bytes) -> int:
        i = C.c_uint32()
        self._check(self._lib.emqxgm_route_ref(self._h, f, len(f), C.byref(i)), "route_ref")
        return i.value

    def route_unref(self, f: bytes) -> None:
        self._check(self._lib.emqxgm_route_unref(self._h, f, len(f)), "route_unref")

    # ---- the level-triggered mirror (emqxgm_route_set: the NIF's sync process) ----
    def route_set(self, f: bytes, present: bool) -> None:
        self._check(self._lib.emqxgm_route_set(self._h, f, len(f), 1 if present else 0), "route_set")

    def route_set_many(self, buf: np.ndarray, off: np.ndarray, present: bool) -> None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        self._check(self._lib.emqxgm_route_set_many(self._h, _ptr(buf), _ptr(off), len(off) - 1,
                                                     1 if present else 0), "route_set_many")

    def route_set_batch(self, items: Sequence[Tuple[bytes, bool]], commit: bool = True) -> int:
        """emqxgm_route_set_batch: the membership of several filters, and (commit) visible to
        every match started after the return -- never waiting for a background full build
        unless the current tables cannot take the delta.  Returns the epoch."""
        buf, off = pack([f for f, _ in items], np.uint64)
        pr = np.fromiter((1 if p else 0 for _, p in items), dtype=np.uint8, count=len(items))
        e = C.c_uint64()
        self._check(self._lib.emqxgm_route_set_batch(self._h, _ptr(buf), _ptr(off), _ptr(pr),
                                                      len(items), SET_COMMIT if commit else 0,
                                                      C.byref(e)), "route_set_batch")
        return e.value

    def route_dests_batch(self, items: Sequence[Tuple[bytes, Sequence[Tuple[int, int]]]],
                          commit: bool = True) -> int:
        """emqxgm_route_dests_batch: each filter gets exactly these (node, group) dest handles
        (group NONE: a node dest) -- its rows of the route bag -- and its route key / trie
        membership while it has any; (commit) visible on return.  Returns the epoch."""
        buf, off = pack([f for f, _ in items], np.uint64)
        dptr = np.zeros(len(items) + 1, np.uint32)
        np.cumsum([len(d) for _, d in items], out=dptr[1:])
        node = np.array([n for _, d in items for n, _ in d], np.uint32)
        group = np.array([g for _, d in items for _, g in d], np.uint32)
        e = C.c_uint64()
        self._check(self._lib.emqxgm_route_dests_batch(
            self._h, _ptr(buf), _ptr(off), len(items), _ptr(dptr), _ptr(node), _ptr(group),
            SET_COMMIT if commit else 0, C.byref(e)), "route_dests_batch")
        return e.value

    def subscribers_batch(self, items: Sequence[Tuple[bytes, Sequence[int]]],
                          commit: bool = True) -> int:
        """emqxgm_subscribers_batch: each filter gets exactly these local subscriber handles."""
        buf, off = pack([f for f, _ in items], np.uint64)
        sptr = np.zeros(len(items) + 1, np.uint32)
        np.cumsum([len(x) for _, x in items], out=sptr[1:])
        subs = np.array([v for _, x in items for v in x], np.uint32)
        e = C.c_uint64()
        self._check(self._lib.emqxgm_subscribers_batch(
            self._h, _ptr(buf), _ptr(off), len(items), _ptr(sptr), _ptr(subs),
            SET_COMMIT if commit else 0, C.byref(e)), "subscribers_batch")
        return e.value

    def sync_begin(self) -> int:
        g = C.c_uint32()
        self._check(self._lib.emqxgm_route_sync_begin(self._h, C.byref(g)), "route_sync_begin")
        return int(g.value)

    def sync_end(self, gen: int) -> int:
        """Ends a resync: route keys not set present since sync_begin are removed; how many."""
        k = C.c_uint64()
        self._check(self._lib.emqxgm_route_sync_end(self._h, gen, C.byref(k)), "route_sync_end")
        return int(k.value)

    def route_member(self, f: bytes) -> bool:
        return bool(self._check(self._lib.emqxgm_route_member(self._h, f, len(f)), "route_member"))

    # ---- publish fan-out registry (emqx_router do_add_route/do_delete_route, subscribers) ----
    def route_add(self, f: bytes, node: int, group: int = NONE) -> None:
        self._check(self._lib.emqxgm_route_add(self._h, f, len(f), node, group), "route_add")

    def route_delete(self, f: bytes, node: int, group: int = NONE) -> None:
        self._check(self._lib.emqxgm_route_delete(self._h, f, len(f), node, group), "route_delete")

    def set_local_node(self, node: int) -> None:
        self._check(self._lib.emqxgm_set_local_node(self._h, node), "set_local_node")

    def subscriber_add(self, f: bytes, sub: int) -> None:
        self._check(self._lib.emqxgm_subscriber_add(self._h, f, len(f), sub), "subscriber_add")

    def subscriber_delete(self, f: bytes, sub: int) -> None:
        self._check(self._lib.emqxgm_subscriber_delete(self._h, f, len(f), sub),
                    "subscriber_delete")

    def publish(self, topics: Sequence[bytes]) -> PublishResult:
        buf, off = pack(list(topics), np.uint64)
        if len(buf) > 0xFFFFFFFF:
            raise EngineError("batch larger than 4 GiB: split it")
        off32 = np.ascontiguousarray(off, dtype=np.uint32)
        n = len(off32) - 1
        o = _PubOut()
        self._check(self._lib.emqxgm_publish_batch(self._h, _ptr(buf), _ptr(off32), n,
                                                   C.byref(o)), "publish_batch")

        def arr(p, k, dt):
            return np.ctypeslib.as_array(p, shape=(k,)).copy() if k else np.zeros(0, dt)
        return PublishResult(arr(o.route_ptr, n + 1, np.uint64),
                             arr(o.route_filter, o.n_routes, np.uint32),
                             arr(o.route_dest, o.n_routes, np.uint32),
                             arr(o.deliver_ptr, n + 1, np.uint64),
                             arr(o.deliver_filter, o.n_deliveries, np.uint32),
                             arr(o.deliver_sub, o.n_deliveries, np.uint32))

    def trie_insert_many(self, buf: np.ndarray, off: np.ndarray) -> np.ndarray:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        ids = np.empty(len(off) - 1, dtype=np.uint32)
        self._check(self._lib.emqxgm_trie_insert_many(self._h, _ptr(buf), _ptr(off), len(ids),
                                                       _ptr(ids)), "trie_insert_many")
        return ids

    def route_ref_many(self, buf: np.ndarray, off: np.ndarray) -> np.ndarray:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        ids = np.empty(len(off) - 1, dtype=np.uint32)
        self._check(self._lib.emqxgm_route_ref_many(self._h, _ptr(buf), _ptr(off), len(ids),
                                                     _ptr(ids)), "route_ref_many")
        return ids

    def commit(self) -> int:
        e = C.c_uint64()
        self._check(self._lib.emqxgm_commit(self._h, C.byref(e)), "commit")
        return e.value

    def snapshot_save(self, path: str) -> None:
        """emqxgm_snapshot_save: commit, then write the committed index to `path`."""
        self._check(self._lib.emqxgm_snapshot_save(self._h, os.fsencode(path)), "snapshot_save")

    def snapshot_load(self, path: str) -> None:
        """emqxgm_snapshot_load: restore a snapshot into this fresh engine (no rebuild)."""
        self._check(self._lib.emqxgm_snapshot_load(self._h, os.fsencode(path)), "snapshot_load")

    def trie_empty(self) -> bool:
        return bool(self._check(self._lib.emqxgm_trie_empty(self._h), "trie_empty"))

    def trie_member(self, f: bytes) -> bool:
        return bool(self._check(self._lib.emqxgm_trie_member(self._h, f, len(f)), "trie_member"))

    def lookup_id(self, f: bytes) -> Optional[int]:
        i = C.c_uint32()
        rc = self._lib.emqxgm_lookup_id(self._h, f, len(f), C.byref(i))
        return None if rc == -errno.ENOENT else (self._check(rc, "lookup_id") or i.value)

    def filter_bytes(self, fid: int) -> bytes:
        """The bytes of filter id `fid`, copied under the engine's registry lock
        (emqxgm_filter_copy: a pointer into the registry could dangle once a writer grows it)."""
        n = C.c_uint32()
        buf = C.create_string_buffer(256)
        rc = self._lib.emqxgm_filter_copy(self._h, fid, buf, len(buf), C.byref(n))
        if rc == -errno.ENOSPC:
            buf = C.create_string_buffer(n.value)
            rc = self._lib.emqxgm_filter_copy(self._h, fid, buf, len(buf), C.byref(n))
        self._check(rc, "filter_copy")
        return buf.raw[:n.value]

    def filters_bytes(self, ids) -> List[bytes]:
        """The bytes of many filter ids at once (emqxgm_filters_copy)."""
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        off = np.zeros(len(ids) + 1, np.uint64)
        cap = 64 * max(1, len(ids))
        for _ in range(2):
            buf = np.empty(max(cap, 1), np.uint8)
            rc = self._lib.emqxgm_filters_copy(self._h, _ptr(ids), len(ids), _ptr(buf), cap, _ptr(off))
            if rc != -errno.ENOSPC:
                break
            cap = int(off[-1])
        self._check(rc, "filters_copy")
        raw = buf.tobytes()
        return [raw[int(off[i]):int(off[i + 1])] for i in range(len(ids))]

    # ---- match ----
    def match_packed(self, buf: np.ndarray, off: np.ndarray, copy: bool = True) -> MatchResult:
        """emqxgm_match_batch over packed topics.  copy=False returns views of the handle's
        pinned result buffers (valid until the next call on this handle)."""
        off32 = np.ascontiguousarray(off, dtype=np.uint32)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        n = len(off32) - 1
        out = _Out()
        self._check(self._lib.emqxgm_match_batch(self._h, _ptr(buf), _ptr(off32), n,
                                                 C.byref(out)), "match_batch")
        cp = (lambda a: a.copy()) if copy else (lambda a: a)  # noqa: E731
        row = cp(np.ctypeslib.as_array(out.row_ptr, shape=(n + 1,)))
        fid = (cp(np.ctypeslib.as_array(out.filter_id, shape=(out.n_pairs,)))
               if out.n_pairs else np.zeros(0, np.uint32))
        ex = (cp(np.ctypeslib.as_array(out.exact_id, shape=(n,))) if n
              else np.zeros(0, np.uint32))
        return MatchResult(row, fid, ex)

    def pinned(self, n: int, dtype=np.uint8) -> np.ndarray:
        """A numpy array in pinned host memory (emqxgm_host_alloc), freed with the engine."""
        nbytes = max(1, int(n) * np.dtype(dtype).itemsize)
        p = self._lib.emqxgm_host_alloc(self._h, nbytes)
        if not p:
            raise EngineError("emqxgm_host_alloc failed")
        self._pinned.append(p)
        arr = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(p))
        return arr.view(dtype)[:int(n)]

    def match(self, topics: Sequence[bytes]) -> MatchResult:
        buf, off = pack(list(topics), np.uint64)
        if len(buf) > 0xFFFFFFFF:
            raise EngineError("batch larger than 4 GiB: split it")
        return self.match_packed(buf, off)

    def match_device(self, d_bytes: int, d_off: int, n: int, bytes_len: int) -> DeviceResult:
        o = _DevOut()
        self._check(self._lib.emqxgm_match_device(self._h, C.c_void_p(d_bytes), C.c_void_p(d_off),
                                                  n, bytes_len, C.byref(o)), "match_device")
        return DeviceResult(o.n, o.n_pairs, o.row_ptr or 0, o.filter_id or 0, o.exact_id or 0,
                            o.n_words or 0)

    PIPES = 2  # EMQXGM_PIPES (each engine reads its library's: emqxgm_device_pipes)

    def match_device_submit(self, d_bytes: int, d_off: int, n: int, bytes_len: int) -> int:
        """emqxgm_match_device_submit: enqueue a device pass, return its ticket (pipelined: up
        to PIPES passes in flight; ticket k's result stays valid until ticket k + PIPES)."""
        t = C.c_uint64(0)
        self._check(self._lib.emqxgm_match_device_submit(
            self._h, C.c_void_p(d_bytes), C.c_void_p(d_off), n, bytes_len, C.byref(t)),
            "match_device_submit")
        return int(t.value)

    def match_device_wait(self, ticket: int) -> DeviceResult:
        """emqxgm_match_device_wait: complete a submitted pass; its device-resident result."""
        o = _DevOut()
        self._check(self._lib.emqxgm_match_device_wait(self._h, ticket, C.byref(o)),
                    "match_device_wait")
        return DeviceResult(o.n, o.n_pairs, o.row_ptr or 0, o.filter_id or 0, o.exact_id or 0,
                            o.n_words or 0)

    HOST_PIPES = 3  # EMQXGM_HOST_PIPES

    def match_batch_submit(self, buf: np.ndarray, off: np.ndarray, filters: bool = False) -> int:
        """emqxgm_match_batch_submit: host-in pass (H2D, device pass, results to pinned host
        memory) enqueued on one of HOST_PIPES streams.  `buf` / `off` (uint8 / uint32, off[0] ==
        0) must stay alive and unchanged until the wait: keep a reference.  filters=True:
        emqxgm_match_batch_submit_filters (the filter-byte gather and every copy behind the pass,
        for match_batch_wait_filters)."""
        assert off.dtype == np.uint32 and buf.dtype == np.uint8
        t = C.c_uint64(0)
        fn = (self._lib.emqxgm_match_batch_submit_filters if filters
              else self._lib.emqxgm_match_batch_submit)
        self._check(fn(self._h, _ptr(buf), _ptr(off), len(off) - 1, C.byref(t)), "match_batch_submit")
        return int(t.value)

    def match_batch_wait_filters(self, ticket: int):
        """emqxgm_match_batch_wait_filters: (MatchResult, byte offsets [n_pairs + 1], filter
        bytes), copies."""
        o = _BatchOut()
        fo, fb = _U32P(), _U8P()
        self._check(self._lib.emqxgm_match_batch_wait_filters(self._h, ticket, C.byref(o),
                                                              C.byref(fo), C.byref(fb)),
                    "match_batch_wait_filters")
        n, m = o.n, o.n_pairs
        row = np.ctypeslib.as_array(o.row_ptr, shape=(n + 1,)).astype(np.uint64)
        fid = np.ctypeslib.as_array(o.filter_id, shape=(m,)).copy() if m else np.zeros(0, np.uint32)
        ex = np.ctypeslib.as_array(o.exact_id, shape=(n,)).copy() if n else np.zeros(0, np.uint32)
        foff = np.ctypeslib.as_array(fo, shape=(m + 1,)).copy()
        nb = int(foff[-1])
        fbytes = np.ctypeslib.as_array(fb, shape=(nb,)).copy() if nb else np.zeros(0, np.uint8)
        return MatchResult(row, fid, ex), foff, fbytes

    def match_batch_wait(self, ticket: int, copy: bool = True) -> MatchResult:
        """emqxgm_match_batch_wait: the host-resident result (row pointers as uint64 when copied;
        copy=False gives views of the pipe's pinned buffers, u32 rows, valid until ticket +
        HOST_PIPES is submitted)."""
        o = _BatchOut()
        self._check(self._lib.emqxgm_match_batch_wait(self._h, ticket, C.byref(o)),
                    "match_batch_wait")
        n = o.n
        row = np.ctypeslib.as_array(o.row_ptr, shape=(n + 1,))
        fid = (np.ctypeslib.as_array(o.filter_id, shape=(o.n_pairs,)) if o.n_pairs
               else np.zeros(0, np.uint32))
        ex = np.ctypeslib.as_array(o.exact_id, shape=(n,)) if n else np.zeros(0, np.uint32)
        if copy:
            return MatchResult(row.astype(np.uint64), fid.copy(), ex.copy())
        return MatchResult(row, fid, ex)

    def key_owners(self, buf: np.ndarray, off: np.ndarray, parts: int) -> np.ndarray:
        """emqxgm_key_owners: the key shard of each packed key (u8 bytes, u64 offsets[n+1])."""
        off = np.ascontiguousarray(off, dtype=np.uint64)
        out = np.empty(len(off) - 1, np.uint32)
        self._check(self._lib.emqxgm_key_owners(self._h, _ptr(np.ascontiguousarray(buf, np.uint8)),
                                                _ptr(off), len(off) - 1, parts, _ptr(out)),
                    "key_owners")
        return out

    def exact_owned_device(self, d_bytes: int, d_off: int, n: int, parts: int, part: int,
                           d_out: int) -> None:
        """emqxgm_exact_owned_device: route-key ids of the names key shard `part` owns."""
        self._check(self._lib.emqxgm_exact_owned_device(self._h, d_bytes, d_off, n, parts, part,
                                                        d_out), "exact_owned_device")

    def export(self, r: "DeviceResult", id_map: int, row: int, fid: int, exact: int) -> None:
        """emqxgm_export: copy a device-resident result into device buffers (pointers), ids
        mapped through the device array id_map (0 = identity)."""
        o = _DevOut(r.n, r.n_pairs, r.row_ptr or None, r.filter_id or None, r.exact_id or None,
                    r.n_words or None)
        self._check(self._lib.emqxgm_export(self._h, C.byref(o), C.c_void_p(id_map or None),
                                            C.c_void_p(row), C.c_void_p(fid or None),
                                            C.c_void_p(exact or None)), "export")

    def merge(self, rows: Sequence[int], fids: Sequence[int], exacts: Sequence[int], n: int,
              out_row: int, out_fid: int, out_exact: int) -> int:
        """emqxgm_merge: merge per-shard device CSRs (device pointers) into out_*; returns the
        merged pair count."""
        k = len(rows)
        arr = C.c_void_p * max(k, 1)
        tot = C.c_uint32(0)
        self._check(self._lib.emqxgm_merge(self._h, k, arr(*rows), arr(*[f or None for f in fids]),
                                           arr(*exacts), n, C.c_void_p(out_row),
                                           C.c_void_p(out_fid or None), C.c_void_p(out_exact or None),
                                           C.byref(tot)), "merge")
        return int(tot.value)

    WIRE_CNT2 = 1  # EMQXGM_WIRE_CNT2
    WIRE_ID24 = 2  # EMQXGM_WIRE_ID24

    def export_wire(self, r: "DeviceResult", id_map: int, flags: int, cnt: int, fid: int, xs: int,
                    ovf: int) -> Tuple[int, int]:
        """emqxgm_export_wire: a device-resident result in its compact wire form (device
        pointers); returns (exact entries, overflow entries)."""
        o = _DevOut(r.n, r.n_pairs, r.row_ptr or None, r.filter_id or None, r.exact_id or None,
                    r.n_words or None)
        c = (C.c_uint32 * 2)()
        self._check(self._lib.emqxgm_export_wire(self._h, C.byref(o), C.c_void_p(id_map or None),
                                                 flags, C.c_void_p(cnt or None),
                                                 C.c_void_p(fid or None), C.c_void_p(xs or None),
                                                 C.c_void_p(ovf or None), c), "export_wire")
        return int(c[0]), int(c[1])

    def merge_wire(self, flags: Sequence[int], cnts: Sequence[int], fids: Sequence[int],
                   pairs: Sequence[int], xss: Sequence[int], n_xs: Sequence[int],
                   ovfs: Sequence[int], n_ovf: Sequence[int], n: int, out_row: int, out_fid: int,
                   out_exact: int) -> int:
        """emqxgm_merge_wire: merge per-shard wire results (device pointers); returns pairs."""
        k = len(cnts)
        arr = C.c_void_p * max(k, 1)
        u32 = C.c_uint32 * max(k, 1)
        tot = C.c_uint32(0)
        nz = lambda xs: arr(*[x or None for x in xs])  # noqa: E731
        self._check(self._lib.emqxgm_merge_wire(
            self._h, k, u32(*flags), nz(cnts), nz(fids), u32(*pairs), nz(xss), u32(*n_xs),
            nz(ovfs), u32(*n_ovf), n, C.c_void_p(out_row), C.c_void_p(out_fid or None),
            C.c_void_p(out_exact or None), C.byref(tot)), "merge_wire")
        return int(tot.value)

    def walk_census(self, d_bytes: int, d_off: int, n: int, bytes_len: int) -> dict:
        """Instrumented pass: {'states': sum S(t), 'slot_loads', 'pairs', 'words',
        'lane_iters', 'wave_iters'}."""
        out = (C.c_uint64 * 6)()
        self._check(self._lib.emqxgm_walk_census(self._h, C.c_void_p(d_bytes), C.c_void_p(d_off),
                                                 n, bytes_len, out), "walk_census")
        lv = (C.c_uint64 * 32)()
        self._check(self._lib.emqxgm_walk_census_levels(self._h, lv, 32), "walk_census_levels")
        return {"states": out[0], "slot_loads": out[1], "pairs": out[2], "words": out[3],
                "lane_iters": out[4], "wave_iters": out[5],
                "loads_by_level": {"literal": list(lv[:16]), "plus": list(lv[16:32])}}

    def match_rules(self, names: Sequence[bytes], rules: Sequence[bytes],
                    flags: Sequence[int]) -> np.ndarray:
        """emqxgm_match_rules: index of the first rule matching each name (NONE if none)."""
        nb, no = pack(list(names), np.uint32)
        rb, ro = pack(list(rules), np.uint32)
        fl = np.asarray(flags, dtype=np.uint32)
        assert len(fl) == len(rules)
        out = np.empty(len(names), np.uint32)
        self._check(self._lib.emqxgm_match_rules(self._h, _ptr(nb), _ptr(no), len(names), _ptr(rb),
                                                 _ptr(ro), _ptr(fl), len(rules), _ptr(out)),
                    "match_rules")
        return out

    def health(self) -> dict:
        """emqxgm_get_health: {stale (EMQXGM_STALE_* bits, 0 = healthy), last_error, marks,
        repairs, refused} (include/emqx_gpumatch.h "Health")."""
        h = _Health()
        self._check(self._lib.emqxgm_get_health(self._h, C.byref(h)), "health")
        return {k: getattr(h, k) for k, _ in _Health._fields_}

    def mark_stale(self, err: int = errno.ETIMEDOUT) -> None:
        self._check(self._lib.emqxgm_mark_stale(self._h, -abs(err)), "mark_stale")

    def tune(self, key: str, value: int) -> None:
        self._check(self._lib.emqxgm_tune(self._h, key.encode(), int(value)), f"tune({key})")

    def set_profiling(self, on: bool) -> None:
        self._check(self._lib.emqxgm_set_profiling(self._h, 1 if on else 0), "set_profiling")

    def stats(self) -> dict:
        s = _Stats()
        self._check(self._lib.emqxgm_get_stats(self._h, C.byref(s)), "stats")
        return {k: getattr(s, k) for k, _ in _Stats._fields_}


@dataclass
class Window:
    """A collected batcher window: per topic (in add order) its tag, its trie filters' bytes
    and its exact route key id (NONE: none); flush -> completion latency in ns."""
    tag: np.ndarray        # uint64 [n]
    row: np.ndarray        # uint32 [n+1]
    filter_id: np.ndarray  # uint32 [n_pairs]
    foff: np.ndarray       # uint32 [n_pairs+1]
    fbytes: bytes
    exact_id: np.ndarray   # uint32 [n]
    latency_ns: int

    def filters(self, i: int) -> List[bytes]:
        a, b = int(self.row[i]), int(self.row[i + 1])
        return [self.fbytes[int(self.foff[j]):int(self.foff[j + 1])] for j in range(a, b)]


class Batcher:
    """emqxgm_batcher_*: the NIF batcher core (include/emqx_gpumatch.h) over an Engine."""

    def __init__(self, engine: Engine, window_topics: int = 0, window_bytes: int = 0,
                 window_us: int = 0):
        self._lib = engine._lib
        self._eng = engine  # the batcher's pinned windows belong to the engine's device
        cfg = _BatcherCfg(window_topics, window_bytes, window_us, 0)
        b = C.c_void_p()
        engine._check(self._lib.emqxgm_batcher_create(engine._h, C.byref(cfg), C.byref(b)),
                      "batcher_create")
        self._b = b

    def close(self):
        if getattr(self, "_b", None):
            self._lib.emqxgm_batcher_destroy(self._b)
            self._b = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, topic: bytes, tag: int) -> bool:
        """Appends a topic to the open window; True when the window is now full."""
        s = C.c_uint32()
        return bool(self._eng._check(self._lib.emqxgm_batcher_add(self._b, topic, len(topic), tag,
                                                                  C.byref(s)), "batcher_add"))

    def add_many(self, buf: np.ndarray, off: np.ndarray, tag0: int = 0) -> int:
        """Appends packed topics (uint8 bytes, uint32 offsets[n+1]) until the window is full;
        how many were added."""
        off = np.ascontiguousarray(off, dtype=np.uint32)
        return self._eng._check(self._lib.emqxgm_batcher_add_many(
            self._b, _ptr(np.ascontiguousarray(buf, dtype=np.uint8)), _ptr(off), len(off) - 1,
            tag0), "batcher_add_many")

    def due(self, now_ns: int) -> bool:
        return bool(self._eng._check(self._lib.emqxgm_batcher_due(self._b, now_ns), "batcher_due"))

    def flush(self) -> int:
        """Submits the open window; its id (0: it was empty)."""
        w = C.c_uint64()
        self._eng._check(self._lib.emqxgm_batcher_flush(self._b, C.byref(w)), "batcher_flush")
        return int(w.value)

    def collect(self, window: int, materialize: bool = True):
        """The window's result as a Window (copies); materialize=False only completes it and
        returns (topics, pairs, filter bytes, flush -> collected ns) without reading it."""
        o = _WindowOut()
        self._eng._check(self._lib.emqxgm_batcher_collect(self._b, window, C.byref(o)),
                         "batcher_collect")
        n, m = o.n, o.n_pairs
        if not materialize:
            return n, m, (int(o.foff[m]) if m else 0), int(o.done_ns - o.flush_ns)

        def arr(p, k, dt):
            return np.ctypeslib.as_array(p, shape=(k,)).copy() if k else np.zeros(0, dt)
        nb = int(o.foff[m]) if m else 0
        return Window(arr(o.tag, n, np.uint64), arr(o.row, n + 1, np.uint32),
                      arr(o.filter_id, m, np.uint32), arr(o.foff, m + 1, np.uint32),
                      C.string_at(o.fbytes, nb) if nb else b"", arr(o.exact_id, n, np.uint32),
                      int(o.done_ns - o.flush_ns))


@dataclass
class AsyncResult:
    """One reported call of the concurrent entry: its trie filters' bytes (None: the window
    failed, status < 0) and its exact route key id; a publish layer's call its aggre/1 entries
    [(To bytes, dest handle)] and local dispatches [(To bytes, subscriber handle)]."""
    tag: int
    owner: int
    status: int
    filters: Optional[List[bytes]]
    exact_id: int
    device_index: int
    latency_ns: int  # first call of its window -> its window's result complete
    routes: Optional[List[Tuple[bytes, int]]] = None
    deliveries: Optional[List[Tuple[bytes, int]]] = None


class AsyncMatcher:
    """emqxgm_async_*: the concurrent publish entry (what the NIF's match_async/3 calls) over
    one or more engines (one per GPU, each holding the whole index).  `callback(results)` gets
    the reported calls of each completed window (a list of AsyncResult), from an engine
    completer thread; the default callback stores them in ``self.results`` by (tag, owner)."""

    def __init__(self, engines: Sequence[Engine], callback=None, window_topics: int = 0,
                 window_bytes: int = 0, window_us: int = 0, max_levels: int = 0,
                 queued_windows: int = 0, publish: bool = False, deliver_threads: int = 0,
                 fail_threshold: int = 0, eager: bool = False):
        import threading
        self._engines = list(engines)  # kept alive: the layer uses their handles
        self._lib = self._engines[0]._lib
        self.results = {}
        self._cv = threading.Condition()
        self._user_cb = callback

        def on_window(_user, wp):
            w = wp.contents
            out = []
            for i in range(w.n):
                tag = w.tag[i]
                if tag == TAG_CANCELLED:
                    continue
                rt = dl = None
                if w.status:
                    fl, ex = None, NONE
                elif publish:
                    fl, ex = None, NONE

                    def to(j):
                        a, b = w.rfoff[j], w.rfoff[j + 1]
                        return C.string_at(C.addressof(w.rfbytes.contents) + a, b - a) if b > a else b""
                    a, b = w.route_ptr[i], w.route_ptr[i + 1]
                    rt = [(to(j), w.route_dest[j]) for j in range(a, b)]
                    names = {w.route_filter[j]: to(j) for j in range(a, b)}
                    dl = [(names[w.deliver_filter[j]], w.deliver_sub[j])
                          for j in range(w.deliver_ptr[i], w.deliver_ptr[i + 1])]
                else:
                    fl = [C.string_at(C.addressof(w.fbytes.contents) + w.foff[j],
                                      w.foff[j + 1] - w.foff[j]) if w.foff[j + 1] > w.foff[j] else b""
                          for j in range(w.row[i], w.row[i + 1])]
                    ex = w.exact_id[i]
                out.append(AsyncResult(tag, w.owner[i], w.status, fl, ex, w.device_index,
                                       w.done_ns - w.first_ns, rt, dl))
            if self._user_cb is not None:
                self._user_cb(out)
            else:
                with self._cv:
                    for r in out:
                        self.results[(r.tag, r.owner)] = r
                    self._cv.notify_all()
        self._cb = ASYNC_CB(on_window)  # kept alive as long as the layer
        cfg = _AsyncCfg(window_topics, window_bytes, window_us, max_levels, queued_windows,
                        (ASYNC_PUBLISH if publish else 0) | (ASYNC_EAGER if eager else 0),
                        deliver_threads, fail_threshold)
        arr = (C.c_void_p * len(self._engines))(*[e._h for e in self._engines])
        a = C.c_void_p()
        self._engines[0]._check(self._lib.emqxgm_async_create(arr, len(self._engines), C.byref(cfg),
                                                              self._cb, None, C.byref(a)),
                                "async_create")
        self._a = a

    def match(self, topic: bytes, tag: int, owner: int = 0) -> int:
        """0: accepted (reported later); -E2BIG / -EBUSY / -ESTALE / -EINVAL: the caller answers
        it."""
        return self._lib.emqxgm_async_match(self._a, topic, len(topic), tag, owner)

    def cancel(self, tag: int, owner: int = 0) -> bool:
        return bool(self._engines[0]._check(self._lib.emqxgm_async_cancel(self._a, tag, owner),
                                            "async_cancel"))

    def wait(self, keys, timeout: float = 30.0) -> bool:
        """Default callback only: until every (tag, owner) in keys was reported."""
        import time
        end = time.time() + timeout
        with self._cv:
            while not all(k in self.results for k in keys):
                left = end - time.time()
                if left <= 0:
                    return False
                self._cv.wait(left)
        return True

    def stats(self) -> dict:
        v = (C.c_uint64 * 8)()
        self._engines[0]._check(self._lib.emqxgm_async_stats(self._a, v), "async_stats")
        return dict(zip(("calls", "windows", "reported", "busy", "cancelled", "too_deep",
                         "failed", "outstanding"), list(v)))

    def health(self) -> dict:
        """emqxgm_async_health: handles stale now, timeouts and failed windows counted, calls
        refused with -ESTALE."""
        v = (C.c_uint64 * 4)()
        self._lib.emqxgm_async_health(self._a, v)
        return dict(zip(("stale_handles", "timeouts", "failed_windows", "refused"), list(v)))

    def close(self):
        if getattr(self, "_a", None):
            self._lib.emqxgm_async_destroy(self._a)  # reports every accepted call first
            self._a = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HandleRegistry:
    """emqxgm_handles_*: the 32-bit names of dest and subscriber terms, reused once every window
    the layers submitted before a release has been answered (include/emqx_gpumatch.h "Handle
    registry"; the NIF's alloc_handle/2, release_handle/3, reset_handles/1)."""
    KINDS = {"node": 0, "group": 1, "sub": 2}

    def __init__(self, layers: Sequence["AsyncMatcher"] = (), library: Optional[C.CDLL] = None):
        self._layers = list(layers)  # kept alive: the registry reads their windows
        self._lib = library or (self._layers[0]._lib if self._layers else lib())
        arr = (C.c_void_p * max(1, len(self._layers)))(*[x._a for x in self._layers])
        r = C.c_void_p()
        rc = self._lib.emqxgm_handles_create(arr, len(self._layers), C.byref(r))
        if rc:
            raise EngineError(f"handles_create: {errno.errorcode.get(-rc, rc)}")
        self._r = r

    def _chk(self, rc, what):
        if rc < 0:
            raise EngineError(f"{what}: {errno.errorcode.get(-rc, rc)}")
        return rc

    def alloc(self, kind: str) -> int:
        h = C.c_uint32()
        self._chk(self._lib.emqxgm_handles_alloc(self._r, self.KINDS[kind], C.byref(h)), "alloc")
        return int(h.value)

    def release(self, kind: str, h: int) -> None:
        self._chk(self._lib.emqxgm_handles_release(self._r, self.KINDS[kind], h), "release")

    def reset(self) -> None:
        self._chk(self._lib.emqxgm_handles_reset(self._r), "reset")

    def stats(self, kind: str) -> dict:
        v = (C.c_uint64 * 4)()
        self._chk(self._lib.emqxgm_handles_stats(self._r, self.KINDS[kind], v), "stats")
        return dict(zip(("made", "live", "waiting", "free"), list(v)))

    def close(self):
        if getattr(self, "_r", None):
            self._lib.emqxgm_handles_destroy(self._r)
            self._r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
