"""The retainer's mnesia backend on the device (apps/emqx_retainer/src/emqx_retainer_mnesia.erl),
SURVEY 8f rank 4: retained topics (messages stay with the caller) and the reverse match
``match_messages`` -- a subscription filter to the stored topics it selects -- in batches.

The selected set is ``search_table/3``'s (:300-330) with expiry 0 or > now and no '$' rule:
with index specs configured -- by default the reference's ``[[1,2,3],[1,3],[2,3],[3]]``
(emqx_retainer_schema.erl:24-29) -- the index path of the best-scoring index
(emqx_retainer_index.erl:83-91, 141-200: ``a/+`` also selects ``a/x/y`` under ``[1,2,3]``);
with ``index_specs=[]``, or when no index scores, the full scan of ``condition/1`` (:97-112:
'+' any one word, a last '#' any tail).  See DESIGN.md 6c.

    r = Retainer()
    r.store_retained(b"sensor/1/temp", expiry_ms=0)
    r.match_messages(b"sensor/+/temp", now_ms)   # -> [b"sensor/1/temp"]
"""
from __future__ import annotations

import ctypes as C
import time
from typing import List, Optional, Sequence

import numpy as np

from . import engine as E


def _now_ms() -> int:
    return int(time.time() * 1000)


DEFAULT_INDEX_SPECS = ((1, 2, 3), (1, 3), (2, 3), (3,))  # emqx_retainer_schema.erl:24-29


class Retainer:
    def __init__(self, device: int = 0, index_specs: Sequence[Sequence[int]] = DEFAULT_INDEX_SPECS):
        self._lib = E.lib()
        h = C.c_void_p()
        rc = self._lib.emqxgm_retain_create(device, C.byref(h))
        if rc != 0:
            raise E.EngineError(f"emqxgm_retain_create failed: {rc}")
        self._h = h
        self._dirty = False
        self.set_index_specs(index_specs)

    def set_index_specs(self, specs: Sequence[Sequence[int]]) -> None:
        """retainer.backend.index_specs (config_indices/0); [] = the full scan only."""
        pos = np.array([p for s in specs for p in s], np.uint32)
        off = np.zeros(len(specs) + 1, np.uint32)
        np.cumsum([len(s) for s in specs], out=off[1:])
        self._check(self._lib.emqxgm_retain_set_indices(self._h, E._ptr(pos), E._ptr(off),
                                                        len(specs)), "retain_set_indices")

    def close(self):
        if self._h:
            self._lib.emqxgm_retain_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc < 0:
            raise E.EngineError(f"{what} failed: {rc}")
        return rc

    # ---- emqx_retainer_mnesia API ----
    def store_retained(self, topic: bytes, expiry_ms: int = 0) -> int:
        i = C.c_uint32()
        self._check(self._lib.emqxgm_retain_store(self._h, topic, len(topic), expiry_ms,
                                                  C.byref(i)), "retain_store")
        self._dirty = True
        return i.value

    def delete_message(self, topic: bytes) -> None:
        """:166-180: a wildcard deletes every stored topic it selects (Now = 0)."""
        if _wild(topic):
            for t in self.match_messages(topic, 0):
                self._check(self._lib.emqxgm_retain_delete(self._h, t, len(t)), "retain_delete")
        else:
            self._check(self._lib.emqxgm_retain_delete(self._h, topic, len(topic)),
                        "retain_delete")
        self._dirty = True

    def clean(self) -> None:
        self._check(self._lib.emqxgm_retain_clean(self._h), "retain_clean")
        self._dirty = True

    def commit(self) -> None:
        if self._dirty:
            self._check(self._lib.emqxgm_retain_commit(self._h), "retain_commit")
            self._dirty = False

    def tune(self, key: str, value: int) -> None:
        self._check(self._lib.emqxgm_retain_tune(self._h, key.encode(), int(value)), "retain_tune")

    def stats(self) -> dict:
        a = (C.c_uint64 * 4)()
        self._check(self._lib.emqxgm_retain_stats(self._h, a), "retain_stats")
        return {"full_builds": a[0], "delta_commits": a[1], "base_topics": a[2],
                "delta_topics": a[3]}

    def size(self) -> int:
        self.commit()
        n = C.c_uint64()
        self._check(self._lib.emqxgm_retain_size(self._h, C.byref(n)), "retain_size")
        return n.value

    def topic(self, i: int) -> bytes:
        p, n = E._U8P(), C.c_uint32()
        self._check(self._lib.emqxgm_retain_topic(self._h, i, C.byref(p), C.byref(n)),
                    "retain_topic")
        return C.string_at(p, n.value)

    def read_message(self, topic: bytes, now_ms: Optional[int] = None) -> List[bytes]:
        """:182-183 / read_messages/1 :372-382 (expiry 0 or >= now)."""
        self.commit()
        i = C.c_uint32()
        rc = self._check(self._lib.emqxgm_retain_read(
            self._h, topic, len(topic), _now_ms() if now_ms is None else now_ms, C.byref(i)),
            "retain_read")
        return [topic] if rc == 1 else []

    def match_ids(self, filters: Sequence[bytes], now_ms: Optional[int] = None):
        """One device pass: (ptr[n+1] u64, ids u32) -- filter i selects ids[ptr[i]:ptr[i+1]]."""
        self.commit()
        buf, off = E.pack(list(filters), np.uint32)
        out = E._RetOut()
        self._check(self._lib.emqxgm_retain_match(
            self._h, E._ptr(buf), E._ptr(off), len(filters),
            _now_ms() if now_ms is None else now_ms, C.byref(out)), "retain_match")
        n = len(filters)
        ptr = np.ctypeslib.as_array(out.ptr, shape=(n + 1,)).copy()
        ids = (np.ctypeslib.as_array(out.id, shape=(out.n_ids,)).copy() if out.n_ids
               else np.zeros(0, np.uint32))
        return ptr, ids

    def match_messages_batch(self, filters: Sequence[bytes],
                             now_ms: Optional[int] = None) -> List[List[bytes]]:
        ptr, ids = self.match_ids(filters, now_ms)
        return [[self.topic(int(i)) for i in ids[ptr[k]:ptr[k + 1]]] for k in range(len(filters))]

    def match_messages(self, topic: bytes, now_ms: Optional[int] = None) -> List[bytes]:
        """:185-195 (all remaining answers at once)."""
        return self.match_messages_batch([topic], now_ms)[0]


def _wild(topic: bytes) -> bool:
    return any(w in (b"+", b"#") for w in topic.split(b"/"))
