"""``emqx_trie`` contract on the MI355X engine (apps/emqx/src/emqx_trie.erl).

Same names, argument meaning and error behaviour as the reference module:

* ``insert(Topic) -> ok``            emqx_trie.erl:113-127 (idempotent per filter)
* ``delete(Topic) -> ok``            emqx_trie.erl:130-144 (absent filter: no-op)
* ``match(Topic) -> [Filter]``       emqx_trie.erl:147-169 (wildcard topic name -> [])
* ``empty() -> boolean()``           emqx_trie.erl:172-178
* ``match_batch([Topic]) -> [[Filter]]`` -- the batched form the engine exists for.

Mutations inside the reference happen in mria transactions and become visible at commit
(emqx_router_utils.erl:74-135); here they land in the engine's pending registry and become
visible at ``commit()``.  ``match``/``empty`` commit pending changes first, which is what a
caller sees after its own transaction returned.  ``transaction()`` groups several mutations
into one commit.  ``set_compact`` exists for API parity: trie compaction changes the
reference's key layout, never its match results (both test groups of emqx_trie_SUITE assert
the same answers), and the device index has one layout.
"""
from __future__ import annotations

import contextlib
from typing import List, Sequence

from .engine import NONE, Engine, MatchResult


class Trie:
    def __init__(self, engine: Engine = None, device: int = 0, **engine_kw):
        self.engine = engine or Engine(device=device, **engine_kw)
        self._depth = 0
        self._compact = True

    # --- emqx_trie:is_compact/0, set_compact/1 (emqx_trie.erl:350-354) ---
    def is_compact(self) -> bool:
        return self._compact

    def set_compact(self, flag: bool) -> None:
        self._compact = bool(flag)

    @contextlib.contextmanager
    def transaction(self):
        self._depth += 1
        try:
            yield self
        finally:
            self._depth -= 1
            if self._depth == 0:
                self.engine.commit()

    def _maybe_commit(self):
        if self._depth == 0:
            self.engine.commit()

    def insert(self, topic: bytes) -> str:
        self.engine.trie_insert(topic)
        return "ok"

    def delete(self, topic: bytes) -> str:
        self.engine.trie_delete(topic)
        return "ok"

    def empty(self) -> bool:
        self._maybe_commit()
        return self.engine.trie_empty()

    def match(self, topic: bytes) -> List[bytes]:
        return self.match_batch([topic])[0]

    def match_batch(self, topics: Sequence[bytes]) -> List[List[bytes]]:
        self._maybe_commit()
        res = self.engine.match(topics)
        return [[self.engine.filter_bytes(int(f)) for f in res.row(i)] for i in range(len(topics))]

    def match_ids(self, topics: Sequence[bytes]) -> MatchResult:
        self._maybe_commit()
        return self.engine.match(topics)

    # ---- the session trie (emqx_trie.erl:84-100, 117-119, 135-137, 151-153, 175-176): the same
    # operations on a second table, used when persistent sessions are enabled
    # (emqx_session_router.erl:147-159).  Here: a second engine index on the same device,
    # created on first use. ----
    def _session(self) -> "Trie":
        s = getattr(self, "_session_trie", None)
        if s is None:
            s = self._session_trie = Trie(device=self.engine.device)
            s._compact = self._compact
        return s

    def insert_session(self, topic: bytes) -> str:
        return self._session().insert(topic)

    def delete_session(self, topic: bytes) -> str:
        return self._session().delete(topic)

    def match_session(self, topic: bytes) -> List[bytes]:
        return self._session().match(topic)

    def match_session_batch(self, topics: Sequence[bytes]) -> List[List[bytes]]:
        return self._session().match_batch(topics)

    def empty_session(self) -> bool:
        return self._session().empty()

    def lookup_topic(self, topic: bytes) -> List[bytes]:
        """emqx_trie.erl:267-271 -- whether the committed trie holds the key {Topic, 1}."""
        self._maybe_commit()
        return [topic] if self.engine.trie_member(topic) else []
