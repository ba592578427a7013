"""``emqx_trie_gpu_sync`` (src/emqx_trie_gpu_sync.erl) restated over the engine's C-ABI: the
level-triggered mirror of a committed route table into the device index.

The reference keeps a route key while its filter has a route and a wildcard filter in the trie
while it has one (emqx_router_utils.erl:34-39, 57-71).  The mirror follows that as a STATE:
whatever event arrives for topic T -- a write, a delete_object, a delete of the key, in any
number and order -- it reads the table as it is now and calls ``emqxgm_route_set(T,
has_routes(T))``.  A full resync (at start and then periodically) is ``sync_begin``, every topic
of the table set present, ``sync_end``, which removes the route keys the scan did not see.
Events queued while a resync runs are handled after it, against the table as it is then.

``table`` is anything with ``has_routes(topic)`` and ``topics()`` -- ``oracle.emqx_ref.Router``
in the tests (the route bag ``emqx_route``, emqx_router.erl:155-161, 186-188).  ``engines``: one
or more engines holding the same index (the NIF's resource: one engine per GPU).
"""
from __future__ import annotations

from collections import deque
from typing import Deque, Sequence, Tuple


class RouteTableMirror:
    def __init__(self, engines: Sequence, table):
        self.engines = list(engines)
        self.table = table
        self.queue: Deque[Tuple[str, bytes]] = deque()  # the process's mailbox of table events
        self.dirty = False

    # -- mnesia table events: {write, Route, _} / {delete_object, Route, _} / {delete, {Tab, T}, _}
    def event(self, kind: str, topic: bytes) -> None:
        """Queues a table event (it is handled later, like a message in the process's mailbox)."""
        assert kind in ("write", "delete_object", "delete")
        self.queue.append((kind, topic))

    def handle_events(self, limit: int = -1) -> int:
        """Handles up to `limit` queued events (all: -1), as handle_info/2 does: each sets its
        topic's membership from the table's CURRENT state."""
        k = 0
        while self.queue and k != limit:
            _kind, topic = self.queue.popleft()
            self.set(topic)
            k += 1
        return k

    def set(self, topic: bytes) -> None:
        present = bool(self.table.has_routes(topic))
        for e in self.engines:
            e.route_set(topic, present)
        self.dirty = True

    def resync(self) -> int:
        """A full resync: every topic of the table set present, every other route key removed.
        Returns how many route keys the sweep removed (engine 0's count)."""
        gens = [e.sync_begin() for e in self.engines]
        for t in self.table.topics():
            for e in self.engines:
                e.route_set(t, True)
        removed = [e.sync_end(g) for e, g in zip(self.engines, gens)]
        self.dirty = True
        return removed[0] if removed else 0

    def commit(self) -> None:
        for e in self.engines:
            e.commit()
        self.dirty = False

    def init(self) -> None:
        """init/1: (subscribed first,) one full resync, then the first commit; the index is
        published only after it."""
        self.resync()
        self.commit()
