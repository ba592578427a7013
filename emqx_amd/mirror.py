"""``emqx_trie_gpu_sync`` and the writing node's hooks (src/emqx_trie_gpu_sync.erl,
src/emqx_trie_gpu.erl) restated over the engine's C-ABI: the level-triggered mirror of the
committed route table (and the local subscriber bag) into the device index.

The reference keeps a route key while its filter has a route and a wildcard filter in the trie
while it has one (emqx_router_utils.erl:34-39, 57-71).  The mirror follows that as a STATE:
whatever event arrives for topic T -- a write, a delete_object, a delete of the key, in any
number and order -- it reads the table as it is now and sets T's dests on the device
(``emqxgm_route_dests_batch``: the route key and the trie membership follow from them).

* ``handle_events``: the queued events become ONE device call committed before it returns
  (``EMQXGM_SET_COMMIT``) -- no tick; a full build running in the background is not waited for.
* ``route_changed(T)`` / ``subscribers_changed(T)``: the writing node's hooks after
  emqx_router:do_add_route/2, do_delete_route/2 and emqx_broker's subscribe / unsubscribe
  (emqx_router.erl:124-138, 171-179; emqx_broker.erl:160-212): committed before they return, so
  the node's next publish sees the change (emqx_broker.erl:163-168).
* ``resync``: ``sync_begin``, every topic of the table in chunks of ``chunk`` distinct topics per
  call, ``sync_end`` (removes every route key the scan did not see), then the subscriber lists.

``table`` is anything with ``lookup_routes(topic)`` ([(topic, dest)]; a dest is a node name or a
``(group, node)`` tuple) and ``topics()`` -- ``oracle.emqx_ref.Router`` in the tests (the route bag
``emqx_route``, emqx_router.erl:155-161, 186-188).  ``subscribers``: topic -> local subscriber
names (the ``emqx_subscriber`` bag), optional.  ``engines``: one or more engines holding the
same index (the NIF's resource: one engine per GPU).
"""
from __future__ import annotations

from collections import deque
from typing import Deque, Dict, Hashable, List, Optional, Sequence, Tuple

from .engine import NONE


class Handles:
    """The engine's 32-bit names of dests (nodes, groups) and subscribers (emqx_trie_gpu's
    handles table; the NIF maps them back to terms)."""

    def __init__(self):
        self.ids: Dict[Tuple[str, Hashable], int] = {}
        self.names: Dict[str, List[Hashable]] = {"node": [], "group": [], "sub": []}

    def __call__(self, kind: str, name: Hashable) -> int:
        k = (kind, name)
        if k not in self.ids:
            self.ids[k] = len(self.names[kind])
            self.names[kind].append(name)
        return self.ids[k]

    def dest(self, d) -> Tuple[int, int]:
        if isinstance(d, tuple):  # {Group, Node}
            return self("node", d[1]), self("group", d[0])
        return self("node", d), NONE


class RouteTableMirror:
    def __init__(self, engines: Sequence, table, subscribers: Optional[Dict] = None,
                 local_node: Hashable = "n1", chunk: int = 65536):
        self.engines = list(engines)
        self.table = table
        self.subscribers = subscribers
        self.handles = Handles()
        self.chunk = chunk
        self.queue: Deque[Tuple[str, bytes]] = deque()  # the process's mailbox of table events
        self.local = self.handles("node", local_node)  # set on the engines by init()

    # -- mnesia table events: {write, Route, _} / {delete_object, Route, _} / {delete, {Tab, T}, _}
    def event(self, kind: str, topic: bytes) -> None:
        """Queues a table event (it is handled later, like a message in the process's mailbox)."""
        assert kind in ("write", "delete_object", "delete")
        self.queue.append((kind, topic))

    def handle_events(self, limit: int = -1) -> int:
        """Handles up to `limit` queued events (all: -1) as handle_info/2 + collect/2 do: one
        batch, each topic's dests read from the table's CURRENT state, committed at once."""
        topics = set()
        k = 0
        while self.queue and k != limit:
            topics.add(self.queue.popleft()[1])
            k += 1
        if topics:
            self.sync(sorted(topics))
        return k

    def items(self, topics) -> list:
        return [(t, [self.handles.dest(d) for _, d in self.table.lookup_routes(t)]) for t in topics]

    def sync(self, topics, commit: bool = True) -> None:
        items = self.items(topics)
        for e in self.engines:
            e.route_dests_batch(items, commit=commit)

    # -- the writing node's hooks (src/emqx_trie_gpu.erl route_changed/1, subscribers_changed/1)
    def route_changed(self, topic: bytes) -> None:
        self.sync([topic])

    def subscribers_changed(self, topic: bytes, commit: bool = True) -> None:
        subs = [self.handles("sub", s) for s in (self.subscribers or {}).get(topic, [])]
        for e in self.engines:
            e.subscribers_batch([(topic, subs)], commit=commit)

    def resync(self) -> int:
        """A full resync: every topic of the table in chunks, every other route key removed,
        every subscriber list set.  Returns how many route keys the sweep removed."""
        gens = [e.sync_begin() for e in self.engines]
        topics = list(self.table.topics())
        for i in range(0, len(topics), self.chunk):
            self.sync(topics[i:i + self.chunk], commit=False)
        removed = [e.sync_end(g) for e, g in zip(self.engines, gens)]
        for t in sorted(self.subscribers or {}):
            self.subscribers_changed(t, commit=False)
        return removed[0] if removed else 0

    def commit(self) -> None:
        for e in self.engines:
            e.commit()

    def init(self, snapshot: Optional[str] = None) -> None:
        """handle_continue(open): fresh engines start from `snapshot` (broker.perf.gpu_match.
        snapshot_dir) when there is one -- no full build --, then (subscribed first,) one full
        resync and the first commit, which is then a delta of what changed since the save; the
        index is published only after it."""
        if snapshot is not None:
            import os
            if os.path.isfile(snapshot):
                for e in self.engines:
                    try:
                        e.snapshot_load(snapshot)
                    except Exception:  # another configuration's snapshot: the resync builds
                        pass
        # prepare/2: the local node after the load (it makes the engines dirty, and a snapshot
        # loads into fresh engines only)
        for e in self.engines:
            e.set_local_node(self.local)
        self.resync()
        self.commit()

    def save(self, snapshot: str) -> None:
        """terminate/2: the committed index to `snapshot` (engine 0: they all hold the same)."""
        self.engines[0].snapshot_save(snapshot)
