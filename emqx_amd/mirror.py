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

Failing closed (r06, SURVEY 5 "Failure detection").  A device call the engine refuses never
crashes the mirror or a hook, and never leaves publishers on an index that lacks a committed
change: the engine marks itself stale on the failed commit (include/emqx_gpumatch.h "Health") and
refuses every match until a repair, so publishers take the reference's path meanwhile; the
hooks return ``ok`` whatever happened; the mirror repairs (a full resync and a commit) with
backoff until the engine is healthy again; the index is published only after its first
successful repair.

``table`` is anything with ``lookup_routes(topic)`` ([(topic, dest)]; a dest is a node name or a
``(group, node)`` tuple) and ``topics()`` -- ``oracle.emqx_ref.Router`` in the tests (the route bag
``emqx_route``, emqx_router.erl:155-161, 186-188).  ``subscribers``: topic -> local subscriber
names (the ``emqx_subscriber`` bag), optional.  ``engines``: one or more engines holding the
same index (the NIF's resource: one engine per GPU).
"""
from __future__ import annotations

from collections import deque
from typing import Deque, Dict, Hashable, List, Optional, Sequence, Tuple

from .engine import NONE, EngineError


class Handles:
    """The engine's 32-bit names of dests (nodes, groups) and subscribers (emqx_trie_gpu's
    handles table; the NIF maps them back to terms).  Numbers come from the handle registry
    (emqxgm_handles_*: a released number is reused once the windows submitted before its release
    were answered); without one, from a counter."""

    def __init__(self, registry=None):
        self.ids: Dict[Tuple[str, Hashable], int] = {}
        self.names: Dict[str, Dict[int, Hashable]] = {"node": {}, "group": {}, "sub": {}}
        self.registry = registry
        self._next = {"node": 0, "group": 0, "sub": 0}

    def __call__(self, kind: str, name: Hashable) -> int:
        k = (kind, name)
        if k not in self.ids:
            if self.registry is not None:
                h = self.registry.alloc(kind)
            else:
                h = self._next[kind]
                self._next[kind] += 1
            self.ids[k] = h
            self.names[kind][h] = name
        return self.ids[k]

    def release(self, kind: str, name: Hashable) -> None:
        """term gone (emqx_trie_gpu:subscriber_down/1 -> the NIF's release_handle/3)."""
        h = self.ids.pop((kind, name), None)
        if h is None:
            return
        del self.names[kind][h]
        if self.registry is not None:
            self.registry.release(kind, h)

    def dest(self, d) -> Tuple[int, int]:
        if isinstance(d, tuple):  # {Group, Node}
            return self("node", d[1]), self("group", d[0])
        return self("node", d), NONE


class RouteTableMirror:
    BACKOFF_MS = (100, 30000)  # the repair's first retry and its cap (emqx_trie_gpu_sync.erl)

    def __init__(self, engines: Sequence, table, subscribers: Optional[Dict] = None,
                 local_node: Hashable = "n1", chunk: int = 65536, registry=None):
        self.engines = list(engines)
        self.table = table
        self.subscribers = subscribers
        self.handles = Handles(registry)
        self.chunk = chunk
        self.queue: Deque[Tuple[str, bytes]] = deque()  # the process's mailbox of table events
        self.local = self.handles("node", local_node)  # set on the engines by init()
        self.published = False      # persistent_term {emqx_trie_gpu, route} set
        self.repair_pending = False  # a `resync` cast queued (repair/1)
        self.backoff_ms = 0          # the next retry's delay after a failed repair (0: none due)
        self.errors = 0              # device calls refused so far

    def _refused(self) -> None:
        """check/2, sync_result/1: the engine refused (it marked itself stale): a repair."""
        self.errors += 1
        self.repair_pending = True

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

    def _each(self, f) -> None:
        """f(engine) on EVERY engine, then the first error raised: an engine that refused is
        stale, the others must still get the change (the NIF's on_engines)."""
        err = None
        for e in self.engines:
            try:
                f(e)
            except EngineError as ex:
                err = err or ex
        if err is not None:
            raise err

    def _dests(self, topics, commit: bool) -> None:
        items = self.items(topics)
        self._each(lambda e: e.route_dests_batch(items, commit=commit))

    def sync(self, topics, commit: bool = True) -> bool:
        """sync/2 + check/2: the topics' state := the table's now; False: refused (repair due)."""
        try:
            self._dests(topics, commit)
        except EngineError:
            self._refused()
            return False
        return True

    # -- the writing node's hooks (src/emqx_trie_gpu.erl route_changed/1, subscribers_changed/1):
    # "ok" whatever the device did (a refused change is repaired; the engine refuses matches
    # until then)
    def route_changed(self, topic: bytes) -> str:
        self.sync([topic])
        return "ok"

    def _subs(self, topic: bytes, commit: bool) -> None:
        subs = [self.handles("sub", s) for s in (self.subscribers or {}).get(topic, [])]
        self._each(lambda e: e.subscribers_batch([(topic, subs)], commit=commit))

    def subscribers_changed(self, topic: bytes, commit: bool = True) -> str:
        try:
            self._subs(topic, commit)
        except EngineError:
            self._refused()
        return "ok"

    def subscriber_down(self, sub: Hashable) -> str:
        """emqx_trie_gpu:subscriber_down/1, after emqx_broker:subscriber_down/1 removed the
        subscriber's rows and each of its topics' subscribers_changed/1 committed: its handle goes
        back to the registry (emqx_broker.erl:361-380)."""
        self.handles.release("sub", sub)
        return "ok"

    def resync(self) -> int:
        """A full resync: every topic of the table in chunks, every other route key removed,
        every subscriber list set.  Returns how many route keys the sweep removed; raises
        EngineError when the engine refuses a step (resync/1 returns {error, _})."""
        gens = [e.sync_begin() for e in self.engines]
        topics = list(self.table.topics())
        for i in range(0, len(topics), self.chunk):
            self._dests(topics[i:i + self.chunk], commit=False)
        # the subscriber lists before sync_end, which clears every list the resync did not give
        for t in sorted(self.subscribers or {}):
            self._subs(t, commit=False)
        removed = [e.sync_end(g) for e, g in zip(self.engines, gens)]
        return removed[0] if removed else 0

    def commit(self) -> None:
        """Raises EngineError; -ESTALE: committed, but an engine is still stale (no resync since
        its last mark, or its streams did not answer)."""
        self._each(lambda e: e.commit())

    def repair(self) -> bool:
        """handle_cast(resync) / handle_info(repair): a full resync and a commit.  True: every
        engine healthy (and the index published, if it was not yet); False: the next try is due
        after ``backoff_ms`` (doubling from BACKOFF_MS[0] up to BACKOFF_MS[1])."""
        self.repair_pending = False
        try:
            self.resync()
            self.commit()
        except EngineError:
            self.errors += 1
            lo, hi = self.BACKOFF_MS
            self.backoff_ms = min(hi, max(lo, 2 * self.backoff_ms))
            return False
        self.backoff_ms = 0
        self.published = True
        return True

    def healthy(self) -> bool:
        return all(e.health()["stale"] == 0 for e in self.engines)

    def device_offered(self) -> bool:
        """Whether a publisher's call may be answered by the device: the index is published and
        some engine is not stale (emqxgm_async_match refuses -ESTALE when none is)."""
        return self.published and any(e.health()["stale"] == 0 for e in self.engines)

    def match_routes(self, topic: bytes):
        """emqx_trie_gpu:match_routes/1 with one engine's synchronous match standing in for the
        NIF's window: [(topic, dest)] in match_routes order (the topic's own rows, then each matched
        filter's).  The table's own match_routes (the reference's path) answers before the first
        repair and whenever the device refuses (-ESTALE) or fails (a repair is then due)."""
        if not self.published:
            return list(self.table.match_routes(topic))
        try:
            r = self.engines[0].match([topic])
        except EngineError as ex:
            if "ESTALE" not in str(ex):
                self._refused()
            return list(self.table.match_routes(topic))
        filters = self.engines[0].filters_bytes(r.row(0).tolist())
        exact = int(r.exact_id[0]) != NONE
        heads = ([topic] if exact else []) + list(filters)
        return [rt for f in heads for rt in self.table.lookup_routes(f)]

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
        if not self.repair():  # unpublished: publishers take the reference's path until it works
            self.repair_pending = True

    def save(self, snapshot: str) -> None:
        """terminate/2: the committed index to `snapshot` (engine 0: they all hold the same)."""
        self.engines[0].snapshot_save(snapshot)


class LoadAdaptive:
    """emqx_trie_gpu's load-adaptive choice (low_load/0, sample_load/2): every publish counts
    itself; a sample every `sample_ms` sets whether the rate since the last sample is under
    `below_rate` publishes/s -- then the reference path answers (at idle its walk on the
    publisher's core is ~4x faster than a device window: bench.py's `crossover`).  0 = always the
    device.  `clock` (ms) is injectable for tests."""

    def __init__(self, below_rate: int = 0, sample_ms: int = 100, clock=None):
        import time
        self.below_rate = below_rate
        self.sample_ms = sample_ms
        self.clock = clock or (lambda: time.monotonic() * 1e3)
        self.count = 0
        self.low = False
        self._last = (0, self.clock())

    def note(self) -> bool:
        """One publish: True when it takes the reference path."""
        self.count += 1
        return self.low

    def sample(self) -> None:
        c0, t0 = self._last
        t1 = self.clock()
        rate = (self.count - c0) * 1000 // max(1, int(t1 - t0))
        self.low = self.below_rate > 0 and rate < self.below_rate
        self._last = (self.count, t1)
