"""``emqx_router`` contract on the MI355X engine (apps/emqx/src/emqx_router.erl).

* ``add_route(Topic[, Dest])`` / ``do_add_route``  emqx_router.erl:111-138
* ``delete_route(Topic[, Dest])`` / ``do_delete_route``  emqx_router.erl:163-179
* ``match_routes(Topic) -> [#route{}]``  emqx_router.erl:141-146
* ``lookup_routes(Topic)``, ``has_routes(Topic)``, ``topics()``  emqx_router.erl:155-161, 186-188
* ``match_routes_batch([Topic])`` -- the batched publish path.

The route bag (filter -> dests) stays on the host, as ``emqx_route`` is an ETS bag on the node
(emqx_router.erl:78-92).  The engine holds the two indexes that the match reads: every route
key (exact table, so ``lookup_routes(Topic)`` of the published name is a device probe) and the
trie of wildcard route keys, kept exactly as emqx_router_utils does it (trie insert on the
first dest of a wildcard filter, delete on the last: emqx_router_utils.erl:34-39, 57-71).
Routes are returned as ``(topic, dest)`` tuples standing for ``#route{topic, dest}``.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

from .engine import NONE, Engine

Route = Tuple[bytes, object]


def wildcard(topic: bytes) -> bool:
    """emqx_topic:wildcard/1 (emqx_topic.erl:54-64) -- a host-side control-plane decision."""
    return any(w in (b"+", b"#") for w in topic.split(b"/"))


class Router:
    def __init__(self, engine: Engine = None, node: object = "node", device: int = 0,
                 **engine_kw):
        self.engine = engine or Engine(device=device, **engine_kw)
        self.node = node
        self._bag: Dict[bytes, List[object]] = {}
        self._dirty = False

    # ---- writes (emqx_router.erl:111-138, 163-179) ----
    def add_route(self, topic: bytes, dest: object = None) -> str:
        dest = self.node if dest is None else dest
        dests = self._bag.get(topic)
        if dests is not None and dest in dests:
            return "ok"
        if dests is None:
            self._bag[topic] = dests = []
            self.engine.route_ref(topic)
            if wildcard(topic):
                self.engine.trie_insert(topic)
        dests.append(dest)
        self._dirty = True
        return "ok"

    do_add_route = add_route

    def delete_route(self, topic: bytes, dest: object = None) -> str:
        dest = self.node if dest is None else dest
        dests = self._bag.get(topic)
        if not dests or dest not in dests:
            return "ok"
        dests.remove(dest)
        if not dests:
            del self._bag[topic]
            self.engine.route_unref(topic)
            if wildcard(topic):
                self.engine.trie_delete(topic)
        self._dirty = True
        return "ok"

    do_delete_route = delete_route

    def commit(self) -> None:
        if self._dirty:
            self.engine.commit()
            self._dirty = False

    # ---- reads ----
    def lookup_routes(self, topic: bytes) -> List[Route]:
        return [(topic, d) for d in self._bag.get(topic, [])]

    def has_routes(self, topic: bytes) -> bool:
        return topic in self._bag

    def topics(self) -> List[bytes]:
        return list(self._bag)

    def match_routes(self, topic: bytes) -> List[Route]:
        return self.match_routes_batch([topic])[0]

    def match_routes_batch(self, topics: Sequence[bytes]) -> List[List[Route]]:
        """Per topic: lookup_routes(Topic) ++ [lookup_routes(F) || F <- emqx_trie:match(Topic)]
        (emqx_router.erl:141-146; an empty trie matches nothing, :149-153)."""
        self.commit()
        res = self.engine.match(list(topics))
        out: List[List[Route]] = []
        fb = self.engine.filter_bytes
        for i, t in enumerate(topics):
            routes: List[Route] = []
            if int(res.exact_id[i]) != NONE:
                routes += self.lookup_routes(t)
            for f in res.row(i):
                routes += self.lookup_routes(fb(int(f)))
            out.append(routes)
        return out


class SessionRouter(Router):
    """``emqx_session_router`` (apps/emqx/src/emqx_session_router.erl), the router of persistent
    sessions: the same route assembly over a second route bag (``emqx_session_route_ram/disc``)
    whose wildcard filters live in the session trie (``emqx_trie:insert_session/1`` via
    emqx_router_utils:insert_session_trie_route, :41-46; delete via delete_session_trie_route,
    :54-71).  Dests are session ids.

    * ``do_add_route(Topic, SessionID)``     emqx_session_router.erl:126-143
    * ``do_delete_route(Topic, SessionID)``  :168-176
    * ``match_routes(Topic)``                :146-151 (match_trie :154-159 reads the session
      trie: [] when it is empty)
    * ``delete_routes(SessionID, Topics)``   :162-163 (asynchronous there: a cast to the pool)

    Given a :class:`emqx_amd.Trie`, the router writes that Trie's session table, so
    ``Trie.match_session`` and this router read one index, as emqx_trie's session_trie() is the
    table emqx_router_utils writes; otherwise it owns a second engine index."""

    def __init__(self, trie=None, device: int = 0, **engine_kw):
        engine = trie._session().engine if trie is not None else None
        super().__init__(engine=engine, node=None, device=device, **engine_kw)
        self.trie = trie

    def do_add_route(self, topic: bytes, session_id: object) -> str:
        return Router.add_route(self, topic, session_id)

    def do_delete_route(self, topic: bytes, session_id: object) -> str:
        return Router.delete_route(self, topic, session_id)

    add_route = do_add_route
    delete_route = do_delete_route

    def delete_routes(self, session_id: object, topics: Sequence[bytes]) -> str:
        for t in topics:
            self.do_delete_route(t, session_id)
        return "ok"

