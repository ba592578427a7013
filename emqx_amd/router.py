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
