"""``emqx_broker`` publish fan-out on the MI355X engine (apps/emqx/src/emqx_broker.erl).

* ``subscribe(Topic, Sub)`` / ``unsubscribe(Topic, Sub)`` -- the local subscriber bag
  (emqx_broker.erl:150-214) plus the route {Topic, node()} while Topic has local subscribers.
* ``add_route(Topic, Dest)`` / ``delete_route(Topic, Dest)`` -- routes to other nodes or shared
  groups (``Dest = Node`` or ``(Group, Node)``), emqx_router:do_add_route/do_delete_route
  (emqx_router.erl:124-138, 171-179).
* ``publish(Topic)`` / ``publish_batch([Topic])`` -- route(aggre(match_routes(Topic))) of
  emqx_broker:publish/1 (:218-300): per topic the aggre/1 entries ``(To, Node | Group)`` and the
  local dispatches ``(To, Sub)`` of the entries ``{To, node()}`` (dispatch/2, :326-355).

The match, aggre and the per-subscriber expansion all run on the device
(``emqxgm_publish_batch``); this class only maps node / group / subscriber names to the
engine's 32-bit handles.  Entries are returned in the engine's deterministic order; the
reference's order is that of its fold, and route/2 treats them as a set.
"""
from __future__ import annotations

from typing import Dict, Hashable, List, Sequence, Tuple

from .engine import DEST_GROUP, NONE, Engine


class _Names:
    def __init__(self):
        self.ids: Dict[Hashable, int] = {}
        self.names: List[Hashable] = []

    def id(self, name: Hashable) -> int:
        i = self.ids.get(name)
        if i is None:
            i = self.ids[name] = len(self.names)
            self.names.append(name)
        return i


class Broker:
    def __init__(self, engine: Engine = None, node: str = "node@local", device: int = 0,
                 **engine_kw):
        self.engine = engine or Engine(device=device, **engine_kw)
        self.node = node
        self._nodes, self._groups, self._subs = _Names(), _Names(), _Names()
        self._local: Dict[bytes, set] = {}
        self.engine.set_local_node(self._nodes.id(node))
        self._dirty = True

    # ---- routes to other nodes / shared groups ----
    def _dest(self, dest) -> Tuple[int, int]:
        if isinstance(dest, tuple):  # {Group, Node}
            return self._nodes.id(dest[1]), self._groups.id(dest[0])
        return self._nodes.id(dest), NONE

    def add_route(self, topic: bytes, dest=None) -> str:
        n, g = self._dest(self.node if dest is None else dest)
        self.engine.route_add(topic, n, g)
        self._dirty = True
        return "ok"

    def delete_route(self, topic: bytes, dest=None) -> str:
        n, g = self._dest(self.node if dest is None else dest)
        self.engine.route_delete(topic, n, g)
        self._dirty = True
        return "ok"

    # ---- local subscriptions ----
    def subscribe(self, topic: bytes, sub: Hashable) -> str:
        subs = self._local.setdefault(topic, set())
        if sub not in subs:
            subs.add(sub)
            self.engine.subscriber_add(topic, self._subs.id(sub))
            if len(subs) == 1:  # first local subscriber: route {Topic, node()}
                self.add_route(topic)
            self._dirty = True
        return "ok"

    def unsubscribe(self, topic: bytes, sub: Hashable) -> str:
        subs = self._local.get(topic)
        if subs and sub in subs:
            subs.remove(sub)
            self.engine.subscriber_delete(topic, self._subs.id(sub))
            if not subs:
                del self._local[topic]
                self.delete_route(topic)
            self._dirty = True
        return "ok"

    def subscribers(self, topic: bytes) -> List[Hashable]:
        return sorted(self._local.get(topic, ()), key=repr)

    # ---- publish ----
    def commit(self) -> None:
        if self._dirty:
            self.engine.commit()
            self._dirty = False

    def publish_batch(self, topics: Sequence[bytes]):
        """[(aggre entries [(To, Node | Group)], local dispatches [(To, Sub)])] per topic."""
        self.commit()
        res = self.engine.publish(list(topics))
        fb = self.engine.filter_bytes
        out = []
        for i in range(len(topics)):
            entries = []
            for f, d in res.routes(i):
                to = fb(f)
                entries.append((to, self._groups.names[d & ~DEST_GROUP] if d & DEST_GROUP
                                else self._nodes.names[d]))
            deliveries = [(fb(f), self._subs.names[s]) for f, s in res.deliveries(i)]
            out.append((entries, deliveries))
        return out

    def publish(self, topic: bytes):
        return self.publish_batch([topic])[0]
