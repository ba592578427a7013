"""CPU restatement of the reference's publish-match semantics -- TEST INFRASTRUCTURE ONLY.

This module is the *checker* for the MI355X engine.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and
only to compute expected results.  The product package ``emqx_amd`` never imports it.

It is a line-by-line restatement (pure Python, small cases only) of:

* ``apps/emqx/src/emqx_topic.erl``   -- ``wildcard/1`` 54-64, ``match/2`` 67-89,
  ``validate/1,2`` 92-130, ``prepend/2`` 134-149, ``levels/1`` 151-153, ``tokens/1`` 155-159,
  ``words/1``/``word/1`` 162-169, ``join/1`` 188-204, ``parse/1,2`` 206-233;
* ``apps/emqx/src/emqx_trie.erl``    -- key model 54-60, ``insert`` 121-127, ``delete`` 139-144,
  ``match/2`` 155-169, ``empty`` 178, ``make_keys/compact/do_compact/join/make_prefixes``
  195-240, ``insert_key/delete_key`` 242-260, ``lookup_topic`` 264-271, ``has_prefix``
  274-280, ``do_match`` 282-297, ``match_no_compact`` 299-325, ``match_compact`` 327-344,
  ``'match_#'`` 346-348;
* ``apps/emqx/src/emqx_router.erl``  -- ``do_add_route`` 124-138, ``match_routes`` 141-146,
  ``match_trie`` 149-153, ``lookup_routes`` 155-157, ``has_routes`` 159-161,
  ``do_delete_route`` 171-179, ``topics`` 186-188;
* ``apps/emqx/src/emqx_router_utils.erl`` -- ``insert_direct_route`` 31-32,
  ``insert_trie_route`` 34-39, ``delete_direct_route`` 48-49, ``delete_trie_route`` 57-71;
* ``apps/emqx/src/emqx_broker.erl``  -- ``aggre/1`` 284-300.

Pinning: every vector transcribed from the reference's own suites
(``emqx_topic_SUITE``, ``emqx_trie_SUITE`` in both groups, ``emqx_router_SUITE:t_match_routes``,
the ``emqx_trie`` eunit key-layout tests, ``emqx_client_SUITE`` TOPICS x WILD_TOPICS) lives in
``tests/golden/reference_vectors.json`` and is asserted by ``tests/test_oracle_golden.py``.
The Erlang reference itself cannot run in this image (no ``erl``/``erlc``), so
there is no ``oracle/_ref`` build.

Erlang word representation used here: a word is ``bytes`` for a binary, or one of the str
atoms ``''``, ``'+'``, ``'#'`` (``emqx_topic:word/1``).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

Word = Union[bytes, str]
EMPTY, PLUS, HASH = "", "+", "#"
MAX_TOPIC_LEN = 65535  # emqx_topic.erl:47


class TopicError(Exception):
    """Mirrors the ``error(Reason)`` raised by emqx_topic:validate/parse."""


# ----------------------------------------------------------------------------------------
# emqx_topic
# ----------------------------------------------------------------------------------------

def tokens(topic: bytes) -> List[bytes]:
    """emqx_topic.erl:155-159 -- ``binary:split(Topic, <<"/">>, [global])`` (keeps empties)."""
    return topic.split(b"/")


def word(w: bytes) -> Word:
    """emqx_topic.erl:166-169."""
    if w == b"":
        return EMPTY
    if w == b"+":
        return PLUS
    if w == b"#":
        return HASH
    return w


def words(topic: bytes) -> List[Word]:
    """emqx_topic.erl:162-164."""
    return [word(w) for w in tokens(topic)]


def levels(topic: bytes) -> int:
    """emqx_topic.erl:151-153."""
    return len(tokens(topic))


def wildcard(topic: Union[bytes, Sequence[Word]]) -> bool:
    """emqx_topic.erl:54-64."""
    ws = words(topic) if isinstance(topic, (bytes, bytearray)) else topic
    for w in ws:
        if w == HASH or w == PLUS:
            return True
    return False


def _bin(w: Word) -> bytes:
    """emqx_topic.erl:145-149."""
    if isinstance(w, str):
        return w.encode()
    return bytes(w)


def join(ws: Sequence[Word]) -> bytes:
    """emqx_topic.erl:188-204."""
    if not ws:
        return b""
    return b"/".join(_bin(w) for w in ws)


def prepend(parent, w) -> bytes:
    """emqx_topic.erl:134-143 (``undefined`` is passed as ``None``)."""
    if parent is None or parent == b"":
        return _bin(w)
    p = _bin(parent)
    if p[-1:] == b"/":
        return p + _bin(w)
    return p + b"/" + _bin(w)


def match(name: Union[bytes, Sequence[Word]], filt: Union[bytes, Sequence[Word]]) -> bool:
    """emqx_topic.erl:67-89 -- the MQTT predicate (set-semantics oracle)."""
    if isinstance(name, (bytes, bytearray)) and isinstance(filt, (bytes, bytearray)):
        # 70-73: a name starting with '$' never matches a filter starting with '+' or '#'
        if name[:1] == b"$" and filt[:1] in (b"+", b"#"):
            return False
        return _match_words(words(name), words(filt))
    return _match_words(list(name), list(filt))


def _match_words(n: List[Word], f: List[Word]) -> bool:
    i = 0
    while True:
        if i == len(n) and i == len(f):  # match([], []) -> true
            return True
        if i < len(n) and i < len(f) and n[i] == f[i]:  # match([H|T1], [H|T2])
            i += 1
            continue
        if i < len(n) and i < len(f) and f[i] == PLUS:  # match([_H|T1], ['+'|T2])
            i += 1
            continue
        if len(f) - i == 1 and f[i] == HASH:  # match(_, ['#']) -> true
            return True
        return False  # remaining clauses are all false


def validate(topic, kind: Optional[str] = None) -> bool:
    """emqx_topic.erl:92-130.  ``validate(B)`` == ``validate(filter, B)``;
    ``validate(('name', B))`` form is accepted too."""
    if kind is None:
        if isinstance(topic, tuple):
            kind, topic = topic
        else:
            kind = "filter"
    if topic == b"":
        raise TopicError("empty_topic")
    if len(topic) > MAX_TOPIC_LEN:
        raise TopicError("topic_too_long")
    ws = words(topic)
    if kind == "filter":
        return _validate2(ws)
    if kind == "name":
        # validate2(Words) andalso (not wildcard(Words)) orelse error(topic_name_error)
        if _validate2(ws) and not wildcard(ws):
            return True
        raise TopicError("topic_name_error")
    raise ValueError(kind)


def _validate2(ws: List[Word]) -> bool:
    for idx, w in enumerate(ws):
        if w == HASH:
            if idx != len(ws) - 1:
                raise TopicError("topic_invalid_#")
            return True
        if w == EMPTY or w == PLUS:
            continue
        _validate3(w)
    return True


def _validate3(w: bytes) -> bool:
    # validate3 walks utf8 code points; '#', '+' and NUL are single bytes in utf8 and cannot
    # occur inside a multi-byte sequence, so a bytewise scan is equivalent on valid utf8.
    for c in w:
        if c in (0x23, 0x2B, 0x00):
            raise TopicError("topic_invalid_char")
    return True


def parse(topic_filter, options: Optional[dict] = None) -> Tuple[bytes, dict]:
    """emqx_topic.erl:206-233."""
    if isinstance(topic_filter, tuple):
        topic_filter, options = topic_filter
    options = dict(options or {})
    if topic_filter.startswith(b"$share/"):
        if "share" in options:
            raise TopicError(("invalid_topic_filter", topic_filter))
        rest = topic_filter[len(b"$share/"):]
        parts = rest.split(b"/", 1)
        if len(parts) == 1:
            raise TopicError(("invalid_topic_filter", topic_filter))
        share, filt = parts
        if b"+" in share or b"#" in share:
            raise TopicError(("invalid_topic_filter", topic_filter))
        options["share"] = share
        return parse(filt, options)
    if topic_filter.startswith(b"$exclusive/"):
        t = topic_filter[len(b"$exclusive/"):]
        if t == b"":
            raise TopicError(("invalid_topic_filter", topic_filter))
        options["is_exclusive"] = True
        return t, options
    return topic_filter, options


# ----------------------------------------------------------------------------------------
# emqx_trie
# ----------------------------------------------------------------------------------------

_ROOT = object()  # the atom 'empty' used as the virtual root prefix (emqx_trie.erl:212,274)


def _tjoin(prefix, w: Word) -> bytes:
    """emqx_trie.erl:223-227."""
    if prefix is _ROOT:
        if w == PLUS:
            return b"+"
        if w == HASH:
            return b"#"
        if w == EMPTY:
            return b""
        return w
    return join([prefix, w])


def do_compact(ws: Sequence[Word]) -> List[bytes]:
    """emqx_trie.erl:211-221: segments, each ending with one wildcard word."""
    seg = _ROOT
    acc: List[bytes] = []
    for w in ws:
        if w == PLUS or w == HASH:
            acc.append(_tjoin(seg, w))
            seg = _ROOT
        else:
            seg = _tjoin(seg, w)
    if seg is not _ROOT:
        acc.append(seg)
    return acc


class Trie:
    """emqx_trie with its ETS ``ordered_set`` of ``{Key, Count}`` (emqx_trie.erl:54-60).

    ``compact`` mirrors ``broker.perf.trie_compaction`` (emqx_trie.erl:350-354); it is read at
    insert/delete time (make_keys) and at match time (do_match), like the reference.
    """

    def __init__(self, compact: bool = True):
        self.compact = compact
        self.tab: Dict[Tuple[bytes, int], int] = {}

    # --- key model ---------------------------------------------------------------------
    def make_keys(self, topic: bytes):
        """emqx_trie.erl:195-197."""
        return (topic, 1), [(p, 0) for p in self.make_prefixes(words(topic))]

    def make_prefixes(self, ws: Sequence[Word]) -> List[bytes]:
        """emqx_trie.erl:229-240 (longest prefix first, like the reference)."""
        segs = do_compact(ws) if self.compact else list(ws)
        out = []
        for i in range(len(segs) - 1, 0, -1):
            out.append(join(segs[:i]))
        return out

    def insert(self, topic: bytes) -> None:
        """emqx_trie.erl:121-127 (idempotent per filter)."""
        tk, pks = self.make_keys(topic)
        if tk in self.tab:
            return
        for k in [tk] + pks:
            self.tab[k] = self.tab.get(k, 0) + 1  # insert_key 242-250

    def delete(self, topic: bytes) -> None:
        """emqx_trie.erl:139-144 (no-op for a filter that is not in the trie)."""
        tk, pks = self.make_keys(topic)
        if tk not in self.tab:
            return
        for k in [tk] + pks:  # delete_key 252-260
            c = self.tab.get(k)
            if c is None:
                continue
            if c > 1:
                self.tab[k] = c - 1
            else:
                del self.tab[k]

    def empty(self) -> bool:
        """emqx_trie.erl:178."""
        return not self.tab

    # --- lookups -----------------------------------------------------------------------
    def lookup_topic(self, topic: bytes, is_wildcard: bool = True) -> List[bytes]:
        """emqx_trie.erl:264-271."""
        if not is_wildcard:
            return []
        c = self.tab.get((topic, 1))
        return [topic] if c is not None and c > 0 else []

    def has_prefix(self, prefix) -> bool:
        """emqx_trie.erl:274-280."""
        if prefix is _ROOT:
            return True
        c = self.tab.get((prefix, 0))
        return c is not None and c > 0

    def _match_hash(self, prefix) -> List[bytes]:
        """'match_#' emqx_trie.erl:346-348."""
        return self.lookup_topic(_tjoin(prefix, HASH))

    # --- match -------------------------------------------------------------------------
    def match(self, topic: bytes) -> List[bytes]:
        """emqx_trie.erl:155-169."""
        ws = words(topic)
        if wildcard(ws):
            return []
        return self._do_match(ws)

    def _do_match(self, ws: List[Word]) -> List[bytes]:
        """emqx_trie.erl:282-297."""
        first = ws[0]
        if isinstance(first, bytes) and first[:1] == b"$":
            rest = ws[1:]
            head = self.lookup_topic(first) if not rest else []
            return head + self._walk(rest, first)
        return self._walk(ws, _ROOT)

    def _walk(self, ws, prefix):
        if self.compact:
            return self._match_compact(ws, 0, prefix, False, [])
        return self._match_no_compact(ws, 0, prefix, False, [])

    def _match_no_compact(self, ws, i, prefix, is_wild, acc):
        """emqx_trie.erl:299-325."""
        if i == len(ws):
            return self._match_hash(prefix) + self.lookup_topic(prefix, is_wild) + acc
        if self.has_prefix(prefix):
            acc1 = self._match_hash(prefix) + acc
            acc2 = self._match_no_compact(ws, i + 1, _tjoin(prefix, PLUS), True, acc1)
            return self._match_no_compact(ws, i + 1, _tjoin(prefix, ws[i]), is_wild, acc2)
        return acc

    def _match_compact(self, ws, i, prefix, is_wild, acc):
        """emqx_trie.erl:327-344."""
        if i == len(ws):
            return self._match_hash(prefix) + self.lookup_topic(prefix, is_wild) + acc
        acc1 = self._match_hash(prefix) + acc
        acc2 = self._match_compact(ws, i + 1, _tjoin(prefix, ws[i]), is_wild, acc1)
        wprefix = _tjoin(prefix, PLUS)
        if i + 1 == len(ws) or self.has_prefix(wprefix):
            return self._match_compact(ws, i + 1, wprefix, True, acc2)
        return acc2

    def filters(self) -> List[bytes]:
        return sorted(k for (k, t) in self.tab if t == 1)


def trie_match_bruteforce(topic: bytes, filters: Iterable[bytes],
                          nonwild_in_trie: Iterable[bytes] = ()) -> List[bytes]:
    """The set statement of SURVEY 8a' item 1/3: trie(t) = {f wildcard : match(t,f)}, plus the
    single-word '$' literal quirk (emqx_trie.erl:286-287); [] for a wildcard topic."""
    ws = words(topic)
    if wildcard(ws):
        return []
    out = [f for f in filters if wildcard(f) and match(topic, f)]
    if len(ws) == 1 and isinstance(ws[0], bytes) and ws[0][:1] == b"$":
        out += [f for f in nonwild_in_trie if f == topic]
    return out


# ----------------------------------------------------------------------------------------
# emqx_router (+ emqx_router_utils) and emqx_broker:aggre
# ----------------------------------------------------------------------------------------

class Router:
    """Route bag ``emqx_route`` (filter -> #route{topic, dest}) plus the trie."""

    def __init__(self, compact: bool = True):
        self.trie = Trie(compact)
        self.bag: Dict[bytes, List[object]] = {}

    def lookup_routes(self, topic: bytes) -> List[Tuple[bytes, object]]:
        """emqx_router.erl:155-157."""
        return [(topic, d) for d in self.bag.get(topic, [])]

    def has_routes(self, topic: bytes) -> bool:
        return topic in self.bag

    def topics(self) -> List[bytes]:
        return list(self.bag)

    def add_route(self, topic: bytes, dest: object = "node") -> None:
        """emqx_router.erl:124-138 (do_add_route)."""
        if dest in self.bag.get(topic, []):
            return
        if wildcard(topic):
            # insert_trie_route (emqx_router_utils.erl:34-39)
            if topic not in self.bag:
                self.trie.insert(topic)
        self.bag.setdefault(topic, []).append(dest)

    def delete_route(self, topic: bytes, dest: object = "node") -> None:
        """emqx_router.erl:171-179 (do_delete_route)."""
        routes = self.bag.get(topic, [])
        if wildcard(topic):
            # delete_trie_route (emqx_router_utils.erl:57-71)
            if routes == [dest]:
                del self.bag[topic]
                self.trie.delete(topic)
                return
        if dest in routes:
            routes.remove(dest)
            if not routes:
                del self.bag[topic]

    def match_trie(self, topic: bytes) -> List[bytes]:
        """emqx_router.erl:149-153."""
        return [] if self.trie.empty() else self.trie.match(topic)

    def match_routes(self, topic: bytes) -> List[Tuple[bytes, object]]:
        """emqx_router.erl:141-146."""
        matched = self.match_trie(topic)
        if not matched:
            return self.lookup_routes(topic)
        out: List[Tuple[bytes, object]] = []
        for to in [topic] + matched:
            out += self.lookup_routes(to)
        return out


def aggre(routes: List[Tuple[bytes, object]]) -> list:
    """emqx_broker.erl:284-300.  A dest is a node (str) or a ``(group, node)`` tuple."""
    if not routes:
        return []
    if len(routes) == 1:
        to, d = routes[0]
        return [(to, d)] if not isinstance(d, tuple) else [(to, d[0])]
    acc: list = []
    for to, d in routes:
        if not isinstance(d, tuple):
            acc = [(to, d)] + acc
        else:
            acc = sorted(set([(to, d[0])] + acc), key=_erl_order)
    return acc


def _erl_order(entry):
    """Erlang term order for ``{To, Node | Group}``: binaries compare bytewise and an atom
    (node, str here) sorts before a binary (group)."""
    to, x = entry
    return (to, (0, x.encode()) if isinstance(x, str) else (1, bytes(x)))


def publish(router: "Router", topic: bytes, local_node: object,
            subscribers: Dict[bytes, List[object]]) -> Tuple[list, list]:
    """emqx_broker:publish/1 (emqx_broker.erl:218-232) as far as routing goes:
    ``route(aggre(match_routes(Topic)), Delivery)`` (:262-282).  Returns the aggre/1 entries
    and the local dispatches: every ``{To, Node}`` entry with ``Node =:= node()`` goes to
    dispatch(To) = each subscriber of To (subscribers/1, :546-552); other nodes are forwarded to
    and groups go to emqx_shared_sub (outside the node's own fan-out)."""
    entries = aggre(router.match_routes(topic))
    deliveries = []
    for to, dest in entries:
        if dest == local_node:
            deliveries += [(to, s) for s in subscribers.get(to, [])]
    return entries, deliveries


# ----------------------------------------------------------------------------------------
# emqx_retainer_index / emqx_retainer_mnesia: the reverse match (a subscription filter ->
# the stored retained topics it selects), an ETS match-spec search over word lists
# ----------------------------------------------------------------------------------------

ANY = "_"  # the match-spec wildcard '_' (a str, never equal to a binary word)


class Improper:
    """An improper list pattern ``[P1, ..., Pk | '_']`` (``L ++ '_'`` in the reference)."""

    def __init__(self, items):
        self.items = list(items)

    def __eq__(self, other):
        return isinstance(other, Improper) and self.items == other.items

    def __repr__(self):
        return f"Improper({self.items!r})"


def _app_any(items: list):
    """``L ++ '_'``: '_' itself for an empty L."""
    return ANY if not items else Improper(items)


def _concat(items: list, pat):
    """``L ++ Pattern`` for a proper list L."""
    if pat == ANY:
        return _app_any(items)
    if isinstance(pat, Improper):
        return Improper(items + pat.items)
    return items + list(pat)


def retainer_condition(toks: Sequence[Word]):
    """emqx_retainer_index.erl:97-112 condition/1: '+' -> '_', a last '#' -> an any tail."""
    t1 = [ANY if w == PLUS else w for w in toks]
    if not (len(t1) > 0 and t1[-1] == HASH):
        return t1
    rest = list(t1)
    rest.remove(HASH)  # Tokens1 -- ['#'] drops the first '#'
    return _app_any(rest)


def retainer_condition_index(index: Sequence[int], toks: Sequence[Word]):
    """emqx_retainer_index.erl:93-95, 174-200 condition/2: the index-key pattern."""
    def go(ix, ts, n, im, om):
        if ix and ts and ts[0] == HASH:  # :174-175
            return (_app_any(im[::-1]), _app_any(om[::-1]))
        if not ix and ts and ts[0] == HASH:  # :176-177
            return (im[::-1], _app_any(om[::-1]))
        if not ix:  # :178-179
            return (im[::-1], _concat(om[::-1], retainer_condition(ts)))
        if not ts:  # :180-181
            return (_app_any(im[::-1]), om[::-1])
        t = ts[0]
        if t == PLUS:
            if ix[0] == n:  # :182-185
                return go(ix[1:], ts[1:], n + 1, [ANY] + im, om)
            return go(ix, ts[1:], n + 1, im, [ANY] + om)  # :186-187
        if ix[0] == n:  # :188-191
            return go(ix[1:], ts[1:], n + 1, [t] + im, om)
        return go(ix, ts[1:], n + 1, im, [t] + om)  # :192-195
    return (tuple(index), go(list(index), list(toks), 1, [], []))


def retainer_to_index_key(index: Sequence[int], toks: Sequence[Word]):
    """emqx_retainer_index.erl:66-68, 130-139 to_index_key/2 + split_index_tokens/5."""
    ix, ts, n, it, ot = list(index), list(toks), 1, [], []
    while True:
        if not ix:
            return (tuple(index), (tuple(it), tuple(ot + ts)))
        if not ts:
            return (tuple(index), (tuple(it), tuple(ot)))
        if ix[0] == n:
            it.append(ts[0])
            ix = ix[1:]
        else:
            ot.append(ts[0])
        ts = ts[1:]
        n += 1


def retainer_index_score(index: Sequence[int], toks: Sequence[Word]) -> int:
    """emqx_retainer_index.erl:79-81, 141-152 index_score/2."""
    ix, ts, n, score = list(index), list(toks), 1, 0
    while ix and ts:
        if ix[0] == n and ts[0] in (PLUS, HASH):
            return score
        if ix[0] == n:
            ix, score = ix[1:], score + 1
        ts, n = ts[1:], n + 1
    return score


def retainer_select_index(toks: Sequence[Word], indices: Sequence[Sequence[int]]):
    """emqx_retainer_index.erl:83-91, 154-165 select_index/2 (None = undefined)."""
    best, sel = 0, None
    for ix in indices:
        s = retainer_index_score(ix, toks)
        if s > best:
            best, sel = s, list(ix)
    return sel


def retainer_restore_topic(key) -> List[Word]:
    """emqx_retainer_index.erl:118-121, 202-209 restore_topic/1."""
    index, (it, ot) = key
    ix, it, ot, n, out = list(index), list(it), list(ot), 1, []
    while it:
        if ix and ix[0] == n:
            out.append(it[0])
            ix, it = ix[1:], it[1:]
        else:
            out.append(ot[0])
            ot = ot[1:]
        n += 1
    return out + ot


def ets_match(pat, term) -> bool:
    """ETS match-spec head matching of the patterns above against stored keys."""
    if pat == ANY:
        return True
    if isinstance(pat, Improper):
        term = list(term) if isinstance(term, (list, tuple)) else None
        return (term is not None and len(term) >= len(pat.items)
                and all(ets_match(p, t) for p, t in zip(pat.items, term)))
    if isinstance(pat, list):
        term = list(term) if isinstance(term, (list, tuple)) else None
        return term is not None and len(term) == len(pat) and all(
            ets_match(p, t) for p, t in zip(pat, term))
    if isinstance(pat, tuple):
        return isinstance(term, tuple) and len(term) == len(pat) and all(
            ets_match(p, t) for p, t in zip(pat, term))
    return pat == term


class Retainer:
    """emqx_retainer_mnesia (apps/emqx_retainer/src/emqx_retainer_mnesia.erl) over dicts:
    ?TAB_MESSAGE (word tuple -> expiry) and ?TAB_INDEX (index key -> expiry) for the configured
    index specs (config_indices/0, sorted).  Messages are represented by their topics."""

    def __init__(self, index_specs: Sequence[Sequence[int]] = ()):
        self.msgs: Dict[tuple, int] = {}
        self.index: Dict[tuple, int] = {}
        self.indices = sorted(list(ix) for ix in index_specs)

    def store_retained(self, topic: bytes, expiry: int = 0) -> None:
        """:138-152, 262-292 (the table-full check is the caller's)."""
        toks = tuple(words(topic))
        self.msgs[toks] = expiry
        for ix in self.indices:
            self.index[retainer_to_index_key(ix, toks)] = expiry

    def _delete(self, toks: tuple) -> None:
        """:351-362 delete_message_with_indices/2."""
        self.msgs.pop(toks, None)
        for ix in self.indices:
            self.index.pop(retainer_to_index_key(ix, toks), None)

    def delete_message(self, topic: bytes) -> None:
        """:166-180: an exact topic, or every message a wildcard selects (Now = 0)."""
        if not wildcard(topic):
            self._delete(tuple(words(topic)))
        else:
            for t in self.search_table(words(topic), 0):
                self._delete(tuple(words(t)))

    def read_message(self, topic: bytes, now: int) -> List[bytes]:
        """:182-183, 372-382 (note ``Et >= Now`` here, ``>`` in the match specs)."""
        et = self.msgs.get(tuple(words(topic)))
        return [] if et is None or not (et == 0 or et >= now) else [topic]

    def search_table(self, toks: Sequence[Word], now: int) -> List[bytes]:
        """:300-330 search_table/2,3: the index path when an index scores > 0, else a scan of
        the message table with condition/1; both keep expiry 0 or > Now."""
        ix = retainer_select_index(toks, self.indices)
        if ix is None:
            ms = retainer_condition(toks)
            return [join(t) for t, et in self.msgs.items()
                    if ets_match(ms, list(t)) and (et == 0 or et > now)]
        ms = retainer_condition_index(ix, toks)
        out = []
        for key, et in self.index.items():
            if ets_match(ms, key) and (et == 0 or et > now):
                t = tuple(retainer_restore_topic(key))
                met = self.msgs.get(t)
                if met is not None and (met == 0 or met > now):
                    out.append(join(t))
        return out

    def match_messages(self, topic: bytes, now: int) -> List[bytes]:
        """:185-195 (all remaining answers at once)."""
        return self.search_table(words(topic), now)

    def size(self) -> int:
        return len(self.msgs)

    def clean(self) -> None:
        self.msgs.clear()
        self.index.clear()


def retained_match_indexed(filt: bytes, topics: Iterable[bytes],
                           index_specs: Sequence[Sequence[int]]) -> List[bytes]:
    """The set ``Retainer(index_specs).match_messages`` selects (expiry aside), as a predicate
    over the stored topics, derived from select_index/2 and condition/2
    (emqx_retainer_index.erl:83-91, 141-200) and checked against ``Retainer.search_table`` by
    tests/test_oracle_golden.py: with no index scoring > 0 the full scan; on the index path a
    first '#' (any position) makes the words before it a prefix with any tail, and a filter that
    ends while index positions remain selects topics up to the run of index positions right
    after its last word longer (any words there)."""
    toks = words(filt)
    ix = retainer_select_index(toks, sorted(list(s) for s in index_specs))
    if ix is None:
        return retained_match(filt, topics)
    rest = list(ix)
    for n, w in enumerate(toks, 1):
        if w == HASH:  # condition/5 :174-177, before the index is used up or right at it
            pre = toks[:n - 1]
            return [t for t in topics if len(words(t)) >= len(pre) and all(
                f == PLUS or f == x for f, x in zip(pre, words(t)))]
        if not rest:  # :178-179: the rest through condition/1, i.e. the full scan's pattern
            return retained_match(filt, topics)
        if rest[0] == n:
            rest = rest[1:]
    k, tail = len(toks), 0
    for p in rest:
        if p == k + 1 + tail:
            tail += 1
    return [t for t in topics if k <= len(words(t)) <= k + tail and all(
        f == PLUS or f == w for f, w in zip(toks, words(t)))]


def retained_match(filt: bytes, topics: Iterable[bytes]) -> List[bytes]:
    """The set match_messages selects, as a predicate: the topics whose word lists the
    condition/1 pattern of ``filt`` matches (``+`` any one word, a last ``#`` any tail, the
    '$' clauses of emqx_topic:match/2 NOT applied)."""
    ms = retainer_condition(words(filt))
    return [t for t in topics if ets_match(ms, words(t))]
