"""Ordered topic rules matched on the device: the scalar
``emqx_topic:match/2`` loops outside the router, one device pass per batch of names.

* ``authz_match_topics(names, filters)`` -- ``emqx_authz_rule:match_topics/3``
  (apps/emqx_authz/src/emqx_authz_rule.erl:201-214): True if any rule filter matches; a rule
  ``("eq", F)`` matches only the name ``F`` itself, other filters by ``match/2`` on word lists
  (``match_topic(emqx_topic:words(Topic), TopicFilter)``, so the binary '$' clauses of
  emqx_topic.erl:70-73 do not apply).
* ``rewrite_rule(names, filters)`` -- the rule ``emqx_rewrite:match_and_rewrite/3``
  (apps/emqx_modules/src/emqx_rewrite.erl:145-150) applies to each name: the first whose filter
  matches under ``match/2`` on binaries ('$' clauses apply), or None.

Both are ``TopicRules.first_match`` with the matching flags; the regex rewrite itself and the
``${clientid}``/``${username}`` placeholder feed (``feed_var/2``) stay with the caller.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

from .engine import NONE, RULE_EQ, RULE_WORDS, Engine

Rule = Union[bytes, tuple]


class TopicRules:
    def __init__(self, rules: Sequence[Rule], words: bool = False, engine: Engine = None,
                 device: int = 0):
        self.engine = engine or Engine(device=device)
        self.filters: List[bytes] = []
        self.flags: List[int] = []
        for r in rules:
            if isinstance(r, tuple):
                kind, f = r
                if kind != "eq":
                    raise ValueError(f"unknown rule kind {kind!r}")
                self.filters.append(bytes(f))
                self.flags.append(RULE_EQ)
            else:
                self.filters.append(bytes(r))
                self.flags.append(RULE_WORDS if words else 0)

    def first_match(self, names: Sequence[bytes]) -> List[Optional[int]]:
        out = self.engine.match_rules(names, self.filters, self.flags)
        return [None if int(i) == NONE else int(i) for i in out]


def authz_match_topics(names: Sequence[bytes], filters: Sequence[Rule],
                       engine: Engine = None) -> List[bool]:
    return [i is not None for i in TopicRules(filters, words=True, engine=engine).first_match(names)]


def rewrite_rule(names: Sequence[bytes], filters: Sequence[bytes],
                 engine: Engine = None) -> List[Optional[int]]:
    return TopicRules(filters, words=False, engine=engine).first_match(names)
