"""Writes ``reference_vectors.json``: known-answer vectors TRANSCRIBED from the reference's own
test suites (data only -- inputs and the expected outputs the reference asserts).

Every table below cites the suite file:line it was transcribed from (paths relative to the
reference checkout).  The reference cannot run in this image (no Erlang), so these asserted
values are the pins for the oracle (``oracle/emqx_ref.py``) and, through it, for the GPU engine.

Run:  python tests/golden/make_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

# apps/emqx/test/emqx_topic_SUITE.erl:45-115 -- (name, filter, expected) for emqx_topic:match/2
MATCH = [
    # t_match1 51-64
    ("a/b/c", "a/b/+", True), ("a/b/c", "a/#", True), ("abcd/ef/g", "#", True),
    ("abc/de/f", "abc/de/f", True), ("abc", "+", True), ("a/b/c", "a/b/c", True),
    ("a/b/c", "a/c/d", False), ("$share/x/y", "+", False), ("$share/x/y", "+/x/y", False),
    ("$share/x/y", "#", False), ("$share/x/y", "+/+/#", False),
    ("house/1/sensor/0", "house/+", False), ("house", "house/+", False),
    # t_match2 66-83
    ("sport/tennis/player1", "sport/tennis/player1/#", True),
    ("sport/tennis/player1/ranking", "sport/tennis/player1/#", True),
    ("sport/tennis/player1/score/wimbledon", "sport/tennis/player1/#", True),
    ("sport", "sport/#", True), ("sport", "#", True), ("/sport/football/score/1", "#", True),
    ("Topic/C", "+/+", True), ("TopicA/B", "+/+", True), ("TopicA/C", "+/+", True),
    ("abc", "+", True), ("a/b/c", "a/b/c", True), ("a/b/c", "a/c/d", False),
    ("$share/x/y", "+", False), ("$share/x/y", "+/x/y", False), ("$share/x/y", "#", False),
    ("$share/x/y", "+/+/#", False), ("house/1/sensor/0", "house/+", False),
    # t_match3 85-91
    ("device/60019423a83c/fw", "device/60019423a83c/#", True),
    ("device/60019423a83c/$fw", "device/60019423a83c/#", True),
    ("device/60019423a83c/$fw/fw", "device/60019423a83c/$fw/#", True),
    ("device/60019423a83c/fw/checksum", "device/60019423a83c/#", True),
    ("device/60019423a83c/$fw/checksum", "device/60019423a83c/#", True),
    ("device/60019423a83c/dust/type", "device/60019423a83c/#", True),
    # t_sigle_level_match 93-102
    ("sport/tennis/player1", "sport/tennis/+", True),
    ("sport/tennis/player1/ranking", "sport/tennis/+", False),
    ("sport", "sport/+", False), ("sport/", "sport/+", True), ("/finance", "+/+", True),
    ("/finance", "/+", True), ("/finance", "+", False),
    ("/devices/$dev1", "/devices/+", True), ("/devices/$dev1/online", "/devices/+/online", True),
    # t_sys_match 104-108
    ("$SYS/broker/clients/testclient", "$SYS/#", True), ("$SYS/broker", "$SYS/+", True),
    ("$SYS/broker", "+/+", False), ("$SYS/broker", "#", False),
    # 't_#_match' 110-115
    ("a/b/c", "#", True), ("a/b/c", "+/#", True), ("$SYS/brokers", "#", False),
    ("a/b/$c", "a/b/#", True), ("a/b/$c", "a/#", True),
    # t_match_perf 117-121
    ("a/b/ccc", "a/#", True),
    ("/abkc/19383/192939/akakdkkdkak/xxxyyuya/akakak", "/abkc/19383/+/akakdkkdkak/#", True),
]

# emqx_topic_SUITE.erl:45-49 t_wildcard
WILDCARD = [("a/b/#", True), ("a/+/#", True), ("", False), ("a/b/c", False)]

# emqx_topic_SUITE.erl:159-171 t_tokens / t_words ; atoms encoded as {"atom": ...}
WORDS = [
    ("/a/+/#", [{"atom": ""}, "a", {"atom": "+"}, {"atom": "#"}]),
    ("/abkc/19383/+/akakdkkdkak/#",
     [{"atom": ""}, "abkc", "19383", {"atom": "+"}, "akakdkkdkak", {"atom": "#"}]),
]
TOKENS = [("a/b/+/#", ["a", "b", "+", "#"])]
LEVELS = [("a/+/#", 3), ("a/b/c/d", 4)]  # t_levels 154-156

# emqx_topic_SUITE.erl:173-180 t_join: (words, expected)
JOIN = [
    ([], ""), (["x"], "x"), ([{"atom": "#"}], "#"),
    ([{"atom": "+"}, {"atom": ""}, {"atom": "#"}], "+//#"),
    (["x", "y", "z", {"atom": "+"}], "x/y/z/+"),
    ({"words_of": "/ab/cd/ef/"}, "/ab/cd/ef/"), ({"words_of": "ab/+/#"}, "ab/+/#"),
]

# emqx_topic_SUITE.erl:124-152 t_validate / t_sigle_level_validate: (kind, topic, ok|error)
VALIDATE = [
    ("filter", "a/+/#", True), ("filter", "a/b/c/d", True), ("name", "abc/de/f", True),
    ("filter", "abc/+/f", True), ("filter", "abc/#", True), ("filter", "x", True),
    ("name", "x//y", True), ("filter", "sport/tennis/#", True),
    ("name", "", "empty_topic"), ("name", "abc/#", "topic_name_error"),
    ("name", {"long_topic": True}, "topic_too_long"),
    ("filter", "abc/#/1", "topic_invalid_#"), ("filter", "abc/#xzy/+", "topic_invalid_char"),
    ("filter", "abc/xzy/+9827", "topic_invalid_char"),
    ("filter", "sport/tennis#", "topic_invalid_char"),
    ("filter", "sport/tennis/#/ranking", "topic_invalid_#"),
    ("filter", "+", True), ("filter", "+/tennis/#", True), ("filter", "sport/+/player1", True),
    ("filter", "sport+", "topic_invalid_char"),
]

# emqx_topic_SUITE.erl:154-160 t_prepend: (parent|None, word, expected)
PREPEND = [(None, "ab", "ab"), ("", "a/b", "a/b"), ("x/", "a/b", "x/a/b"),
           ("x/y", "a/b", "x/y/a/b"), ({"atom": "+"}, "a/b", "+/a/b")]

# emqx_topic_SUITE.erl:209-228 t_parse: (input, options, expected (topic, opts) | error)
PARSE = [
    ("$share/g/t", {"share": "g"}, {"error": "$share/g/t"}),
    ("$share/t", {}, {"error": "$share/t"}),
    ("$share/+/t", {}, {"error": "$share/+/t"}),
    ("a/b/+/#", {}, ["a/b/+/#", {}]),
    ("a/b/+/#", {"qos": 1}, ["a/b/+/#", {"qos": 1}]),
    ("$share/group/topic", {}, ["topic", {"share": "group"}]),
    ("$local/topic", {}, ["$local/topic", {}]),
    ("$local/$share/group/a/b/c", {}, ["$local/$share/group/a/b/c", {}]),
    ("$fastlane/topic", {}, ["$fastlane/topic", {}]),
]

# apps/emqx/test/emqx_trie_SUITE.erl:62-186 -- run in BOTH groups (compact, not_compact; 25-40).
# Each case: a list of steps; "insert"/"delete" mutate, "match" asserts the sorted result,
# "match_len" asserts only the length (t_match3 72), "lookup_topic" asserts lookup_topic/2.
TRIE_CASES = {
    "t_insert": [
        ["insert", ["sensor/1/metric/2", "sensor/+/#", "sensor/#"]],
        ["match", "sensor", ["sensor/#"]]],
    "t_match": [
        ["insert", ["sensor/1/metric/2", "sensor/+/#", "sensor/#"]],
        ["match", "sensor/1", ["sensor/#", "sensor/+/#"]]],
    "t_match_invalid": [
        ["insert", ["sensor/1/metric/2", "sensor/+/#", "sensor/#"]],
        ["match", "sensor/+", []], ["match", "#", []]],
    "t_match2": [
        ["insert", ["#", "+/#", "+/+/#"]],
        ["match", "a/b/c", ["#", "+/#", "+/+/#"]],
        ["match", "$SYS/broker/zenmq", []]],
    "t_match3": [
        ["insert", ["d/#", "a/b/+", "a/#", "#", "$SYS/#"]],
        ["match_len", "a/b/c", 3],
        ["match", "$SYS/a/b/c", ["$SYS/#"]]],
    "t_match4": [
        ["insert", ["/#", "/+", "/+/a/b/c"]],
        ["match", "/0/a/b/c", ["/#", "/+/a/b/c"]]],
    "t_match5": [
        ["insert", ["#", "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z/#",
                    "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z/+"]],
        ["match", "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z",
         ["#", "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z/#"]],
        ["match", "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z/1",
         ["#", "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z/#",
          "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z/+"]]],
    "t_match6": [
        ["insert", ["+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/#"]],
        ["match", "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z",
         ["+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/#"]]],
    "t_match7": [
        ["insert", ["a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#"]],
        ["match", "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z",
         ["a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#"]]],
    "t_empty": [
        ["empty", True], ["insert", ["topic/x/#"]], ["empty", False],
        ["delete", ["topic/x/#"]], ["empty", True]],
    "t_delete": [
        ["insert", ["sensor/1/#", "sensor/1/metric/2", "sensor/1/metric/3"]],
        ["delete", ["sensor/1/metric/2", "sensor/1/metric", "sensor/1/metric"]],
        ["match", "sensor/1/x", ["sensor/1/#"]]],
    "t_delete2": [
        ["insert", ["sensor", "sensor/1/metric/2", "sensor/+/metric/3"]],
        ["delete", ["sensor", "sensor/1/metric/2", "sensor/+/metric/3", "sensor/+/metric/3"]],
        ["match", "sensor", []], ["match", "sensor/1", []]],
    "t_delete3": [
        ["insert", ["sensor/+", "sensor/+/metric/2", "sensor/+/metric/3"]],
        ["delete", ["sensor/+/metric/2", "sensor/+/metric/3", "sensor", "sensor/+",
                    "sensor/+/unknown"]],
        ["match", "sensor", []], ["lookup_topic", "sensor/+", []]],
}

# apps/emqx/src/emqx_trie.erl:365-415 eunit key layout: (compact, filter, topic_key, prefixes)
MAKE_KEYS = [
    [False, "#", "#", []], [False, "a/+", "a/+", ["a"]], [False, "+", "+", []],
    [True, "#", "#", []], [True, "a/+", "a/+", []], [True, "+", "+", []],
    [True, "a/+/c", "a/+/c", ["a/+"]],
]
MAKE_PREFIXES = [
    [False, "a/b/+", ["a/b", "a"]], [False, "a/b/+/c/#", ["a/b/+/c", "a/b/+", "a/b", "a"]],
    [True, "a/b/+", []], [True, "a/b/+/c/#", ["a/b/+"]],
]
DO_COMPACT = [
    ["/+", ["/+"]], ["/#", ["/#"]], ["a/b/+/c", ["a/b/+", "c"]],
    ["a/+/+/b", ["a/+", "+", "b"]], ["a/+/+/+/+/b", ["a/+", "+", "+", "+", "b"]],
]

# apps/emqx/test/emqx_router_SUITE.erl:91-109 t_match_routes
ROUTER_CASES = {
    "t_match_routes": [
        ["add_route", [["a/b/c", "node"], ["a/+/c", "node"], ["a/b/#", "node"], ["#", "node"]]],
        ["match_routes", "a/b/c", [["#", "node"], ["a/+/c", "node"], ["a/b/#", "node"],
                                   ["a/b/c", "node"]]],
        ["delete_route", [["a/b/c", "node"], ["a/+/c", "node"], ["a/b/#", "node"],
                          ["#", "node"]]],
        ["match_routes", "a/b/c", []]],
}

# apps/emqx/test/emqx_client_SUITE.erl:28-44 TOPICS x WILD_TOPICS, plus the '$' publish at
# 255-270 ("$" ++ nth(2, TOPICS) is not delivered to nth(6, WILD_TOPICS) = "+/+").
CLIENT_TOPICS = ["TopicA", "TopicA/B", "Topic/C", "TopicA/C", "/TopicA"]
CLIENT_WILD = ["TopicA/+", "+/C", "#", "/#", "/+", "+/+", "TopicA/#"]
CLIENT_DOLLAR = [["$TopicA/B", "+/+", False]]

# apps/emqx/src/emqx_broker_bench.erl:33-34,163-170: each publisher topic has exactly 1 route
BENCH_PATTERNS = {"sub_ptn": "device/{{id}}/+/{{num}}/#",
                  "pub_ptn": "device/{{id}}/foo/{{num}}/bar/1/2/3/4/5",
                  "expect_routes_per_lookup": 1}


# apps/emqx_retainer/test/emqx_retainer_index_SUITE.erl:32-210 -- emqx_retainer_index.
# Words: strings are binaries, {"atom": x} the atoms '' '+' '#' and the match-spec '_';
# {"improper": [...]} is the improper list [... | '_'].
_A = {"atom": "_"}
RETAINER_INDEX = {
    # t_foreach_index_key 32-43, t_to_index_key 45-61: (index, topic words, key)
    "to_index_key": [
        ([1, 3], ["a", "b", "c"], [[1, 3], [["a", "c"], ["b"]]]),
        ([1, 4], ["a", "b", "c"], [[1, 4], [["a"], ["b", "c"]]]),
    ],
    # t_index_score 63-110: (index, filter words, score)
    "index_score": [
        ([1, 4], [{"atom": "+"}, "a", "b", {"atom": "+"}], 0),
        ([1, 2], [{"atom": "+"}, "a", "b", {"atom": "+"}], 0),
        ([1, 2], ["a", "b", {"atom": "+"}], 2),
        ([1, 2], ["a"], 1),
        ([2, 3, 4, 5], [{"atom": "+"}, "a", {"atom": "#"}], 1),
        ([2, 3, 4, 5], [{"atom": "+"}, "a", "b", {"atom": "+"}], 2),
    ],
    # t_select_index 112-132: (filter words, indices, selected or None)
    "select_index": [
        ([{"atom": "+"}, "a", "b", {"atom": "+"}], [[1, 4], [2, 3, 4, 5], [1, 2]], [2, 3, 4, 5]),
        ([{"atom": "+"}, "a", "b", {"atom": "+"}], [[1, 4]], None),
    ],
    # t_condition 134-147: (filter words, pattern)
    "condition": [
        ([{"atom": "+"}, "a", "b", {"atom": "+"}], [_A, "a", "b", _A]),
        ([{"atom": "+"}, "a", {"atom": "#"}], {"improper": [_A, "a"]}),
    ],
    # t_condition_index 149-207: (index, filter words, pattern {Index, {IndexPart, OtherPart}})
    "condition_index": [
        ([2, 3], [{"atom": "+"}, "a", "b", {"atom": "+"}], [[2, 3], [["a", "b"], [_A, _A]]]),
        ([3, 4], [{"atom": "+"}, "a", "b", {"atom": "+"}], [[3, 4], [["b", _A], [_A, "a"]]]),
        ([3, 5], [{"atom": "+"}, "a", "b", {"atom": "+"}],
         [[3, 5], [{"improper": ["b"]}, [_A, "a", _A]]]),
        ([3, 5], [{"atom": "+"}, "a", "b", {"atom": "#"}],
         [[3, 5], [{"improper": ["b"]}, {"improper": [_A, "a"]}]]),
        ([3, 4], [{"atom": "+"}, "a", "b", {"atom": "#"}],
         [[3, 4], [{"improper": ["b"]}, {"improper": [_A, "a"]}]]),
        ([1], ["a", {"atom": "#"}], [[1], [["a"], _A]]),
        ([1, 2, 3], [{"atom": ""}, "saya", {"atom": "+"}],
         [[1, 2, 3], [[{"atom": ""}, "saya", _A], []]]),
    ],
    # t_restore_topic 209-228: (key, topic words)
    "restore_topic": [
        ([[2, 3], [["a", "b"], ["x", "y"]]], ["x", "a", "b", "y"]),
        ([[3, 4], [["b", "y"], ["x", "a"]]], ["x", "a", "b", "y"]),
        ([[3, 5], [["b"], ["x", "a", "y"]]], ["x", "a", "b", "y"]),
    ],
}

# apps/emqx_retainer/test/emqx_retainer_SUITE.erl: retained stores and what a subscriber gets.
# Each case: steps of ["store", topic, expiry_ms] / ["delete", topic] / ["clean"] /
# ["match", [filters], now_ms, expected message count over all filters].
RETAINER_CASES = {
    # t_store_and_clean 124-153 (an empty retained payload deletes: emqx_retainer.erl)
    "store_and_clean": [["store", "retained", 0], ["match", ["retained"], 1, 1],
                        ["delete", "retained"], ["match", ["retained"], 1, 0],
                        ["store", "retained", 0], ["clean"], ["match", ["retained"], 1, 0]],
    # t_wildcard_subscription 203-240
    "wildcard_subscription": [
        ["store", "retained/0", 0], ["store", "retained/1", 0], ["store", "retained/a/b/c", 0],
        ["store", "/x/y/z", 0],
        ["match", ["retained/+", "retained/+/b/#", "/+/y/#"], 1, 4]],
    # t_message_expiry 242-296: expiry = publish time (0) + Message-Expiry-Interval * 1000
    # (emqx_retainer.erl:130-141; interval 0 or absent with the default config: never)
    "message_expiry": [
        ["store", "retained/0", 0], ["store", "retained/1", 2000], ["store", "retained/2", 5000],
        ["store", "retained/3", 0], ["store", "$SYS/retained/4", 0],
        ["match", ["retained/+", "$SYS/retained/+"], 1, 5],
        ["match", ["retained/+", "$SYS/retained/+"], 3000, 4]],
}


def main():
    out = {
        "source": "transcribed from fengyangdi/emqx @ 5.0.14 test suites (see make_golden.py)",
        "match": MATCH, "wildcard": WILDCARD, "words": WORDS, "tokens": TOKENS,
        "levels": LEVELS, "join": JOIN, "validate": VALIDATE, "prepend": PREPEND,
        "parse": PARSE, "trie_cases": TRIE_CASES, "make_keys": MAKE_KEYS,
        "make_prefixes": MAKE_PREFIXES, "do_compact": DO_COMPACT,
        "router_cases": ROUTER_CASES, "client_topics": CLIENT_TOPICS,
        "client_wild": CLIENT_WILD, "client_dollar": CLIENT_DOLLAR,
        "bench_patterns": BENCH_PATTERNS, "retainer_index": RETAINER_INDEX,
        "retainer_cases": RETAINER_CASES,
    }
    with open(os.path.join(HERE, "reference_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
