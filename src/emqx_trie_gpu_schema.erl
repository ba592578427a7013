%%--------------------------------------------------------------------
%% emqx_trie_gpu_schema -- broker.perf.gpu_match, beside broker.perf.route_lock_type and
%% broker.perf.trie_compaction (apps/emqx/src/emqx_schema.erl:1259-1273).  A maintainer adds
%% {"gpu_match", sc(ref(emqx_trie_gpu_schema, "gpu_match"), #{})} to fields("broker_perf").
%%
%% How each field reaches the engine (include/emqx_gpumatch.h):
%%   enable          -> whether emqx_trie_gpu answers emqx_trie:match/1 at all
%%   devices         -> emqxgm_cfg.device (the first; one index per node)
%%   batch_max       -> emqxgm_batcher_cfg.window_topics = emqxgm_cfg.batch_max
%%                      (window_bytes = 64 x batch_max)
%%   batch_window_us -> emqxgm_batcher_cfg.window_us
%%   max_levels      -> topics deeper than this take emqx_trie:match/1 (the zone's
%%                      mqtt.max_topic_levels, emqx_schema.erl:405-412, default 128)
%%   delta_commit    -> emqxgm_tune(h, "delta_commit", V)
%% emqx_amd/config.py is the same table for the Python mirror (tests/test_config.py).
%%--------------------------------------------------------------------
-module(emqx_trie_gpu_schema).

-include_lib("typerefl/include/types.hrl").
-include_lib("hocon/include/hoconsc.hrl").

-export([fields/1]).

fields("gpu_match") ->
    [
        {"enable", hoconsc:mk(boolean(), #{default => false})},
        {"devices", hoconsc:mk(hoconsc:array(non_neg_integer()), #{default => [0]})},
        {"batch_max",
            hoconsc:mk(range(1, 4194304), #{default => 65536})},
        {"batch_window_us", hoconsc:mk(range(1, 1000000), #{default => 50})},
        {"max_levels", hoconsc:mk(range(1, 65535), #{default => 128})},
        {"delta_commit", hoconsc:mk(hoconsc:enum([never, small, always]), #{default => small})}
    ].
