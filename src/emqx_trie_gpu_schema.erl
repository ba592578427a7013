%%--------------------------------------------------------------------
%% emqx_trie_gpu_schema -- broker.perf.gpu_match, beside broker.perf.route_lock_type and
%% broker.perf.trie_compaction (apps/emqx/src/emqx_schema.erl:1259-1273).  A maintainer adds
%% {"gpu_match", sc(ref(emqx_trie_gpu_schema, "gpu_match"), #{})} to fields("broker_perf").
%%
%% How each field reaches the engine (include/emqx_gpumatch.h):
%%   enable              -> whether emqx_trie_gpu answers emqx_trie:match/1 at all
%%   devices             -> one engine per device (emqxgm_cfg.device), each holding the whole
%%                          index; windows go round robin to the engines (emqxgm_async_create)
%%   batch_max           -> emqxgm_async_cfg.window_topics = emqxgm_cfg.batch_max
%%                          (window_bytes = 64 x batch_max)
%%   batch_window_us     -> emqxgm_async_cfg.window_us: a window is submitted at most this long
%%                          after its first topic
%%   max_levels          -> emqxgm_async_cfg.max_levels: deeper topics take emqx_trie:match/1
%%                          (the zone's mqtt.max_topic_levels, emqx_schema.erl:405-412)
%%   delta_commit        -> emqxgm_tune(h, "delta_commit", never 0 | small 1 | always 2)
%%   bg_build            -> emqxgm_tune(h, "bg_build"): full builds of registries of at least this
%%                          many filters run in the background while commits patch the index
%%   publish             -> a publish_async layer (EMQXGM_ASYNC_PUBLISH) for emqx_trie_gpu:route/2
%%   spin_us             -> emqxgm_tune(h, "spin_us"): a completer thread polls a window's pass
%%                          this long before it blocks (0: block at once -- no core taken from the
%%                          schedulers; ADVICE r04)
%%   report_threads      -> emqxgm_async_cfg.deliver_threads: a window's calls are answered (terms,
%%                          enif_send) by up to this many threads, not by one completer per GPU
%%   snapshot_dir        -> emqxgm_snapshot_save at the mirror's shutdown, emqxgm_snapshot_load at
%%                          its next start (no full build; the resync commits the difference)
%%   timeout_ms          -> how long a publisher waits for the device before it cancels and takes
%%                          the reference's path (r06: 500, was 5000)
%%   fail_threshold      -> emqxgm_async_cfg.fail_threshold: that many timed-out calls or failed
%%                          windows in a row mark the engines stale, so every later call is refused
%%                          at once until the mirror's repair (include/emqx_gpumatch.h "Health")
%%   eager_windows       -> emqxgm_async_cfg.flags EMQXGM_ASYNC_EAGER: a window is submitted as
%%                          soon as a pipe is free instead of batch_window_us after its first call
%%                          (an idle broker answers in one pass; a loaded one still batches)
%%   adaptive_below_rate -> publishes per second under which the reference path answers (its
%%                          ~22 us on the publisher's core beats the device's window at idle);
%%                          0 = always the device (emqx_trie_gpu "Load-adaptive choice")
%%   resync_interval_ms  -> period of emqx_trie_gpu_sync's full resync (emqxgm_route_sync_*);
%%                          default 0 (none) on a core node, whose table events all arrive, and
%%                          30000 on a replicant
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
        {"delta_commit", hoconsc:mk(hoconsc:enum([never, small, always]), #{default => small})},
        {"bg_build", hoconsc:mk(non_neg_integer(), #{default => 16384})},
        {"publish", hoconsc:mk(boolean(), #{default => true})},
        {"spin_us", hoconsc:mk(range(0, 1000000), #{default => 0})},
        {"report_threads", hoconsc:mk(range(0, 64), #{default => 8})},
        {"snapshot_dir", hoconsc:mk(string(), #{required => false})},
        {"timeout_ms", hoconsc:mk(range(1, 600000), #{default => 500})},
        {"fail_threshold", hoconsc:mk(range(0, 1000000), #{default => 3})},
        {"eager_windows", hoconsc:mk(boolean(), #{default => true})},
        {"adaptive_below_rate", hoconsc:mk(non_neg_integer(), #{default => 0})},
        {"resync_interval_ms", hoconsc:mk(range(0, 86400000), #{required => false})}
    ].
