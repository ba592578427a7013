"""``broker.perf.gpu_match`` -- the configuration surface of the device match path, beside the
reference's ``broker.perf.route_lock_type`` / ``trie_compaction`` (apps/emqx/src/emqx_schema.erl:
1259-1273; SURVEY 5 "Config / flags"), and how each field reaches the engine.  The same table as
``src/emqx_trie_gpu_schema.erl`` (the HOCON fields a maintainer adds to ``fields("broker_perf")``):

================== ================== ======================================================
field              default            engine
================== ================== ======================================================
enable             false              the device answers ``emqx_trie:match/1`` at all
devices            [0]                one engine per device (``emqxgm_cfg.device``), each with
                                      the whole index; windows round robin over them
                                      (``emqxgm_async_create``)
batch_max          65536              ``emqxgm_cfg.batch_max`` = ``emqxgm_async_cfg.window_topics``
                                      (``window_bytes`` = 64 x batch_max)
batch_window_us    50                 ``emqxgm_async_cfg.window_us``
max_levels         128                ``emqxgm_async_cfg.max_levels``: deeper topics take the
                                      reference's ``emqx_trie:match/1`` (``mqtt.max_topic_levels``,
                                      emqx_schema.erl:405-412)
delta_commit       small              ``emqxgm_tune("delta_commit", never 0 / small 1 / always 2)``
bg_build           16384              ``emqxgm_tune("bg_build")``: full builds of registries of at
                                      least this many filters run in the background (r05)
publish            true               a publish layer (``EMQXGM_ASYNC_PUBLISH``) beside the match one
spin_us            0                  ``emqxgm_tune("spin_us")``: completer threads block at once
report_threads     8                  ``emqxgm_async_cfg.deliver_threads``: a window's calls are
                                      answered by up to this many threads (the NIF's per-call
                                      terms and enif_send), not by one completer per GPU
snapshot_dir       (none)             ``emqxgm_snapshot_save`` at the mirror's shutdown,
                                      ``emqxgm_snapshot_load`` at its next start (no full build)
timeout_ms         500                a publisher's wait before it cancels and takes the
                                      reference's match (src/emqx_trie_gpu.erl)
fail_threshold     3                  ``emqxgm_async_cfg.fail_threshold``: that many timed-out
                                      calls or failed windows in a row mark the engines stale
                                      (every later call refused at once until the mirror's
                                      repair; include/emqx_gpumatch.h "Health")
eager_windows      true               ``EMQXGM_ASYNC_EAGER``: a window goes to the device as soon
                                      as a pipe is free, not batch_window_us after its first call
                                      (an idle broker answers in one pass; a loaded one batches)
adaptive_below_rate 0                 publishes/s under which the reference path answers (its
                                      ~22 us on the publisher's core beats the device's window
                                      at idle); 0 = always the device (``LoadAdaptive``)
resync_interval_ms (role)             period of the mirror's full resync (``emqxgm_route_sync_begin``
                                      / ``_end``): none (0) on a core node, 30000 on a replicant
================== ================== ======================================================
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Mapping, Optional

DELTA_COMMIT = {"never": 0, "small": 1, "always": 2}


@dataclass(frozen=True)
class GpuMatchConfig:
    enable: bool = False
    devices: List[int] = field(default_factory=lambda: [0])
    batch_max: int = 65536
    batch_window_us: int = 50
    max_levels: int = 128
    delta_commit: str = "small"
    bg_build: int = 16384
    publish: bool = True
    spin_us: int = 0
    report_threads: int = 8
    snapshot_dir: Optional[str] = None
    timeout_ms: int = 500
    fail_threshold: int = 3
    eager_windows: bool = True
    adaptive_below_rate: int = 0
    resync_interval_ms: Optional[int] = None  # None: by the node's mria role

    @classmethod
    def from_map(cls, conf: Mapping) -> "GpuMatchConfig":
        """A ``broker.perf.gpu_match`` map (HOCON keys) -> a checked config; ValueError on a
        value the schema's ranges reject (emqx_trie_gpu_schema.erl)."""
        known = {f for f in cls.__dataclass_fields__}
        extra = set(conf) - known
        if extra:
            raise ValueError(f"unknown broker.perf.gpu_match fields: {sorted(extra)}")
        c = cls(**{k: (list(v) if k == "devices" else v) for k, v in conf.items()})
        c.check()
        return c

    def check(self) -> None:
        def rng(name, v, lo, hi):
            if not isinstance(v, int) or isinstance(v, bool) or not lo <= v <= hi:
                raise ValueError(f"broker.perf.gpu_match.{name} = {v!r}: expected {lo}..{hi}")
        if not isinstance(self.enable, bool):
            raise ValueError("broker.perf.gpu_match.enable: expected a boolean")
        if not self.devices:
            raise ValueError("broker.perf.gpu_match.devices: at least one device")
        for d in self.devices:
            rng("devices[]", d, 0, 1023)
        rng("batch_max", self.batch_max, 1, 4 << 20)
        rng("batch_window_us", self.batch_window_us, 1, 1_000_000)
        rng("max_levels", self.max_levels, 1, 65535)
        rng("timeout_ms", self.timeout_ms, 1, 600_000)
        rng("fail_threshold", self.fail_threshold, 0, 1_000_000)
        rng("adaptive_below_rate", self.adaptive_below_rate, 0, 1 << 40)
        if self.resync_interval_ms is not None:
            rng("resync_interval_ms", self.resync_interval_ms, 0, 86_400_000)
        rng("bg_build", self.bg_build, 0, 1 << 62)
        rng("report_threads", self.report_threads, 0, 64)
        rng("spin_us", self.spin_us, 0, 1_000_000)
        if not isinstance(self.publish, bool):
            raise ValueError("broker.perf.gpu_match.publish: expected a boolean")
        if not isinstance(self.eager_windows, bool):
            raise ValueError("broker.perf.gpu_match.eager_windows: expected a boolean")
        if self.delta_commit not in DELTA_COMMIT:
            raise ValueError(f"broker.perf.gpu_match.delta_commit: one of {sorted(DELTA_COMMIT)}")

    def engine_kwargs(self) -> List[Dict[str, int]]:
        """``emqxgm_cfg`` fields (emqx_amd.Engine keywords), one engine per device."""
        return [{"device": d, "batch_max": self.batch_max} for d in self.devices]

    def async_kwargs(self) -> Dict[str, int]:
        """``emqxgm_async_cfg`` fields (emqx_amd.AsyncMatcher keywords)."""
        return {"window_topics": self.batch_max, "window_bytes": 64 * self.batch_max,
                "window_us": self.batch_window_us, "max_levels": self.max_levels,
                "deliver_threads": self.report_threads, "fail_threshold": self.fail_threshold,
                "eager": self.eager_windows}

    def batcher_kwargs(self) -> Dict[str, int]:
        """``emqxgm_batcher_cfg`` fields (emqx_amd.Batcher keywords: the single-driver batcher
        core the bench's window sweep uses)."""
        return {"window_topics": self.batch_max, "window_bytes": 64 * self.batch_max,
                "window_us": self.batch_window_us}

    def tunes(self) -> Dict[str, int]:
        """``emqxgm_tune`` knobs."""
        return {"delta_commit": DELTA_COMMIT[self.delta_commit], "bg_build": self.bg_build,
                "spin_us": self.spin_us}

    def resync_ms(self, role: str = "core") -> int:
        """The mirror's resync period on a node of this mria role (0: none)."""
        if self.resync_interval_ms is not None:
            return self.resync_interval_ms
        return 30000 if role == "replicant" else 0

    def open(self, callback):
        """The engines and their concurrent entry as the NIF's open/6 makes them
        (emqx_trie_gpu_sync:init/1): one Engine per device, tuned, and an AsyncMatcher over them
        reporting completed windows to `callback`."""
        from .engine import AsyncMatcher, Engine
        engines = [Engine(**kw) for kw in self.engine_kwargs()]
        for eng in engines:
            for k, v in self.tunes().items():
                eng.tune(k, v)
        return engines, AsyncMatcher(engines, callback, **self.async_kwargs())
