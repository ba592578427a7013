"""broker.perf.gpu_match (emqx_amd/config.py, src/emqx_trie_gpu_schema.erl): defaults, range
checks, and the mapping onto emqxgm_cfg / emqxgm_batcher_cfg / emqxgm_tune."""
import pytest

from emqx_amd.config import GpuMatchConfig


def test_defaults_map_onto_the_engine():
    c = GpuMatchConfig.from_map({})
    assert not c.enable and c.devices == [0] and c.max_levels == 128
    assert c.engine_kwargs() == [{"device": 0, "batch_max": 65536}]
    assert c.async_kwargs() == {"window_topics": 65536, "window_bytes": 64 * 65536,
                                "window_us": 50, "max_levels": 128, "deliver_threads": 8,
                                "fail_threshold": 3, "eager": True}
    assert c.timeout_ms == 500 and c.resync_ms("core") == 0 and c.resync_ms("replicant") == 30000
    assert c.tunes() == {"delta_commit": 1, "bg_build": 16384, "spin_us": 0} and c.publish


def test_values_and_ranges():
    c = GpuMatchConfig.from_map({"enable": True, "devices": [3, 1], "batch_max": 16384,
                                 "batch_window_us": 200, "delta_commit": "always"})
    assert c.engine_kwargs() == [{"device": 3, "batch_max": 16384}, {"device": 1, "batch_max": 16384}]
    assert c.async_kwargs()["window_us"] == 200 and c.tunes()["delta_commit"] == 2
    for bad in ({"batch_max": 0}, {"batch_max": 5 << 20}, {"batch_window_us": 0},
                {"max_levels": 0}, {"devices": []}, {"devices": [-1]}, {"enable": 1},
                {"delta_commit": "sometimes"}, {"batch_size": 3}, {"batch_max": True},
                {"timeout_ms": 0}, {"resync_interval_ms": -1}, {"spin_us": -1},
                {"publish": 1}, {"bg_build": -5}, {"report_threads": 65},
                {"fail_threshold": -1}, {"adaptive_below_rate": -1}, {"eager_windows": 1}):
        with pytest.raises(ValueError):
            GpuMatchConfig.from_map(bad)


def test_erlang_schema_lists_the_same_fields():
    import os
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "src", "emqx_trie_gpu_schema.erl")).read()
    fields = re.findall(r'\{"([a-z_]+)",', src.split("fields(\"gpu_match\") ->")[1])
    assert fields == list(GpuMatchConfig.__dataclass_fields__)


def test_load_adaptive_choice():
    """emqx_trie_gpu's low_load/0 + sample_load/2 (restated in emqx_amd.mirror.LoadAdaptive):
    under the rate the reference path answers, over it the device; 0 = always the device."""
    from emqx_amd.mirror import LoadAdaptive
    now = [0.0]
    la = LoadAdaptive(below_rate=20000, sample_ms=100, clock=lambda: now[0])
    for _ in range(500):   # 500 publishes in 100 ms = 5k/s: under
        la.note()
    now[0] += 100
    la.sample()
    assert la.note() is True
    for _ in range(10000):  # 10k in 100 ms = 100k/s: over
        la.note()
    now[0] += 100
    la.sample()
    assert la.note() is False
    off = LoadAdaptive(below_rate=0, clock=lambda: now[0])
    now[0] += 100
    off.sample()
    assert off.note() is False
