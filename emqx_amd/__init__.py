"""emqx_amd -- MI355X-native batched MQTT topic matching behind the EMQX routing API.

The product is ``libemqx_gpumatch.so`` (gfx950 HIP kernels + host index builder + C-ABI,
``include/emqx_gpumatch.h``).  This package is the host-side mirror of the reference's
``emqx_trie`` / ``emqx_router`` / ``emqx_broker`` (publish fan-out) modules over that library:

    from emqx_amd import Trie, Router, Broker, Engine
"""
from .broker import Broker  # noqa: F401
from .engine import NONE, AsyncMatcher, AsyncResult, Batcher, DeviceResult, Engine, EngineError, MatchResult, PublishResult, Window  # noqa: F401
from .router import Router, SessionRouter  # noqa: F401
from .retainer import Retainer  # noqa: F401
from .rules import TopicRules  # noqa: F401
from .trie import Trie  # noqa: F401

__all__ = ["Engine", "EngineError", "MatchResult", "DeviceResult", "PublishResult", "Trie",
           "Router", "SessionRouter", "Broker", "TopicRules", "Retainer", "Batcher", "Window",
           "AsyncMatcher", "AsyncResult", "NONE"]
