// gm_internal.h -- entry points of the engine (gm_engine.cpp) that only the library's own layers
// use (the concurrent publish entry, gm_async.cpp); not part of the C-ABI.  The async layer's
// host harness (tests/host_harness/async_harness.cpp) defines them over its mock engine.
#pragma once
#include <stdint.h>

#include "../../include/emqx_gpumatch.h"

// emqxgm_match_batch_submit_filters for a window whose offsets the caller built increasing
// (no O(n) check)
int gm_submit_window(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets, uint32_t n,
                     uint64_t* ticket);
// every host pipe of h sized for windows of n topics / nb bytes (no reallocation later)
int gm_reserve_windows(emqxgm_t* h, uint32_t n, uint64_t nb);
// whether h's index is stale (include/emqx_gpumatch.h "Health"): one atomic load, per call
int gm_stale(emqxgm_t* h);
