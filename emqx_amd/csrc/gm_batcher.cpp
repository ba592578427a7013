// gm_batcher.cpp -- the NIF batcher core (include/emqx_gpumatch.h "NIF batcher core"), a layer
// over the engine's public C-ABI: publish topics of concurrent callers are packed into a window
// in pinned host memory, a window is submitted whole through the host pipes
// (emqxgm_match_batch_submit_filters / _wait_filters), and a collected window comes back with every
// pair's filter bytes, gathered on the device.
//
// The reference matches each publish in the publisher's own process
// (emqx_broker:publish/1 -> emqx_router:match_routes/1 -> emqx_trie:match/1,
// apps/emqx/src/emqx_broker.erl:218-232, emqx_router.erl:141-157, emqx_trie.erl:147-169); the
// NIF (c_src/emqx_trie_gpu_nif.c) hands this core one topic per caller and answers each caller
// from its window's result.
#include <errno.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/emqx_gpumatch.h"

namespace {

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

constexpr uint32_t SLOTS = EMQXGM_HOST_PIPES + 1;  // the open window + the ones in flight

// One window slot: its packed topics (pinned, the H2D source of its pass) and, once collected,
// its result (host copies: the pipe's pinned result buffers are reused HOST_PIPES flushes on).
struct Window {
  uint8_t* bytes = nullptr;  // pinned [window_bytes]
  uint32_t* off = nullptr;   // pinned [window_topics + 1]
  std::vector<uint64_t> tag;
  uint32_t n = 0;
  uint64_t first_ns = 0;
  uint64_t id = 0, ticket = 0;
  int state = 0;  // 0 open / free, 1 in flight, 2 collected, 3 being collected
  uint64_t flush_ns = 0, done_ns = 0;
  // the collected result: tags copied (the slot's tag list is refilled when it reopens), the
  // rest read in place from the host pipe's pinned buffers, valid until EMQXGM_HOST_PIPES more
  // windows are flushed (the pipe's next ticket)
  std::vector<uint64_t> r_tag;
  emqxgm_batch_out r{};
  const uint32_t* r_foff = nullptr;
  const uint8_t* r_fb = nullptr;
};

}  // namespace

struct emqxgm_batcher {
  emqxgm_t* h = nullptr;
  emqxgm_batcher_cfg cfg{};
  Window w[SLOTS];
  uint32_t open = 0;      // slot of the open window
  uint64_t next_id = 1;
  uint32_t in_flight = 0;
  std::mutex mu;
};

extern "C" {

int emqxgm_batcher_create(emqxgm_t* h, const emqxgm_batcher_cfg* cfg, emqxgm_batcher_t** out) {
  if (!h || !out) return -EINVAL;
  *out = nullptr;
  emqxgm_batcher* b = new (std::nothrow) emqxgm_batcher();
  if (!b) return -ENOMEM;
  b->h = h;
  if (cfg) b->cfg = *cfg;
  if (!b->cfg.window_topics) b->cfg.window_topics = 65536;
  if (!b->cfg.window_bytes) b->cfg.window_bytes = 64u * b->cfg.window_topics;
  if (!b->cfg.window_us) b->cfg.window_us = 50;
  for (Window& w : b->w) {
    w.bytes = (uint8_t*)emqxgm_host_alloc(h, b->cfg.window_bytes);
    w.off = (uint32_t*)emqxgm_host_alloc(h, ((uint64_t)b->cfg.window_topics + 1) * 4);
    if (!w.bytes || !w.off) {
      emqxgm_batcher_destroy(b);
      return -ENOMEM;
    }
    w.off[0] = 0;
    w.tag.reserve(b->cfg.window_topics);
  }
  *out = b;
  return 0;
}

void emqxgm_batcher_destroy(emqxgm_batcher_t* b) {
  if (!b) return;
  for (Window& w : b->w) {
    if (w.state == 1) {  // a pass still reads the window's pinned bytes: complete it first
      emqxgm_batch_out o;
      (void)emqxgm_match_batch_wait(b->h, w.ticket, &o);
    }
    emqxgm_host_free(b->h, w.bytes);
    emqxgm_host_free(b->h, w.off);
  }
  delete b;
}

int emqxgm_batcher_add(emqxgm_batcher_t* b, const uint8_t* topic, uint32_t len, uint64_t tag,
                       uint32_t* slot) {
  if (!b || (!topic && len)) return -EINVAL;
  std::lock_guard<std::mutex> g(b->mu);
  if (len > b->cfg.window_bytes) return -E2BIG;
  Window& w = b->w[b->open];
  const uint32_t used = w.off[w.n];
  if (w.n >= b->cfg.window_topics || len > b->cfg.window_bytes - used) return -ENOSPC;
  if (w.n == 0) w.first_ns = mono_ns();
  if (len) memcpy(w.bytes + used, topic, len);
  w.off[w.n + 1] = used + len;
  w.tag.push_back(tag);
  if (slot) *slot = w.n;
  w.n += 1;
  // full: no room for another topic (the next one may be as long as the longest seen so far;
  // the caller retries a -ENOSPC add after a flush anyway)
  return (w.n == b->cfg.window_topics || w.off[w.n] == b->cfg.window_bytes) ? 1 : 0;
}

int emqxgm_batcher_add_many(emqxgm_batcher_t* b, const uint8_t* bytes, const uint32_t* offsets,
                            uint32_t n, uint64_t tag0) {
  if (!b || (n && (!offsets || (!bytes && offsets[n] != offsets[0])))) return -EINVAL;
  std::lock_guard<std::mutex> g(b->mu);
  Window& w = b->w[b->open];
  // the run of topics that fits, then one copy of its bytes (a copy per topic cost ~15 ns each:
  // ~1 ms per 64k-topic window, r03)
  const uint32_t used = w.off[w.n];
  const uint32_t room_t = b->cfg.window_topics - w.n;
  uint32_t k = 0;
  int err = 0;
  for (; k < n && k < room_t; ++k) {
    if (offsets[k + 1] < offsets[k]) {
      err = -EINVAL;
      break;
    }
    const uint32_t len = offsets[k + 1] - offsets[k];
    if (len > b->cfg.window_bytes) {
      err = -E2BIG;
      break;
    }
    if ((uint64_t)offsets[k + 1] - offsets[0] > (uint64_t)b->cfg.window_bytes - used) break;
  }
  if (k == 0) return err;
  if (w.n == 0) w.first_ns = mono_ns();
  const uint32_t o0 = offsets[0];
  if (offsets[k] != o0) memcpy(w.bytes + used, bytes + o0, offsets[k] - o0);
  for (uint32_t j = 1; j <= k; ++j) w.off[w.n + j] = used + (offsets[j] - o0);
  for (uint32_t j = 0; j < k; ++j) w.tag.push_back(tag0 + j);
  w.n += k;
  return (int)k;
}

int emqxgm_batcher_due(emqxgm_batcher_t* b, uint64_t now_ns) {
  if (!b) return -EINVAL;
  std::lock_guard<std::mutex> g(b->mu);
  const Window& w = b->w[b->open];
  return (w.n > 0 && now_ns >= w.first_ns + 1000ull * b->cfg.window_us) ? 1 : 0;
}

int emqxgm_batcher_flush(emqxgm_batcher_t* b, uint64_t* window) {
  if (!b || !window) return -EINVAL;
  std::lock_guard<std::mutex> g(b->mu);
  *window = 0;
  Window& w = b->w[b->open];
  if (w.n == 0) return 0;
  if (b->in_flight >= EMQXGM_HOST_PIPES) return -EBUSY;
  uint64_t tk = 0;
  // the filter-byte gather and every result copy go behind the pass: one synchronisation at
  // collect (emqxgm_match_batch_wait_filters)
  const int rc = emqxgm_match_batch_submit_filters(b->h, w.bytes, w.off, w.n, &tk);
  if (rc) return rc;
  w.ticket = tk;
  w.id = b->next_id++;
  w.state = 1;
  w.flush_ns = mono_ns();
  b->in_flight += 1;
  *window = w.id;
  // the next open window: a slot not in flight (SLOTS = HOST_PIPES + 1 guarantees one)
  for (uint32_t k = 1; k <= SLOTS; ++k) {
    const uint32_t s = (b->open + k) % SLOTS;
    if (b->w[s].state != 1 && b->w[s].state != 3) {
      b->open = s;
      Window& nw = b->w[s];
      nw.n = 0;
      nw.off[0] = 0;
      nw.tag.clear();
      // a collected window reopened: its old id no longer names a result (-ENOENT)
      nw.state = 0;
      nw.id = 0;
      break;
    }
  }
  return 0;
}

int emqxgm_batcher_collect(emqxgm_batcher_t* b, uint64_t window, emqxgm_window_out* out) {
  if (!b || !out || !window) return -EINVAL;
  std::unique_lock<std::mutex> g(b->mu);
  Window* wp = nullptr;
  for (Window& w : b->w)
    if (w.id == window && w.state != 0) wp = &w;
  if (!wp) return -ENOENT;
  Window& w = *wp;
  if (w.state == 3) return -EBUSY;  // another thread is collecting it right now
  if (w.state == 1) {
    // the stream wait runs without the batcher lock (adds of other threads go on); state 3
    // keeps the slot from being reopened or collected twice meanwhile
    w.state = 3;
    const uint64_t tk = w.ticket;
    g.unlock();
    emqxgm_batch_out r{};
    const uint32_t* foff = nullptr;
    const uint8_t* fb = nullptr;
    // every pair's filter bytes gathered on the device from its copy of the string pool (the
    // host registry per pair costs two random DRAM reads: ~250 ns per cfg3 topic, r03)
    const int rc = emqxgm_match_batch_wait_filters(b->h, tk, &r, &foff, &fb);
    g.lock();
    b->in_flight -= 1;
    if (rc) {
      // the window is gone (its callers are answered some other way): free its slot
      w.state = 0;
      w.id = 0;
      return rc;
    }
    w.r = r;
    w.r_foff = foff;
    w.r_fb = fb;
    w.r_tag = w.tag;
    w.state = 2;
    w.done_ns = mono_ns();
  }
  out->n = w.r.n;
  out->n_pairs = w.r.n_pairs;
  out->tag = w.r_tag.data();
  out->row = w.r.row_ptr;
  out->filter_id = w.r.filter_id;
  out->foff = w.r_foff;
  out->fbytes = w.r_fb;
  out->exact_id = w.r.exact_id;
  out->flush_ns = w.flush_ns;
  out->done_ns = w.done_ns;
  return 0;
}

}  // extern "C"
