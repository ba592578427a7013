// gm_roctx.h -- roctx ranges (rocprofv3 --marker-trace) around the engine's host phases and
// markers at each kernel launch, when a handle's profiling markers are on (emqxgm_tune
// "roctx" = 1, or EMQXGM_ROCTX=1 in the environment at emqxgm_create).  The roctx library is
// resolved with dlopen on first use, so the engine has no link-time dependency on it (and the
// host sanitizer harness builds without it); when it is missing the calls do nothing.
#pragma once
#include <dlfcn.h>

#include <mutex>

namespace gm {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
};

inline const Roctx& roctx_lib() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                           "libroctx64.so.4", "libroctx64.so"};
    for (const char* n : names) {
      void* l = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      if (!l) continue;
      r.push = (int (*)(const char*))dlsym(l, "roctxRangePushA");
      r.pop = (int (*)())dlsym(l, "roctxRangePop");
      r.mark = (void (*)(const char*))dlsym(l, "roctxMarkA");
      if (r.push && r.pop && r.mark) break;
      r = Roctx{};
    }
  });
  return r;
}

// A range for one scope (no-op unless `on`).
struct RoctxRange {
  bool on;
  RoctxRange(bool enabled, const char* name) : on(enabled && roctx_lib().push) {
    if (on) roctx_lib().push(name);
  }
  ~RoctxRange() {
    if (on) roctx_lib().pop();
  }
};

inline void roctx_mark(bool enabled, const char* name) {
  if (enabled && roctx_lib().mark) roctx_lib().mark(name);
}

}  // namespace gm
