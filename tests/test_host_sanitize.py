"""The engine's host code (registry, trie model, delta commits, exact-table and fan-out
bookkeeping, epochs) under AddressSanitizer + UndefinedBehaviorSanitizer, on the CPU.

tests/host_harness/harness.cpp includes emqx_amd/csrc/gm_engine.cpp and runs it against a fake
HIP runtime (device memory = host memory, k_patch applied on the CPU): random subscribe /
unsubscribe / route-key / route / subscriber churn on a delta-committing engine and a rebuilding
one, every commit's device tables walked on the CPU as k_walk walks them and compared with the
oracle (oracle/ref_trie.cpp, restating emqx_trie.erl:113-144, 242-260, 282-348), the exact table
probed as k_exact probes it, every fan-out entry compared with the registry; halfway through,
the delta-committing engine is saved to a snapshot and replaced by a fresh engine loaded from it.
Any sanitizer report or mismatch fails the run.

tests/host_harness/bg_harness.cpp (r05) is the subscribe-then-publish visibility check while full
builds run in the background: single subscribes / unsubscribes through
emqxgm_route_set_batch(.., EMQXGM_SET_COMMIT) during a bulk commit's build, during a build the
tables' load started, and a batch too large for a delta during a build -- each checked on the
epoch readers have right after the call (the reference's subscriber has its route before SUBACK,
emqx_broker.erl:163-168, emqx_router.erl:124-138) -- under ThreadSanitizer and ASan + UBSan."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = os.path.join(ROOT, "tests", "host_harness")
OUT = os.path.join(H, "build", "harness_asan")
SRCS = [os.path.join(H, "harness.cpp"), os.path.join(H, "fake_hip.cpp"),
        os.path.join(ROOT, "oracle", "ref_trie.cpp")]
DEPS = SRCS + [os.path.join(H, "fakehip", "hip", "hip_runtime.h"), os.path.join(H, "harness_walk.h")] + [
    os.path.join(ROOT, "emqx_amd", "csrc", f) for f in ("gm_engine.cpp", "gm_common.h", "gm_kernels.h")
] + [os.path.join(ROOT, "include", "emqx_gpumatch.h")]


SAN = {"asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                "-fno-omit-frame-pointer"],
       "tsan": ["-fsanitize=thread"]}


def _build(main="harness.cpp", san="asan"):
    out = OUT if (main, san) == ("harness.cpp", "asan") else os.path.join(
        H, "build", main.replace(".cpp", "") + "_" + san)
    srcs = [os.path.join(H, main)] + SRCS[1:]
    deps = DEPS + [srcs[0]]
    if os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O1", "-g"] + SAN[san] + [
        "-Wno-subobject-linkage", "-I", os.path.join(H, "fakehip")] + srcs + ["-pthread", "-o", out]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert r.returncode == 0, r.stdout[-4000:]
    return out


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed,rounds,hash_bits,keyed", [(11, 25, 0, 1), (12, 12, 3, 1),
                                                         (13, 20, 0, 2), (14, 10, 3, 2)])
def test_engine_host_code_under_asan_ubsan(seed, rounds, hash_bits, keyed, tmp_path):
    """keyed 2: every eligible trie node token-keyed (gm_common.h edge_home), so the CPU walk
    and the delta commits run over keyed placements."""
    exe = _build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, str(seed), str(rounds), str(hash_bits), str(tmp_path), str(keyed)],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env,
                       timeout=540)
    assert r.returncode == 0, r.stdout[-6000:]
    last = r.stdout.strip().splitlines()[-1].split()
    assert last[0] == "OK", r.stdout[-2000:]
    commits, delta, full, checks = map(int, last[1:])
    assert commits > 0 and checks > 0  # (the counts are the restored engine's: it replaced the first)
    if hash_bits == 0:
        assert delta > 0 and full > 0  # both commit paths ran


@pytest.mark.timeout(900)
@pytest.mark.parametrize("san,seed,delta_max", [("tsan", 21, 300), ("asan", 22, 400)])
def test_subscribe_visible_during_background_builds(san, seed, delta_max):
    """Each single subscribe / unsubscribe committed with EMQXGM_SET_COMMIT is visible on the
    next match while a full build runs in the background; the bulk that started the build is
    visible exactly from its install on; a batch the current tables cannot take waits for the
    install and is visible after it.  The printed latency is the single subscribes' during
    builds (fake HIP runtime: host-side cost only).  delta_max: the changes a delta takes
    (tune "delta_max"; 0 = the default bound, 4096 at these sizes) -- small under TSan to keep
    the bulk small."""
    exe = _build("bg_harness.cpp", san)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([exe, str(seed), str(delta_max)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, env=env, timeout=840)
    assert r.returncode == 0, r.stdout[-6000:]
    last = r.stdout.strip().splitlines()[-1].split()
    assert last[0] == "OK", r.stdout[-2000:]
    checks, builds, waits = map(int, last[1:4])
    assert checks > 500 and builds >= 3 and waits >= 1
