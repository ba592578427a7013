"""The engine's host code (registry, trie model, delta commits, exact-table and fan-out
bookkeeping, epochs) under AddressSanitizer + UndefinedBehaviorSanitizer, on the CPU.

tests/host_harness/harness.cpp includes emqx_amd/csrc/gm_engine.cpp and runs it against a fake
HIP runtime (device memory = host memory, k_patch applied on the CPU): random subscribe /
unsubscribe / route-key / route / subscriber churn on a delta-committing engine and a rebuilding
one, every commit's device tables walked on the CPU as k_walk walks them and compared with the
oracle (oracle/ref_trie.cpp, restating emqx_trie.erl:113-144, 242-260, 282-348), the exact table
probed as k_exact probes it, every fan-out entry compared with the registry; halfway through,
the delta-committing engine is saved to a snapshot and replaced by a fresh engine loaded from it.
Any sanitizer report or mismatch fails the run."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = os.path.join(ROOT, "tests", "host_harness")
OUT = os.path.join(H, "build", "harness_asan")
SRCS = [os.path.join(H, "harness.cpp"), os.path.join(H, "fake_hip.cpp"),
        os.path.join(ROOT, "oracle", "ref_trie.cpp")]
DEPS = SRCS + [os.path.join(H, "fakehip", "hip", "hip_runtime.h")] + [
    os.path.join(ROOT, "emqx_amd", "csrc", f) for f in ("gm_engine.cpp", "gm_common.h", "gm_kernels.h")
] + [os.path.join(ROOT, "include", "emqx_gpumatch.h")]


def _build():
    if os.path.exists(OUT) and all(os.path.getmtime(d) <= os.path.getmtime(OUT) for d in DEPS):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-Wno-subobject-linkage",
           "-I", os.path.join(H, "fakehip")] + SRCS + ["-pthread", "-o", OUT]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert r.returncode == 0, r.stdout[-4000:]
    return OUT


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
