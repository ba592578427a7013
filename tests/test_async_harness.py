"""The concurrent publish entry (emqx_amd/csrc/gm_async.cpp: emqxgm_async_*, the NIF's
match_async/3) under ThreadSanitizer and AddressSanitizer + UBSan, on the CPU.

tests/host_harness/async_harness.cpp links gm_async.cpp against a mock engine whose pass is the
oracle's restatement of emqx_trie:match/1 + the route-key lookup (oracle/ref_trie.cpp), with the
engine's pipe contract enforced (-EBUSY beyond EMQXGM_HOST_PIPES tickets, released results
poisoned, waits of random length).  16-64 publisher threads call one topic at a time and cancel
some calls; every reported result must equal the oracle's, every accepted call be reported
exactly once unless cancelled, none after a successful cancel, and the layer must never overrun
a handle's pipes.  TSan uses clang's runtime: GCC 11's libtsan does not intercept
pthread_cond_clockwait (std::condition_variable::wait_for) and reports false double locks."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = os.path.join(ROOT, "tests", "host_harness")
SRCS = [os.path.join(H, "async_harness.cpp"), os.path.join(ROOT, "emqx_amd", "csrc", "gm_async.cpp"),
        os.path.join(ROOT, "oracle", "ref_trie.cpp")]
DEPS = SRCS + [os.path.join(ROOT, "include", "emqx_gpumatch.h")]
CLANG = "/opt/rocm/llvm/bin/clang++"


def _build(name, cxx, flags):
    out = os.path.join(H, "build", name)
    if os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in DEPS):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-pthread", "-DGM_DELIVER_MIN=4"] + flags + SRCS +
                       ["-o", out],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert r.returncode == 0, r.stdout[-4000:]
    return out


def _run(exe, args, env=None):
    r = subprocess.run([exe] + [str(a) for a in args], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0 and "WARNING" not in r.stdout, r.stdout[-6000:]
    last = r.stdout.strip().splitlines()[-1].split()
    assert last[0] == "OK", r.stdout[-2000:]
    accepted, reported, cancelled, busy, too_deep = map(int, last[1:])
    assert accepted > 0 and reported + cancelled == accepted
    return accepted, reported, cancelled, busy, too_deep


@pytest.mark.skipif(not os.path.exists(CLANG), reason="clang++ (ThreadSanitizer runtime) absent")
@pytest.mark.parametrize("seed,threads,handles,window,calls", [
    (1, 16, 2, 64, 2000), (2, 64, 1, 256, 600), (3, 16, 3, 8, 1500), (4, 4, 1, 4096, 3000)])
def test_async_layer_under_tsan(seed, threads, handles, window, calls):
    exe = _build("async_tsan", CLANG, ["-fsanitize=thread"])
    _run(exe, [seed, threads, handles, window, calls], {"TSAN_OPTIONS": "halt_on_error=1"})


@pytest.mark.parametrize("seed,threads,handles,window,calls", [(5, 16, 2, 32, 1500),
                                                               (6, 64, 1, 16, 400)])
def test_async_layer_under_asan(seed, threads, handles, window, calls):
    exe = _build("async_asan", shutil.which("g++") or "g++",
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    _run(exe, [seed, threads, handles, window, calls],
         {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})


@pytest.mark.skipif(not os.path.exists(CLANG), reason="clang++ (ThreadSanitizer runtime) absent")
@pytest.mark.parametrize("seed,threads,handles,window", [(7, 16, 2, 64), (8, 8, 1, 16)])
def test_hung_device_costs_one_timeout_then_refuses(seed, threads, handles, window):
    """Health mode: the device hangs; publishers that time out cancel; after
    fail_threshold timeouts every handle is stale and later calls are refused at once (-ESTALE);
    after the repair calls are answered correctly again."""
    exe = _build("async_tsan", CLANG, ["-fsanitize=thread"])
    _run(exe, [seed, threads, handles, window, 0, 0, "health"], {"TSAN_OPTIONS": "halt_on_error=1"})


@pytest.mark.skipif(not os.path.exists(CLANG), reason="clang++ (ThreadSanitizer runtime) absent")
def test_handle_registry_waits_for_windows_in_flight():
    """emqxgm_handles_* over a real layer: a number released while a window
    submitted before the release is in flight is not reused until that window was reported."""
    exe = _build("async_tsan", CLANG, ["-fsanitize=thread"])
    _run(exe, [9, 1, 1, 64, 0, 0, "handles"], {"TSAN_OPTIONS": "halt_on_error=1"})
