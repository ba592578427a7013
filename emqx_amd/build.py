"""Builds every native artefact in-tree (run: ``python -m emqx_amd.build``).

* ``emqx_amd/libemqx_gpumatch.so`` -- the engine: gfx950 HIP kernels + host builder + C-ABI
  (hipcc --offload-arch=gfx950).  This is the product.
* ``oracle/build/libemqx_ref.so`` -- the C++ restatement of the reference (test checker and
  CPU baseline only; g++).
* ``workloads/libemqx_workload.so`` -- deterministic synthetic workload generator (g++).
* ``tests/host_harness/lib/libasync_load.so`` -- publisher threads driving the engine's concurrent
  entry (tests/host_harness/async_load.cpp; test and bench infrastructure, linked against the
  engine).

Outputs are git-ignored and travel to the GPU box with the tree.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "emqx_amd", "csrc")
ENGINE_SO = os.path.join(ROOT, "emqx_amd", "libemqx_gpumatch.so")
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "libemqx_ref.so")
WORKLOAD_SO = os.path.join(ROOT, "workloads", "libemqx_workload.so")
LOAD_SO = os.path.join(ROOT, "tests", "host_harness", "lib", "libasync_load.so")

ENGINE_SRCS = ["gm_kernels.hip", "gm_engine.cpp", "gm_retain.cpp", "gm_batcher.cpp", "gm_async.cpp"]
ENGINE_DEPS = sorted(set(ENGINE_SRCS) | {f for f in os.listdir(CSRC) if f.endswith((".h", ".inc"))})


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _stale(out: str, deps) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("build failed: " + " ".join(cmd))
    return r.stdout


def build_engine(force: bool = False) -> str:
    deps = [os.path.join(CSRC, s) for s in ENGINE_DEPS] + [
        os.path.join(ROOT, "include", "emqx_gpumatch.h")]
    if force or _stale(ENGINE_SO, deps):
        _run([_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-Wall", "-Wno-unused-function", "-Wno-unused-result", "-pthread"]
             + [os.path.join(CSRC, s) for s in ENGINE_SRCS] + ["-o", ENGINE_SO])
    return ENGINE_SO


def build_oracle(force: bool = False) -> str:
    src = os.path.join(ROOT, "oracle", "ref_trie.cpp")
    if force or _stale(ORACLE_SO, [src]):
        os.makedirs(os.path.dirname(ORACLE_SO), exist_ok=True)
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-pthread", "-shared", "-Wall", src, "-o",
              ORACLE_SO])
    return ORACLE_SO


def build_workloads(force: bool = False) -> str:
    src = os.path.join(ROOT, "workloads", "gen.cpp")
    if force or _stale(WORKLOAD_SO, [src]):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", src, "-o", WORKLOAD_SO])
    return WORKLOAD_SO


def build_load_harness(force: bool = False) -> str:
    src = os.path.join(ROOT, "tests", "host_harness", "async_load.cpp")
    deps = [src, ENGINE_SO, os.path.join(ROOT, "include", "emqx_gpumatch.h")]
    if force or _stale(LOAD_SO, deps):
        os.makedirs(os.path.dirname(LOAD_SO), exist_ok=True)
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", src,
              "-L", os.path.dirname(ENGINE_SO), "-l:libemqx_gpumatch.so",
              "-Wl,-rpath,$ORIGIN/../../../emqx_amd", "-o", LOAD_SO])
    return LOAD_SO


def build_all(force: bool = False):
    return (build_engine(force), build_oracle(force), build_workloads(force),
            build_load_harness(force))


if __name__ == "__main__":
    for p in build_all(force="--force" in sys.argv):
        print(p)
