"""The NIF (c_src/emqx_trie_gpu_nif.c) compiles: no Erlang runtime exists in this image, so it is
checked with gcc -fsyntax-only against tests/nif_stub/erl_nif.h (the erl_nif declarations it
uses, OTP's signatures) and include/emqx_gpumatch.h.  Warnings are errors."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_nif_compiles_against_erl_nif_declarations():
    r = subprocess.run(["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(ROOT, "tests", "nif_stub"),
                        "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "c_src", "emqx_trie_gpu_nif.c")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
