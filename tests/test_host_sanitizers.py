"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer.

The sensor core (data_t codec, shared BPF filter header, chain tracker) and the token-automaton compiler are linked
into one -fsanitize=address,undefined executable (csrc/tests/host_sanitize.cpp) and driven with adversarial inputs;
any sanitizer report aborts it with a non-zero status."""
import os
import shutil
import subprocess

import pytest


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_cores_clean_under_asan_ubsan():
    from chronos import native

    exe = native.build_sanitize_harness()
    # verify_asan_link_order=0: the environment may preload its own (non-sanitizer) library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "host_sanitize ok" in out.stdout
