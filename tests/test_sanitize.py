"""ASan/UBSan: the CPU oracle (oracle/khipu_oracle.cc, oracle/batch_root.cc)
and the host replay of the device per-thread code (tests/emu: trie_ops.h, keccak.h,
nodedata.h, synth.h) built with -fsanitize=address,undefined into one driver
(tests/sanitize/driver.cc) and run over random, deep-prefix, variable-length and
malformed inputs, with the roots cross-checked.  The HIP host half of libkhst.so needs
the HIP runtime and a GPU, so it is exercised by the -m gpu suite instead."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(HERE, "sanitize")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sanitized_oracle_and_replay():
    subprocess.check_call(["make", "-s", "-C", SAN])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(SAN, "san_driver")], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "all checks clean" in r.stdout
