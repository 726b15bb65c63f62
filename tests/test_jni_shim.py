"""CPU: the JNI shim (jni/khst_jni.c) compiles against include/khst.h and
links against libkhst.so with no undefined symbol, and wraps every host-buffer entry point
the header declares -- so a changed khst.h signature, or a new host entry point without a
JVM binding, fails here.  The image has no JDK: tests/jni_stub/jni.h declares the JNI types
and JNIEnv functions the shim uses (with the JDK's signatures)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "jni", "khst_jni.c")
HEADER = os.path.join(ROOT, "include", "khst.h")
LIB = os.path.join(ROOT, "khipu_amd", "libkhst.so")

# entry points taking device buffers or a caller-owned context: the JVM uses the _host forms
# (kh_fold_root16 is the host fold kh_trie_root_sharded already applies inside the library)
DEVICE_ONLY = {"kh_trie_open", "kh_trie_open_nodes", "kh_trie_apply", "kh_forest_apply", "kh_block_commit",
               "kh_trie_root_of", "kh_trie_get", "kh_fold_root16"}


def _cc():
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    return cc


def test_shim_compiles_against_the_header(tmp_path):
    out = tmp_path / "khst_jni.o"
    r = subprocess.run([_cc(), "-std=c99", "-Wall", "-Wextra", "-Werror", "-fPIC", "-c",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"),
                        SHIM, "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_shim_links_against_libkhst(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("libkhst.so not built (__graft_entry__.build())")
    out = tmp_path / "libkhst_jni.so"
    r = subprocess.run([_cc(), "-std=c99", "-Wall", "-Werror", "-fPIC", "-shared",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"),
                        SHIM, "-L", os.path.dirname(LIB), "-lkhst", "-Wl,--no-undefined",
                        "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    nm = subprocess.run(["nm", "-D", "--defined-only", str(out)], capture_output=True, text=True)
    exported = set(re.findall(r"\b(Java_khipu_trie_gpu_Khst_\w+)", nm.stdout))
    assert "Java_khipu_trie_gpu_Khst_blockCommit" in exported and len(exported) >= 30, sorted(exported)


def test_every_host_entry_point_has_a_wrapper():
    with open(HEADER) as f:
        hdr = f.read()
    with open(SHIM) as f:
        shim = f.read()
    declared = set(re.findall(r"^(?:int|const char\*)\s+(kh_\w+)\s*\(", hdr, re.M))
    host = {d for d in declared if not d.startswith(("kh_dev_", "kh_ctx_")) and d not in DEVICE_ONLY}
    called = set(re.findall(r"\b(kh_\w+)\s*\(", shim))
    missing = sorted(host - called)
    assert not missing, missing
    # the per-block calls the reference's persist / flush / genesis paths use
    for fn in ("kh_block_commit_host", "kh_trie_emit_nodes", "kh_trie_root_nodes", "kh_trie_open_host",
               "kh_trie_open_nodes_host", "kh_kec256_batch", "kh_trie_usage", "kh_trie_compact", "kh_trie_free"):
        assert fn in called, fn


def test_free_zeroes_the_box_before_freeing():
    """The idempotent free: the Java-side handle is read, zeroed, then freed (a second call
    sees 0 and returns)."""
    with open(SHIM) as f:
        shim = f.read()
    body = shim[shim.index("Java_khipu_trie_gpu_Khst_free("):]
    body = body[:body.index("\n}\n")]
    assert body.index("SetLongArrayRegion") < body.index("kh_trie_free(")
    assert "if (!h) return;" in body


def _driver():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "jni_stub")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return os.path.join(ROOT, "tests", "jni_stub", "jni_driver")


def test_no_critical_regions():
    """a wrapper may wait for the context's mutex and run seconds of GPU work, so no
    JNI critical region may be held across a library call (the stub jni.h no longer declares the
    critical functions, so a use would not compile either)."""
    with open(SHIM) as f:
        code = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    assert "GetPrimitiveArrayCritical" not in code and "ReleasePrimitiveArrayCritical" not in code
    for w in ("trieRootDirect", "trieRootNodesDirect", "openHostDirect", "trieRootShardedDirect"):
        assert "Java_khipu_trie_gpu_Khst_" + w + "(" in code, w


def test_shim_argument_checks_through_a_jnienv():
    """The wrappers run through an in-process JNIEnv (tests/jni_stub/fake_env.c): a heap array or
    a short buffer handed to a *Direct wrapper, and a short root hash, raise
    IllegalArgumentException before any library call; the empty trie needs no device."""
    import json
    if not os.path.exists(LIB):
        pytest.skip("libkhst.so not built (__graft_entry__.build())")
    r = subprocess.run([_driver(), "cpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    got = {d["check"]: d for d in map(json.loads, r.stdout.split("\n")[:-1])}
    for c in ("direct_keys_not_direct", "direct_voff_short", "direct_vals_short", "open_nodes_short_root"):
        assert got[c]["pending"] == 1 and got[c]["exc"] == "java/lang/IllegalArgumentException", got[c]
    empty = "56e81f171bcc55a6ff8345e692c0f86e5b48e01b996cadc001622fb5e363b421"
    assert got["direct_empty"]["root"] == empty and got["array_empty"]["root"] == empty
