"""CPU: the loopback RCCL's matching rules (tests/loopback/loopback_rccl.cpp), which the GPU test
tests/test_gpu_loopback_rccl.py relies on to run kh_trie_root_sharded's RCCL branch on one GPU:
an unmatched send or receive, a size or type mismatch, or a call outside a group fails the
group the way RCCL refuses it; a peer outside the communicator is an invalid argument.  None of
these reach a HIP call (no device here)."""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OK, INVALID_ARGUMENT, INVALID_USAGE = 0, 4, 5
UINT8, UINT64 = 1, 5


@pytest.fixture(scope="module")
def lb():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "loopback")], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("loopback RCCL not built: " + r.stderr[-300:])
    L = ctypes.CDLL(os.path.join(ROOT, "tests", "loopback", "librccl.so"))
    for f in ("ncclSend", "ncclRecv"):
        getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p]
    L.ncclGetErrorString.restype = ctypes.c_char_p
    return L


def _comms(lb, devs):
    arr = (ctypes.c_void_p * len(devs))()
    dv = (ctypes.c_int * len(devs))(*devs)
    assert lb.ncclCommInitAll(arr, len(devs), dv) == OK
    return arr


def test_repeated_devices_are_accepted(lb):
    c = _comms(lb, [0] * 8)
    assert all(c[i] for i in range(8))


def test_unmatched_send_fails_the_group(lb):
    c = _comms(lb, [0, 0])
    buf = ctypes.create_string_buffer(64)
    assert lb.ncclGroupStart() == OK
    assert lb.ncclSend(buf, 4, UINT8, 1, c[0], None) == OK
    assert lb.ncclGroupEnd() == INVALID_USAGE
    assert b"unmatched" in lb.ncclGetErrorString(INVALID_USAGE)


def test_size_and_type_mismatch_fail(lb):
    c = _comms(lb, [0, 0, 0])
    buf = ctypes.create_string_buffer(64)
    assert lb.ncclGroupStart() == OK
    assert lb.ncclSend(buf, 4, UINT8, 2, c[0], None) == OK
    assert lb.ncclRecv(buf, 5, UINT8, 0, c[2], None) == OK
    assert lb.ncclGroupEnd() == INVALID_USAGE
    assert lb.ncclGroupStart() == OK
    assert lb.ncclSend(buf, 1, UINT64, 2, c[0], None) == OK
    assert lb.ncclRecv(buf, 8, UINT8, 0, c[2], None) == OK
    assert lb.ncclGroupEnd() == INVALID_USAGE


def test_peer_range_and_grouping(lb):
    c = _comms(lb, [0, 0])
    buf = ctypes.create_string_buffer(64)
    assert lb.ncclSend(buf, 4, UINT8, 1, c[0], None) == INVALID_USAGE  # outside a group
    assert lb.ncclGroupStart() == OK
    assert lb.ncclSend(buf, 4, UINT8, 2, c[0], None) == INVALID_ARGUMENT  # no rank 2
    assert lb.ncclGroupEnd() == OK  # (nothing posted)
    assert lb.ncclGroupEnd() == INVALID_USAGE  # no open group


def test_zero_byte_pair_matches_without_a_copy(lb):
    c = _comms(lb, [0, 0])
    buf = ctypes.create_string_buffer(8)
    o, b, g = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lb.loopback_stats(ctypes.byref(o), ctypes.byref(b), ctypes.byref(g))
    assert lb.ncclGroupStart() == OK and lb.ncclGroupStart() == OK  # nested groups end together
    assert lb.ncclSend(buf, 0, UINT8, 1, c[0], None) == OK
    assert lb.ncclRecv(buf, 0, UINT8, 0, c[1], None) == OK
    assert lb.ncclGroupEnd() == OK and lb.ncclGroupEnd() == OK
    o2, b2, g2 = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lb.loopback_stats(ctypes.byref(o2), ctypes.byref(b2), ctypes.byref(g2))
    assert (o2.value, b2.value, g2.value) == (o.value, b.value, g.value + 1)
