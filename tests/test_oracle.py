"""The oracle, pinned: in-tree known answers of the reference, FIPS SHA3 cross-check
of the permutation, the RLP / hex-prefix byte contract, and
the mainnet genesis state root + block hash (GenesisDataLoader.scala:139-165,
EtcHandshake.scala:52)."""
import hashlib
import json
import os
import random

import pytest

from khipu_amd import codec

HERE = os.path.dirname(os.path.abspath(__file__))
GENESIS_ROOT = "d7f8974fb5ac78d9ac099b9ad5018bedc2ce0a72dad1827a1709da30580f0544"
GENESIS_BLOCK_HASH = "d4e56740f876aef8c010b86a40d5f56745a118d0906a34e69aec8c0db1cb8fa3"


def test_kec256_known_answers(oracle):
    assert oracle.kec256(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert oracle.kec256(b"\x80") == codec.EMPTY_TRIE_HASH
    assert oracle.kec256(b"\xc0") == codec.EMPTY_LIST_HASH


@pytest.mark.parametrize("L", [0, 1, 7, 8, 55, 56, 134, 135, 136, 137, 271, 272, 273, 407, 408, 1000])
def test_permutation_vs_fips_sha3(oracle, L):
    """Same Keccak-f[1600] and rate as FIPS SHA3-256; only the domain byte differs."""
    m = bytes(random.Random(L).getrandbits(8) for _ in range(L))
    assert oracle.keccak256_pad(m, 0x06) == hashlib.sha3_256(m).digest()
    assert oracle.keccak256_pad(m, 0x01) == oracle.kec256(m)


def test_rlp_contract(oracle):
    # RLP.scala:141-150, 157-169
    assert oracle.rlp_str(b"") == b"\x80"
    assert oracle.rlp_str(b"\x00") == b"\x00"
    assert oracle.rlp_str(b"\x7f") == b"\x7f"
    assert oracle.rlp_str(b"\x80") == b"\x81\x80"
    assert oracle.rlp_str(b"a" * 55)[:1] == b"\xb7"
    assert oracle.rlp_str(b"a" * 56)[:2] == b"\xb8\x38"
    assert oracle.rlp_str(b"a" * 255)[:2] == b"\xb8\xff"
    assert oracle.rlp_str(b"a" * 256)[:3] == b"\xb9\x01\x00"
    assert oracle.rlp_list(b"") == b"\xc0"
    assert oracle.rlp_list(b"a" * 55)[:1] == b"\xf7"
    assert oracle.rlp_list(b"a" * 56)[:2] == b"\xf8\x38"
    assert oracle.rlp_list(b"a" * 1024)[:3] == b"\xf9\x04\x00"
    for b in [b"", b"\x01", b"\x80", b"x" * 55, b"x" * 56, b"x" * 300]:
        assert codec.rlp_str(b) == oracle.rlp_str(b)


def test_hex_prefix(oracle):
    # HexPrefix.scala:11-21: flag nibble 2*leaf + odd, a 0 pad nibble when even
    assert oracle.hp_encode(b"", True) == b"\x20"
    assert oracle.hp_encode(b"", False) == b"\x00"
    assert oracle.hp_encode(b"\x0a", True) == b"\x3a"
    assert oracle.hp_encode(b"\x0a", False) == b"\x1a"
    assert oracle.hp_encode(b"\x01\x02", True) == b"\x20\x12"
    assert oracle.hp_encode(b"\x01\x02\x03", False) == b"\x11\x23"
    # one-byte HP is emitted raw inside a node (RLP.scala:142-143)
    assert oracle.rlp_str(oracle.hp_encode(b"\x0a", True)) == b"\x3a"


def test_storage_value_double_wrap(oracle):
    # value RLP(trimmed int) wrapped again as a string in the leaf
    assert codec.storage_value_rlp(1) == b"\x01"
    assert oracle.rlp_str(codec.storage_value_rlp(1)) == b"\x01"
    assert oracle.rlp_str(codec.storage_value_rlp(0x80)) == b"\x82\x81\x80"
    assert len(oracle.rlp_str(codec.storage_value_rlp(2 ** 256 - 1))) == 34


def _genesis(oracle):
    t = oracle.Trie()
    with open(os.path.join(HERE, "golden", "genesis_alloc.txt")) as f:
        for line in f:
            a, b = line.split()
            # GenesisDataLoader.scala:141-146: fresh trie per account, put(kec256(addr)), persist
            t.reopen()
            t.put(oracle.kec256(bytes.fromhex(a)), codec.account_rlp(0, int(b)))
            t.persist()
    return t.root_hash()


def test_genesis_state_root_and_block_hash(oracle):
    root = _genesis(oracle)
    assert root.hex() == GENESIS_ROOT
    with open(os.path.join(HERE, "golden", "genesis_header.json")) as f:
        h = json.load(f)

    def hx(s):
        return bytes.fromhex(s[2:] if s.startswith("0x") else s)

    R = codec.rlp_str
    U = codec.uint_bytes
    # BlockHeader RLP (PV62.scala:116-122), fields from GenesisDataLoader.scala:149-165
    header = codec.rlp_list(
        R(hx(h["parentHash"])), R(hx(h["ommersHash"])), R(hx(h["coinbase"])), R(root),
        R(codec.EMPTY_TRIE_HASH), R(codec.EMPTY_TRIE_HASH), R(b"\0" * 256),
        R(U(int(h["difficulty"], 16))), R(U(0)), R(U(int(h["gasLimit"], 16))), R(U(0)),
        R(U(int(h["timestamp"], 16))), R(hx(h["extraData"])), R(hx(h["mixHash"])), R(hx(h["nonce"])))
    assert oracle.kec256(header).hex() == GENESIS_BLOCK_HASH


def test_sequential_modes_agree(oracle):
    """TrieAccounts.flush pattern (one instance) == GenesisDataLoader pattern (instance per put)."""
    r = random.Random(1)
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(300)]
    vals = [codec.account_rlp(i, i * 7) for i in range(300)]
    assert oracle.seq_root(keys, vals, mode=0) == oracle.seq_root(keys, vals, mode=1)


def test_remove_restores_root(oracle):
    r = random.Random(2)
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(200)]
    vals = [codec.storage_value_rlp(i + 1) for i in range(200)]
    full = oracle.seq_root(keys, vals)
    extra = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(50)]
    xvals = [codec.storage_value_rlp(1000 + i) for i in range(50)]
    # put 250 keys, then remove the 50 extra ones (fix() collapses, MerklePatriciaTrie.scala:430-477)
    got = oracle.seq_root(keys + extra + extra, vals + xvals + [b""] * 50, dels=[0] * 250 + [1] * 50)
    assert got == full
    # deleting everything gives the empty root
    assert oracle.seq_root(keys + keys, vals + [b""] * 200, dels=[0] * 200 + [1] * 200) == codec.EMPTY_TRIE_HASH


def test_get_and_reachable(oracle):
    r = random.Random(3)
    t = oracle.Trie()
    kv = {bytes(r.getrandbits(8) for _ in range(32)): codec.storage_value_rlp(r.randrange(1, 1 << 64))
          for _ in range(100)}
    for k, v in kv.items():
        t.put(k, v)
    for k, v in kv.items():
        assert t.get(k) == v
    assert t.get(b"\0" * 32) is None
    nodes = t.reachable()
    assert t.root_hash() in nodes
    assert all(oracle.kec256(e) == h for h, e in nodes.items())


def test_identical_subtree_quirk(oracle):
    """Reference quirk kept by the restatement: two leaves with the same path suffix and
    value share a node hash; replacing one logs Removed(hash), after which reading the
    other fails (MerklePatriciaTrie.scala:491-516, getNode :536-537).  The GPU path
    builds the canonical trie and is unaffected."""
    def key(b30, b31):
        b = bytearray(32)
        b[30], b[31] = b30, b31
        return bytes(b)
    same = codec.account_rlp(1, 2)
    keys = [key(0x10, 0x05), key(0x20, 0x05), key(0x10, 0x06), key(0x20, 0x07)]
    vals = [same, same, codec.account_rlp(3, 4), codec.account_rlp(5, 6)]
    with pytest.raises(oracle.OracleError):
        oracle.seq_root(keys, vals)


def test_reference_value_branch_quirk(oracle):
    """Pins what the oracle (and khipu) does on a re-put of a key whose leaf has an empty
    remaining path: putInLeafNode with ml == 0 and an empty existingKey builds
    BranchNode.withValueOnly and puts into it (MerklePatriciaTrie.scala:187-199,258-262),
    so the root differs from the canonical trie of the same (key, value) set.  The GPU
    resident commit reproduces it (tests/test_gpu_resident.py::test_value_only_branch_*)."""
    import random
    r = random.Random(63)
    k1 = bytearray(r.getrandbits(8) for _ in range(32))
    k2 = bytearray(k1)
    k2[31] ^= 0x01
    k1, k2 = bytes(k1), bytes(k2)
    t = oracle.Trie()
    t.put(k1, b"\x01")
    t.put(k2, b"\x02")
    t.put(k1, b"\x03")
    canonical = oracle.batch_root([k1, k2], [b"\x03", b"\x02"])
    assert t.root_hash() != canonical
    assert t.get(k1) == b"\x03"
    fresh = oracle.Trie()
    fresh.put(k2, b"\x02")
    fresh.put(k1, b"\x03")
    assert fresh.root_hash() == canonical
