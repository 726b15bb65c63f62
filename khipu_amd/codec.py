"""Host-side key/value codecs for the state-root path (pure Python, no GPU).

These serialise what khipu hands to ``MerklePatriciaTrie.put`` as bytes, so
callers of the C-ABI (and the tests) can build inputs the same way the reference
does.  Reference files (under /root/reference/):

* RLP string / list framing: khipu-base/.../rlp/RLP.scala:116-169
* account body RLP[nonce, balance, stateRoot, codeHash]:
  khipu-eth/.../network/p2p/messages/PV63.scala:46-51 (AccountEnc),
  values via rlp.toRLPEncodable(DataWord) (rlp/package.scala:56-57) =
  DataWord.nonZeroLeadingBytes (DataWord.scala:175-188), zero -> empty string
* storage value = rlp.encode(toRLPEncodable(DataWord)) (trie/package.scala:28-32)
* EMPTY_TRIE_HASH / EMPTY_CODE_HASH: domain/Account.scala:13-17
"""

EMPTY_TRIE_HASH = bytes.fromhex("56e81f171bcc55a6ff8345e692c0f86e5b48e01b996cadc001622fb5e363b421")
EMPTY_CODE_HASH = bytes.fromhex("c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470")
EMPTY_LIST_HASH = bytes.fromhex("1dcc4de8dec75d7aab85b567b6ccd41ad312451b948a7413f0a142fd40d49347")


def _len_prefix(n: int, offset: int) -> bytes:
    """RLP.encodeLength (RLP.scala:157-169)."""
    if n < 56:
        return bytes([n + offset])
    be = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([len(be) + offset + 55]) + be


def rlp_str(b: bytes) -> bytes:
    """RLPValue encoding (RLP.scala:141-150): one byte < 0x80 is its own encoding."""
    if len(b) == 1 and b[0] < 0x80:
        return bytes(b)
    return _len_prefix(len(b), 0x80) + bytes(b)


def rlp_list(*items: bytes) -> bytes:
    """RLPList of already-encoded items (RLP.scala:118-139)."""
    payload = b"".join(items)
    return _len_prefix(len(payload), 0xC0) + payload


def uint_bytes(v: int) -> bytes:
    """Minimal big-endian bytes; 0 -> b'' (DataWord.nonZeroLeadingBytes / isZero)."""
    if v < 0:
        raise ValueError("negative")
    return v.to_bytes((v.bit_length() + 7) // 8, "big") if v else b""


def account_rlp(nonce: int, balance: int, state_root: bytes = EMPTY_TRIE_HASH,
                code_hash: bytes = EMPTY_CODE_HASH) -> bytes:
    """Account body bytes, as Account.accountSerializer.toBytes (PV63.scala:46-51)."""
    return rlp_list(rlp_str(uint_bytes(nonce)), rlp_str(uint_bytes(balance)),
                    rlp_str(state_root), rlp_str(code_hash))


def storage_value_rlp(v: int) -> bytes:
    """Storage slot value bytes, as rlpDataWordSerializer.toBytes (trie/package.scala:28-32)."""
    return rlp_str(uint_bytes(v))
