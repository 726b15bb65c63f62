"""The storage write-back contract, shared by the GPU tests.

After one block, the engine's delta D (hash -> encoding, kh_trie_emit_nodes) must satisfy,
against the khipu-faithful oracle (oracle/khipu_oracle.cc, MerklePatriciaTrie.scala:491-516
updateNodesToLogs; BlockWorldState.scala:312-330 hands the Updated entries to
NodeStorage.update):

1. every emitted pair is an `Updated` entry of that block's log, with the same bytes;
2. every emitted pair is reachable from the new root of a trie the block touched;
3. every node reachable from a touched trie's new root is in the store or in D (the store
   after the hand-off holds every touched trie whole).

Test infrastructure only.
"""
EMPTY_TRIE_HASH = bytes.fromhex("56e81f171bcc55a6ff8345e692c0f86e5b48e01b996cadc001622fb5e363b421")


def reachable(o):
    """The oracle trie's reachable node set ({} for an empty trie)."""
    return o.reachable() if o.root_hash() != EMPTY_TRIE_HASH else {}


def check_delta(delta, tries, store, what=""):
    """delta: {hash: enc}; tries: the oracle tries the block touched (their logs not yet
    reset); store: {hash: enc} before the hand-off.  Raises AssertionError naming the first
    violation; returns the reachable union (for the caller's store update)."""
    upd, reach = {}, {}
    for o in tries:
        upd.update(o.updated())
        reach.update(reachable(o))
    not_logged = [h.hex() for h, e in delta.items() if upd.get(h) != e]
    assert not not_logged, (what, "emitted but not an Updated entry", len(not_logged), not_logged[:3])
    unreachable = [h.hex() for h, e in delta.items() if reach.get(h) != e]
    assert not unreachable, (what, "emitted but unreachable", len(unreachable), unreachable[:3])
    missing = [h.hex() for h in reach if h not in store and h not in delta]
    assert not missing, (what, "reachable, new, not emitted", len(missing), missing[:3])
    return reach


def settle(tries):
    """persist() + reopen every oracle trie: the next block's log starts empty."""
    for o in tries:
        o.persist().reopen()
