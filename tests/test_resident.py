"""Incremental commit over a resident trie: the host replay of the
device pipeline (tests/emu; same per-element ops as the kh_trie_apply kernels) against
the oracle trie folded put-by-put / remove-by-remove (MerklePatriciaTrie.scala:157-477)."""
import pytest

from tests import cases as C


@pytest.mark.parametrize("sc", C.commit_scenarios(), ids=lambda s: s[0])
def test_emu_commits_vs_oracle(oracle, sc):
    from tests.emu import emu
    name, ks, vs, batches = sc
    want = C.oracle_commits(oracle, ks, vs, batches)
    t = emu.ResidentTrie(ks, vs)
    assert t.root == want[0], name
    for i, (ups, dels) in enumerate(batches):
        got = t.commit(ups, dels)
        assert got == want[i + 1], (name, i)


def test_emu_commit_rehashes_only_changed_paths(oracle):
    """One updated account in a 5,000-account trie re-hashes its leaf and its
    ancestors only (the reference's put path), not the whole trie."""
    import random
    from tests.emu import emu
    r = random.Random(4)
    ks = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(5000)]
    vs = [C.account_value(r) for _ in ks]
    t = emu.ResidentTrie(ks, vs)
    batch = ([(ks[123], C.account_value(r))], [])
    got = t.commit(*batch)
    assert got == C.oracle_commits(oracle, ks, vs, [batch])[1]
    hashes = int(t.stats[2])
    assert 2 <= hashes <= 8, hashes  # the leaf + its ~log16(5000) ancestors
