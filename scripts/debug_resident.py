"""Step-by-step resident-trie commits on the GPU vs the host replay and the oracle
(prints per-commit counts; used to localise a device/replay divergence)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import khipu_amd  # noqa: E402,F401
from khipu_amd._lib import KhStats  # noqa: E402
from khipu_amd.device import Ctx, ResidentTrie  # noqa: E402
from oracle import oracle  # noqa: E402
from tests import cases as C  # noqa: E402
from tests.emu import emu  # noqa: E402

only = sys.argv[1:] or None
ctx = Ctx(0)
for name, ks, vs, batches in C.commit_scenarios():
    if only and name not in only:
        continue
    want = C.oracle_commits(oracle, ks, vs, batches)
    e = emu.ResidentTrie(ks, vs)
    t = ResidentTrie(ctx, ks, vs)
    print(name, "open", t.root == want[0], e.root == want[0], len(t), flush=True)
    for i, (ups, dels) in enumerate(batches):
        er = e.commit(ups, dels)
        st = KhStats()
        try:
            g = t.commit(ups, dels, stats=st)
        except Exception as ex:  # noqa: BLE001
            print(name, i, "DEVICE ERROR", ex, "emu m2/nd", list(e.stats), flush=True)
            break
        print(name, i, "gpu", g == want[i + 1], "emu", er == want[i + 1], "gpu m2", st.n_leaves, "emu m2/nd",
              list(e.stats), "hashes", st.n_node_hashes, flush=True)
