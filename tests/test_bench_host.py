"""Host-side checks of bench.py's roofline plumbing (no GPU): the PMC traffic lookup
reads the committed per-size summary, and scripts/pmc_summary.py's --json argument is
not mistaken for the build count."""
import json
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pmc_traffic_reads_committed_summary():
    t = bench.pmc_traffic("k_leaf_fused", 100_000_000)
    assert t is not None and t > 0
    # per launch: hbm_bytes / calls_per_build of the newest summary that has the kernel
    with open(os.path.join(ROOT, "profiles", "r1l_pmc_traffic_100000000.json")) as fh:
        row = json.load(fh)["kernels"]["k_leaf_fused"]
    assert abs(t - row["hbm_bytes"] / row["calls_per_build"]) < 1.0


def test_pmc_traffic_unknown_size_is_none():
    assert bench.pmc_traffic("k_leaf_fused", 12345) is None


def test_pmc_summary_json_arg(tmp_path):
    out = tmp_path / "t.json"
    r = subprocess.run([sys.executable, "scripts/pmc_summary.py", "no_such_tag", "--json", str(out)],
                       cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert "invalid literal" not in r.stderr
    assert r.returncode == 0, r.stderr
    with open(out) as fh:
        assert "kernels" in json.load(fh)


def test_pmc_round_order():
    """Newest summary by round number, not by file-name string order (r10a after r2a)."""
    names = ["profiles/r1l_pmc_traffic_5.json", "profiles/r10a_pmc_traffic_5.json", "profiles/r2b_pmc_traffic_5.json",
             "profiles/r2a_pmc_traffic_5.json"]
    assert sorted(names, key=bench.round_key)[-1].endswith("r10a_pmc_traffic_5.json")
    assert sorted(names, key=bench.round_key)[0].endswith("r1l_pmc_traffic_5.json")


def test_extrapolation_fit():
    """us/put = a + b*log16(n) through exact samples recovers a and b."""
    import math
    a, b = 3.0, 4.0
    samples = [(n, n * (a + b * math.log(n, 16)) * 1e-6) for n in (20000, 50000, 100000)]
    fa, fb, res = bench.fit_put_cost(samples)
    assert abs(fa - a) < 1e-6 and abs(fb - b) < 1e-6
    assert max(abs(r) for r in res) < 1e-6


def test_seq_root_hashes_keys_in_c(oracle):
    """mode 2 (keys hashed inside the C put loop) == hashing them first."""
    import numpy as np
    from khipu_amd import codec
    rnd = np.random.default_rng(5)
    addrs = [rnd.integers(0, 256, 20, dtype=np.uint8).tobytes() for _ in range(300)]
    vals = [codec.account_rlp(i, 10 ** 18 + i) for i in range(300)]
    vo = np.zeros(301, np.uint64)
    vo[1:] = np.cumsum([len(v) for v in vals])
    a = np.frombuffer(b"".join(addrs), np.uint8)
    vb = np.frombuffer(b"".join(vals), np.uint8)
    assert oracle.seq_root_packed(a, 20, vb, vo, 300, mode=2) == \
        oracle.seq_root([oracle.kec256(x) for x in addrs], vals)


def test_storage_ranges_balanced():
    """bench.py --workload storage: slot-balanced contiguous trie ranges cover every trie once."""
    import numpy as np
    r = np.random.default_rng(1)
    for nt, world in ((100_000, 8), (10, 16), (1, 4), (1000, 1), (5000, 3)):
        cnt = np.exp(r.uniform(0, np.log(10_001), nt)).astype(np.int64).clip(1, 10_000)
        so = np.concatenate([[0], np.cumsum(cnt)])
        b = bench.storage_ranges(so, world)
        assert b[0] == 0 and b[-1] == nt and all(b[g] <= b[g + 1] for g in range(world))
        slots = [int(so[b[g + 1]] - so[b[g]]) for g in range(world)]
        assert sum(slots) == int(so[-1])
        if nt >= 100 * world:
            assert max(slots) <= 1.02 * so[-1] / world + 10_000
