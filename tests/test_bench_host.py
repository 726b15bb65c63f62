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
