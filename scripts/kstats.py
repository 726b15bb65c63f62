"""Per-kernel time per build from a rocprofv3 --kernel-trace CSV (full-size launches only).

usage: python scripts/kstats.py <rocprof output dir> [min_ms]
Dispatches shorter than min_ms (default 0) are kept; each kernel's total is divided by the
number of builds = launches of k_leaf_in (one per plain root build; key hashing of host inputs
is one launch per arriving part since round 6), else of k_hash_keys / k_hash_keys_ck."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))


def kname(full):
    return full.split("(")[0].replace("void ", "").split("<")[0].replace("khst::", "").strip()


tot = collections.defaultdict(float)
cnt = collections.defaultdict(int)
for r in rows:
    k = kname(r["Kernel_Name"])
    tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    cnt[k] += 1
builds = cnt.get("k_leaf_in", 0) or max(cnt.get("k_hash_keys", 0), cnt.get("k_hash_keys_ck", 0), 1)
print(f"builds={builds}  (ms per build, launches per build)")
for k in sorted(tot, key=lambda x: -tot[x]):
    print(f"{k[:34]:34s} {tot[k] / builds:9.3f} ms  {cnt[k] / builds:7.1f}")
