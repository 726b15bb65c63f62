"""The last block of a scripts/gpu_bc_pmc.sh run (configs[2] commits under FETCH_SIZE /
WRITE_SIZE passes), per kernel: dispatches, summed duration (the --pmc passes serialise the
kernels), corrected read bytes (2 x FETCH_SIZE, MI355X_MICROARCH.md) and write bytes.
Windows are cut at idle gaps > 3 ms.  Measurement only.

  python scripts/pmc_last_block.py <tag>
"""
import csv, sys, collections
tag = sys.argv[1]
def load(p, cname):
    rows = []
    for r in csv.DictReader(open(f"gpurun_out/{tag}_{p}/pmc_counter_collection.csv")):
        if r["Counter_Name"] == cname:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0], float(r["Counter_Value"]), r["Queue_Id"], int(r["Grid_Size"])))
    rows.sort()
    # cut into windows by gaps > 3 ms; last window
    wins, cur = [], []
    for e in rows:
        if cur and e[0] - max(x[1] for x in cur[-8:]) > 3e6:
            wins.append(cur); cur = []
        cur.append(e)
    wins.append(cur)
    return wins
w1 = load("p1", "FETCH_SIZE")
w2 = load("p2", "WRITE_SIZE")
print("windows", len(w1), [len(w) for w in w1[-4:]])
last = w1[-1]; lastw = w2[-1]
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for a, b in zip(last, lastw):
    k = a[2]
    agg[k][0] += 1; agg[k][1] += (a[1]-a[0])/1e3; agg[k][2] += 2*a[3]/1e3; agg[k][3] += b[3]/1e3
tot = [0,0,0,0]
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:28s} {v[0]:3d} {v[1]:8.1f}us read {v[2]:8.2f}MB write {v[3]:8.2f}MB")
    for i in range(4): tot[i] += v[i]
print("total", tot)
