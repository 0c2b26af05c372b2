"""Per-kernel-name HBM bytes of a ResNet-20 PMC run (FETCH_SIZE / WRITE_SIZE passes, KB) over the
last quarter of the dispatches (steady state): MB per call, GB/s over the kernel's own duration."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:60]


def load(name):
    f = glob.glob(f"{root}/pmc_{name}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(float)
    meta = {}
    for r in csv.DictReader(open(f)):
        d = int(r["Dispatch_Id"])
        per[d] += float(r["Counter_Value"])
        meta[d] = (short(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                   r["Grid_Size"])
    ids = sorted(per)[len(per) * 3 // 4:]
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for d in ids:
        k = (meta[d][0], meta[d][2])
        agg[k][0] += 1
        agg[k][1] += per[d]
        agg[k][2] += meta[d][1]
    return agg


fetch, write = load("fetch"), load("write")
print(f"{'kernel':60s} {'grid':>9s} {'calls':>5s} {'read MB':>8s} {'write MB':>8s} {'us':>7s} {'TB/s':>6s}")
rows = []
for k, (n, kb, ns) in fetch.items():
    w = write.get(k, [n, 0.0, ns])
    rd, wr = kb / n / 1024, w[1] / max(w[0], 1) / 1024
    us = ns / n / 1e3
    rows.append((ns, k, n, rd, wr, us))
for ns, k, n, rd, wr, us in sorted(rows, reverse=True)[:25]:
    print(f"{k[0]:60s} {k[1]:>9s} {n:5d} {rd:8.1f} {wr:8.1f} {us:7.1f} {(rd + wr) / us:6.2f}")
