"""Per-interval stream concurrency of a rocprofv3 kernel trace of bench.py: time with 0 / 1 / 2 /
3 hardware queues busy, and each queue's first / last kernel within the interval."""
import csv
import sys
from collections import Counter, defaultdict

r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x["Start_Timestamp"]))
t0 = int(r[0]["Start_Timestamp"])
mlp = [x for x in r if "mlp_" in x["Kernel_Name"]]
# interval starts: a train kernel after a gap of > 300 us with no kernel running
starts, end = [], 0
for x in mlp:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    if s - end > 300_000:
        starts.append(s)
    end = max(end, e)
tot = Counter()
for lo, hi in zip(starts, starts[1:]):
    ev, span = [], defaultdict(lambda: [1e30, 0])
    for x in mlp:
        s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        if lo <= s < hi:
            ev += [(s, 1, x["Queue_Id"]), (e, -1, x["Queue_Id"])]
            sp = span[x["Queue_Id"]]
            sp[0], sp[1] = min(sp[0], s), max(sp[1], e)
    ev.sort()
    act, dur, last = Counter(), Counter(), lo
    for t, d, q in ev:
        dur[sum(1 for v in act.values() if v > 0)] += t - last
        last = t
        act[q] += d
    tot.update(dur)
    print(f"interval at {(lo - t0) / 1e6:8.2f} ms: busy-queue ms",
          {k: round(v / 1e6, 2) for k, v in sorted(dur.items())},
          "queue spans", {q: (round((a - lo) / 1e6, 2), round((b - lo) / 1e6, 2))
                          for q, (a, b) in sorted(span.items())})
print("all intervals:", {k: round(v / 1e6, 2) for k, v in sorted(tot.items())})
