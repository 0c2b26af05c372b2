"""Summarise a gpu_profile.sh output directory into markdown + JSON for profiles/.

Per kernel (from the kernel_bench PMC passes): duration, HBM bytes (FETCH_SIZE x2, the gfx950
half-counting of wide loads, plus WRITE_SIZE), achieved bandwidth, MFMA busy share, LDS bank
conflict cycles per LDS instruction; plus the kernel-time table of the bench trace.
"""
import collections
import csv
import json
import os
import sys


def _short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].strip()


def load(path):
    rows = list(csv.DictReader(open(path)))
    out = collections.defaultdict(list)
    for r in rows:
        name = _short(r["Kernel_Name"])
        key = (name.strip(), int(r["Grid_Size"]))
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        out[key].append((r["Counter_Name"], float(r["Counter_Value"]), dur))
    return out


def main(d, out_prefix):
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for sub in ("pmc_fetch", "pmc_write", "pmc_mfma", "pmc_lds"):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for key, vals in load(f).items():
            for name, v, dur in vals:
                counters[key][name].append(v)
                durs[key].append(dur)
    table = []
    for key in sorted(counters, key=lambda k: -sum(durs[k]) / max(len(durs[k]), 1)):
        name, grid = key
        if not any(t in name for t in ("mlp_", "multi_copy", "attn", "rmsnorm", "adamw", "im2col",
                                       "bn_", "swiglu", "ce_", "rope", "embed", "hyper", "sgd")):
            continue
        c = {k: sum(v) / len(v) for k, v in counters[key].items()}
        dur = sorted(durs[key])[len(durs[key]) // 2]
        fetch = 2 * c.get("FETCH_SIZE", 0) * 1024
        write = c.get("WRITE_SIZE", 0) * 1024
        row = {"kernel": name, "workgroups": grid // 256, "median_us": round(dur, 1),
               "hbm_read_MB": round(fetch / 1e6, 1), "hbm_write_MB": round(write / 1e6, 1),
               "hbm_TBps": round((fetch + write) / (dur * 1e-6) / 1e12, 2) if dur else None}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("SQ_BUSY_CYCLES"):
            row["mfma_busy_pct"] = round(100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] /
                                         (c["GRBM_GUI_ACTIVE"] * 256 * 4), 2) \
                if c.get("GRBM_GUI_ACTIVE") else None
        if c.get("SQ_INSTS_LDS"):
            row["lds_conflict_cycles_per_inst"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) /
                                                        c["SQ_INSTS_LDS"], 3)
        table.append(row)
    trace = []
    tf = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(tf):
        for r in list(csv.DictReader(open(tf)))[:12]:
            trace.append({"kernel": _short(r["Name"])[:60], "calls": int(r["Calls"]),
                          "avg_us": round(float(r["AverageNs"]) / 1e3, 1),
                          "pct": round(float(r["Percentage"]), 2)})
    bench = json.load(open(os.path.join(d, "bench.json")))
    kb = json.load(open(os.path.join(d, "kbench.json"))) if os.path.exists(
        os.path.join(d, "kbench.json")) else None
    summary = {"bench": bench, "kernel_bench": kb, "pmc": table, "bench_trace_top": trace}
    json.dump(summary, open(out_prefix + ".json", "w"), indent=1)
    with open(out_prefix + ".md", "w") as f:
        f.write(f"# Profile summary ({os.path.basename(out_prefix)})\n\n")
        f.write(f"bench: **{bench['value']} {bench['metric'].split('(')[0].strip()}**, "
                f"{bench['ms_per_step']} ms/step, host ms per sync {bench.get('host_ms_per_sync')}\n\n")
        f.write("## PMC per kernel (kernel_bench, one population step)\n\n")
        keys = ["kernel", "workgroups", "median_us", "hbm_read_MB", "hbm_write_MB", "hbm_TBps",
                "mfma_busy_pct", "lds_conflict_cycles_per_inst"]
        f.write("| " + " | ".join(keys) + " |\n|" + "---|" * len(keys) + "\n")
        for r in table:
            f.write("| " + " | ".join(str(r.get(k, "")) for k in keys) + " |\n")
        f.write("\n## Bench kernel trace (rocprofv3 --kernel-trace --stats)\n\n")
        f.write("| kernel | calls | avg us | % |\n|---|---|---|---|\n")
        for r in trace:
            f.write(f"| {r['kernel']} | {r['calls']} | {r['avg_us']} | {r['pct']} |\n")
    print(open(out_prefix + ".md").read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
