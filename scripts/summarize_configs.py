"""Summarise the config-3/5 kernel traces (scripts/trace_configs.sh), the population-GEMM bench
(scripts/gemm_bench.py) and its PMC passes (scripts/pmc_gemm.sh) into one markdown file.

    python scripts/summarize_configs.py gpurun_out/trace2 gpurun_out/gemm2.json \
        gpurun_out/pmc2 profiles/configs_r1.md
"""
import collections
import csv
import json
import os
import sys


def _short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].strip()[:70]


def trace_table(path, top=14):
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"GPU kernel time {total / 1e6:.1f} ms over the traced run\n",
           "| kernel | calls | avg us | % |", "|---|---|---|---|"]
    for r in rows[:top]:
        out.append(f"| {_short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                   f"{float(r['Percentage']):.1f} |")
    return "\n".join(out)


def pmc_table(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ("mfma", "lds", "fetch"):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if "pgemm_kernel" not in r["Kernel_Name"]:
                continue
            key = (r["Kernel_Name"].split("pgemm_kernel")[1].split(">")[0] + ">",
                   int(r["Grid_Size"]) // 256)
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = ["| pgemm instance <srcA, srcB, TA, TB, WM, FM, FN> | workgroups | "
           "LDS bank-conflict cycles / LDS instr | VALU instr / LDS instr | HBM read MB |",
           "|---|---|---|---|---|"]
    for (inst, wg), c in sorted(agg.items(), key=lambda kv: -kv[0][1]):
        m = {k: sum(v) / len(v) for k, v in c.items()}
        lds = max(m.get("SQ_INSTS_LDS", 1), 1)
        out.append(f"| {inst} | {wg} | {m.get('SQ_LDS_BANK_CONFLICT', 0) / lds:.2f} | "
                   f"{m.get('SQ_INSTS_VALU', 0) / lds:.1f} | {2 * m.get('FETCH_SIZE', 0) / 1e3:.0f} |")
    return "\n".join(out)


def gemm_table(path):
    rows = json.load(open(path))
    out = ["| shape | P | M | N | K | plan (cfg, splits, k/split) | pgemm us | pgemm TFLOP/s | "
           "hipBLASLt NN (materialised) us | TFLOP/s |", "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| {r['shape']} | {r['P']} | {r['M']} | {r['N']} | {r['K']} | {r['plan']} | "
                   f"{r['pgemm_us']} | {r['pgemm_tflops']} | {r.get('bmm_nn_us', '')} | "
                   f"{r.get('bmm_nn_tflops', '')} |")
    return "\n".join(out)


def main(trace_dir, gemm_json, pmc_dir, out):
    parts = ["# Config 3 / 5 kernel profiles (MI355X, one GPU)\n"]
    for name, title in (("resnet20", "ResNet-20 population (config 3: 32 trials x 128 images)"),
                        ("lm125m", "Llama-style 125M LM population (config 5: 8 trials x 8 x 512 "
                                   "tokens)")):
        f = os.path.join(trace_dir, name, "run_kernel_stats.csv")
        if os.path.exists(f):
            parts += [f"## {title}\n", trace_table(f), ""]
    if os.path.exists(gemm_json):
        parts += ["## Population GEMM (csrc/pgemm.hip) vs hipBLASLt\n", gemm_table(gemm_json), ""]
    if os.path.isdir(pmc_dir):
        parts += ["## Population GEMM PMC counters (rocprofv3 --pmc, gemm_bench shapes)\n",
                  pmc_table(pmc_dir), ""]
    open(out, "w").write("\n".join(parts) + "\n")
    print(open(out).read())


if __name__ == "__main__":
    main(*sys.argv[1:5])
