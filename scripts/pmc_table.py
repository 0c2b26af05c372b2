"""Per-dispatch table of a rocprofv3 --pmc CSV (run_counter_collection.csv): one row per kernel
dispatch with its counters summed over the dimension instances.

    python scripts/pmc_table.py gpurun_out/x/sq/run_counter_collection.csv [--filter dconv]
"""
import argparse
import collections
import csv
import re
import sys


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--filter", default="")
    a = ap.parse_args(argv)
    data = collections.OrderedDict()
    for r in csv.DictReader(open(a.csv)):
        k = (int(r["Dispatch_Id"]), short(r["Kernel_Name"]), r["LDS_Block_Size"], r["VGPR_Count"],
             r["Grid_Size"])
        d = data.setdefault(k, {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k, d in data.items():
        if a.filter not in k[1]:
            continue
        cs = " ".join(f"{c}={v / 1e6:.2f}M" if v >= 1e5 else f"{c}={v:.0f}" for c, v in d.items())
        print(f"{k[0]:4d} {k[1][:44]:44s} lds={k[2]:>6s} vgpr={k[3]:>4s} grid={k[4]:>8s} {cs}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
