"""Summarise rocprofv3 --pmc CSVs per kernel (mean over dispatches of each counter)."""
import collections
import csv
import glob
import sys


def summarise(root, filt=("k_vpass", "k_hpass", "k_wta", "k_raw_cost", "k_support")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            key = next((k for k in filt if k in name), None)
            if key is None:
                continue
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1])
    for k, cs in res.items():
        print(f"== {k}")
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {v:16.1f}")
