"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE runs of bench.py into profiles/traffic.json.

    python tools/traffic_json.py gpurun_out/pmc_<tag> [--key c4_n1] [--out profiles/traffic.json]

Corrections per MI355X_MICROARCH.md (HBM section): the counters are in KB;
FETCH_SIZE on gfx950 reports half the bytes of a 16-B-per-lane streaming read, so
it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  The aggregation
passes stream the cost volume with 16-B-per-lane loads and stores, which is the
calibrated case.  Reported per launch, averaged over every k_vpass/k_hpass
dispatch, like bench.py's `achieved`.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_kernel(root, counter):
    vals = {}
    for f in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            k = "k_vpass" if "k_vpass" in name else "k_hpass" if "k_hpass" in name else None
            if k:
                # one row per dispatch (values summed over instances by rocprofv3)
                d = vals.setdefault(k, {})
                d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: statistics.mean(v.values()) * 1024.0 for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--key", default="c4_n1")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "traffic.json"))
    a = ap.parse_args()
    fetch = per_kernel(a.root, "FETCH_SIZE")
    write = per_kernel(a.root, "WRITE_SIZE")
    entry = {"source": a.root, "corrections": "FETCH_SIZE x2 (gfx950 16B/lane reads), KB->bytes"}
    tot = []
    for k in ("k_vpass", "k_hpass"):
        if k in fetch and k in write:
            r, w = 2 * fetch[k], write[k]
            entry[k] = {"read_bytes": round(r), "write_bytes": round(w), "total_bytes": round(r + w)}
            tot.append(r + w)
    entry["hbm_bytes_per_pass"] = round(statistics.mean(tot)) if tot else None
    try:
        data = json.load(open(a.out))
    except (OSError, ValueError):
        data = {}
    data[a.key] = entry
    json.dump(data, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps({a.key: entry}))


if __name__ == "__main__":
    main()
