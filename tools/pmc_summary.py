"""Summarise rocprofv3 --pmc runs per kernel instance and derive the roofline figures.

    python tools/pmc_summary.py gpurun_out/<tag>/pmc [--json out.json]

Each pmc/p<i>/run_counter_collection.csv holds one counter set (tools/gpu.sh pmc).
Rows are grouped by kernel name with its template arguments (so k_vpass9<35,16,2,...>
(den-read) and <35,16,1,...> (den-write) stay apart) and averaged over dispatches.

Derived (MI355X_MICROARCH.md §HBM, §PMC; calibration of the counters for the access
shapes of these kernels: tools/ubench/fetch_calib.hip, profiles/r02/calib.json):
  hbm_read_B  = FETCH_SIZE * 1024 * 2  (FETCH_SIZE reads 1/2 of the bytes for both
                4-B/lane and 16-B/lane coalesced streaming reads on gfx950)
  hbm_write_B = WRITE_SIZE * 1024      (exact for 4-B and 16-B/lane stores)
  valu_busy   = SQ_ACTIVE_INST_VALU * 4 / (SQ_BUSY_CYCLES * 4 SIMDs * 32 CUs/SE ...)
is NOT attempted (gfx950 has no derived-counter section in ROCm 7.2); instead the
per-wave instruction mix and the wait/active split of wave cycles are reported.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name: str) -> str:
    m = re.search(r"(k_\w+)(<[^>(]*>)?", name)
    if not m:
        return name[:60]
    return m.group(1) + (m.group(2) or "")


def collect(root: str) -> dict:
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> counter -> dispatch -> sum
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            d = per[k][r["Counter_Name"]]
            key = (f, r["Dispatch_Id"])
            d[key] = d.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for k, cs in per.items():
        out[k] = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    return out


def derive(c: dict) -> dict:
    d = {}
    if "FETCH_SIZE" in c:
        d["hbm_read_B"] = c["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in c:
        d["hbm_write_B"] = c["WRITE_SIZE"] * 1024
    if "hbm_read_B" in d and "hbm_write_B" in d:
        d["hbm_total_B"] = d["hbm_read_B"] + d["hbm_write_B"]
    w = c.get("SQ_WAVES")
    if w:
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH"):
            if n in c:
                d[n.replace("SQ_INSTS_", "per_wave_")] = c[n] / w
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM"):
            if n in c:
                d[n.replace("SQ_", "frac_wave_cycles_")] = c[n] / wc
    if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
        tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
        d["l2_hit_rate"] = c["TCC_HIT_sum"] / tot if tot else None
    if c.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    ap.add_argument("--filter", default="k_")
    a = ap.parse_args()
    raw = collect(a.root)
    res = {}
    for k in sorted(raw):
        if a.filter not in k:
            continue
        res[k] = {"counters": raw[k], "derived": derive(raw[k])}
        print(f"== {k}")
        for n, v in sorted(raw[k].items()):
            print(f"   {n:28s} {v:18.1f}")
        for n, v in sorted(res[k]["derived"].items()):
            print(f"   > {n:26s} {v if v is None else round(v, 4)}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
