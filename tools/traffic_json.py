"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE runs of bench.py into profiles/traffic.json.

    python tools/traffic_json.py gpurun_out/<tag>/pmc [--key c4_n1] [--out profiles/traffic.json]

<root>/p*/ hold one --pmc counter set each (tools/gpu.sh "pmc" step, or any
directory of rocprofv3 CSVs).  Corrections, calibrated on this hardware for the
kernels' own access shapes (tools/ubench/fetch_calib.hip, profiles/r02/calib.json):
the counters are in KB; FETCH_SIZE reads exactly half the bytes of a coalesced
streaming read, for 4-B/lane (the cost-volume loads) as for 16-B/lane loads, so
it is doubled; WRITE_SIZE is exact for 4-B and 16-B/lane stores.

Entries are per kernel and den mode, averaged over dispatches, keyed like
bench.py's roofline.kernel: "k_vpass10<DM_READ>", "k_hpass9<DM_WRITE>", ...
"""
import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import collect  # noqa: E402

DM = {0: "DM_NONE", 1: "DM_WRITE", 2: "DM_READ"}


def key_of(name: str):
    """k_vpass10<35, 16, 2, ...> -> k_vpass10<T=35,DM_READ>; k_hpass9<35, 4, 40, 2> ->
    k_hpass9<T=35,DM_READ>; k_hpass11<35, 4, 2, ...> -> k_hpass11<T=35,DM_READ> (template
    argument order of each kernel; bench.py looks the kernel asw_pass_kernel names up this way)."""
    m = re.match(r"(k_vpass10|k_hpass9|k_hpass11_wr|k_hpass11|k_vpass32|k_hpass32)<([^>]*)>", name)
    if not m:
        return None
    args = [a.strip() for a in m.group(2).split(",")]
    if m.group(1) == "k_hpass11_wr":  # the last H pass with the WTA's own scan (den-read)
        return f"k_hpass11_wr<T={args[0]},DM_READ>"
    dm = int(args[3]) if m.group(1) == "k_hpass9" else int(args[2])
    # the first V pass over the uint16 raw costs: k_vpass10<..., C16 = true> (its last
    # argument), k_vpass32<T, NW, DM, CP, NPH, RB, PS, C16[, HS]> (the eighth)
    if m.group(1) == "k_vpass32":
        c16 = len(args) > 7 and args[7] == "true"
    else:
        c16 = m.group(1) == "k_vpass10" and args[-1] == "true"
    return f"{m.group(1)}{'_c16' if c16 else ''}<T={args[0]},{DM[dm]}>"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--key", default="c4_n1")
    ap.add_argument("--source", default="", help="the tracked copy of root under profiles/ (recorded as the source)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "traffic.json"))
    a = ap.parse_args()
    raw = collect(a.root)
    entry = {"source": a.source or a.root,
             "corrections": "hbm_read = 2 x FETCH_SIZE x 1024, hbm_write = WRITE_SIZE x 1024 "
                            "(calibrated: profiles/r02/calib.json)"}
    for name, c in raw.items():
        k = key_of(name)
        if not k or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        r, w = 2 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
        entry[k] = {"read_bytes": round(r), "write_bytes": round(w), "total_bytes": round(r + w)}
    try:
        data = json.load(open(a.out))
    except (OSError, ValueError):
        data = {}
    data[a.key] = entry
    json.dump(data, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps({a.key: entry}, indent=1))


if __name__ == "__main__":
    main()
