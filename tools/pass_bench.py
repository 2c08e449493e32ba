"""Aggregation-pass microbenchmark over the compiled kernel variants (GPU).

    python tools/pass_bench.py [--workload c4] [--reps 10] [--variants 0,1,2,...]

For each variant (asw_tune_set(ASW_TUNE_PASS_VARIANT, v)) times the V and the H
pass on the same realistic inputs (raw cost + supports of the synthetic C4 pair),
interleaved over reps in one process, and checks every variant's output is
bit-identical to variant 0.  Prints one JSON line per (variant, direction) with
the median / min ms and the algorithmic GB/s (8*D*S + 8*T*S per launch).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import WORKLOADS  # noqa: E402
from stereo_matchin_amd import StereoMatcher, make_params  # noqa: E402
from stereo_matchin_amd import _lib  # noqa: E402
from stereo_matchin_amd import kernels as K  # noqa: E402
from stereo_matchin_amd.synthetic import make_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--den", action="store_true", help="also time the cached-denominator modes (write, read)")
    ap.add_argument("--ndisp", type=int, default=0, help="override D (e.g. a d-shard's local planes)")
    ap.add_argument("--planes", type=int, default=0,
                    help="time the shard [0, planes) of the D planes (<= 32: pitch 32, the asw_pass32.h passes)")
    args = ap.parse_args()
    W, H, D, T, iters, lr, desc = WORKLOADS[args.workload]
    D = args.ndisp or D
    dev = torch.device("cuda:0")
    Lh, Rh, _ = make_pair(W, H, D, 0)
    p = make_params(W, H, ndisp=D, taps=T, iters=iters, flags=_lib.FLAG_RAW_F32)  # c0 = the float raw costs
    if args.planes:
        p.d_begin, p.d_end = 0, args.planes
    m = StereoMatcher(p, dev)
    Ld, Rd = torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev)
    m.raw_and_support(Ld, Rd)
    torch.cuda.synchronize()
    cin = m.c0
    out = torch.empty_like(cin)
    variants = [int(v) for v in args.variants.split(",")]
    modes = [0, 1, 2] if args.den else [0]  # ASW_DEN_NONE / WRITE / READ
    dens = {"v": torch.empty_like(cin), "h": torch.empty_like(cin)} if args.den else {}
    lib = _lib.lib()
    S = W * H
    nloc = p.d_stop - p.d_begin
    nbytes = 8 * nloc * S + 8 * T * S
    dirs = ("v", "h")
    ref = {}
    kname = {}
    times = {(v, d, dm): [] for v in variants for d in dirs for dm in modes}
    for rep in range(args.reps + 1):
        for v in variants:
            lib.asw_tune_set(1, v)
            forms = [("v", K.asw_vCostAggregation, m.wvl, m.wvr), ("h", K.asw_hCostAggregation, m.whl, m.whr)]
            for d, fn, wl, wr in forms:
                for dm in modes:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn(p, wl, wr, cin, out=out, den=dens.get(d), den_mode=dm)
                    e1.record()
                    torch.cuda.synchronize()
                    if rep == 0:
                        kname[(d, dm)] = K.pass_kernel(0 if d == "v" else 1, dm)
                        if v == variants[0] and dm == 0:
                            ref[d] = out.clone()
                        elif not torch.equal(out, ref[d]):
                            print(json.dumps({"variant": v, "dir": d, "den_mode": dm,
                                              "error": "output differs from variant 0"}))
                    else:
                        times[(v, d, dm)].append(e0.elapsed_time(e1))
    lib.asw_tune_set(1, 0)
    for (v, d, dm), ts in times.items():
        med = float(np.median(ts))
        print(json.dumps({"workload": args.workload, "ndisp": D, "planes": nloc, "variant": v, "dir": d, "den_mode": dm,
                          "kernel": kname.get((d, dm)),
                          "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                          "GBps": round(nbytes / med / 1e6, 1),
                          "frac_of_8TBps": round(nbytes / med / 1e6 / 8000, 4)}))


if __name__ == "__main__":
    main()
