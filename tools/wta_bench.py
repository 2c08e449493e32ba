"""asw_WTA microbenchmark (GPU): the WTA variants (ASW_TUNE_WTA_VARIANT) on the final
C4 volume of a synthetic pair (raw cost -> supports -> 7 x (V, H)), each checked
identical to variant 0.

    python tools/wta_bench.py [--variants 0,2] [--reps 20]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereo_matchin_amd import StereoMatcher, _lib, make_params  # noqa: E402
from stereo_matchin_amd import kernels as K  # noqa: E402
from stereo_matchin_amd.synthetic import make_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,2")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    W, H, D, T = 1920, 1080, 256, 35
    Lh, Rh, _ = make_pair(W, H, D, 0)
    p = make_params(W, H, ndisp=D, taps=T, iters=7)
    m = StereoMatcher(p, dev)
    m.raw_and_support(torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev))
    cost = m.aggregate()
    torch.cuda.synchronize()
    lib = _lib.lib()
    ref = None
    for v in [int(x) for x in a.variants.split(",")]:
        old = lib.asw_tune_set(2, v)
        ts = []
        try:
            for r in range(a.reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                out = K.asw_WTA(p, cost)
                e1.record()
                torch.cuda.synchronize()
                if r:
                    ts.append(e0.elapsed_time(e1))
        finally:
            lib.asw_tune_set(2, old)
        got = [o.clone() for o in out]
        same = ref is None or all(torch.equal(g, q) for g, q in zip(got, ref))
        ref = ref or got
        print(json.dumps({"variant": v, "ms_median": round(float(np.median(ts)), 4), "ms_min": round(min(ts), 4),
                          "identical_to_first": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
