"""Support-weight kernel microbenchmark (GPU): asw_support_all at C4 per variant.

    python tools/support_bench.py [--variants 0] [--taps 35] [--reps 20]

Variant = an ASW_TUNE_WTA_VARIANT value set around the launches (none select a
support kernel today; the hook stays for the next experiment).
Checks every variant's four arrays are identical to variant 0's.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereo_matchin_amd import _lib, make_params  # noqa: E402
from stereo_matchin_amd import kernels as K  # noqa: E402
from stereo_matchin_amd.synthetic import make_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0",
                    help="asw_tune_set(ASW_TUNE_PASS_VARIANT) values (none select a support form since round 5: "
                         "the EXPD form is tools/exp/exp_forms.hip)")
    ap.add_argument("--c5", action="store_true", help="3840x2160 (default 1920x1080)")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--taps", type=int, default=35)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    W, H = (3840, 2160) if a.c5 else (1920, 1080)
    Lh, Rh, _ = make_pair(W, H, 256, 0)
    p = make_params(W, H, ndisp=256, taps=a.taps, iters=1)
    L, R = torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev)
    lut = K.support_lut(p, dev)
    ws = [K.new_support(p, dev) for _ in range(4)]
    lib = _lib.lib()
    ref = None
    for v in [int(x) for x in a.variants.split(",")]:
        old = lib.asw_tune_set(1, v)
        ts = []
        for r in range(a.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            K.support_all(p, L, R, lut, *ws)
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        lib.asw_tune_set(1, old)
        got = [w.clone() for w in ws]
        same = ref is None or all(torch.equal(g, q) for g, q in zip(got, ref))
        ref = ref or got
        print(json.dumps({"variant": v, "taps": a.taps, "ms_median": round(float(np.median(ts)), 4),
                          "ms_min": round(min(ts), 4), "identical_to_first": bool(same)}))


if __name__ == "__main__":
    main()
