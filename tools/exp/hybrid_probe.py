"""Would a V pass that caches the denominators of only some of its plane blocks be
faster?  A den-read pass is bound by its memory stream (cost in, den in, out), a
den-none pass by VALU (3 instead of 2 per voxel-tap); mixing the two modes in one
launch would balance the two pipes.  Probe without a new kernel: the C4 frame's planes
as two 128-plane halves (two d-shard matchers, pitch 128), their V passes on two
streams at once, in every pair of den modes, against the two halves one after the
other.  GPU only; not part of the product.

    python tools/exp/hybrid_probe.py [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from stereo_matchin_amd import StereoMatcher, _lib, make_params  # noqa: E402
from stereo_matchin_amd import kernels as K  # noqa: E402
from stereo_matchin_amd.synthetic import make_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dir", default="v", choices=["v", "h"])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    W, H, D, T = 1920, 1080, 256, 35
    Lh, Rh, _ = make_pair(W, H, D, 0)
    L, R = torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev)
    ms = []
    for d0, d1 in ((0, 128), (128, 256)):
        p = make_params(W, H, ndisp=D, taps=T, iters=7, d_begin=d0, d_end=d1, flags=_lib.FLAG_RAW_F32)
        m = StereoMatcher(p, dev)
        m.raw_and_support(L, R)
        ms.append(m)
    f = K.asw_vCostAggregation if a.dir == "v" else K.asw_hCostAggregation

    def run(m, mode):
        wl, wr = (m.wvl, m.wvr) if a.dir == "v" else (m.whl, m.whr)
        den = m.den_v if a.dir == "v" else m.den_h
        f(m.p, wl, wr, m.c0, out=m.c1, den=den if mode else None, den_mode=mode)

    for m in ms:
        run(m, _lib.DEN_WRITE)  # the cached denominators
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cases = {"seq read+read": None, "par read|read": (2, 2), "par read|none": (2, 0), "par none|read": (0, 2),
             "par none|none": (0, 0), "seq none+none": "nn"}
    res = {k: [] for k in cases}
    for _ in range(a.reps + 1):
        for name, c in cases.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if c is None or c == "nn":
                mode = _lib.DEN_READ if c is None else _lib.DEN_NONE
                run(ms[0], mode)
                run(ms[1], mode)
            else:
                cur = torch.cuda.current_stream(dev)
                for st, m, mode in ((s0, ms[0], c[0]), (s1, ms[1], c[1])):
                    st.wait_stream(cur)
                    with torch.cuda.stream(st):
                        run(m, mode)
                cur.wait_stream(s0)
                cur.wait_stream(s1)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1))
    for name, ts in res.items():
        print(json.dumps({"dir": a.dir, "case": name, "ms_median": round(float(np.median(ts[1:])), 4),
                          "ms_min": round(min(ts[1:]), 4)}), flush=True)


if __name__ == "__main__":
    main()
