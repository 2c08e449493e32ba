"""C5 k_vpass10 den-read forms (tools/exp/libexp_c5vpx.so, EXP_C5VPX in exp_lib.hip:
deeper cost prefetch, one barrier per row): each form checked bit-exact against the
production pass, then timed.  Not part of the product.

    python tools/exp/c5v_bench.py [--reps 8] [--forms 2,1,81]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from stereo_matchin_amd import StereoMatcher, _lib, make_params  # noqa: E402
from stereo_matchin_amd import kernels as K  # noqa: E402
from stereo_matchin_amd.synthetic import make_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--forms", default="")
    args = ap.parse_args()
    W, H, D, T = 3840, 2160, 512, 51
    forms = [int(f) for f in (args.forms or "2,1,81").split(",")]
    dev = torch.device("cuda:0")
    Lh, Rh, _ = make_pair(W, H, D, 0)
    p = make_params(W, H, ndisp=D, taps=T, iters=7, flags=_lib.FLAG_RAW_F32)
    m = StereoMatcher(p, dev)
    m.raw_and_support(torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev))
    cin = m.c0  # the raw costs as the V input
    den = torch.empty_like(cin)
    ref = m.c1
    K.asw_vCostAggregation(p, m.wvl, m.wvr, cin, out=ref, den=den, den_mode=1)
    K.asw_vCostAggregation(p, m.wvl, m.wvr, cin, out=ref, den=den, den_mode=2)
    torch.cuda.synchronize()
    print("prod", K.pass_kernel(0, 2), flush=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_c5vpx.so"))
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    pp = ctypes.byref(p)
    out = torch.empty_like(cin)
    st = torch.cuda.current_stream()

    def launch(f):
        if f < 0:
            K.asw_vCostAggregation(p, m.wvl, m.wvr, cin, out=out, den=den, den_mode=2)
        else:
            rc = lib.exp_c5vpx(f, pp, P(m.wvl), P(m.wvr), P(cin), P(out), P(den), ctypes.c_void_p(st.cuda_stream))
            assert rc == 0, (f, rc)

    runs = [-1] + forms
    for f in runs:
        out.zero_()
        launch(f)
        torch.cuda.synchronize()
        print(json.dumps({"form": "prod" if f < 0 else f, "bit_exact": bool(torch.equal(out, ref))}), flush=True)
    times = {f: [] for f in runs}
    for rep in range(args.reps + 1):
        for f in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch(f)
            e1.record()
            e1.synchronize()
            if rep >= 1:
                times[f].append(e0.elapsed_time(e1))
    for f, t in times.items():
        t.sort()
        print(json.dumps({"form": "prod" if f < 0 else f, "ms_median": round(t[len(t) // 2], 4),
                          "ms_min": round(t[0], 4)}), flush=True)


if __name__ == "__main__":
    main()
