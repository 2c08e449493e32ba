"""k_hpass32 occupancy experiment (tools/exp/libexp_h32.so, EXP_H32 in exp_lib.hip) on the
C4 8-way shard (1920x1080, planes [0, 32) of D = 256, T = 35, den-none): each form and
segment count is checked bit-exact against the production pass, then timed.  Not part
of the product.

    python tools/exp/h32_bench.py [--reps 30] [--runs 0:0,1:0,2:0,2:6]
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
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--runs", default="0:0,1:0,1:6,2:0,2:6,2:7,3:0",
                    help="form:nseg,... (form 0 = shipped; nseg 0 = the form's slot rule)")
    args = ap.parse_args()
    W, H, D, T = 1920, 1080, 256, 35
    dev = torch.device("cuda:0")
    Lh, Rh, _ = make_pair(W, H, D, 0)
    p = make_params(W, H, ndisp=D, taps=T, iters=7, flags=_lib.FLAG_RAW_F32)
    p.d_begin, p.d_end = 0, 32
    m = StereoMatcher(p, dev)
    m.raw_and_support(torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev))
    cin = torch.empty_like(m.c0)
    K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=cin)  # a realistic H input
    ref = torch.empty_like(cin)
    K.asw_hCostAggregation(p, m.whl, m.whr, cin, out=ref)
    torch.cuda.synchronize()
    print("prod", K.pass_kernel(1, 0), flush=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_h32.so"))
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    pp = ctypes.byref(p)
    out = torch.empty_like(cin)
    runs = [tuple(int(v) for v in r.split(":")) for r in args.runs.split(",")]
    st = torch.cuda.current_stream()

    def launch(form, nseg):
        if form < 0:
            K.asw_hCostAggregation(p, m.whl, m.whr, cin, out=out)
            return
        rc = lib.exp_h32(form, nseg, 0, pp, P(m.whl), P(m.whr), P(cin), P(out), None, ctypes.c_void_p(st.cuda_stream))
        assert rc == 0, (form, nseg, rc)

    runs = [(-1, 0)] + runs
    for form, nseg in runs:
        out.zero_()
        launch(form, nseg)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), f"form {form} nseg {nseg}: not bit-exact"
    print("all forms bit-exact", flush=True)
    times = {r: [] for r in runs}
    for rep in range(args.reps + 2):
        for r in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch(*r)
            e1.record()
            e1.synchronize()
            if rep >= 2:
                times[r].append(e0.elapsed_time(e1))
    for (form, nseg), t in times.items():
        t.sort()
        print(json.dumps({"form": "prod" if form < 0 else form, "nseg": nseg, "ms_median": round(t[len(t) // 2], 4),
                          "ms_min": round(t[0], 4)}), flush=True)


if __name__ == "__main__":
    main()
