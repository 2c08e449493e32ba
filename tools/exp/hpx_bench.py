"""k_hpass11 den-read with a deeper cost prefetch (tools/exp/libexp_hpx.so, EXP_HPX in
exp_lib.hip): each form checked bit-exact against the production pass, then timed.
Not part of the product.

    python tools/exp/hpx_bench.py --c5 [--reps 10] [--forms 0,1,2,3,4]
    python tools/exp/hpx_bench.py [--forms 10,11]          (C4)
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
    ap.add_argument("--c5", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--forms", default="")
    args = ap.parse_args()
    W, H, D, T = (3840, 2160, 512, 51) if args.c5 else (1920, 1080, 256, 35)
    forms = [int(f) for f in (args.forms or ("0,1,2,3,4" if args.c5 else "10,11")).split(",")]
    dev = torch.device("cuda:0")
    Lh, Rh, _ = make_pair(W, H, D, 0)
    p = make_params(W, H, ndisp=D, taps=T, iters=7, flags=_lib.FLAG_RAW_F32)
    m = StereoMatcher(p, dev)
    m.raw_and_support(torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev))
    cin = torch.empty_like(m.c0)
    K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=cin)  # a realistic H input
    del m.c1
    den = torch.empty_like(cin)
    ref = m.c0  # (the raw volume is not needed any more)
    K.asw_hCostAggregation(p, m.whl, m.whr, cin, out=ref, den=den, den_mode=1)
    K.asw_hCostAggregation(p, m.whl, m.whr, cin, out=ref, den=den, den_mode=2)
    torch.cuda.synchronize()
    print("prod", K.pass_kernel(1, 2), flush=True)
    wform = any(f >= 20 for f in forms)  # den-write forms (libexp_hpxw.so): out and den checked
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_hpxw.so" if wform else "libexp_hpx.so"))
    if wform:
        ref_w, den_ref = torch.empty_like(cin), torch.empty_like(cin)
        K.asw_hCostAggregation(p, m.whl, m.whr, cin, out=ref_w, den=den_ref, den_mode=1)
        ref, den_o = ref_w, torch.empty_like(cin)
        del ref_w
        torch.cuda.synchronize()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    pp = ctypes.byref(p)
    out = torch.empty_like(cin)
    st = torch.cuda.current_stream()

    def launch(f):
        if f < 0 and wform:
            K.asw_hCostAggregation(p, m.whl, m.whr, cin, out=out, den=den_o, den_mode=1)
        elif f < 0:
            K.asw_hCostAggregation(p, m.whl, m.whr, cin, out=out, den=den, den_mode=2)
        elif wform:
            rc = lib.exp_hpxw(f, pp, P(m.whl), P(m.whr), P(cin), P(out), P(den_o), ctypes.c_void_p(st.cuda_stream))
            assert rc == 0, (f, rc)
        else:
            rc = lib.exp_hpx(f, pp, P(m.whl), P(m.whr), P(cin), P(out), P(den), ctypes.c_void_p(st.cuda_stream))
            assert rc == 0, (f, rc)

    runs = [-1] + forms
    for f in runs:
        out.zero_()
        launch(f)
        torch.cuda.synchronize()
        ok = bool(torch.equal(out, ref)) and (not wform or bool(torch.equal(den_o, den_ref)))
        print(json.dumps({"form": "prod" if f < 0 else f, "bit_exact": ok}), flush=True)
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
