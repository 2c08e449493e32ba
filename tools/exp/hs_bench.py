"""Half-size tap-major supports on the C4 8-way shard V pass (tools/exp/libexp_hs.so,
EXP_HS in exp_lib.hip).  Checks the half arrays rebuild the full
ones element for element (symmetry + border rule of hs_index), k_vpass32<HS> bit-exact
against the production pass, then times both.  Not part of the product.

    python tools/exp/hs_bench.py [--reps 30]
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
    args = ap.parse_args()
    W, H, D, T = 1920, 1080, 256, 35
    R = T // 2
    dev = torch.device("cuda:0")
    Lh, Rh, _ = make_pair(W, H, D, 0)
    p = make_params(W, H, ndisp=D, taps=T, iters=7, flags=_lib.FLAG_RAW_F32)
    p.d_begin, p.d_end = 0, 32
    m = StereoMatcher(p, dev)
    m.raw_and_support(torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev))
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_hs.so"))
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    pp = ctypes.byref(p)
    st = torch.cuda.current_stream()
    cs = ctypes.c_void_p(st.cuda_stream)
    halves = []
    for full in (m.wvl, m.wvr):
        h = torch.empty(H * (R + 1) * W, dtype=torch.float32, device=dev)
        assert lib.exp_hs_convert(0, P(full), P(h), W, H, cs) == 0
        back = torch.empty_like(full)
        assert lib.exp_hs_convert(1, P(h), P(back), W, H, cs) == 0
        torch.cuda.synchronize()
        nbad = int((back.view(-1) != full.view(-1)).sum())
        print(json.dumps({"check": "half rebuilds full", "mismatches": nbad, "bytes_full": full.numel() * 4,
                          "bytes_half": h.numel() * 4}), flush=True)
        assert nbad == 0
        halves.append(h)
    hl, hr = halves
    ref = torch.empty_like(m.c0)
    K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=ref)
    torch.cuda.synchronize()
    print("prod", K.pass_kernel(0, 0), flush=True)
    out = torch.empty_like(ref)

    def launch(form):
        if form == "prod":
            K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=out)
        elif form == "full":
            assert lib.exp_v32hs(0, pp, P(m.wvl), P(m.wvr), P(m.c0), P(out), cs) == 0
        else:
            assert lib.exp_v32hs(1, pp, P(hl), P(hr), P(m.c0), P(out), cs) == 0

    forms = ["prod", "full", "half"]
    for f in forms:
        out.zero_()
        launch(f)
        torch.cuda.synchronize()
        ok = bool(torch.equal(out, ref))
        print(json.dumps({"form": f, "bit_exact": ok}), flush=True)
    times = {f: [] for f in forms}
    for rep in range(args.reps + 2):
        for f in forms:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch(f)
            e1.record()
            e1.synchronize()
            if rep >= 2:
                times[f].append(e0.elapsed_time(e1))
    for f, t in times.items():
        t.sort()
        print(json.dumps({"form": f, "ms_median": round(t[len(t) // 2], 4), "ms_min": round(t[0], 4)}), flush=True)


if __name__ == "__main__":
    main()
