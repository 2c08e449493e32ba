"""Checks and times the measured-negative forms kept in tools/exp/libforms.so
(exp_forms.hip) against the shipped ones of libasw_hip.so, bit for bit.  GPU only;
not part of the product (their tests moved here with them).

    make -C tools/exp libforms.so && python tools/exp/exp_forms.py [--reps 10]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from stereo_matchin_amd import make_params  # noqa: E402
from stereo_matchin_amd import kernels as K  # noqa: E402
from stereo_matchin_amd.synthetic import make_pair  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(HERE, "libforms.so"))
    vp = ctypes.c_void_p
    lib.forms_support_expd.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                       ctypes.c_float, vp]
    lib.forms_wta_wave.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp]
    dev = torch.device("cuda:0")
    ok = True
    # k_support's EXPD form, T = 35 (C4) and 51 (C5)
    for (W, H, D, T) in ((1920, 1080, 256, 35), (3840, 2160, 512, 51)):
        Lh, _, _ = make_pair(W, H, D, 0)
        p = make_params(W, H, ndisp=D, taps=T)
        img = torch.from_numpy(Lh).to(dev)
        lut = K.support_lut(p, dev)
        for direction in (0, 1):
            f = K.asw_vSupport if direction == 0 else K.asw_hSupport
            ref = f(p, img, lut)
            got = torch.empty_like(ref)
            run = lambda: lib.forms_support_expd(img.data_ptr(), got.data_ptr(), W, H, T, direction,  # noqa: E731
                                                 p.gamma_c, p.gamma_g, None)
            assert run() == 0
            torch.cuda.synchronize()
            same = bool(torch.equal(got, ref))
            ok &= same
            t_expd = timed(run, a.reps)
            t_lut = timed(lambda: f(p, img, lut, out=ref), a.reps)
            print(json.dumps({"form": "k_support EXPD", "W": W, "H": H, "T": T, "dir": direction, "bit_exact": same,
                              "ms_expd": round(t_expd, 4), "ms_shipped_lut": round(t_lut, 4)}), flush=True)
    # the wave-per-pixel asw_WTA against the shipped scan: tie-heavy random volumes and a C4-size one
    rng = np.random.default_rng(7)
    for (H, W, D) in ((5, 67, 61), (13, 129, 256), (3, 200, 300), (2, 700, 128), (1080, 1920, 256)):
        p = make_params(W, H, ndisp=D, taps=3)
        Dp = K.cost_shape(p)[2]
        vol = np.zeros((H, W, Dp), np.float32)
        vol[..., :D] = rng.integers(1, 9, (H, W, D)).astype(np.float32)
        cost = torch.from_numpy(vol).to(dev)
        ref = K.asw_WTA(p, cost)
        outs = [torch.empty((H, W), dtype=dt, device=dev) for dt in (torch.int32, torch.float32, torch.int32,
                                                                      torch.float32)]
        run = lambda: lib.forms_wta_wave(cost.data_ptr(), W, H, Dp, D, *[o.data_ptr() for o in outs], None)  # noqa: E731
        assert run() == 0
        torch.cuda.synchronize()
        same = all(bool(torch.equal(g, r)) for g, r in zip(outs, ref[:4]))
        ok &= same
        line = {"form": "asw_WTA wave per pixel", "H": H, "W": W, "D": D, "bit_exact": same}
        if H * W >= 1 << 20:
            line["ms_wave"] = round(timed(run, a.reps), 4)
            line["ms_shipped_scan"] = round(timed(lambda: K.asw_WTA(p, cost), a.reps), 4)
        print(json.dumps(line), flush=True)
    print(json.dumps({"all_bit_exact": ok}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
