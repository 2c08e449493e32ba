"""Drives tools/exp/libexp.so (experimental pass kernels) on the real C4 inputs and
checks every experiment bit-exact against the production pass.  Not part of the product.

    python tools/exp/exp_bench.py [--reps 8]
"""
import argparse
import ctypes
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
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--v", action="store_true", help="V-pass experiments")
    ap.add_argument("--lib", default="libexp.so")
    ap.add_argument("--c5", action="store_true", help="C5 block-shape experiments (T = 51)")
    ap.add_argument("--c5s", default="", help="C5 V strip experiments: nstrip:kbi,... (libexp_c5s.so)")
    ap.add_argument("--c5libs", default="libexp_c5_1641.so:1641")
    ap.add_argument("--vexps", default="prod_read,v12_read,prod_none")
    ap.add_argument("--h", action="store_true", help="H-pass experiments")
    ap.add_argument("--vprobe", default="", help="V resource probes dm:probe,... (libexp_vprobe.so)")
    ap.add_argument("--vdma", default="", help="LDS-DMA V pass forms f,... (libexp_vdma.so)")
    ap.add_argument("--hwta", default="", help="fused-WTA H pass variants vg,... (libexp_hwta.so)")
    args = ap.parse_args()
    W, H, D, T = (3840, 2160, 512, 51) if args.c5 else (1920, 1080, 256, 35)
    dev = torch.device("cuda:0")
    Lh, Rh, _ = make_pair(W, H, D, 0)
    p = make_params(W, H, ndisp=D, taps=T, iters=7, flags=_lib.FLAG_RAW_F32)  # c0 = the float raw costs
    m = StereoMatcher(p, dev)
    m.raw_and_support(torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev))
    # a realistic H input: one V pass of the raw cost
    cin = torch.empty_like(m.c0)
    K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=cin)
    den = torch.empty_like(cin)
    ref = torch.empty_like(cin)
    K.asw_hCostAggregation(p, m.whl, m.whr, cin, out=ref, den=den, den_mode=1)
    torch.cuda.synchronize()
    lib = None if args.c5 or args.lib == "none" else ctypes.CDLL(os.path.join(ROOT, "tools", "exp", args.lib))
    pp = ctypes.byref(p)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = torch.empty_like(cin)

    def h(nkw, dm, kbg0, nkbg, st):
        rc = lib.exp_h11(nkw, dm, pp, P(m.whl), P(m.whr), P(cin), P(out), P(den), kbg0, nkbg,
                         ctypes.c_void_p(st.cuda_stream))
        assert rc == 0, rc

    if args.c5 and not args.v:
        # V den-read at T = 51: production pass against k_vpass10 shapes, one library each
        # (--c5libs lib:shape,...; shape = NW*100 + NPH*10 + RB)
        cur = torch.cuda.current_stream().cuda_stream
        exps = [(lb, int(sh)) for lb, sh in (x.split(":") for x in args.c5libs.split(","))] if not args.c5s else []
        libs = {lb: ctypes.CDLL(os.path.join(ROOT, "tools", "exp", lb)) for lb, _ in exps}
        if args.c5s:  # (nstrip, kbi) pairs through libexp_c5s.so, shape code = nstrip * 10 + kbi
            ls = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_c5s.so"))
            for x in args.c5s.split(","):
                ns, kb = (int(v) for v in x.split(":"))
                libs[f"s{ns}:{kb}"] = ls
                exps.append((f"s{ns}:{kb}", ns * 10 + kb))
        den_d = torch.empty_like(cin)
        ref_d = torch.empty_like(cin)
        K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=ref_d, den=den_d, den_mode=1)
        K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=ref_d, den=den_d, den_mode=2)
        torch.cuda.synchronize()
        print("prod", K.pass_kernel(0, 2), flush=True)
        res = {}
        for rep in range(args.reps + 1):
            for lb, sh in [(None, 0)] + exps:
                out.zero_()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if lb is None:
                    K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=out, den=den_d, den_mode=2)
                elif lb.startswith("s"):
                    assert libs[lb].exp_c5s(sh // 10, sh % 10, pp, P(m.wvl), P(m.wvr), P(m.c0), P(out), P(den_d),
                                            ctypes.c_void_p(cur)) == 0
                else:
                    assert libs[lb].exp_c5(0, sh, 2, pp, P(m.wvl), P(m.wvr), P(m.c0), P(out), P(den_d),
                                           ctypes.c_void_p(cur)) == 0
                e1.record()
                torch.cuda.synchronize()
                name = f"v_read_{sh or 'prod'}"
                if rep == 0:
                    if not torch.equal(out, ref_d):
                        print(json.dumps({"exp": name, "error": "differs"}), flush=True)
                else:
                    res.setdefault(name, []).append(e0.elapsed_time(e1))
        for name, ts in res.items():
            print(json.dumps({"exp": name, "ms_median": round(float(np.median(ts)), 4)}), flush=True)
        return
    if args.hwta:
        # the last H pass with the WTA's own scan fused (asw_hwta.h) against the production
        # den-read H pass + asw_wta_local, bit-exact (volume, key, m1, m2); then the frame's
        # WTA tail both ways: asw_WTA (k_wta_scan: own + target scan) against the fused
        # pass's scan + asw_wta_target_local + asw_wta_finalize
        lx = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_hwta.so"))
        key_r, m1_r, m2_r = K.wta_local(p, ref)
        Hh, Wh = p.height, p.width
        key = torch.empty((Hh, Wh), dtype=torch.int64, device=dev)
        m1 = torch.empty((Hh, Wh), dtype=torch.float32, device=dev)
        m2 = torch.empty((Hh, Wh), dtype=torch.float32, device=dev)
        wta_ref = K.asw_WTA(p, ref)
        torch.cuda.synchronize()
        vgs = [int(v) for v in args.hwta.split(",")]
        res = {}
        cur = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
        for rep in range(args.reps + 1):
            cases = [("h_read_prod", None)] + [(f"h_read_wta_vg{v}", v) for v in vgs]
            for name, vg in cases:
                out.zero_()
                key.zero_()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if vg is None:
                    K.asw_hCostAggregation(p, m.whl, m.whr, cin, out=out, den=den, den_mode=2)
                else:
                    rc = lx.exp_hwta(vg, pp, P(m.whl), P(m.whr), P(cin), P(out), P(den), P(key), P(m1), P(m2), cur())
                    assert rc == 0, (name, rc)
                e1.record()
                torch.cuda.synchronize()
                if rep == 0:
                    ok = bool(torch.equal(out, ref))
                    if vg is not None:
                        ok = ok and bool(torch.equal(key, key_r)) and bool(torch.equal(m1, m1_r)) and \
                            bool(torch.equal(m2, m2_r))
                        got = K.wta_from_local(p, out, key, m1, m2)
                        ok = ok and all(bool(torch.equal(a_, b_)) for a_, b_ in zip(got, wta_ref))
                    print(json.dumps({"exp": name, "bit_exact": ok}), flush=True)
                else:
                    res.setdefault(name, []).append(e0.elapsed_time(e1))
            # the WTA tails on the same volume
            for name in ("wta_scan", "wta_target_finalize"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if name == "wta_scan":
                    K.asw_WTA(p, ref)
                else:
                    K.wta_from_local(p, ref, key_r, m1_r, m2_r)
                e1.record()
                torch.cuda.synchronize()
                if rep:
                    res.setdefault(name, []).append(e0.elapsed_time(e1))
        for name, ts in res.items():
            print(json.dumps({"exp": name, "ms_median": round(float(np.median(ts)), 4), "ms_min": round(min(ts), 4)}),
                  flush=True)
        return
    if args.vdma:
        # the LDS-DMA-staged V pass (asw_vdma.h) against the production pass, every den mode:
        # bit-exact outputs (and den-write's den), then median times
        lx = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_vdma.so"))
        denv = torch.empty_like(cin)
        refv = torch.empty_like(cin)
        K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=refv, den=denv, den_mode=1)
        denw = torch.empty_like(cin)
        torch.cuda.synchronize()
        forms = [int(f) for f in args.vdma.split(",")]
        cases = [("prod", dm, None) for dm in (0, 1, 2)] + [(f"vdma{f}", dm, f) for f in forms for dm in (0, 1, 2)]
        res = {}
        for rep in range(args.reps + 1):
            for name, dm, f in cases:
                out.zero_()
                torch.cuda.synchronize()
                dbuf = denw if dm == 1 else denv
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if f is None:
                    K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=out, den=dbuf if dm else None, den_mode=dm)
                else:
                    rc = lx.exp_vdma(f, dm, pp, P(m.wvl), P(m.wvr), P(m.c0), P(out), P(dbuf),
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0, (name, dm, rc)
                e1.record()
                torch.cuda.synchronize()
                if rep == 0:
                    ok = bool(torch.equal(out, refv)) and (dm != 1 or bool(torch.equal(denw, denv)))
                    rec = {"exp": name, "dm": dm, "bit_exact": ok}
                    if not ok:
                        bad = (out != refv).nonzero()
                        rec.update(n=int(bad.shape[0]), first=bad[:4].tolist())
                    print(json.dumps(rec), flush=True)
                else:
                    res.setdefault((name, dm), []).append(e0.elapsed_time(e1))
        for (name, dm), ts in res.items():
            print(json.dumps({"exp": name, "dm": dm, "ms_median": round(float(np.median(ts)), 4),
                              "ms_min": round(min(ts), 4)}), flush=True)
        return
    if args.vprobe:
        # k_vpass10 resource probes (asw_vprobe.h): probe 0 must equal the production pass,
        # the others are timed only
        lx = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_vprobe.so"))
        denv = torch.empty_like(cin)
        refv = torch.empty_like(cin)
        K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=refv, den=denv, den_mode=1)
        torch.cuda.synchronize()
        # "dm:probe" (k_vprobe) or "kd:N" (the den-read pass with an N-row den prefetch ring)
        cases = [("prod", 0, None), ("prod", 2, None)]
        for x in args.vprobe.split(","):
            a, b = x.split(":")
            cases.append((f"kd{b}", 2, -int(b)) if a == "kd" else (f"probe{b}", int(a), int(b)))
        res = {}
        for rep in range(args.reps + 1):
            for name, dm, pr in cases:
                out.zero_()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if pr is None:
                    K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=out, den=denv if dm else None, den_mode=dm)
                elif pr < 0:
                    rc = lx.exp_vkd(-pr, pp, P(m.wvl), P(m.wvr), P(m.c0), P(out), P(denv),
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0, (name, rc)
                else:
                    rc = lx.exp_vprobe(pr, dm, pp, P(m.wvl), P(m.wvr), P(m.c0), P(out), P(denv),
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0, (name, dm, rc)
                e1.record()
                torch.cuda.synchronize()
                if rep == 0 and (pr is None or pr <= 0 or pr & 128):  # (128: the staggered form, exact)
                    print(json.dumps({"exp": name, "dm": dm, "bit_exact": bool(torch.equal(out, refv))}), flush=True)
                elif rep:
                    res.setdefault((name, dm), []).append(e0.elapsed_time(e1))
        for (name, dm), ts in res.items():
            print(json.dumps({"exp": name, "dm": dm, "ms_median": round(float(np.median(ts)), 4),
                              "ms_min": round(min(ts), 4)}), flush=True)
        return
    # V pass experiments: the production den-write pass gives den_v, the production
    # den-read pass the reference output
    if args.v:
        denv = torch.empty_like(cin)
        denw = torch.empty_like(cin)
        refv = torch.empty_like(cin)
        K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=refv, den=denv, den_mode=1)
        torch.cuda.synchronize()
        vres = {}
        pxlibs = {}
        allv = {"prod_read": (None, 2, 0), "prod_none": (None, 0, 0), "prod_write": (None, 1, 0),
                "v12_read": (12, 2, 0), "v12_read_s1": (12, 2, 1), "v12_read_s3": (12, 2, 3),
                "v12_none": (12, 0, 0), "v12_write": (12, 1, 0),
                "vpx0": ("px0", 2, 0), "vpx4": ("px4", 2, 0), "vpx8": ("px8", 2, 0),
                "vpx_e": ("px_e", 2, 0), "vpx_f": ("px_f", 2, 0), "vpx_g": ("px_g", 2, 0),
                # round 4: 8-column blocks at 4 waves per SIMD (two blocks per CU)
                "vpx_n8w4": ("px_n8w4", 2, 0),
                # round 5: XCD-round tiles of TK plane blocks x 32/TK column groups (libexp_vtile.so)
                "vtile1": (("tile", 1), 2, 0), "vtile2": (("tile", 2), 2, 0), "vtile4": (("tile", 4), 2, 0),
                "vtile8": (("tile", 8), 2, 0)}
        vexps = [(n,) + allv[n] for n in args.vexps.split(",")]
        for rep in range(args.reps + 1):
            for name, kind, dm, ns in vexps:
                out.zero_()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if kind is None:
                    K.asw_vCostAggregation(p, m.wvl, m.wvr, m.c0, out=out, den=denv if dm else None, den_mode=dm)
                elif isinstance(kind, tuple):  # k_vpass10 in XCD-round tiles (libexp_vtile.so)
                    lx = pxlibs.setdefault("tile", ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_vtile.so")))
                    rc = lx.exp_vtile(kind[1], pp, P(m.wvl), P(m.wvr), P(m.c0), P(out), P(denv),
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0, rc
                elif isinstance(kind, str):  # k_vpass10 with extra cost prefetch (libexp_vpx<N>.so)
                    lx = pxlibs.setdefault(kind, ctypes.CDLL(os.path.join(ROOT, "tools", "exp", f"libexp_v{kind}.so")))
                    rc = lx.exp_vpx(dm, pp, P(m.wvl), P(m.wvr), P(m.c0), P(out), P(denv),
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0, rc
                else:
                    # den-write experiments write a scratch den (compared below), never denv
                    rc = lib.exp_v12(0, dm, ns, pp, P(m.wvl), P(m.wvr), P(m.c0), P(out),
                                     P(denw if dm == 1 else denv),
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0, rc
                e1.record()
                torch.cuda.synchronize()
                if rep == 0:
                    if dm == 1 and kind is not None and not torch.equal(denw, denv):
                        print(json.dumps({"exp": name, "error": "den differs"}), flush=True)
                    if not torch.equal(out, refv):
                        bad = (out != refv).nonzero()
                        print(json.dumps({"exp": name, "error": "differs", "n": int(bad.shape[0]),
                                          "first": bad[:4].tolist()}), flush=True)
                else:
                    vres.setdefault(name, []).append(e0.elapsed_time(e1))
        for name, ts in vres.items():
            print(json.dumps({"exp": name, "ms_median": round(float(np.median(ts)), 4), "ms_min": round(min(ts), 4)}),
                  flush=True)
        if not args.h:
            return
    nkb = 4
    exps = {
        "read_nkw4": [(4, 2, 0, 1, 0)],
        "none_nkw4": [(4, 0, 0, 1, 0)],
        "read_nkw1": [(1, 2, 0, 4, 0)],
        "none_nkw1": [(1, 0, 0, 4, 0)],
        "mix2_nkw2_2streams": [(2, 2, 0, 1, 0), (2, 0, 1, 1, 1)],
        "mix2_nkw2_serial": [(2, 2, 0, 1, 0), (2, 0, 1, 1, 0)],
        "mix3r1n_nkw1_2streams": [(1, 2, 0, 3, 0), (1, 0, 3, 1, 1)],
        "mix1r3n_nkw1_2streams": [(1, 2, 0, 1, 0), (1, 0, 1, 3, 1)],
        "mix2_nkw1_2streams": [(1, 2, 0, 2, 0), (1, 0, 2, 2, 1)],
    }
    del nkb
    res = {k: [] for k in exps}
    cur = torch.cuda.current_stream()
    for rep in range(args.reps + 1):
        for name, launches in exps.items():
            out.zero_()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            for st in (s1, s2):
                st.wait_event(e0)
            for nkw, dm, kbg0, nkbg, si in launches:
                h(nkw, dm, kbg0, nkbg, (s1, s2)[si])
            for st in (s1, s2):
                cur.wait_stream(st)
            e1.record(cur)
            torch.cuda.synchronize()
            if rep == 0:
                ok = torch.equal(out, ref)
                if not ok:
                    print(json.dumps({"exp": name, "error": "differs from the production pass"}), flush=True)
            else:
                res[name].append(e0.elapsed_time(e1))
    for name, ts in res.items():
        print(json.dumps({"exp": name, "ms_median": round(float(np.median(ts)), 4), "ms_min": round(min(ts), 4)}),
              flush=True)


if __name__ == "__main__":
    main()
