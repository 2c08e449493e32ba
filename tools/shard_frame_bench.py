"""One rank's share of a d-sharded C4 frame on one GPU (no collective: the MIN
all-reduces are identities without torch.distributed), for rocprofv3 kernel stats
of the sharded WTA kernels and the replicated side kernels.

    python tools/shard_frame_bench.py [--world 4] [--rank 1] [--reps 5] [--variants 0,3145728 --rounds 2]

--variants: asw_tune_set(ASW_TUNE_PASS_VARIANT) values, timed in turn (interleaved over
--rounds) on one matcher, one JSON line each.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereo_matchin_amd import make_params  # noqa: E402
from stereo_matchin_amd.distributed import PipelinedMatcher, ShardedStereoMatcher  # noqa: E402
from stereo_matchin_amd.synthetic import make_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--workload", default="c4", choices=["c4", "c5"],
                    help="c4: 1920x1080 D256 T35; c5: 3840x2160 D512 T51 (native LR)")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--pipeline", default="",
                    help="also time the frames streamed through distributed.PipelinedMatcher (2 sets of volumes, "
                         "the tail on a side stream): comma list of overlap_prep values, e.g. 0,1")
    ap.add_argument("--flags", default="0",
                    help="asw_params.flags values (ASW_FLAG_*), timed in turn like the variants, e.g. 0,64 "
                         "(64 = ASW_FLAG_RAW_F32: the float raw-cost volume)")
    ap.add_argument("--rounds", type=int, default=1)
    a = ap.parse_args()
    from stereo_matchin_amd import _lib
    lib = _lib.lib()
    dev = torch.device("cuda:0")
    W, H, D, T, r = (1920, 1080, 256, 35, 7) if a.workload == "c4" else (3840, 2160, 512, 51, 7)
    Lh, Rh, _ = make_pair(W, H, D, 0)
    L, R = torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev)
    ms_ = {}
    for f in [int(x) for x in a.flags.split(",")]:
        p = make_params(W, H, ndisp=D, taps=T, iters=r, lr_check=1, lr_mode=1 if D > 256 else 0, flags=f)
        ms_[f] = ShardedStereoMatcher(p, a.rank, a.world, dev)
    for _ in range(a.rounds):
        for v, f in [(int(x), f) for x in a.variants.split(",") for f in ms_]:
            m = ms_[f]
            old = lib.asw_tune_set(1, v)
            m.match(L, R)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                m.match(L, R)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.reps
            lib.asw_tune_set(1, old)
            print(json.dumps({"workload": a.workload, "world": a.world, "rank": a.rank,
                              "planes": m.p.d_stop - m.p.d_begin, "variant": v, "flags": f,
                              "raw16": m.matcher.raw16,
                              "ms_per_shard_frame_no_collective": round(ms, 3)}), flush=True)
    # streamed frames (what bench.py --gpus N runs per rank), per overlap_prep value
    for ov in [int(x) for x in a.pipeline.split(",") if x != ""]:
        p = make_params(W, H, ndisp=D, taps=T, iters=r, lr_check=1, lr_mode=1 if D > 256 else 0)
        pm = PipelinedMatcher(p, a.rank, a.world, dev, overlap_prep=bool(ov))
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for _ in range(2):
                pm.submit(L, R)
            pm.flush()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                pm.submit(L, R)
            pm.flush()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.reps
            print(json.dumps({"workload": a.workload, "world": a.world, "rank": a.rank, "pipelined": True,
                              "overlap_prep": ov, "planes": pm.p.d_stop - pm.p.d_begin,
                              "ms_per_shard_frame_no_collective": round(ms, 3)}), flush=True)
        del pm


if __name__ == "__main__":
    main()
