"""Benchmark of the MI355X ASW stereo hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c2|c3|c5]

One step = one disparity map per frame group: raw cost -> 4 support launches ->
r x (V, H) aggregation passes -> WTA (+ target map) -> LR consistency, on a
synthetic stereo pair already resident in HBM (main.cpp:463-537 minus the
refinement loop, the span of SURVEY §8d).  N > 1 GPUs (one process per GPU,
launched by torch.distributed.run) shard the disparity axis of a frame over a
group of G ranks with RCCL MIN all-reduces for the WTA; G = plan_groups(D, N)
keeps >= 64 planes per rank (the pass kernels' plane block), so D=256 runs one
frame on 2 or 4 GPUs ("scaling": "strong") and two concurrent frames, each
d-sharded 4 ways, on 8 GPUs ("weak" from 4 to 8: the per-GPU share stays 1/4
frame).  `value` counts every frame all groups finished.

Rank 0 prints ONE JSON line.  ``roofline`` is the aggregation pass (the dominant
kernel, 94 % of the reference's ASW time): algorithmic bytes per launch
``8*n*S + 8*T*S`` (read + write the n local cost planes, read both support
arrays) over the launch's average duration from HIP events recorded
on the stream the passes run on, inside the timed region.  ``cpu_baseline`` is the
CPU oracle (oracle/, a scalar-semantics C/OpenMP restatement of the reference
kernels) timed on this host on a bounded strip of the same frame.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "disparity maps/sec + ms/frame, 1920×1080 d=256 ASW win=35, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

WORKLOADS = {
    # name: (W, H, D, T, iters, lr, description)
    "c4": (1920, 1080, 256, 35, 7, True, "C4 synthetic 1920x1080 d=256 win=35 r=7 + LR check"),
    "c2": (450, 375, 64, 35, 7, False, "C2-size synthetic 450x375 d=64 win=35 r=7"),
    "c3": (450, 375, 64, 35, 7, True, "C3-size synthetic 450x375 d=64 win=35 r=7 + LR check"),
    "c5": (3840, 2160, 512, 51, 7, True, "C5 synthetic 3840x2160 d=512 win=51 r=7 + LR check (1 pair/step)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-rows", type=int, default=128, help="rows of the frame timed on the CPU oracle (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(HERE, "profiles", "traffic.json"))
    ap.add_argument("--group-size", type=int, default=0,
                    help="ranks per d-sharded frame (0: plan_groups, >= 64 planes per rank)")
    return ap.parse_args()


def cpu_baseline(Lh, Rh, D, T, iters, rows):
    """Oracle (oracle/asw_oracle.c, OpenMP) on rows [0, rows) of the frame, scaled to a full frame."""
    from oracle import oracle as O
    threads = O.set_threads(0)
    H = Lh.shape[0]
    rows = min(rows, H)
    Ls, Rs = np.ascontiguousarray(Lh[:rows]), np.ascontiguousarray(Rh[:rows])
    t0 = time.perf_counter()
    O.match(Ls, Rs, D, T, iters)
    dt = time.perf_counter() - t0
    frame_s = dt * H / rows
    return {
        "value": round(1.0 / frame_s, 6), "unit": "maps/s", "cores": int(threads), "kind": "port",
        "sample": f"{Lh.shape[1]}x{rows} strip (rows 0-{rows - 1}) of the same frame, full pipeline r={iters}, "
                  f"{dt:.2f} s measured, scaled x{H}/{rows} to one map; {frame_s * 1000:.0f} ms/map",
    }


def load_traffic(path, workload, n_gpus):
    try:
        with open(path) as f:
            t = json.load(f)
        e = t.get(f"{workload}_n{n_gpus}")
        return None if e is None else e.get("hbm_bytes_per_pass")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} (launch N>1 with torch.distributed.run)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from stereo_matchin_amd import make_params
    from stereo_matchin_amd.distributed import ShardedStereoMatcher, plan_groups
    from stereo_matchin_amd.pipeline import StereoMatcher
    from stereo_matchin_amd.synthetic import make_pair

    W, H, D, T, iters, lr, desc = WORKLOADS[args.workload]
    G = args.group_size or plan_groups(D, world)
    if world % G != 0:
        raise SystemExit(f"--group-size {G} does not divide {world} ranks")
    groups, gid, grank = world // G, rank // G, rank % G
    pg = None
    if world > 1 and G > 1:
        # every rank creates every group, in the same order (torch.distributed rule)
        subs = [dist.new_group(list(range(g * G, (g + 1) * G))) for g in range(groups)]
        pg = subs[gid]
    Lh, Rh, _ = make_pair(W, H, D, gid)  # one synthetic pair per group
    L = torch.from_numpy(Lh).to(dev)
    R = torch.from_numpy(Rh).to(dev)
    p = make_params(W, H, ndisp=D, taps=T, iters=iters, lr_check=int(lr))
    if G > 1:
        m = ShardedStereoMatcher(p, grank, G, dev, group=pg)
        nloc = m.p.d_stop - m.p.d_begin
    else:
        m = StereoMatcher(p, dev)
        nloc = D

    def step(events=None):
        return m.match(L, R, events=events)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    evs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ev = []
        step(ev)
        evs.append(ev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    torch.cuda.synchronize()

    # per-launch aggregation-pass durations from the events around each pass
    v_ms, h_ms, frame_ms = [], [], []
    for ev in evs:
        prev = dict(ev)["support"]
        for name, e in ev:
            if name in ("v", "h"):
                (v_ms if name == "v" else h_ms).append(prev.elapsed_time(e))
                prev = e
        frame_ms.append(ev[0][1].elapsed_time(ev[-1][1]))
    pass_ms = float(np.mean(v_ms + h_ms))
    stats = torch.tensor([elapsed, pass_ms, float(np.mean(v_ms)), float(np.mean(h_ms))], dtype=torch.float64,
                         device=dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    elapsed, pass_ms, v_avg, h_avg = stats.tolist()

    if rank == 0:
        S = W * H
        bytes_per_pass = 8 * nloc * S + 8 * T * S
        achieved = bytes_per_pass / (pass_ms * 1e-3) / 1e9
        maps_per_s = groups * args.steps / elapsed
        out = {
            "metric": METRIC,
            "value": round(maps_per_s, 4),
            "unit": "maps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000, 4),
            "higher_is_better": True,
            "scaling": "strong" if groups == 1 else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": desc, "width": W, "height": H, "ndisp": D, "taps": T, "iters": iters,
                       "lr_check": lr, "local_planes": nloc, "frames_per_step": groups,
                       "parallelism": (f"{groups} frame(s) per step, each d-sharded over {G} GPU(s)"
                                       if world > 1 else "single GPU")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(args.traffic, args.workload, world),
                         "kernel": "aggregation pass (k_vpass/k_hpass), mean over all V+H launches",
                         "bytes_per_launch": bytes_per_pass, "avg_launch_ms": round(pass_ms, 4),
                         "v_avg_ms": round(v_avg, 4), "h_avg_ms": round(h_avg, 4)},
            "frame_ms_events": round(float(np.median(frame_ms)), 4),
        }
        if world == 1 and not args.no_cpu and args.cpu_rows > 0:
            out["cpu_baseline"] = cpu_baseline(Lh, Rh, D, T, iters, args.cpu_rows)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
