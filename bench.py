"""Benchmark of the MI355X ASW stereo hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c1|c2|c3|c5] [--api stage|frame]

One step = one disparity map per frame group (C5: a batch of 8 pairs): raw cost
-> 4 support launches -> r x (V, H) aggregation passes -> WTA (+ target map) ->
LR consistency, on a synthetic stereo pair already resident in HBM
(main.cpp:463-537 minus the refinement loop, the span of SURVEY §8d).  C1 is the
reference's own Tsukuba pair (tests/golden/tsukuba.npz), D16 T5.

``--api frame`` times the C-ABI drop-in instead (asw_create + asw_match, host
RGBA8 in, host maps out, as main.cpp's replacement would call it): ``value``
stays the device-resident rate (the sum of asw_match's own HIP-event spans,
h2d end -> consistency end), the PCIe-inclusive wall rate is reported beside it.  N > 1 GPUs (one process per GPU,
launched by torch.distributed.run) shard the disparity axis of ONE frame over all
N ranks with RCCL MIN all-reduces for the WTA (BASELINE.json config 4: "d-axis
sharded across 8x MI355X via RCCL"; at N = 8 each rank owns 32 of the 256 planes
and runs the half-wave passes of asw_pass32.h): "scaling": "strong", the frame's
total work is fixed.  ``--group-size G`` splits the N ranks into N/G concurrent
frames of G shards instead; without it, the layout with the most maps/s,
plan_groups(D, N) ranks per frame, is timed after the main run and reported beside
``value`` as ``frame_groups`` (not as ``value``).  On N > 1 the frames are streamed
(``--pipeline``, default on there): frame k's WTA tail — the four RCCL all-reduces with
the target scan between them, and the LR check — runs on a side stream while frame
k+1 aggregates in a second set of volumes (distributed.PipelinedMatcher), so the
exchange is hidden behind the next frame's passes; every frame's work is inside the
timed region (the side stream is joined before the closing synchronize).

Rank 0 prints ONE JSON line.  ``roofline`` is the dominant kernel: the
(direction, den mode) of aggregation pass with the most pass time per frame — on
one GPU the V pass with cached denominators (k_vpass10, DEN_READ: r-1 of the 2r
launches), on an 8-way C4 shard the den-none 32-plane pass (k_hpass32 / k_vpass32)
— named by asw_pass_kernel right after the timed region, every other kind reported
beside it.  achieved = algorithmic bytes per launch ``8*n*S + 8*T*S`` (read + write the
n local cost planes, read both support arrays of the direction) over
the launch's average duration from HIP events recorded on the stream the passes
run on, inside the timed region.  ``traffic`` = that kernel's HBM bytes per
launch from rocprofv3 PMC (profiles/traffic.json, tools/traffic_json.py).
``cpu_baseline`` is the CPU oracle (oracle/, a scalar-semantics C/OpenMP
restatement of the reference kernels) on this host: a full frame with every
OpenMP thread (C5: a strip), and a 1-thread strip (median of 3).
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
    "c1": (384, 288, 16, 5, 7, True, "C1 Tsukuba 384x288 d=16 win=5 r=7 + LR check (the reference pair)"),
    "c2": (450, 375, 64, 35, 7, False, "C2-size synthetic 450x375 d=64 win=35 r=7"),
    "c3": (450, 375, 64, 35, 7, True, "C3-size synthetic 450x375 d=64 win=35 r=7 + LR check"),
    "c5": (3840, 2160, 512, 51, 7, True, "C5 synthetic 3840x2160 d=512 win=51 r=7 + native LR check, batch of 8 pairs"),
}
for _scene, (_w, _h) in {"tsukuba": (384, 288), "cones": (450, 375), "teddy": (450, 375),
                         "laundry": (450, 372), "art": (450, 359)}.items():
    # the reference's own configuration on its own scenes (D61 T33 r7 k6 +
    # median, main.cpp:176-178): the span its published "ASW total" times
    WORKLOADS[f"ref-{_scene}"] = (_w, _h, 61, 33, 7, True,
                                  f"reference {_scene} {_w}x{_h} d=61 win=33 r=7 + LR + refinement k=6 + median")
REFINE = {k: 6 for k in WORKLOADS if k.startswith("ref-")}  # refinement iterations per workload
BATCH = {"c5": 8}  # pairs per step


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-rows", type=int, default=0,
                    help="rows of the frame timed on the CPU oracle with every thread (0: the full frame; C5: 96)")
    ap.add_argument("--api", default="stage", choices=["stage", "frame"],
                    help="stage: device-resident StereoMatcher; frame: the C-ABI asw_match (host buffers)")
    ap.add_argument("--graph", action="store_true",
                    help="with --api frame: asw_set_graph (the device work replayed from HIP graphs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pipeline", default="auto", choices=["auto", "on", "off"],
                    help="stream the frames through two sets of volumes: frame k's WTA tail (the RCCL exchange, "
                         "target scan, LR check) on a side stream overlapping frame k+1's aggregation "
                         "(distributed.PipelinedMatcher; stage API).  auto: on for N > 1 (it hides the exchange), "
                         "off on one GPU (measured the same there: 23.63 vs 23.59 ms, profiles/r04/pipeline_r10h.log)")
    ap.add_argument("--overlap-prep", type=int, default=1,
                    help="with the pipeline: run frame k+1's raw cost and supports on a third stream beside frame "
                         "k's passes (distributed.PipelinedMatcher overlap_prep; 0: after them)")
    ap.add_argument("--traffic", default=os.path.join(HERE, "profiles", "traffic.json"))
    ap.add_argument("--flags", type=int, default=0,
                    help="asw_params.flags (ASW_FLAG_*): opt-in forms, e.g. 64 = ASW_FLAG_RAW_F32 (the float "
                         "raw-cost volume) for an A/B; 0 = the shipped default")
    ap.add_argument("--group-size", type=int, default=0,
                    help="ranks per d-sharded frame (0: one frame over all ranks; the plan_groups layout is timed "
                         "beside it as frame_groups)")
    return ap.parse_args()


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(Lh, Rh, D, T, iters, rows, lr_mode):
    """Oracle (oracle/asw_oracle.c, OpenMP): rows [0, rows) of the frame (the full
    frame when rows >= H) with every OpenMP thread, and a 1-thread strip (median of
    3), each scaled to one map.  The oracle is the reference's arithmetic restated in
    C (the reference's own CPU path is OpenCL-on-CPU, which this image cannot run)."""
    from oracle import oracle as O
    H = Lh.shape[0]

    def timed(r):
        Ls, Rs = np.ascontiguousarray(Lh[:r]), np.ascontiguousarray(Rh[:r])
        t0 = time.perf_counter()
        O.match(Ls, Rs, D, T, iters)
        return time.perf_counter() - t0

    threads = O.set_threads(0)
    aff = sorted(os.sched_getaffinity(0))
    rows = min(rows, H)
    dt = timed(rows)
    what = "the full frame" if rows == H else f"a {Lh.shape[1]}x{rows} strip (rows 0-{rows - 1}), scaled x{H}/{rows}"
    if dt < 2.0:  # small frames: repeat to ~2 s of CPU work, median frame
        n = min(200, int(2.0 / max(dt, 1e-4)) + 1)
        runs = sorted([dt] + [timed(rows) for _ in range(n - 1)])
        dt = runs[len(runs) // 2]
        what += f", median of {n} runs"
    frame_s = dt * H / rows
    # one thread: a strip sized to ~2 s, median of 3
    r1 = max(4, min(H, int(rows * 2.0 / max(dt * threads, 1e-3))))
    O.set_threads(1)
    try:
        t1 = sorted(timed(r1) for _ in range(3))[1]
    finally:
        O.set_threads(threads)
    one_s = t1 * H / r1
    return {
        "value": round(1.0 / frame_s, 6), "unit": "maps/s", "cores": int(threads), "kind": "port",
        "sample": f"{what}: full pipeline r={iters} (raw cost, supports, 2r passes, WTA + target, LR check), "
                  f"{dt:.3f} s measured, {frame_s * 1000:.1f} ms/map",
        "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
        # where `cores` comes from: OpenMP's default team = OMP_NUM_THREADS (the GPU box's job
        # environment sets 16), run inside this process's CPU affinity mask
        "threads_source": f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', '(unset: every CPU of the mask)')}",
        "affinity_cpus": len(aff), "affinity_mask": _ranges(aff),
        # (VERDICT r04 item 7 asked for every CPU of the mask.  The mask is the whole shared
        # host; this pool's rules give one GPU's job a 16-CPU share and fix OMP_NUM_THREADS
        # at 16, so the baseline keeps the job's share.  `one_thread` below scales to any
        # core count: frame time ~ one_thread / cores for this embarrassingly parallel oracle.)
        "cores_policy": "the job's CPU share on the GPU box (16 of the host's CPUs, OMP_NUM_THREADS=16 "
                        "set by the pool); the affinity mask spans the whole shared host",
        "one_thread": {"value": round(1.0 / one_s, 6), "unit": "maps/s",
                       "sample": f"{Lh.shape[1]}x{r1} strip, median of 3 runs ({t1:.2f} s), scaled x{H}/{r1}; "
                                 f"{one_s * 1000:.0f} ms/map"},
    }


def _ranges(cpus):
    """[0, 1, 2, 5] -> "0-2,5" (a CPU affinity mask)."""
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


DM_NAMES = {0: "DM_NONE", 1: "DM_WRITE", 2: "DM_READ"}
DM_LABEL = {0: "den-none", 1: "den-write", 2: "den-read"}


def ran_kernel(direction, den_mode):
    """The instantiation the library last launched for (direction, den_mode) in this process
    (asw_pass_kernel, e.g. "k_hpass11<T=35,NKW=4,DM=2,nt>"), and its traffic.json keys:
    "<kernel><T=..,DM_x>" then the older "<kernel><DM_x>".  Call it right after the timed
    region: a later run (frame_groups) launches other instantiations."""
    from stereo_matchin_amd import kernels as K
    full = K.pass_kernel(direction, den_mode) or "unknown<>"
    base = full.split("<")[0]
    taps = [a for a in full[len(base) + 1:-1].split(",") if a.startswith("T=")]
    dm = DM_NAMES[den_mode]
    keys = ([f"{base}<{taps[0]},{dm}>"] if taps else []) + [f"{base}<{dm}>"]
    return full, keys


def base_matcher(m):
    """The StereoMatcher that runs the passes of a (Pipelined / Sharded) matcher."""
    from stereo_matchin_amd.distributed import PipelinedMatcher, ShardedStereoMatcher
    if isinstance(m, PipelinedMatcher):
        m = m.sets[0]
    if isinstance(m, ShardedStereoMatcher):
        m = m.matcher
    return m


def pass_den_mode(bm, name, it):
    """Den mode of iteration `it`'s pass `name` ("v"/"h") as StereoMatcher.aggregate runs
    it: none without a denominator volume (a 32-plane shard), else write then read."""
    from stereo_matchin_amd import _lib
    den = bm.den_v if name == "v" else bm.den_h
    if den is None:
        return _lib.DEN_NONE
    return _lib.DEN_WRITE if it == 0 else _lib.DEN_READ


def load_traffic(path, workload, n_gpus, keys):
    """Per-launch HBM bytes of the kernel (first of `keys` present) from profiles/traffic.json
    (rocprofv3 PMC)."""
    try:
        with open(path) as f:
            t = json.load(f)
        e = t.get(f"{workload}_n{n_gpus}") or {}
        for k in keys:
            if k in e:
                return e[k].get("total_bytes")
    except (OSError, ValueError):
        pass
    return None


def load_pairs(workload, W, H, D, n):
    """n stereo pairs of the workload (RGBA8 [H][W][4]): the reference's own pairs for C1
    and ref-<scene> (tests/golden/<scene>.npz, the committed fixtures), synthetic otherwise."""
    from stereo_matchin_amd.synthetic import make_pair
    if workload == "c1" or workload.startswith("ref-"):
        scene = "tsukuba" if workload == "c1" else workload[4:]
        z = np.load(os.path.join(HERE, "tests", "golden", f"{scene}.npz"))
        a = np.full(z["left"].shape[:2] + (1,), 255, np.uint8)
        L = np.ascontiguousarray(np.concatenate([z["left"], a], -1))
        R = np.ascontiguousarray(np.concatenate([z["right"], a], -1))
        assert L.shape == (H, W, 4)
        return [(L, R)] * n
    out = []
    for i in range(n):
        L, R, _ = make_pair(W, H, D, i)
        out.append((L, R))
        print(f"[bench] synthetic pair {i + 1}/{n} ready", file=sys.stderr, flush=True)
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} (launch N>1 with torch.distributed.run)")
    # ASW_BENCH_REHEARSAL=1: every rank on GPU 0 with the gloo backend (CUDA tensors
    # staged through the host), to run the N > 1 code path on a one-GPU box; the
    # numbers of such a run are not a scaling measurement
    rehearsal = os.environ.get("ASW_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from stereo_matchin_amd import FrameContext, make_params
    from stereo_matchin_amd.distributed import PipelinedMatcher, ShardedStereoMatcher, plan_groups
    from stereo_matchin_amd.pipeline import StereoMatcher

    W, H, D, T, iters, lr, desc = WORKLOADS[args.workload]
    batch = BATCH.get(args.workload, 1)
    lr_mode = 1 if D > 256 else 0  # the 8-bit codes collide above 256 levels: compare indices
    G = args.group_size or world
    if world % G != 0:
        raise SystemExit(f"--group-size {G} does not divide {world} ranks")
    if args.api == "frame" and world > 1:
        raise SystemExit("--api frame runs on one GPU (multi-GPU frame contexts: asw_create_multi / asw_create_rank)")
    groups, gid, grank = world // G, rank // G, rank % G
    pg = None
    if world > 1 and G > 1:
        # every rank creates every group, in the same order (torch.distributed rule)
        subs = [dist.new_group(list(range(g * G, (g + 1) * G)), backend="gloo" if rehearsal else None)
                for g in range(groups)]
        pg = subs[gid]
    # one set of pairs per frame group (groups run different pairs)
    pairs_h = load_pairs(args.workload, W, H, D, batch) if groups == 1 else \
        [(L, R) for L, R in load_pairs(args.workload, W, H, D, batch * groups)][gid * batch:(gid + 1) * batch]
    p = make_params(W, H, ndisp=D, taps=T, iters=iters, lr_check=int(lr), lr_mode=lr_mode, flags=args.flags)
    frame = args.api == "frame"
    args.pipeline = not frame and not REFINE.get(args.workload, 0) and (
        args.pipeline == "on" or (args.pipeline == "auto" and world > 1))
    if frame:
        fc = FrameContext(p, devices=[local], graph=args.graph)
        nloc = D
    else:
        pairs = [(torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)) for L, R in pairs_h]
        torch.cuda.synchronize()  # resident inputs (PipelinedMatcher overlap_prep does not wait for their copy)
        if args.pipeline:
            # (the pairs are resident and synchronized: the next frame's raw cost and supports
            # may run beside this frame's passes, overlap_prep)
            m = PipelinedMatcher(p, grank, G, dev, group=pg, overlap_prep=args.overlap_prep)
            nloc = m.p.d_stop - m.p.d_begin
        elif G > 1:
            m = ShardedStereoMatcher(p, grank, G, dev, group=pg)
            nloc = m.p.d_stop - m.p.d_begin
        else:
            m = StereoMatcher(p, dev)
            nloc = D
    spans = []  # frame API: asw_match's device-resident spans (ms)
    k_ref = REFINE.get(args.workload, 0)
    if frame and k_ref:
        from stereo_matchin_amd import _lib
        fc.close()
        fc = FrameContext(p, devices=[local], refine=_lib.default_refine_params(iters=k_ref), graph=args.graph)

    def step(events=None):
        for b in range(batch):
            if frame:
                out = fc.match(*pairs_h[b])
                spans.append(out["timings"])
            else:
                ev = [] if events is not None else None
                res = m.submit(*pairs[b], events=ev) if args.pipeline else m.match(*pairs[b], events=ev)
                if k_ref:  # main.cpp:540-623: k x (ref_v, ref_h, WTA_REF, LR) + 3x3 median
                    from stereo_matchin_amd import _lib
                    m.refine(res, *pairs[b], rp=_lib.default_refine_params(iters=k_ref))
                    if ev is not None:
                        from stereo_matchin_amd.pipeline import _record
                        ev.append(("refine", _record()))
                if events is not None:
                    events.append(ev)

    for _ in range(args.warmup):
        step()
    spans.clear()
    if args.pipeline:
        m.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    evs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(evs)
    if args.pipeline:
        m.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    torch.cuda.synchronize()

    # the instantiations the timed frames ran, per (direction, den mode), queried now:
    # the frame_groups run below launches other ones
    from stereo_matchin_amd import _lib
    ran = {(d, dm): ran_kernel(d, dm) for d in (0, 1) for dm in (_lib.DEN_NONE, _lib.DEN_WRITE, _lib.DEN_READ)}
    # per-launch aggregation-pass durations from the events around each pass, classified
    # by the den mode the pass ran: with cached denominators iteration 0 writes them
    # (DEN_WRITE) and iterations 1..r-1 read them; a 32-plane shard runs DEN_NONE throughout
    per_kind = {}  # ("v"|"h", den mode) -> [ms per launch]
    frame_ms, refine_ms = [], []
    if frame:
        for t in spans:
            frame_ms.append(t["total"] + t["refine"])
            if k_ref:
                refine_ms.append(t["refine"])
        per_pass = spans
        if args.graph:  # graph replays time only the coarse spans: passes from eager calls, outside the timed region
            with FrameContext(p, devices=[local]) as eager:
                per_pass = [eager.match(*pairs_h[0])["timings"] for _ in range(3)]
        for t in per_pass:
            # asw_timings keeps the per-direction mean over the r passes of a frame (the
            # context caches denominators for r >= 2: r - 1 of the r are den-read)
            dm_f = _lib.DEN_READ if iters >= 2 else _lib.DEN_NONE
            per_kind.setdefault(("v", dm_f), []).append(t["v_pass_mean"])
            per_kind.setdefault(("h", dm_f), []).append(t["h_pass_mean"])
    else:
        bm = base_matcher(m)
        for ev in evs:
            prev = dict(ev)["support"]
            it = {"v": 0, "h": 0}
            for name, e in ev:
                if name == "refine":
                    refine_ms.append(dict(ev)["consistency"].elapsed_time(e))
                if name in ("v", "h"):
                    kind = (name, pass_den_mode(bm, name, it[name]))
                    per_kind.setdefault(kind, []).append(prev.elapsed_time(e))
                    it[name] += 1
                    prev = e
            frame_ms.append(ev[0][1].elapsed_time(ev[-1][1]))
    # den-none passes beside the shipped den-read ones (report both and ship
    # the faster): one V and one H pass without the cached denominators, on the
    # matcher's own buffers, after the timed region (not part of `value`)
    v_none, h_none = [], []
    if not frame and not args.pipeline and world == 1 and iters >= 2:
        from stereo_matchin_amd import kernels as K
        for _ in range(3):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            K.asw_vCostAggregation(m.p, m.wvl, m.wvr, m.c0, out=m.c1)
            e[1].record()
            K.asw_hCostAggregation(m.p, m.whl, m.whr, m.c1, out=m.c0)
            e[2].record()
            torch.cuda.synchronize()
            v_none.append(e[0].elapsed_time(e[1]))
            h_none.append(e[1].elapsed_time(e[2]))
    # the layout with the most maps/s (plan_groups: N/g concurrent frames of g shards),
    # timed after the main run and reported beside `value`
    frame_groups = None
    g2 = plan_groups(D, world) if world > 1 and not args.group_size and not frame else 1
    if 1 < g2 < world:
        subs2 = [dist.new_group(list(range(g * g2, (g + 1) * g2)), backend="gloo" if rehearsal else None)
                 for g in range(world // g2)]
        if args.pipeline:  # (streamed like the main run)
            m2 = PipelinedMatcher(p, rank % g2, g2, dev, group=subs2[rank // g2], overlap_prep=args.overlap_prep)
            run2 = m2.submit
        else:
            m2 = ShardedStereoMatcher(p, rank % g2, g2, dev, group=subs2[rank // g2])
            run2 = m2.match
        for _ in range(2):
            for b in range(batch):
                run2(*pairs[b])
        if args.pipeline:
            m2.flush()
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            for b in range(batch):
                run2(*pairs[b])
        if args.pipeline:
            m2.flush()
        torch.cuda.synchronize()
        dist.barrier()
        el2 = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        dist.all_reduce(el2, op=dist.ReduceOp.MAX)
        n2 = world // g2 * args.steps * batch
        frame_groups = {"group_size": g2, "frames_per_step": world // g2 * batch,
                        "value": round(n2 / el2.item(), 4), "unit": "maps/s",
                        "ms_per_step": round(el2.item() / args.steps * 1000, 4),
                        "planes_per_rank": m2.p.d_stop - m2.p.d_begin,
                        "note": f"{world // g2} concurrent frames, each d-sharded over {g2} GPUs "
                                "(the most maps/s on N GPUs; not the headline layout)"}
        del m2
    # max over ranks of every per-kind mean (absent kinds: -1) and of the launches per frame
    kinds = [(n, dm) for n in ("v", "h") for dm in (_lib.DEN_READ, _lib.DEN_WRITE, _lib.DEN_NONE)]
    nframes = max(len(frame_ms), 1) if not frame else max(len(per_pass), 1)
    all_pass = [x for xs in per_kind.values() for x in xs]
    vals = [elapsed, float(np.mean(all_pass)) if all_pass else -1.0, float(np.sum(frame_ms))]
    for k in kinds:
        xs = per_kind.get(k, [])
        vals += [float(np.mean(xs)) if xs else -1.0, len(xs) / nframes]
    stats = torch.tensor(vals, dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    vals = stats.tolist()
    elapsed, pass_avg, span_sum = vals[:3]
    kind_ms = {k: vals[3 + 2 * i] for i, k in enumerate(kinds) if vals[3 + 2 * i] >= 0}
    kind_n = {k: vals[4 + 2 * i] for i, k in enumerate(kinds) if vals[3 + 2 * i] >= 0}

    if rank == 0:
        S = W * H
        bytes_per_pass = 8 * nloc * S + 8 * T * S
        gbs = lambda ms: bytes_per_pass / (ms * 1e-3) / 1e9  # noqa: E731
        n_maps = groups * args.steps * batch
        maps_per_s = n_maps / (span_sum / 1e3) if frame else n_maps / elapsed
        # the dominant kernel: the (direction, den mode) with the most pass time per frame
        dom = max(kind_ms, key=lambda k: kind_ms[k] * kind_n[k]) if kind_ms else ("v", _lib.DEN_READ)
        dom_ms = kind_ms.get(dom, float("nan"))
        kname, tkeys = ran[(0 if dom[0] == "v" else 1, dom[1])]
        opt = lambda k: round(kind_ms[k], 4) if k in kind_ms else None  # noqa: E731
        optf = lambda k: round(gbs(kind_ms[k]) / HBM_PEAK_GBS, 4) if k in kind_ms else None  # noqa: E731
        in_frame_none = ("v", _lib.DEN_NONE) in kind_ms or ("h", _lib.DEN_NONE) in kind_ms
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
            "data": ("reference Tsukuba pair (tests/golden)" if args.workload == "c1" else
                     f"reference {args.workload[4:]} pair (tests/golden)" if args.workload.startswith("ref-")
                     else "synthetic"),
            "config": {"workload": desc, "width": W, "height": H, "ndisp": D, "taps": T, "iters": iters,
                       "lr_check": lr, "lr_mode": "native" if lr_mode else "u8", "pairs_per_step": batch,
                       "local_planes": nloc, "frames_per_step": groups * batch, "flags": args.flags,
                       "api": args.api + ("+graph" if frame and args.graph else "") + ("+pipeline" if args.pipeline else "")
                       + ("+overlap_prep" if args.pipeline and args.overlap_prep else ""),
                       "parallelism": (f"{groups} frame group(s), each d-sharded over {G} GPU(s)"
                                       if world > 1 else "single GPU")},
            "roofline": {"bound": "hbm", "achieved": round(gbs(dom_ms), 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs(dom_ms) / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(args.traffic, args.workload, world, tkeys),
                         "kernel": f"{kname}: {'V' if dom[0] == 'v' else 'H'} aggregation pass, "
                                   f"{DM_LABEL[dom[1]]} ({round(kind_n.get(dom, 0))} of the {2 * iters} "
                                   f"launches per frame)",
                         "bytes_per_launch": bytes_per_pass, "avg_launch_ms": round(dom_ms, 4),
                         "v_read_ms": opt(("v", _lib.DEN_READ)), "v_read_frac": optf(("v", _lib.DEN_READ)),
                         "h_read_ms": opt(("h", _lib.DEN_READ)), "h_read_frac": optf(("h", _lib.DEN_READ)),
                         "v_write_ms": opt(("v", _lib.DEN_WRITE)), "h_write_ms": opt(("h", _lib.DEN_WRITE)),
                         "v_none_ms": opt(("v", _lib.DEN_NONE)) if in_frame_none else
                         (round(float(np.median(v_none)), 4) if v_none else None),
                         "v_none_frac": optf(("v", _lib.DEN_NONE)) if in_frame_none else
                         (round(gbs(float(np.median(v_none))) / HBM_PEAK_GBS, 4) if v_none else None),
                         "h_none_ms": opt(("h", _lib.DEN_NONE)) if in_frame_none else
                         (round(float(np.median(h_none)), 4) if h_none else None),
                         "h_none_frac": optf(("h", _lib.DEN_NONE)) if in_frame_none else
                         (round(gbs(float(np.median(h_none))) / HBM_PEAK_GBS, 4) if h_none else None),
                         "kernels_ran": {f"{'VH'[d]} {DM_LABEL[dm]}": ran[(d, dm)][0]
                                         for (n, dm) in kind_ms for d in [0 if n == "v" else 1]},
                         "den_modes": ("the frame's passes run den-none (a 32-plane shard keeps no denominator "
                                       "volumes): v/h_none are those passes, timed inside the timed region"
                                       if in_frame_none else
                                       "the frame ships cached denominators (den-read) for r >= 2: den-none "
                                       "(v/h_none, 3 VALU per voxel-tap instead of 2, 2.1 GB less traffic) is "
                                       "timed beside it outside the timed region"),
                         "all_pass_mean_ms": round(pass_avg, 4),
                         "all_pass_frac": round(gbs(pass_avg) / HBM_PEAK_GBS, 4),
                         "timing": "frame API: asw_timings per-direction means over all r passes" if frame else
                                   "HIP events on the passes' stream inside the timed region"},
            "frame_ms_events": round(float(np.median(frame_ms)), 4),
        }
        if k_ref:
            out["refine"] = {"iters": k_ref, "median_ms": round(float(np.median(refine_ms)), 4),
                             "note": "refinement loop + 3x3 median inside each step (main.cpp:540-623); "
                                     "frame_ms_events = raw cost -> median, the span of the reference's "
                                     "published ASW total (main.cpp:707-708, BASELINE.md §1)"}
        if frame_groups:
            out["frame_groups"] = frame_groups
        if frame:
            out["pcie_inclusive"] = {"value": round(n_maps / elapsed, 4), "unit": "maps/s",
                                     "note": "wall clock of asw_match incl. host->device upload and device->host "
                                             "read-back of every output"}
        if world == 1 and not args.no_cpu:
            rows = args.cpu_rows or (96 if args.workload == "c5" else H)
            out["cpu_baseline"] = cpu_baseline(*pairs_h[0], D, T, iters, rows, lr_mode)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
