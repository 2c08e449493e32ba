"""Disparity-axis sharding of one stereo frame across GPUs (one process per GPU).

The reference runs each OpenCL device independently (main.cpp:158-172); it has
no multi-device path.  Here the frame's disparity range [0, D) is split into
contiguous shards, one per rank (``torch.distributed``, backend "nccl" = RCCL
over xGMI on MI355X):

* raw cost, V and H passes of plane d read only plane d (plus the d-independent
  supports), so every rank aggregates its own planes with NO communication;
* the WTA over d is the one exchange step.  Each rank reduces its planes to a
  partial top-2; partials combine exactly with elementwise MIN all-reduces of
  ``key = (float_bits(m1) << 32) | index`` (ties -> smallest index, which is the
  reference's first-argmin) and of the second-smallest contribution.  The
  target-view scan (K/asw_wta.cl:50-67) needs the global left argmin, so it
  follows the first exchange and repeats the pattern.  Four all-reduces per
  frame: 2 x int64[H*W] + 2 x float32[H*W].

The protocol (:func:`sharded_wta`) is written against two small interfaces so
the same host logic runs on GPU tensors over RCCL (product) and on CPU tensors
over gloo (tests/test_distributed.py).
"""
from __future__ import annotations

from typing import Callable, Protocol

import torch
import torch.distributed as dist

from . import kernels as K
from ._lib import AswParams
from .pipeline import MatchResult, StereoMatcher


def plan_groups(ndisp: int, world: int, min_planes: int = 64) -> int:
    """Ranks per d-sharded frame ("group size") for the most maps/s on `world` ranks:
    the SMALLEST divisor g >= 2 of `world` with ndisp/g >= min_planes (1 if none);
    world/g groups then each match their own frame, concurrently.

    Why the smallest: a shard repeats the frame's d-independent work (supports and
    their per-pass reads, the image staging of the raw cost, the WTA exchange and LR
    check), so the fewest shards per frame give the most frames per GPU-second.
    bench.py's headline layout is NOT this one: it shards ONE frame over all ranks
    (BASELINE.json config 4), and reports this layout beside it as ``frame_groups``.
    """
    for g in range(2, world + 1):
        if world % g == 0 and ndisp / g >= min_planes:
            return g
    return 1


def shard_range(ndisp: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced split of [0, ndisp) into `world` non-empty shards."""
    if world > ndisp:
        raise ValueError(f"cannot split {ndisp} disparities over {world} ranks")
    base, rem = divmod(ndisp, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


class ShardOps(Protocol):
    def local(self, cost): ...                    # -> key, m1, m2
    def target_local(self, cost, key_ref): ...    # -> tkey, t1, t2
    def second(self, key_g, key_l, m1, m2): ...   # -> contribution
    def finalize(self, key, m2, tkey, t2): ...    # -> d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar


def _allreduce_min_factory(group=None) -> Callable[[torch.Tensor], torch.Tensor]:
    def reduce_min(t: torch.Tensor) -> torch.Tensor:
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        return t
    return reduce_min


def sharded_wta(ops: ShardOps, cost, reduce_min: Callable, local: tuple | None = None) -> tuple:
    """Exact WTA over a d-sharded cost volume (see module doc).  ``local``: the
    (key, m1, m2) of ops.local(cost) when already computed."""
    key, m1, m2 = ops.local(cost) if local is None else local
    key_g = reduce_min(key.clone())
    m2_g = reduce_min(ops.second(key_g, key, m1, m2))
    tkey, t1, t2 = ops.target_local(cost, key_g)
    tkey_g = reduce_min(tkey.clone())
    t2_g = reduce_min(ops.second(tkey_g, tkey, t1, t2))
    return ops.finalize(key_g, m2_g, tkey_g, t2_g)


class HipShardOps:
    """The HIP C-ABI stage functions of include/asw.h for one shard."""

    def __init__(self, p: AswParams):
        self.p = p

    def local(self, cost):
        return K.wta_local(self.p, cost)

    def target_local(self, cost, key_ref):
        return K.wta_target_local(self.p, cost, key_ref)

    def second(self, key_g, key_l, m1, m2):
        return K.wta_second(self.p, key_g, key_l, m1, m2)

    def finalize(self, key, m2, tkey, t2):
        return K.wta_finalize(self.p, key, m2, tkey, t2)


class ShardedStereoMatcher:
    """One rank's share of a d-sharded frame."""

    def __init__(self, params: AswParams, rank: int, world: int, device="cuda", group=None):
        p = params.copy()
        p.d_begin, p.d_end = shard_range(params.ndisp, rank, world)
        self.p = p
        self.rank, self.world = rank, world
        self.matcher = StereoMatcher(p, device)
        self.ops = HipShardOps(p)
        self.reduce_min = _allreduce_min_factory(group)

    def match(self, left: torch.Tensor, right: torch.Tensor, events: list | None = None) -> MatchResult:
        m = self.matcher
        if events is not None:
            events.append(("start", _record()))
        m.raw_and_support(left, right)
        if events is not None:
            events.append(("support", _record()))
        cost = m.aggregate(events)
        # (m.local: the local scan, when the last pass ran it)
        d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar = sharded_wta(self.ops, cost, self.reduce_min, m.local)
        if events is not None:
            events.append(("wta", _record()))
        lr = red = None
        if self.p.lr_check:
            lr, red = K.Constistency(self.p, d_ref, d_tar, code_ref, code_tar, conf_ref, conf_tar)
        if events is not None:
            events.append(("consistency", _record()))
        return MatchResult(d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar, lr, red, cost)


def _record():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


class PipelinedMatcher:
    """Frames streamed through ``depth`` sets of volumes, the WTA tail of frame k
    overlapping the aggregation of frame k+1.

    The main stream runs frame k's raw cost, supports, 2r passes and the local WTA scan
    (``asw_wta_local``); a side stream then runs the rest of its WTA — on a d-sharded
    frame the four MIN all-reduces over RCCL with the target scan between them
    (``sharded_wta``), on a whole-range frame ``asw_WTA`` itself — and the consistency
    check, while the main stream goes on with frame k+1 in the other set of volumes.
    A set is reused only after its frame's tail has finished (an event the main stream
    waits for).  Results are bit-identical to ``ShardedStereoMatcher.match`` /
    ``StereoMatcher.match`` (tests/test_gpu_frame.py, tests/test_distributed.py).

    ``submit(left, right)`` returns the frame's ``MatchResult`` (valid once ``flush()``
    or a later ``submit`` into the same set has ordered the caller's stream after it:
    ``flush()`` makes the current stream wait for every submitted tail).  Its maps and
    images are the frame's own tensors, but ``.cost`` is the set's persistent volume:
    the ``depth``-th later ``submit`` (the next one into the same set) overwrites it, so
    a caller that needs the volume (e.g. for ``refine``) copies it before then."""

    def __init__(self, params: AswParams, rank: int = 0, world: int = 1, device="cuda", group=None, depth: int = 2,
                 overlap_prep: bool = False):
        self.device = torch.device(device)
        # overlap_prep: frame k+1's raw cost and support weights (d-independent of frame
        # k's volumes, in the other set's buffers) run on a third stream while frame k's
        # passes run, instead of after them on the main stream.  The caller's images must
        # then be valid when submit() is called (resident inputs, or their producer
        # synchronized): the preparation does not wait for the caller's stream.
        self.overlap_prep = overlap_prep
        self.prep = torch.cuda.Stream(self.device) if overlap_prep else None
        self.sharded = world > 1
        if self.sharded:
            self.sets = [ShardedStereoMatcher(params, rank, world, self.device, group) for _ in range(depth)]
            self.p = self.sets[0].p
        else:
            self.sets = [StereoMatcher(params, self.device) for _ in range(depth)]
            self.p = self.sets[0].p
        self.side = torch.cuda.Stream(self.device)
        self.done: list = [None] * depth
        self.k = 0

    def submit(self, left: torch.Tensor, right: torch.Tensor, events: list | None = None) -> MatchResult:
        """Queue one frame.  ``events``: ("start", "support", "v"/"h" per pass) on the main
        stream and ("consistency") at the end of its tail on the side stream."""
        i = self.k % len(self.sets)
        self.k += 1
        main = torch.cuda.current_stream(self.device)
        if self.done[i] is not None:
            main.wait_event(self.done[i])  # set i's previous tail has finished with its volume
        st = self.sets[i]
        m = st.matcher if self.sharded else st
        if events is not None:
            events.append(("start", _record()))
        if self.overlap_prep:
            # raw cost + supports of this frame on the prep stream, after set i's previous
            # tail (its last reader), beside whatever the main stream is running
            if self.done[i] is not None:
                self.prep.wait_event(self.done[i])
            with torch.cuda.stream(self.prep):
                m.raw_and_support(left, right)
                prepared = torch.cuda.Event()
                prepared.record(self.prep)
            for t in (left, right):
                t.record_stream(self.prep)
            main.wait_event(prepared)
        else:
            m.raw_and_support(left, right)
        if events is not None:
            events.append(("support", _record()))
        cost = m.aggregate(events)
        local = m.local  # the local scan, when a pass already ran it
        if local is None and self.sharded:
            local = st.ops.local(cost)
        ready = torch.cuda.Event()
        ready.record(main)
        p = m.p
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            for t in (local or ()):
                t.record_stream(self.side)
            if self.sharded:
                d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar = sharded_wta(st.ops, cost, st.reduce_min, local)
            elif local is not None:
                d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar = K.wta_from_local(p, cost, *local)
            else:
                d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar = K.asw_WTA(p, cost)
            lr = red = None
            if p.lr_check:
                lr, red = K.Constistency(p, d_ref, d_tar, code_ref, code_tar, conf_ref, conf_tar)
            done = torch.cuda.Event(enable_timing=events is not None)
            done.record(self.side)
        if events is not None:
            events.append(("consistency", done))
        self.done[i] = done
        outs = (d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar, lr, red)
        for t in outs:  # allocated on the side stream, read on the caller's: freed after both
            if t is not None:
                t.record_stream(main)
        return MatchResult(*outs, cost)

    def flush(self) -> None:
        """Order the current stream after every submitted frame's tail."""
        torch.cuda.current_stream(self.device).wait_stream(self.side)
        if self.prep is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.prep)
