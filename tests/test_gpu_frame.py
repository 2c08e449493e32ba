"""FRAME API on the GPU (include/asw.h: asw_create / asw_create_multi / asw_create_rank,
asw_match / asw_match_batch): multi-shard contexts, RCCL, batches, 16-bit outputs.

Every multi-shard result is compared bit for bit with the one-GPU context (itself
checked against the oracle in test_gpu_parity.py) and, at small sizes, with the
oracle directly.
"""
import numpy as np
import pytest

from conftest import load_scene

pytestmark = pytest.mark.gpu


def _p(W, H, D, T, iters, **kw):
    from stereo_matchin_amd import make_params
    return make_params(W, H, ndisp=D, taps=T, iters=iters, **kw)


def _pair(seed, H, W, shift=6):
    rng = np.random.default_rng(seed)
    L = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    R = np.roll(L, -shift, axis=1).copy()
    R[..., :3] = np.clip(R[..., :3].astype(int) + rng.integers(-4, 5, (H, W, 3)), 0, 255).astype(np.uint8)
    L[..., 3] = R[..., 3] = 255
    return L, R


KEYS = ("d_ref", "d_tar", "conf_ref", "conf_tar", "disp_rgba", "lr_rgba", "lr_red_rgba")


def _same(a, b, keys=KEYS):
    for k in keys:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


# several d-shards of one frame on ONE GPU: the COMM_LOCAL exchange (peer copies +
# MIN kernel), same protocol and kernels as the RCCL path
@pytest.mark.parametrize("n", [2, 3, 8])
def test_multi_shard_local_equals_single(gpu, oracle, n):
    from stereo_matchin_amd import FrameContext
    Lh, Rh, _ = load_scene("teddy")
    p = _p(Lh.shape[1], Lh.shape[0], 64, 35, 3)
    with FrameContext(p, devices=[0]) as one:
        ref = one.match(Lh, Rh, want_cost=True, want16=True)
    with FrameContext(p, devices=[0] * n) as fc:
        sh = fc.shards()
        assert len(sh) == n and sh[0][0] == 0 and sh[-1][1] == 64
        assert all(sh[i][1] == sh[i + 1][0] for i in range(n - 1))
        got = fc.match(Lh, Rh, want_cost=True, want16=True)
    _same(got, ref, KEYS + ("disp16", "lr16"))
    assert np.array_equal(got["cost"][:, :, :64], ref["cost"][:, :, :64])
    assert got["timings"]["exchange"] > 0
    o = oracle.match(Lh, Rh, 64, 35, 3)
    assert np.array_equal(got["d_ref"], o["d_ref"]) and np.array_equal(got["lr_red_rgba"], o["lr_red_rgba"])


# C4's D = 256 over 8 shards of 32 planes (pitch 32: the half-wave passes)
def test_multi_shard_d256_eight_way(gpu):
    from stereo_matchin_amd import FrameContext
    Lh, Rh = _pair(7, 96, 320, shift=40)
    p = _p(320, 96, 256, 35, 2)
    with FrameContext(p, devices=[0]) as one:
        ref = one.match(Lh, Rh)
    with FrameContext(p, devices=[0] * 8) as fc:
        assert [e - b for b, e in fc.shards()] == [32] * 8
        got = fc.match(Lh, Rh)
    _same(got, ref)


# RCCL itself on a one-GPU box: a one-rank communicator from asw_comm_unique_id /
# ncclCommInitRank; the four ncclAllReduce(ncclMin) calls of the exchange run
def test_rank_context_rccl_one_rank(gpu):
    from stereo_matchin_amd import FrameContext, comm_unique_id
    Lh, Rh, _ = load_scene("tsukuba")
    p = _p(Lh.shape[1], Lh.shape[0], 16, 5, 7)
    with FrameContext(p, devices=[0]) as one:
        ref = one.match(Lh, Rh)
    cid = comm_unique_id()
    assert len(cid) == 128
    with FrameContext(p, devices=[0], rank=0, nranks=1, comm_id=cid) as fc:
        got = fc.match(Lh, Rh)
    _same(got, ref)
    assert got["timings"]["exchange"] > 0


def test_batch_equals_single_pairs(gpu):
    from stereo_matchin_amd import FrameContext
    pairs = [_pair(s, 40, 90, shift=3 + s) for s in range(3)]
    p = _p(90, 40, 24, 9, 2)
    with FrameContext(p, devices=[0]) as fc:
        single = [fc.match(L, R) for L, R in pairs]
        batch = fc.match_batch(np.stack([L for L, _ in pairs]), np.stack([R for _, R in pairs]))
    assert len(batch) == 3
    for a, b in zip(batch, single):
        _same(a, b)
        assert a["timings"]["total"] > 0


def test_disp16_outputs(gpu, oracle):
    from stereo_matchin_amd import FrameContext
    Lh, Rh, _ = load_scene("cones")
    for lr_mode in (0, 1):
        p = _p(Lh.shape[1], Lh.shape[0], 64, 35, 2, lr_mode=lr_mode)
        with FrameContext(p) as fc:
            out = fc.match(Lh, Rh, want16=True)
        assert out["disp16"].dtype == np.uint16
        assert np.array_equal(out["disp16"], out["d_ref"].astype(np.uint16))
        rgba = out["lr_red_rgba"]
        red = (rgba[..., 0] == 255) & (rgba[..., 1] == 0) & (rgba[..., 2] == 0)
        inconsistent = out["lr16"] == 0xFFFF
        assert np.array_equal(inconsistent, red)
        assert np.array_equal(out["lr16"][~inconsistent], out["d_ref"][~inconsistent].astype(np.uint16))
        if lr_mode == 1:
            want = np.abs(out["d_ref"] - out["d_tar"]) > 1
            assert np.array_equal(inconsistent, want)


# D > 256: the 8-bit codes collide, the 16-bit image and the native LR check do not
def test_d512_native_lr_and_disp16(gpu, oracle):
    from stereo_matchin_amd import FrameContext
    Lh, Rh = _pair(11, 24, 700, shift=300)
    p = _p(700, 24, 512, 9, 1, lr_mode=1)
    with FrameContext(p, devices=[0, 0]) as fc:
        out = fc.match(Lh, Rh, want16=True)
    o = oracle.match(Lh, Rh, 512, 9, 1)
    assert np.array_equal(out["d_ref"], o["d_ref"]) and np.array_equal(out["d_tar"], o["d_tar"])
    assert out["d_ref"].max() > 256
    assert np.array_equal(out["disp16"], o["d_ref"].astype(np.uint16))
    cons = np.abs(o["d_ref"] - o["d_tar"]) <= 1
    assert np.array_equal(out["lr16"], np.where(cons, o["d_ref"], 0xFFFF).astype(np.uint16))


# with refinement on, every non-refinement output is the pre-refinement
# result (copied out before the loop updates its buffers in place)
def test_refine_leaves_pre_refinement_outputs(gpu):
    from stereo_matchin_amd import FrameContext, _lib
    Lh, Rh, _ = load_scene("tsukuba")
    p = _p(Lh.shape[1], Lh.shape[0], 61, 33, 7)
    with FrameContext(p) as fc:
        plain = fc.match(Lh, Rh, want16=True)
    with FrameContext(p, refine=_lib.default_refine_params()) as fc:
        ref = fc.match(Lh, Rh, want16=True)
    _same(ref, plain, KEYS + ("disp16", "lr16"))
    assert ref["timings"]["refine"] > 0
    assert not np.array_equal(ref["final_rgba"], plain["lr_rgba"])


# timings are filled for any iteration count (the event slots are
# sized from iters at create)
def test_timings_for_many_iterations(gpu):
    from stereo_matchin_amd import FrameContext
    Lh, Rh = _pair(3, 20, 40)
    with FrameContext(_p(40, 20, 8, 3, 14)) as fc:
        t = fc.match(Lh, Rh)["timings"]
    for k in ("raw_cost", "support", "v_pass_mean", "h_pass_mean", "aggregation_total", "wta", "total"):
        assert t[k] > 0, k


# the refinement loop on a d-sharded frame (its asw_WTA_REF scans exchanged like the
# WTA): equal to the one-GPU refinement, which test_gpu_refine.py pins to the oracle
@pytest.mark.parametrize("n", [2, 3])
def test_multi_shard_refinement_equals_single(gpu, n):
    from stereo_matchin_amd import FrameContext, _lib
    Lh, Rh, _ = load_scene("tsukuba")
    p = _p(Lh.shape[1], Lh.shape[0], 61, 33, 7)
    rp = _lib.default_refine_params()
    with FrameContext(p, devices=[0], refine=rp) as one:
        ref = one.match(Lh, Rh)
    with FrameContext(p, devices=[0] * n, refine=rp) as fc:
        got = fc.match(Lh, Rh)
    _same(got, ref, KEYS + ("final_rgba", "post_red_rgba"))
    assert got["timings"]["refine"] > 0


def test_rank_context_refinement(gpu):
    from stereo_matchin_amd import FrameContext, _lib, comm_unique_id
    Lh, Rh, _ = load_scene("cones")
    p = _p(Lh.shape[1], Lh.shape[0], 64, 35, 2)
    rp = _lib.default_refine_params(iters=3)
    with FrameContext(p, devices=[0], refine=rp) as one:
        ref = one.match(Lh, Rh)
    with FrameContext(p, devices=[0], rank=0, nranks=1, comm_id=comm_unique_id(), refine=rp) as fc:
        got = fc.match(Lh, Rh)
    _same(got, ref, KEYS + ("final_rgba", "post_red_rgba"))


# asw_set_graph: the device work captured once into HIP graphs and replayed; every
# output equals the eager path's, also for a second pair through the same graphs
def test_graph_mode_equals_eager(gpu):
    from stereo_matchin_amd import FrameContext, _lib
    p = _p(450, 375, 64, 35, 3)
    rp = _lib.default_refine_params(iters=2)
    scenes = [load_scene("cones")[:2], load_scene("teddy")[:2]]
    with FrameContext(p, refine=rp) as eager, FrameContext(p, refine=rp, graph=True) as graphed:
        for Lh, Rh in scenes + scenes[:1]:
            a = eager.match(Lh, Rh, want16=True)
            b = graphed.match(Lh, Rh, want16=True)
            _same(b, a, KEYS + ("final_rgba", "post_red_rgba", "disp16", "lr16"))
            assert b["timings"]["total"] > 0 and b["timings"]["refine"] > 0


# the frame API's raw-cost forms: the uint16 volume (default where asw_raw16_supported)
# against ASW_FLAG_RAW_F32 (the float volume), whole range and 8 shards of 32 planes,
# the final volume included
@pytest.mark.parametrize("devices", [[0], [0] * 8])
def test_raw16_frame_equals_float(gpu, devices):
    from stereo_matchin_amd import FrameContext, _lib
    Lh, Rh = _pair(11, 72, 300, shift=30)
    p = _p(300, 72, 256, 35, 2)
    with FrameContext(p, devices=devices) as fc:
        a = fc.match(Lh, Rh, want_cost=len(devices) == 1)
    q = p.copy()
    q.flags = _lib.FLAG_RAW_F32
    with FrameContext(q, devices=devices) as fc:
        b = fc.match(Lh, Rh, want_cost=len(devices) == 1)
    _same(a, b)
    if len(devices) == 1:
        assert np.array_equal(a["cost"], b["cost"])
