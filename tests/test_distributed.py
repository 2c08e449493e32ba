"""Multi-process (gloo, CPU) tests of the d-sharded WTA protocol (no GPU).

`stereo_matchin_amd.distributed.sharded_wta` is the host logic every rank runs
on the GPU over RCCL.  Here the same function runs in two (and three) real
processes over torch.distributed's gloo backend, with a CPU restatement of the
four per-shard stage kernels (asw_wta_local / _target_local / _second /
_finalize, include/asw.h) written below from the reference's WTA rules
(K/asw_wta.cl:12-82).  The gathered result must equal the oracle's
unsharded WTA (oracle_wta, pinned to the reference in test_oracle_golden.py)
bit for bit, on volumes built with many exact ties and with NaN-free zero gaps.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stereo_matchin_amd.distributed import shard_range, sharded_wta

INIT = np.float32(100000.0)  # K/asw_wta.cl:25-26
NOKEY = np.int64(0x7FFFFFFFFFFFFFFF)


def _key(v: np.ndarray, idx: np.ndarray) -> np.ndarray:
    bits = v.astype(np.float32).view(np.uint32).astype(np.uint64)
    return ((bits << np.uint64(32)) | idx.astype(np.uint64)).astype(np.int64)


def _top2(cands: np.ndarray, ids: np.ndarray):
    """Sequential strict-< scan of K/asw_wta.cl:25-47 over the last axis."""
    m1 = np.full(cands.shape[:-1], INIT, np.float32)
    m2 = np.full(cands.shape[:-1], INIT, np.float32)
    idx = np.full(cands.shape[:-1], -1, np.int64)
    for j in range(cands.shape[-1]):
        t = cands[..., j]
        ok = ~np.isnan(t)
        lt2 = ok & (t < m2)
        m2 = np.where(lt2, t, m2)
        lt1 = ok & (t < m1)
        m2 = np.where(lt1, m1, m2)
        idx = np.where(lt1, ids[..., j], idx)
        m1 = np.where(lt1, t, m1)
    return m1, m2, idx


class CpuShardOps:
    """CPU restatement of the per-shard stage functions (test infrastructure)."""

    def __init__(self, d_begin: int, d_end: int, D: int):
        self.b, self.e, self.D = d_begin, d_end, D

    def local(self, cost):  # cost: [H][W][n] local planes, pixel-major like the product
        c = cost.numpy()
        ids = np.broadcast_to(np.arange(self.b, self.e), c.shape)
        m1, m2, idx = _top2(c, ids)
        key = np.where(idx < 0, NOKEY, _key(m1, np.maximum(idx, 0)))
        return torch.from_numpy(key), torch.from_numpy(m1), torch.from_numpy(m2)

    def target_local(self, cost, key_ref):
        c = cost.numpy()
        H, W, _ = c.shape
        kr = key_ref.numpy()
        md = np.where(kr == NOKEY, 0, kr & 0xFFFFFFFF).astype(np.int64)
        x = np.broadcast_to(np.arange(W), (H, W))
        y = np.broadcast_to(np.arange(H)[:, None], (H, W))
        Dmax = self.D
        i = np.arange(Dmax)
        xq = np.maximum(x[..., None] - i, 0)
        b = md[..., None] + xq - x[..., None]
        valid = (i < md[..., None]) & (b >= self.b) & (b < self.e)
        cand = np.full((H, W, Dmax), np.nan, np.float32)
        yy = np.broadcast_to(y[..., None], cand.shape)
        cand[valid] = c[yy[valid], xq[valid], (b - self.b)[valid]]
        m1, m2, idx = _top2(cand, np.broadcast_to(i, cand.shape))
        tkey = np.where(idx < 0, NOKEY, _key(m1, np.maximum(idx, 0)))
        return torch.from_numpy(tkey), torch.from_numpy(m1), torch.from_numpy(m2)

    def second(self, key_g, key_l, m1, m2):
        return torch.where(key_l == key_g, m2, m1)

    def finalize(self, key, m2, tkey, t2):
        k, tk = key.numpy(), tkey.numpy()
        H, W = k.shape
        x = np.broadcast_to(np.arange(W), (H, W))
        md = np.where(k == NOKEY, 0, k & 0xFFFFFFFF).astype(np.int32)
        m1 = np.where(k == NOKEY, INIT, (k.astype(np.uint64) >> np.uint64(32)).astype(np.uint32).view(np.float32))
        ti = (tk & 0xFFFFFFFF).astype(np.int64)
        mdr = np.where(tk == NOKEY, md, md + np.maximum(x - ti, 0) - x).astype(np.int32)
        tm1 = np.where(tk == NOKEY, INIT,
                       (tk.astype(np.uint64) >> np.uint64(32)).astype(np.uint32).view(np.float32))
        with np.errstate(invalid="ignore", divide="ignore"):
            conf_ref = (m2.numpy() - m1) / m2.numpy()
            conf_tar = (t2.numpy() - tm1) / t2.numpy()
        return md, conf_ref.astype(np.float32), mdr, conf_tar.astype(np.float32)


def _volume(D, H, W, seed):
    rng = np.random.default_rng(seed)
    # few distinct levels -> many exact ties across shards (the tie rules matter)
    C = rng.integers(1, 12, size=(D, H, W)).astype(np.float32) * np.float32(0.25)
    C[:, 0, :3] = 5.0  # a pixel row with an all-equal start
    return C


def _worker(rank, world, store, D, H, W, seed, out_path):
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    try:
        C = _volume(D, H, W, seed)  # plane-major [D][H][W]
        b, e = shard_range(D, rank, world)
        local = torch.from_numpy(np.ascontiguousarray(C[b:e].transpose(1, 2, 0)))

        def reduce_min(t):
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return t

        d_ref, conf_ref, d_tar, conf_tar = sharded_wta(CpuShardOps(b, e, D), local, reduce_min)
        if rank == 0:
            np.savez(out_path, d_ref=d_ref, conf_ref=conf_ref, d_tar=d_tar, conf_tar=conf_tar)
    finally:
        dist.destroy_process_group()


def _group_worker(rank, world, G, store, D, H, W, out_dir):
    """bench.py's layout: world/G frame groups, each d-sharded over its G ranks."""
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    try:
        groups, gid, grank = world // G, rank // G, rank % G
        subs = [dist.new_group(list(range(g * G, (g + 1) * G))) for g in range(groups)]
        pg = subs[gid]
        C = _volume(D, H, W, 777 + gid)  # one frame per group
        b, e = shard_range(D, grank, G)
        local = torch.from_numpy(np.ascontiguousarray(C[b:e].transpose(1, 2, 0)))

        def reduce_min(t):
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=pg)
            return t

        d_ref, conf_ref, d_tar, conf_tar = sharded_wta(CpuShardOps(b, e, D), local, reduce_min)
        stat = torch.tensor([float(rank)])
        dist.all_reduce(stat, op=dist.ReduceOp.MAX)  # the bench's max-over-ranks on the world group
        assert stat.item() == world - 1
        if grank == 0:
            np.savez(os.path.join(out_dir, f"g{gid}.npz"), d_ref=d_ref, d_tar=d_tar, conf_ref=conf_ref,
                     conf_tar=conf_tar)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,G", [(4, 0), (8, 0), (8, 8)])
def test_frame_groups_gloo(oracle, tmp_path, world, G):
    """bench.py --gpus 4 / 8 layouts on gloo: plan_groups' 2-way groups (G = 0), and one
    frame d-sharded 8 ways (--group-size 8)."""
    from stereo_matchin_amd.distributed import plan_groups
    D, H, W = 16, 4, 18
    if not G:
        G = plan_groups(D, world, min_planes=8)
        assert G == 2
    mp.start_processes(_group_worker, args=(world, G, _store(tmp_path), D, H, W, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    for gid in range(world // G):
        got = np.load(tmp_path / f"g{gid}.npz")
        dr, cr, dt, ct = oracle.wta(_volume(D, H, W, 777 + gid))
        assert np.array_equal(got["d_ref"], dr) and np.array_equal(got["d_tar"], dt)
        np.testing.assert_array_equal(got["conf_ref"], cr)
        np.testing.assert_array_equal(got["conf_tar"], ct)


def test_plan_groups():
    from stereo_matchin_amd.distributed import plan_groups
    assert [plan_groups(256, n) for n in (1, 2, 4, 8)] == [1, 2, 2, 2]
    assert plan_groups(512, 8) == 2 and plan_groups(61, 2) == 1 and plan_groups(128, 8) == 2
    assert plan_groups(256, 3) == 3 and plan_groups(100, 3) == 1 and plan_groups(256, 6) == 2


def _store(tmp_path):
    """A FileStore rendezvous file in the test's own directory: no TCP port to pick, so
    concurrent tests (pytest -n) cannot race for one."""
    return str(tmp_path / "rendezvous")


@pytest.mark.parametrize("world,D,H,W", [(2, 16, 6, 20), (3, 13, 5, 17), (2, 61, 4, 70), (8, 64, 4, 40)])
def test_sharded_wta_gloo_matches_oracle(oracle, tmp_path, world, D, H, W):
    seed = 1234 + world + D
    out = str(tmp_path / "res.npz")
    mp.start_processes(_worker, args=(world, _store(tmp_path), D, H, W, seed, out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    dr, cr, dt, ct = oracle.wta(_volume(D, H, W, seed))
    assert np.array_equal(got["d_ref"], dr)
    assert np.array_equal(got["d_tar"], dt)
    np.testing.assert_array_equal(got["conf_ref"], cr)
    np.testing.assert_array_equal(got["conf_tar"], ct)


def test_shard_range_covers_exactly():
    for D in (1, 16, 61, 256, 512):
        for world in range(1, min(D, 9) + 1):
            spans = [shard_range(D, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == D
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(e - b for b, e in spans) - min(e - b for b, e in spans) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 0, 5)
