"""Frames streamed through distributed.PipelinedMatcher — run on an MI355X.

Frame k's WTA tail (the d-sharded exchange of K/asw_wta.cl:34-67's reductions, the
target scan, the LR check of K/consist.cl) runs on a side stream while frame k+1
aggregates in the other set of volumes.  Every frame's maps and images must equal the
plain StereoMatcher's (itself bit-exact against the oracle, test_gpu_parity.py), for a
whole-range matcher and for a 2-rank d-sharded one (gloo over one GPU, as bench.py's
rehearsal).
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ("d_ref", "d_tar", "conf_ref", "conf_tar", "code_ref", "code_tar", "lr_rgba", "lr_red_rgba")


def _pairs(n, H, W, D):
    from stereo_matchin_amd.synthetic import make_pair
    return [make_pair(W, H, D, 11 + k)[:2] for k in range(n)]


def _np(res):
    return {k: getattr(res, k).cpu().numpy() for k in KEYS}


# overlap_prep: frame k+1's raw cost and supports on a third stream beside frame k's
# passes (the inputs are resident and synchronized before the first submit)
@pytest.mark.parametrize("overlap_prep", [False, True])
def test_pipelined_whole_range_equals_match(gpu, overlap_prep):
    import torch

    from stereo_matchin_amd import StereoMatcher, make_params
    from stereo_matchin_amd.distributed import PipelinedMatcher
    H, W, D, T = 96, 320, 64, 9
    p = make_params(W, H, ndisp=D, taps=T, iters=3)
    pairs = [(torch.from_numpy(L).to(gpu), torch.from_numpy(R).to(gpu)) for L, R in _pairs(5, H, W, D)]
    want = [_np(StereoMatcher(p, gpu).match(L, R)) for L, R in pairs]
    torch.cuda.synchronize()
    pm = PipelinedMatcher(p, device=gpu, overlap_prep=overlap_prep)
    got = [pm.submit(L, R) for L, R in pairs]  # 5 frames through 2 sets of volumes
    pm.flush()
    torch.cuda.synchronize()
    for k, res in enumerate(got):  # (each frame's maps are tensors of its own)
        g = _np(res)
        for key in KEYS:
            assert np.array_equal(g[key], want[k][key]), (k, key)


def _rank_main(rank, world, store, out, H, W, D, T, overlap_prep=False):
    import torch
    import torch.distributed as dist

    # a FileStore rendezvous in the test's directory: no TCP port to pick (no race under pytest -n)
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    from stereo_matchin_amd import make_params
    from stereo_matchin_amd.distributed import PipelinedMatcher
    dev = torch.device("cuda:0")
    p = make_params(W, H, ndisp=D, taps=T, iters=3)
    pm = PipelinedMatcher(p, rank, world, dev, overlap_prep=overlap_prep)
    inputs = [(torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)) for L, R in _pairs(4, H, W, D)]
    torch.cuda.synchronize()  # (overlap_prep: the inputs are valid before the first submit)
    res = [pm.submit(L, R) for L, R in inputs]
    pm.flush()
    torch.cuda.synchronize()
    if rank == 0:
        np.savez(out, **{f"{k}_{key}": v for k, r in enumerate(res) for key, v in _np(r).items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap_prep", [False, True])
def test_pipelined_sharded_two_ranks_equals_match(gpu, tmp_path, overlap_prep):
    import torch
    import torch.multiprocessing as tmp

    from stereo_matchin_amd import StereoMatcher, make_params
    H, W, D, T = 64, 256, 64, 9
    out = str(tmp_path / "pipe.npz")
    tmp.spawn(_rank_main, args=(2, str(tmp_path / "rendezvous"), out, H, W, D, T, overlap_prep), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    p = make_params(W, H, ndisp=D, taps=T, iters=3)
    for k, (L, R) in enumerate(_pairs(4, H, W, D)):
        want = _np(StereoMatcher(p, gpu).match(torch.from_numpy(L).to(gpu), torch.from_numpy(R).to(gpu)))
        for key in KEYS:
            assert np.array_equal(got[f"{k}_{key}"], want[key]), (k, key)
