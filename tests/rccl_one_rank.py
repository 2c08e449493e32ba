"""Child process of tests/test_gpu_rccl.py: a one-rank torch.distributed "nccl"
(RCCL) process group, initialised the way bench.py does for N > 1, and the
d-sharded WTA protocol with its four MIN all-reduces forced through RCCL (a
one-rank group would otherwise skip them).  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from stereo_matchin_amd import StereoMatcher, make_params  # noqa: E402
from stereo_matchin_amd.distributed import HipShardOps, sharded_wta  # noqa: E402
from stereo_matchin_amd.synthetic import make_pair  # noqa: E402


def main():
    port = int(sys.argv[1])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    out = {"backend": dist.get_backend()}
    # int64 and float32 MIN: the key and second-minimum exchanges of the protocol
    k = torch.tensor([5, -3, 1 << 40], dtype=torch.int64, device=dev)
    dist.all_reduce(k, op=dist.ReduceOp.MIN)
    f = torch.tensor([1.5, -2.0], dtype=torch.float32, device=dev)
    dist.all_reduce(f, op=dist.ReduceOp.MIN)
    out["int64_min_ok"] = k.tolist() == [5, -3, 1 << 40]
    out["f32_min_ok"] = f.tolist() == [1.5, -2.0]

    def reduce_min(t):
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return t

    W, H, D, T, r = 192, 64, 64, 9, 2
    Lh, Rh, _ = make_pair(W, H, D, 3)
    L, R = torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev)
    # no LR check: Constistency zeroes the confidences of inconsistent pixels in place
    p = make_params(W, H, ndisp=D, taps=T, iters=r, lr_check=0)
    m = StereoMatcher(p, dev)
    whole = m.match(L, R)
    sh = sharded_wta(HipShardOps(m.p), whole.cost, reduce_min)
    torch.cuda.synchronize()
    names = ("d_ref", "conf_ref", "d_tar", "conf_tar", "code_ref", "code_tar")
    out["mismatch"] = {n: int((a != getattr(whole, n)).sum()) for a, n in zip(sh, names)}
    out["protocol_equals_wta"] = not any(out["mismatch"].values())
    dist.destroy_process_group()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
