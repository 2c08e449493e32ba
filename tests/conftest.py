import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
SCENES = ["tsukuba", "cones", "teddy", "laundry", "art"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


def rgba(a):
    a = np.asarray(a, np.uint8)
    return np.ascontiguousarray(np.concatenate([a, np.full(a.shape[:2] + (1,), 255, np.uint8)], -1))


def load_scene(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    return rgba(z["left"]), rgba(z["right"]), z["lr_red"]


def plane_major(cost_hwd, D):
    """device [H][W][Dp] -> oracle [D][H][W]"""
    c = np.asarray(cost_hwd)
    return np.ascontiguousarray(np.transpose(c[:, :, :D], (2, 0, 1)))


def pixel_major(cost_dhw, Dp):
    """oracle [D][H][W] -> device [H][W][Dp] (zero padded)"""
    D, H, W = cost_dhw.shape
    out = np.zeros((H, W, Dp), np.float32)
    out[:, :, :D] = np.transpose(cost_dhw, (1, 2, 0))
    return out


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import stereo_matchin_amd._lib as L
    L.lib()  # loud failure if the HIP library is missing
    return torch.device("cuda:0")


@pytest.fixture
def tune_variant():
    """asw_tune_set(ASW_TUNE_PASS_VARIANT, v) for one test, restored afterwards."""
    from stereo_matchin_amd import _lib
    saved = []

    def set_(v):
        old = _lib.lib().asw_tune_set(1, v)
        assert old >= 0, f"asw_tune_set rejected pass variant {v:#x} ({old})"  # an unknown bit: never applied
        saved.append(old)

    yield set_
    if saved:
        _lib.lib().asw_tune_set(1, saved[0])
