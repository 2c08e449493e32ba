"""The C-ABI library loads and exports every symbol include/asw.h declares (CPU only:
host-side helpers are called, no kernel is launched)."""
import ctypes
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    import stereo_matchin_amd._lib as L
    L.lib()
    return L


def test_every_header_symbol_is_exported(L):
    names = L.header_functions()
    assert len(names) >= 20
    lib = L.lib()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes signature table covers exactly the header
    assert set(names) == set(L.SIGNATURES)


def test_abi_version(L):
    import re
    assert L.lib().asw_abi_version() == 4
    # the binding's mirrored struct layouts are the header's revision (_load refuses others)
    hdr = open(os.path.join(ROOT, "include", "asw.h")).read()
    assert int(re.search(r"#define ASW_ABI_VERSION (\d+)", hdr).group(1)) == L.ABI_VERSION


def test_tune_set_rejects_bits_that_select_nothing(L):
    lib = L.lib()
    assert lib.asw_tune_set(1, 64) == L.ASW_E_INVALID      # round 1's 10-wave H form: no longer built
    assert lib.asw_tune_set(1, 1 << 28) == L.ASW_E_INVALID
    assert lib.asw_tune_set(1, 1 << 26) == 0 and lib.asw_tune_set(1, 0) == 1 << 26  # 32-plane passes: nt flipped
    # round 6: the 32-plane H pass's 4-wave-block (bit 24) and LDS-left-ring (bit 27) forms are no longer built
    assert lib.asw_tune_set(1, 1 << 24) == L.ASW_E_INVALID
    assert lib.asw_tune_set(1, 1 << 27) == L.ASW_E_INVALID
    assert lib.asw_tune_set(2, 5) == L.ASW_E_INVALID
    # WTA variant 1 (wave per pixel) is no longer built (tools/exp/exp_forms.hip)
    assert lib.asw_tune_set(2, 1) == L.ASW_E_INVALID
    assert lib.asw_tune_set(2, 2) == 0 and lib.asw_tune_set(2, 0) == 2
    old = lib.asw_tune_set(1, 128)
    assert lib.asw_tune_set(1, old) == 128


def test_default_params_are_the_reference_values(L):
    p = L.default_params(384, 288)
    # K/asw_aggr.cl:16 (61 levels), K/asw_vcost_aggregation.cl:33 (33 taps), main.cpp:177 (r=7),
    # K/asw_vsupport.cl:22,24 (30.91, 28.21), untruncated AD, LR check with 8-bit codes
    assert (p.ndisp, p.taps, p.iters) == (61, 33, 7)
    assert p.gamma_c == pytest.approx(30.91) and p.gamma_g == pytest.approx(28.21)
    assert p.tad_tau >= 765.0 and p.lr_check == 1 and p.lr_mode == L.LR_U8
    assert p.d_begin == 0 and p.d_stop == 61
    assert L.params_check(p) == L.ASW_OK


@pytest.mark.parametrize("D,T,Dp,Tp", [(61, 33, 64, 36), (16, 5, 64, 12), (64, 35, 64, 36), (256, 35, 256, 36),
                                       (512, 51, 512, 52), (65, 3, 128, 4)])
def test_layout_pitches(L, D, T, Dp, Tp):
    p = L.default_params(100, 50, ndisp=D, taps=T)
    assert L.disp_pitch(p) == Dp and L.tap_pitch(p) == Tp
    assert (Tp // 4) % 2 == 1  # odd number of 16-B slots per support row (LDS banks)
    lib = L.lib()
    assert lib.asw_cost_bytes(ctypes.byref(p)) == 100 * 50 * Dp * 4
    assert lib.asw_support_bytes(ctypes.byref(p)) == 100 * 50 * Tp * 4
    assert lib.asw_lut_bytes(ctypes.byref(p)) == (T // 2 + 1) * 766 * 4


def test_shard_pitch(L):
    p = L.default_params(10, 10, ndisp=256, taps=35, d_begin=64, d_end=128)
    assert L.disp_pitch(p) == 64
    # a shard of <= 32 planes: pitch 32 (the half-wave passes, asw_pass32.h)
    p = L.default_params(10, 10, ndisp=256, taps=35, d_begin=0, d_end=32)
    assert L.disp_pitch(p) == 32
    p = L.default_params(10, 10, ndisp=256, taps=35, d_begin=250, d_end=256)
    assert L.disp_pitch(p) == 32
    p = L.default_params(10, 10, ndisp=32, taps=35)  # the whole range: 64-plane blocks
    assert L.disp_pitch(p) == 64


@pytest.mark.parametrize("field,value", [("width", 0), ("height", -1), ("ndisp", 0), ("taps", 4), ("iters", -1),
                                         ("gamma_c", 0.0), ("d_begin", 70), ("lr_mode", 7)])
def test_params_check_rejects(L, field, value):
    p = L.default_params(32, 32)
    setattr(p, field, value)
    assert L.params_check(p) == L.ASW_E_INVALID


def test_color_space_values(L):
    assert L.params_check(L.default_params(32, 32, color_space=L.COLOR_LAB)) == L.ASW_OK
    assert L.params_check(L.default_params(32, 32, color_space=7)) == L.ASW_E_INVALID


def test_strerror(L):
    for s in (L.ASW_OK, L.ASW_E_INVALID, L.ASW_E_HIP, L.ASW_E_NOMEM, L.ASW_E_UNSUPPORTED):
        assert L.strerror(s)
    assert L.strerror(123) == "unknown status"


def test_stage_api_validates_before_launch(L):
    # invalid parameters / null pointers are rejected host-side, never launched
    lib = L.lib()
    p = L.default_params(0, 0)
    assert lib.asw_raw_cost(ctypes.byref(p), None, None, None, None) == L.ASW_E_INVALID
    p = L.default_params(8, 8)
    assert lib.asw_raw_cost(ctypes.byref(p), None, None, None, None) == L.ASW_E_INVALID
    assert lib.asw_aggregate_pass(ctypes.byref(p), 5, 1, 1, 1, 2, None) == L.ASW_E_INVALID
    assert lib.asw_aggregate_pass(ctypes.byref(p), 0, 1, 1, 1, 1, None) == L.ASW_E_INVALID  # in place
    # cached-denominator pass: bad mode, missing den, den aliasing the output
    assert lib.asw_aggregate_pass_den(ctypes.byref(p), 0, 1, 1, 1, 2, 3, 7, None) == L.ASW_E_INVALID
    assert lib.asw_aggregate_pass_den(ctypes.byref(p), 0, 1, 1, 1, 2, None, L.DEN_READ, None) == L.ASW_E_INVALID
    assert lib.asw_aggregate_pass_den(ctypes.byref(p), 0, 1, 1, 1, 2, 2, L.DEN_WRITE, None) == L.ASW_E_INVALID
    p.d_end = 30
    assert lib.asw_wta(ctypes.byref(p), 1, 1, 1, 1, 1, None, None, None) == L.ASW_E_INVALID  # sharded


def test_pass_rejects_volumes_past_32bit_offsets(L):
    # the pass kernels address up to ~2T+16 cost rows from a 32-bit buffer offset
    # (ADVICE r01): such shapes return ASW_E_UNSUPPORTED before any launch
    lib = L.lib()
    p = L.default_params(7680, 64, ndisp=1280, taps=51)
    assert L.params_check(p) == L.ASW_OK
    assert lib.asw_aggregate_pass(ctypes.byref(p), 0, 1, 1, 1, 2, None) == L.ASW_E_UNSUPPORTED
    assert lib.asw_aggregate_pass_den(ctypes.byref(p), 1, 1, 1, 1, 2, 3, L.DEN_WRITE, None) == L.ASW_E_UNSUPPORTED
    # C5 (3840 x 2160, D 512, T 51) is inside the range; so are the supports (< 2 GiB)
    q = L.default_params(3840, 2160, ndisp=512, taps=51)
    assert 3840 * 512 * 4 * (2 * 51 + 16) < 2 ** 31
    assert lib.asw_support_bytes(ctypes.byref(q)) < 2 ** 31
    # the frame API rejects them at create, before any device call or allocation
    # (an 8K D512 frame used to allocate tens of GB and fail at its
    # first pass); a multi-shard context checks each shard's own pitch
    ctx = ctypes.c_void_p()
    big = L.default_params(7680, 4320, ndisp=512, taps=51)
    assert lib.asw_create(ctypes.byref(big), 0, ctypes.byref(ctx)) == L.ASW_E_UNSUPPORTED and not ctx.value
    ids = (ctypes.c_int * 2)(0, 0)
    wide = L.default_params(7680, 64, ndisp=1280, taps=51)
    assert lib.asw_create_multi(ctypes.byref(wide), ids, 2, ctypes.byref(ctx)) == L.ASW_E_UNSUPPORTED


def test_frame_api_validates_before_allocating(L):
    lib = L.lib()
    p = L.default_params(16, 8, ndisp=16, taps=5)
    ctx = ctypes.c_void_p()
    devs = (ctypes.c_int * 2)(0, 0)
    assert lib.asw_create_multi(ctypes.byref(p), devs, 0, ctypes.byref(ctx)) == L.ASW_E_INVALID
    assert lib.asw_create_multi(ctypes.byref(p), None, 2, ctypes.byref(ctx)) == L.ASW_E_INVALID
    assert lib.asw_create_rank(ctypes.byref(p), 0, 2, 2, b"\0" * 128, ctypes.byref(ctx)) == L.ASW_E_INVALID
    p.d_end = 8  # contexts shard the disparity axis themselves
    assert lib.asw_create(ctypes.byref(p), 0, ctypes.byref(ctx)) == L.ASW_E_INVALID
    assert lib.asw_ctx_shard(None, 0, None, None, None) == L.ASW_E_INVALID
    assert lib.asw_match_batch(None, None, None, 1, None, None) == L.ASW_E_INVALID
    assert L.strerror(L.ASW_E_COMM)


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: without libasw_hip.so every product entry point raises
    AswLibraryError (checked in a child process, ASW_LIB pointing nowhere)."""
    import subprocess
    import sys
    code = (
        "import torch\n"
        "from stereo_matchin_amd import _lib, make_params, StereoMatcher\n"
        "try:\n"
        "    StereoMatcher(make_params(16, 8, ndisp=4, taps=3, iters=1), torch.device('cpu'))\n"
        "    _lib.lib()\n"
        "except _lib.AswLibraryError as e:\n"
        "    print('LOUD', e)\n"
    )
    env = dict(os.environ, ASW_LIB=str(tmp_path / "absent.so"))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert "LOUD" in r.stdout, (r.stdout, r.stderr[-2000:])


def test_params_flags(L):
    """asw_params.flags (ABI 4): the context options; the bits of the forms removed in
    round 6 (measured slower in every shape) and unknown bits are rejected."""
    import re
    p = L.default_params(32, 32)
    assert p.flags == 0
    for f in (L.FLAG_COMM_LOCAL, L.FLAG_RAW_F32, L.FLAG_COMM_LOCAL | L.FLAG_RAW_F32):
        p.flags = f
        assert L.params_check(p) == L.ASW_OK
    for f in (0x1, 0x2, 0x4, 0x8, 0x10, 0x80, 0x100, 0x200):
        p.flags = f
        assert L.params_check(p) == L.ASW_E_INVALID
    hdr = open(os.path.join(ROOT, "include", "asw.h")).read()
    assert sorted(re.findall(r"#define ASW_FLAG_(\w+) ", hdr)) == ["ALL", "COMM_LOCAL", "RAW_F32"]
    for name in ("COMM_LOCAL", "RAW_F32"):
        v = int(re.search(rf"#define ASW_FLAG_{name} (0x[0-9A-Fa-f]+)", hdr).group(1), 16)
        assert v == getattr(L, f"FLAG_{name}")
    # the library reads no environment switch (the flags replaced them)
    src = open(os.path.join(ROOT, "stereo_matchin_amd", "csrc", "asw_frame.cpp")).read()
    assert "getenv" not in src


def test_removed_forms_are_not_exported(L):
    """Round 6 removed the opt-in forms that lost their A/B everywhere (DESIGN.md
    §Keep/drop): their entry points are gone from the library and the header."""
    import re
    hdr = open(os.path.join(ROOT, "include", "asw.h")).read()
    lib = L.lib()
    for name in ("asw_aggregate_pass_otf", "asw_pass_otf_supported", "asw_aggregate_pass_otf_v",
                 "asw_pass_otf_v_supported", "asw_aggregate_pass_raw", "asw_pass_raw_supported",
                 "asw_support_all_fmt", "asw_support_index_bytes", "asw_aggregate_pass_index",
                 "asw_pass_index_supported", "asw_aggregate_pass_wta_local", "asw_pass_wta_local_supported"):
        assert not hasattr(lib, name), name
        assert not re.search(rf"\b{name}\(", hdr), name


def test_raw16_supported_and_validation(L):
    """asw_raw16_supported / asw_raw_cost16 / asw_aggregate_pass_den16 (the uint16 raw
    costs): integral or absent truncation, ring tap counts, a first pass only; rejected
    host-side before any launch."""
    lib = L.lib()
    ok = L.default_params(64, 32, ndisp=64, taps=35)
    assert lib.asw_raw16_supported(ctypes.byref(ok)) == 1
    assert lib.asw_raw16_supported(ctypes.byref(L.default_params(64, 32, ndisp=64, taps=35, tad_tau=40.0))) == 1
    assert lib.asw_raw16_supported(ctypes.byref(L.default_params(64, 32, ndisp=64, taps=35, tad_tau=40.5))) == 0
    assert lib.asw_raw16_supported(ctypes.byref(L.default_params(64, 32, ndisp=64, taps=11))) == 0  # no ring kernel
    assert lib.asw_raw16_supported(ctypes.byref(L.default_params(64, 32, ndisp=64, taps=35, iters=0))) == 0
    shard = L.default_params(64, 32, ndisp=256, taps=35, d_begin=32, d_end=64)  # pitch 32: k_vpass32
    assert lib.asw_raw16_supported(ctypes.byref(shard)) == 1
    x, y = ctypes.c_void_p(1), ctypes.c_void_p(2)
    frac = L.default_params(64, 32, ndisp=64, taps=35, tad_tau=40.5)
    assert lib.asw_raw_cost16(ctypes.byref(frac), x, x, y, None) == L.ASW_E_UNSUPPORTED
    assert lib.asw_raw_cost16(ctypes.byref(ok), None, x, y, None) == L.ASW_E_INVALID
    # den-read is never a first pass; den-write needs a den volume; in place is refused
    assert lib.asw_aggregate_pass_den16(ctypes.byref(ok), x, x, x, y, y, L.DEN_READ, None) == L.ASW_E_INVALID
    assert lib.asw_aggregate_pass_den16(ctypes.byref(ok), x, x, x, y, None, L.DEN_WRITE, None) == L.ASW_E_INVALID
    assert lib.asw_aggregate_pass_den16(ctypes.byref(ok), x, x, y, y, None, L.DEN_NONE, None) == L.ASW_E_INVALID
    q = L.default_params(64, 32, ndisp=64, taps=11)
    assert lib.asw_aggregate_pass_den16(ctypes.byref(q), x, x, x, y, None, L.DEN_NONE, None) == L.ASW_E_UNSUPPORTED
    assert L.FLAG_RAW_F32 == 0x40
