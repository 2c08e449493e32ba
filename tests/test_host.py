"""Host driver (stereo_matchin_amd/host): PNG I/O and the asw_stereo CLI.

The reference decodes/encodes with lodepng (main.cpp:183-186, 621-631); png_io
is an independent implementation over zlib, checked here against PIL on every
colour type / bit depth / interlace combination, and the CLI is checked end to
end (GPU) against the reference's own committed asw_consistency_pre-reff.png.
"""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

from conftest import ROOT, load_scene

PIL = pytest.importorskip("PIL.Image")
PKG = os.path.join(ROOT, "stereo_matchin_amd")
PNG_TOOL = os.path.join(PKG, "png_tool")
CLI = os.path.join(PKG, "asw_stereo")


@pytest.fixture(scope="module")
def tools():
    subprocess.run(["make", "-s", "-C", os.path.join(PKG, "host"), "../png_tool"], check=True)
    return PNG_TOOL


def _decode(tool, path, tmp_path):
    raw = tmp_path / "out.raw"
    r = subprocess.run([tool, "decode", str(path), str(raw)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    w, h = map(int, r.stdout.split())
    return np.fromfile(raw, np.uint8).reshape(h, w, 4)


def _chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def _pack_row(samples, depth):
    if depth == 8:
        return bytes(samples.astype(np.uint8))
    if depth == 16:
        return samples.astype(">u2").tobytes()
    per = 8 // depth
    out = bytearray((len(samples) + per - 1) // per)
    for i, s in enumerate(samples):
        out[i // per] |= int(s) << (8 - depth * (i % per + 1))
    return bytes(out)


def _write_png(path, samples, ctype, depth, interlace=False, plte=None, trns=None, filt=1):
    """Minimal independent PNG writer: samples [H][W][C] integers (all filters exercised)."""
    H, W, C = samples.shape
    bpp = max(1, C * depth // 8)

    def filtered(rows):
        out, prev = b"", None
        for k, r in enumerate(rows):
            r = bytearray(r)
            ft = (filt + k) % 5
            cur = bytearray(r)
            for i in range(len(r)):
                a = r[i - bpp] if i >= bpp else 0
                b = prev[i] if prev is not None else 0
                c = prev[i - bpp] if (prev is not None and i >= bpp) else 0
                if ft == 1:
                    cur[i] = (r[i] - a) & 255
                elif ft == 2:
                    cur[i] = (r[i] - b) & 255
                elif ft == 3:
                    cur[i] = (r[i] - ((a + b) >> 1)) & 255
                elif ft == 4:
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pr = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                    cur[i] = (r[i] - pr) & 255
            out += bytes([ft]) + bytes(cur)
            prev = r
        return out

    raw = b""
    passes = ADAM7 if interlace else [(0, 0, 1, 1)]
    for x0, y0, dx, dy in passes:
        sub = samples[y0::dy, x0::dx]
        if sub.size == 0:
            continue
        raw += filtered([_pack_row(row.reshape(-1), depth) for row in sub])
    ihdr = struct.pack(">IIBBBBB", W, H, depth, ctype, 0, 0, 1 if interlace else 0)
    data = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr)
    if plte is not None:
        data += _chunk(b"PLTE", bytes(plte))
    if trns is not None:
        data += _chunk(b"tRNS", bytes(trns))
    data += _chunk(b"tEXt", b"Comment\x00ancillary chunk") + _chunk(b"IDAT", zlib.compress(raw)) + _chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(data)


CASES = [(0, 1), (0, 2), (0, 4), (0, 8), (0, 16), (2, 8), (2, 16), (3, 1), (3, 4), (3, 8), (4, 8), (4, 16),
         (6, 8), (6, 16)]


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("ctype,depth", CASES)
def test_png_decode_matches_pil(tools, tmp_path, ctype, depth, interlace):
    rng = np.random.default_rng(ctype * 100 + depth + interlace)
    H, W = 13, 11
    C = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    top = (1 << depth) - 1
    plte = trns = None
    if ctype == 3:
        n = 1 << depth
        plte = rng.integers(0, 256, 3 * n).astype(np.uint8)
        trns = rng.integers(0, 256, max(1, n // 2)).astype(np.uint8)
        top = n - 1
    samples = rng.integers(0, top + 1, (H, W, C))
    path = tmp_path / "t.png"
    _write_png(path, samples, ctype, depth, interlace, plte, trns)
    got = _decode(tools, path, tmp_path)
    ref = np.asarray(PIL.open(path).convert("RGBA"))
    if depth == 16 and ctype != 0:
        # PIL reduces 16-bit colour to 8 bits by the high byte, as png_io does
        np.testing.assert_array_equal(got, ref)
    elif depth == 16:
        np.testing.assert_array_equal(got[..., :3], (samples[..., 0] >> 8).astype(np.uint8)[..., None].repeat(3, -1))
    else:
        np.testing.assert_array_equal(got, ref)


def test_png_decode_rejects_corruption(tools, tmp_path):
    p = tmp_path / "c.png"
    _write_png(p, np.zeros((4, 4, 3), int), 2, 8)
    b = bytearray(p.read_bytes())
    b[40] ^= 0xFF  # inside IHDR/IDAT -> CRC mismatch
    p.write_bytes(bytes(b))
    r = subprocess.run([tools, "decode", str(p), str(tmp_path / "x.raw")], capture_output=True, text=True)
    assert r.returncode != 0 and r.stderr


@pytest.mark.parametrize("channels", [1, 4])
def test_png_encode_round_trip(tools, tmp_path, channels):
    rng = np.random.default_rng(channels)
    img = rng.integers(0, 256, (37, 53, channels), dtype=np.uint8)
    img[:10] = 7  # flat rows -> filter choice None vs Paeth both exercised
    raw = tmp_path / "in.raw"
    img.tofile(raw)
    out = tmp_path / "o.png"
    r = subprocess.run([tools, "encode", str(raw), "53", "37", str(channels), str(out)], capture_output=True)
    assert r.returncode == 0
    back = np.asarray(PIL.open(out))
    np.testing.assert_array_equal(back.reshape(img.shape), img)


def test_png_encode16_round_trip(tools, tmp_path):
    # 16-bit grey disparity maps (D > 256: the 8-bit codes collide)
    rng = np.random.default_rng(16)
    img = rng.integers(0, 65536, (29, 41), dtype=np.uint16)
    img[:5] = 511
    img[5, :] = 0xFFFF
    raw = tmp_path / "in16.raw"
    img.tofile(raw)
    out = tmp_path / "o16.png"
    r = subprocess.run([tools, "encode16", str(raw), "41", "29", str(out)], capture_output=True)
    assert r.returncode == 0, r.stderr
    im = PIL.open(out)
    assert im.mode.startswith("I")
    np.testing.assert_array_equal(np.asarray(im).astype(np.uint16), img)


def test_cli_usage_errors(tmp_path):
    subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(PKG, "host")], check=True)
    r = subprocess.run([CLI, "--bogus"], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr
    r = subprocess.run([CLI, "--pics", str(tmp_path / "missing.txt")], capture_output=True, text=True)
    assert r.returncode == 1 and "cannot read" in r.stderr


@pytest.mark.gpu
def test_cli_tsukuba_reproduces_reference_png(tmp_path):
    """pics.txt -> asw_stereo -> asw_consistency_pre-reff.png == the reference's committed file."""
    L, R, dev_red = load_scene("tsukuba")
    d = tmp_path / "tsukuba"
    d.mkdir()
    PIL.fromarray(L[..., :3]).save(d / "im1.png")
    PIL.fromarray(R[..., :3]).save(d / "im5.png")
    (tmp_path / "pics.txt").write_text("tsukuba/im1.png\ntsukuba/im5.png\nmissing/a.png\nmissing/b.png\n")
    tsv = tmp_path / "times.tsv"
    r = subprocess.run([CLI, "--pics", str(tmp_path / "pics.txt"), "--runs", "2", "--tsv", str(tsv)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 1, r.stderr  # the missing pair is reported, the rest still runs
    assert "missing" in r.stderr
    out = np.asarray(PIL.open(d / "asw_consistency_pre-reff.png").convert("RGB"))
    np.testing.assert_array_equal(out, dev_red)
    for name in ("asw_wta_disparity.png", "asw_consistency.png"):
        assert (d / name).exists()
    lines = tsv.read_text().splitlines()
    header = next(ln for ln in lines if ln.startswith("id\t"))
    rows = [ln for ln in lines if ln[:1].isdigit()]
    assert len(rows) == 2 and all(len(ln.split("\t")) == len(header.split("\t")) for ln in rows)


@pytest.mark.gpu
def test_cli_devices_refine_matches_reference(tmp_path):
    """--devices 0,0 with the default --refine 6: the d-sharded refinement writes the
    reference's asw_disparity.png and asw_consistency_post-reff.png (main.cpp:617-631),
    byte-exact against the committed tsukuba files (--devices used to drop
    refinement silently)."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "tsukuba.npz"))
    d = tmp_path / "tsukuba"
    d.mkdir()
    PIL.fromarray(z["left"]).save(d / "im1.png")
    PIL.fromarray(z["right"]).save(d / "im5.png")
    (tmp_path / "pics.txt").write_text("tsukuba/im1.png\ntsukuba/im5.png\n")
    r = subprocess.run([CLI, "--pics", str(tmp_path / "pics.txt"), "--runs", "1", "--devices", "0,0"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "skipped" not in r.stderr
    for name, key in (("asw_disparity.png", "disp_final"), ("asw_consistency_post-reff.png", "lr_post_red"),
                      ("asw_consistency_pre-reff.png", "lr_red")):
        np.testing.assert_array_equal(np.asarray(PIL.open(d / name).convert("RGB")), z[key], err_msg=name)


@pytest.mark.gpu
def test_cli_devices_and_png16(tmp_path):
    """--devices 0,0 (two d-shards on one GPU, asw_create_multi) reproduces the one-GPU
    images; --png16 writes the 16-bit disparity maps (d_ref; 65535 = LR-inconsistent)."""
    L, R, dev_red = load_scene("tsukuba")
    d = tmp_path / "tsukuba"
    d.mkdir()
    PIL.fromarray(L[..., :3]).save(d / "im1.png")
    PIL.fromarray(R[..., :3]).save(d / "im5.png")
    (tmp_path / "pics.txt").write_text("tsukuba/im1.png\ntsukuba/im5.png\n")
    r = subprocess.run([CLI, "--pics", str(tmp_path / "pics.txt"), "--runs", "1", "--devices", "0,0", "--png16",
                        "--refine", "0", "--tsv", str(tmp_path / "t.tsv")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    np.testing.assert_array_equal(np.asarray(PIL.open(d / "asw_consistency_pre-reff.png").convert("RGB")), dev_red)
    d16 = np.asarray(PIL.open(d / "asw_wta_disparity16.png")).astype(np.int64)
    c16 = np.asarray(PIL.open(d / "asw_consistency16.png")).astype(np.int64)
    wta8 = np.asarray(PIL.open(d / "asw_wta_disparity.png").convert("L")).astype(np.int64)
    assert d16.max() <= 60
    np.testing.assert_array_equal((17 * d16 + 1) >> 2, wta8)  # the reference's round-half-down code
    red = (dev_red[..., 0] == 255) & (dev_red[..., 1] == 0) & (dev_red[..., 2] == 0)
    np.testing.assert_array_equal(c16 == 65535, red)
    np.testing.assert_array_equal(c16[~red], d16[~red])
