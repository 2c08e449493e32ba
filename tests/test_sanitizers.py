"""Host sanitizer build (SURVEY §5 "Race detection / sanitizers"):
`make ASAN=1` builds asw_stereo, png_tool and the oracle with
-fsanitize=address,undefined (host code only, g++/gcc; no device code is
sanitized), and these CPU tests run the PNG round trips, a structured PNG fuzz of
the decoder (png_io.cpp parses untrusted chunks), the CLI's error paths and every
oracle entry point under it.  Any sanitizer report aborts the process, so a zero
exit status is the assertion.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from test_host import CASES, _write_png

PIL = pytest.importorskip("PIL.Image")
PKG = os.path.join(ROOT, "stereo_matchin_amd")
PNG_TOOL = os.path.join(PKG, "png_tool_asan")
CLI = os.path.join(PKG, "asw_stereo_asan")
ORACLE = os.path.join(ROOT, "oracle", "_ref", "asan_check")
# the HIP runtime the CLI loads keeps allocations to process exit: leaks are not the question here
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def asan_tools():
    subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(PKG, "host"), "ASAN=1"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ASAN=1"], check=True)
    return PNG_TOOL


def _run(args, **kw):
    r = subprocess.run(args, capture_output=True, text=True, env=ENV, timeout=600, **kw)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, r.stderr[-4000:]
    return r


@pytest.mark.parametrize("interlace", [False, True])
def test_asan_png_decode_all_types(asan_tools, tmp_path, interlace):
    for ctype, depth in CASES:
        rng = np.random.default_rng(ctype * 100 + depth)
        C = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
        top, plte, trns = (1 << depth) - 1, None, None
        if ctype == 3:
            plte = rng.integers(0, 256, 3 << depth).astype(np.uint8)
            trns = rng.integers(0, 256, max(1, (1 << depth) // 2)).astype(np.uint8)
        samples = rng.integers(0, top + 1, (9, 7, C))
        path = tmp_path / f"t{ctype}_{depth}.png"
        _write_png(path, samples, ctype, depth, interlace, plte, trns)
        r = _run([asan_tools, "decode", str(path), str(tmp_path / "o.raw")])
        assert r.returncode == 0, (ctype, depth, r.stderr)
        got = np.fromfile(tmp_path / "o.raw", np.uint8).reshape(9, 7, 4)
        if depth != 16 or ctype != 0:
            np.testing.assert_array_equal(got, np.asarray(PIL.open(path).convert("RGBA")))


def test_asan_png_round_trips(asan_tools, tmp_path):
    rng = np.random.default_rng(5)
    for ch in (1, 4):
        img = rng.integers(0, 256, (23, 31, ch), dtype=np.uint8)
        img.tofile(tmp_path / "in.raw")
        assert _run([asan_tools, "encode", str(tmp_path / "in.raw"), "31", "23", str(ch),
                     str(tmp_path / "o.png")]).returncode == 0
        np.testing.assert_array_equal(np.asarray(PIL.open(tmp_path / "o.png")).reshape(img.shape), img)
    img16 = rng.integers(0, 65536, (17, 19), dtype=np.uint16)
    img16.tofile(tmp_path / "in16.raw")
    assert _run([asan_tools, "encode16", str(tmp_path / "in16.raw"), "19", "17",
                 str(tmp_path / "o16.png")]).returncode == 0
    np.testing.assert_array_equal(np.asarray(PIL.open(tmp_path / "o16.png")).astype(np.uint16), img16)


# seeds of every chunk shape the decoder handles: RGBA8, palette + tRNS, Adam7 grey16,
# 2-bit grey; each gets 20k structured mutants (IHDR fields, chunk order / length /
# duplicates, recompressed random scanlines, truncated zlib streams, CRC flips)
@pytest.mark.parametrize("ctype,depth,interlace", [(6, 8, False), (3, 4, False), (0, 16, True), (0, 2, True)])
def test_asan_png_fuzz(asan_tools, tmp_path, ctype, depth, interlace):
    rng = np.random.default_rng(depth)
    C = {0: 1, 3: 1, 6: 4}[ctype]
    plte = rng.integers(0, 256, 3 << depth).astype(np.uint8) if ctype == 3 else None
    trns = rng.integers(0, 256, 5).astype(np.uint8) if ctype == 3 else None
    seed = tmp_path / "seed.png"
    _write_png(seed, rng.integers(0, 1 << min(depth, 8), (11, 13, C)), ctype, depth, interlace, plte, trns)
    r = _run([asan_tools, "fuzz", str(seed), "20000", str(ctype * 1000 + depth)])
    assert r.returncode == 0, r.stderr[-4000:]
    n, ok = map(int, r.stdout.split())
    assert n == 20000 and 0 < ok < n  # some mutants still decode, most are rejected


def test_asan_cli_error_paths(asan_tools, tmp_path):
    r = _run([CLI, "--bogus"])
    assert r.returncode == 2 and "usage" in r.stderr
    r = _run([CLI, "--pics", str(tmp_path / "missing.txt")])
    assert r.returncode == 1 and "cannot read" in r.stderr
    # a pics.txt whose images are missing or not PNGs: reported per pair, no device work
    (tmp_path / "bad.png").write_bytes(b"\x89PNG\r\n\x1a\nnot really")
    (tmp_path / "pics.txt").write_text("missing/a.png\nmissing/b.png\nbad.png\nbad.png\n")
    r = _run([CLI, "--pics", str(tmp_path / "pics.txt"), "--runs", "1"], cwd=tmp_path)  # (its TSV lands there)
    assert r.returncode == 1 and "missing" in r.stderr


def test_asan_oracle(asan_tools):
    r = _run([ORACLE])
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.count("sum=") == 5 and "shard" in r.stdout
