"""Generate the committed golden fixtures from the reference's own data files.

Run in the survey/build container (where /root/reference exists):

    python tests/golden/make_golden.py

For each Middlebury scene listed in the reference's stereo_matching/pics.txt it
stores, in ``tests/golden/<scene>.npz``:

* ``left``, ``right``: the input pair as RGB u8 [H][W][3] (main.cpp:183-186 decodes
  them with lodepng to RGBA8; alpha is 255 everywhere);
* ``lr_red``: the reference's device-produced ``asw_consistency_pre-reff.png``
  (RGB u8) — the output of ``Constistency`` right after the initial ASW WTA
  (main.cpp:529-537, read back and encoded at :625-627).  This is the hot path's
  own end-to-end output at the reference parameters D=61, T=33, r=7;
* ``lr_post_red``: ``asw_consistency_post-reff.png``, the consistency image after
  the k = 6 refinement iterations (main.cpp:540-613, encoded at :629-631);
* ``disp_final``: ``asw_disparity.png``, the 3x3 median of the refined
  consistency image (main.cpp:615-623).

These are data (inputs and expected outputs), not reference source.
PNG decoding uses PIL, which is only needed to regenerate the fixtures.
"""
from __future__ import annotations

import os
import sys

import numpy as np

REF = "/root/reference/stereo_matching"
OUT = os.path.dirname(os.path.abspath(__file__))


def main() -> int:
    from PIL import Image

    if not os.path.isdir(REF):
        print("reference not present; nothing to do", file=sys.stderr)
        return 1
    with open(os.path.join(REF, "pics.txt")) as f:
        lines = [ln.strip() for ln in f if ln.strip()]
    pairs = list(zip(lines[0::2], lines[1::2]))
    for lp, rp in pairs:
        scene = lp.split("/")[0]
        left = np.array(Image.open(os.path.join(REF, lp)).convert("RGB"))
        right = np.array(Image.open(os.path.join(REF, rp)).convert("RGB"))
        red = np.array(Image.open(os.path.join(REF, scene, "asw_consistency_pre-reff.png")).convert("RGB"))
        # after the k = 6 refinement iterations and the 3x3 median (main.cpp:540-631)
        post = np.array(Image.open(os.path.join(REF, scene, "asw_consistency_post-reff.png")).convert("RGB"))
        final = np.array(Image.open(os.path.join(REF, scene, "asw_disparity.png")).convert("RGB"))
        assert left.shape == right.shape == red.shape == post.shape == final.shape, scene
        np.savez_compressed(os.path.join(OUT, f"{scene}.npz"), left=left, right=right, lr_red=red,
                            lr_post_red=post, disp_final=final,
                            source=np.array(f"{lp} {rp} {scene}/asw_consistency_pre-reff.png "
                                            f"{scene}/asw_consistency_post-reff.png {scene}/asw_disparity.png"))
        print(scene, left.shape)
    return 0


if __name__ == "__main__":
    sys.exit(main())
