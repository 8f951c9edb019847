"""Generate tests/golden/earthmap_rgb8.png: the pixels of the reference's own texture asset.

The reference loads `./assets/earthmap.jpg` with `image::open` (src/textures/image_texture.rs:19-33;
used by generate_earth, src/application.rs:604-612, and generate_final, :897-901) and keeps the
decoded RGB8 bytes (1024x512x3).  This script decodes the same file with Pillow (libjpeg-turbo) and
stores the pixels losslessly as PNG, so the GPU box (which has no /root/reference) renders the Earth
scenes with the reference's texture on both sides of every parity test.

Decoder caveat: the reference decodes with the `jpeg-decoder 0.3.0` crate (Cargo.lock), Pillow with
libjpeg-turbo.  Both are baseline-JPEG IDCT implementations whose outputs can differ by a few levels in
some pixels; no reference output pins the decoded bytes (parity unpinned at this boundary).  The GPU
and the oracle read the SAME bytes, so GPU-vs-oracle parity is unaffected.

Run (in the container that has the reference):  python tests/golden/make_earthmap.py
"""
import os

import numpy as np
from PIL import Image

SRC = "/root/reference/assets/earthmap.jpg"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "earthmap_rgb8.png")


def main():
    im = Image.open(SRC)
    assert im.mode == "RGB", im.mode  # image_texture.rs: components = 3 for this asset
    px = np.asarray(im, dtype=np.uint8)
    Image.fromarray(px, "RGB").save(OUT, optimize=True)
    back = np.asarray(Image.open(OUT), dtype=np.uint8)
    assert np.array_equal(back, px)
    print(OUT, px.shape, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
