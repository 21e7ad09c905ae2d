"""Natural-image fixtures (tests/golden/natural_images.npz + natural_oracle.json).

The reference holds no per-stage vectors (it has no tests; OpenCV is absent), so the ORB /
SGBM kernels are checked against the oracle on real camera statistics here: flat and
saturated regions, FAST / Harris ties at the retainBest cut, repetitive texture.  Inputs are
the public scikit-image sample images present in this build container (SURVEY.md Appendix C;
BSD-licensed data, decoded with PIL):

* camera, grass, gravel, brick (512 x 512 gray) -- ORB at 500 / 1000 features;
* ``montage600``: the four tiled 2 x 2 and cropped to 960 x 600 (the bench geometry);
* the rectified Middlebury "motorcycle" pair (741 x 500 RGB -> gray with OpenCV's 14-bit
  BGR2GRAY weights) and its ground-truth disparity (x16 as uint16, 0 = invalid) -- SGBM.

natural_oracle.json records sha256 digests (+ counts) of the oracle's outputs on them, so
the CPU suite pins the oracle against regressions without committing the large outputs.
Regenerate only on a deliberate oracle change:  python tests/golden/make_golden_natural.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
SK = "/opt/conda/lib/python3.9/site-packages/skimage/data"

import oracle  # noqa: E402


def gray_from_rgb(rgb: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(RGB2GRAY) 8-bit: (R*4899 + G*9617 + B*1868 + 2^13) >> 14."""
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14).astype(np.uint8)


def load_gray(name: str) -> np.ndarray:
    from PIL import Image
    im = np.asarray(Image.open(os.path.join(SK, name)))
    return gray_from_rgb(im) if im.ndim == 3 else im.astype(np.uint8)


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode() + str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def oracle_outputs(imgs: dict) -> dict:
    """The expected outputs the fixtures pin (computed by the oracle)."""
    out = {}
    for name in ("camera", "grass", "gravel", "brick", "montage600"):
        for nf in (500, 1000):
            kp, d = oracle.orb_detect_compute(imgs[name], nf)
            out[f"orb/{name}/{nf}"] = {"n": int(len(kp)), "sha256": digest(kp, d)}
    kp0, d0 = oracle.orb_detect_compute(imgs["moto_L"], 1000)
    kp1, d1 = oracle.orb_detect_compute(imgs["moto_R"], 1000)
    m = oracle.bf_match(d0, d1)
    out["bf/moto_L-moto_R/1000"] = {"n": int(len(m)), "sha256": digest(m)}
    disp = oracle.sgbm(imgs["moto_L"], imgs["moto_R"])
    out["sgbm/moto/96"] = {"sha256": digest(disp)}
    disp128 = oracle.sgbm(imgs["moto_L"], imgs["moto_R"], num_disp=128)
    out["sgbm/moto/128"] = {"sha256": digest(disp128)}
    return out


def main():
    oracle.build()
    imgs = {k: load_gray(k + ".png") for k in ("camera", "grass", "gravel", "brick")}
    mont = np.block([[imgs["camera"], imgs["grass"]], [imgs["gravel"], imgs["brick"]]])
    imgs["montage600"] = np.ascontiguousarray(mont[:600, :960])
    imgs["moto_L"] = load_gray("motorcycle_left.png")
    imgs["moto_R"] = load_gray("motorcycle_right.png")
    gt = np.load(os.path.join(SK, "motorcycle_disp.npz"))["arr_0"].astype(np.float64)
    gt16 = np.where(np.isfinite(gt) & (gt > 0), np.round(gt * 16), 0).astype(np.uint16)
    np.savez_compressed(os.path.join(HERE, "natural_images.npz"), moto_gt16=gt16, **imgs)
    ref = oracle_outputs(imgs)
    with open(os.path.join(HERE, "natural_oracle.json"), "w") as f:
        json.dump(ref, f, indent=1, sort_keys=True)
    print({k: v.get("n") for k, v in ref.items()})


if __name__ == "__main__":
    main()
