"""configs[0] fixture: the Input-data scene (Scene.cpp:3-224 over the
reference's own OBJ files) at 256x256, 4 samples per pixel, 5 bounces, on
the oracle's serial loop (threads=1, the reference's CPU plumbing case).

    python tests/golden/make_configs0.py

Writes tests/golden/configs0_256x256_4spp.json: the image's sha256 (float32
accumulator bytes), its segment count, the per-channel sums and the BMP
payload's sha256 (Renderer::renderImage, Renderer.cpp:15-63, ITER = 4).  A
regression pin of the oracle at this exact config; the oracle itself is
pinned to the reference's Render.bmp (tests/test_oracle_golden.py), and
tests/test_configs0.py checks this render's block means against it too.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

W, H, SPP, BOUNCES = 256, 256, 4, 5


def render():
    import oracle as O
    O.build()
    sc = O.reference_scene(os.path.join(ROOT, "scenes", "input_data"))
    img, seg = O.render(sc, O.RenderConfig(width=W, height=H, iterations=SPP, max_bounces=BOUNCES, threads=1))
    return O, img, seg


def main():
    O, img, seg = render()
    out = {"width": W, "height": H, "spp": SPP, "max_bounces": BOUNCES, "threads": 1, "segments": int(seg),
           "image_sha256": hashlib.sha256(img.tobytes()).hexdigest(),
           "bmp_sha256": hashlib.sha256(O.to_bmp_bytes(img, W, H, SPP)).hexdigest(),
           "channel_sums": [float(x) for x in img.astype("float64").sum(0)]}
    with open(os.path.join(HERE, "configs0_256x256_4spp.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
