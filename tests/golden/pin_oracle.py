"""Pin the CPU oracle against the reference's own output image.

Renders the Scene.cpp scene at the reference's Config.h settings
(1000x800, ITER=500, 5 bounces) with the oracle and compares the BMP bytes
with the reference's committed PathTracerAP/Render.bmp (fixture
tests/golden/reference_render_1000x800_500.npz).  The oracle render takes
~30 min on one core, so the result (the oracle's BMP payload) is cached in
tests/golden/oracle_render_1000x800_500.npz and the statistics are written to
tests/golden/oracle_pin_stats.json; tests/test_oracle_golden.py re-checks the
committed numbers and re-renders a cheap slice.

    python tests/golden/pin_oracle.py [threads]
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle as O  # noqa: E402


def compare(ours: np.ndarray, ref: np.ndarray) -> dict:
    d = np.abs(ours.astype(np.int32) - ref.astype(np.int32))
    return {
        "pixels": int(d.shape[0] * d.shape[1]),
        "exact_byte_fraction": float((d == 0).mean()),
        "within_1_fraction": float((d <= 1).mean()),
        "within_2_fraction": float((d <= 2).mean()),
        "within_4_fraction": float((d <= 4).mean()),
        "mean_abs_diff": float(d.mean()),
        "p99_abs_diff": float(np.percentile(d, 99)),
        "max_abs_diff": int(d.max()),
        "mean_ours": [float(x) for x in ours.reshape(-1, 3).mean(0)],
        "mean_ref": [float(x) for x in ref.reshape(-1, 3).mean(0)],
    }


def main(threads=1):
    sc = O.reference_scene(os.path.join(os.path.dirname(os.path.dirname(HERE)), "scenes", "input_data"))
    cfg = O.RenderConfig(width=1000, height=800, iterations=500, threads=int(threads))
    t = time.time()
    img, seg = O.render(sc, cfg)
    el = time.time() - t
    px = np.frombuffer(O.to_bmp_bytes(img, 1000, 800, 500)[54:], np.uint8).reshape(800, 1000, 3)
    ref = np.load(os.path.join(HERE, "reference_render_1000x800_500.npz"))["bgr"]
    st = compare(px, ref)
    st["oracle_seconds"] = el
    st["segments"] = int(seg)
    np.savez_compressed(os.path.join(HERE, "oracle_render_1000x800_500.npz"), bgr=px)
    with open(os.path.join(HERE, "oracle_pin_stats.json"), "w") as f:
        json.dump(st, f, indent=1)
    print(json.dumps(st, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
