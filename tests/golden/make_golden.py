"""Regenerate the committed golden fixtures from the reference checkout.

Run once in the build container (the GPU box has no /root/reference):

    python tests/golden/make_golden.py [/root/reference/PathTracerAP]

Writes
  scenes/input_data/{enclosing_box,ceiling_light,blender_monkey}.obj
      -- the reference's own scene inputs (data files, copied verbatim);
  tests/golden/reference_render_1000x800_500.npz
      -- the pixel payload of the reference's committed output image
         PathTracerAP/Render.bmp (Renderer::renderImage, 1000x800, ITER=500,
         Scene.cpp scene): key ``bgr`` = uint8 (800, 1000, 3) in file order
         (row 0 = bottom row, bytes in the order the reference wrote them:
         R,G,B of the float accumulator), plus ``header`` = the 54 bytes.
"""
import os
import shutil
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main(ref=None):
    ref = ref or "/root/reference/PathTracerAP"
    for f in ("enclosing_box.obj", "ceiling_light.obj", "blender_monkey.obj"):
        shutil.copyfile(os.path.join(ref, "Input data", f), os.path.join(HERE, "..", "..", "scenes", "input_data", f))
    raw = open(os.path.join(ref, "Render.bmp"), "rb").read()
    w, h = struct.unpack("<ii", raw[18:26])
    off = struct.unpack("<I", raw[10:14])[0]
    px = np.frombuffer(raw[off:off + 3 * w * h], np.uint8).reshape(h, w, 3)
    np.savez_compressed(os.path.join(HERE, "reference_render_1000x800_500.npz"),
                        bgr=px, header=np.frombuffer(raw[:54], np.uint8))
    print("wrote fixtures", w, h)


if __name__ == "__main__":
    main(*sys.argv[1:])
