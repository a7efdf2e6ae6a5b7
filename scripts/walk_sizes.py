"""Distribution of k_trace_gf's walks over hit-set size (stats build, PT_DEBUG_ABLATE=2048):
    PT_LIB_PATH=build_variants/lib_stats.so python scripts/walk_sizes.py"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["PT_DEBUG_ABLATE"] = "2048"
import pathtracerap_amd as P  # noqa: E402
from pathtracerap_amd import synthetic  # noqa: E402

for ntri in (100_000, 1_000_000):
    s = P.Scene(synthetic.diffuse_scene(tempfile.mkdtemp(), ntri=ntri))
    s.build()
    r = P.Renderer(P.RenderConfig(width=1280, height=1024, max_bounces=8))
    r.allocateOnGPU(s)
    r.renderLoop(0, 4)
    c = r.segments_per_bounce(128)
    w = c[51 + 63:55 + 63]
    tot = max(sum(w), 1)
    print(ntri, "walks", sum(w), "per segment", round(sum(w) / r.segments(), 3),
          "share nh=1,2,3,>=4:", [round(x / tot, 3) for x in w], flush=True)
    r.free()
s = P.Scene(os.path.join(ROOT, "scenes", "reference_scene.txt"))
s.build()
r = P.Renderer(P.RenderConfig(width=1280, height=1024, max_bounces=5))
r.allocateOnGPU(s)
r.renderLoop(0, 4)
c = r.segments_per_bounce(128)
w = c[51 + 63:55 + 63]
tot = max(sum(w), 1)
print("reference scene walks", sum(w), "share nh=1,2,3,>=4:", [round(x / tot, 3) for x in w])
