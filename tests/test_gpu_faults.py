"""GPU: failure reporting of the persistent traces and stream/graph hygiene
of the host side.  A trace that hits its iteration cap must make
synchronize() / image() fail instead of shading stale hit records into a
silently wrong image; rebinding the accumulator after a hipGraph capture must
keep results exact."""
import pytest

from helpers import assert_bitexact, flat_from_export, oracle_cfg

pytestmark = pytest.mark.gpu


def _scene(P, synth_dir, seed=3):
    from pathtracerap_amd import synthetic
    s = P.Scene(synthetic.diffuse_scene(synth_dir, ntri=3000, seed=seed))
    s.build(bvh=True)
    return s


@pytest.fixture(scope="module")
def synth_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("synth_faults"))


@pytest.mark.parametrize("accel", [1, 2])
def test_trace_iteration_cap_is_an_error(gpu, pt_mod, synth_dir, monkeypatch, accel):
    P = pt_mod
    monkeypatch.setenv("PT_TRACE_ITER_CAP", "3")      # every wave gives up almost at once
    s = _scene(P, synth_dir)
    r = P.Renderer(P.RenderConfig(width=64, height=48, iterations=1, max_bounces=4, accel=accel, pipelines=2))
    r.allocateOnGPU(s)
    r.renderLoop(0, 2, sync=False)
    with pytest.raises(P.PathTracerError, match="gave up"):
        r.synchronize()
    assert r.trace_faults() > 0
    with pytest.raises(P.PathTracerError, match="image invalid"):
        r.image()
    r.free()


def test_trace_fault_records_the_stuck_lanes(gpu, pt_mod, synth_dir, monkeypatch):
    """A k_trace_gf wave that gives up records its 64 lanes by state in diagnostic
    slots 59..62 (idle, done, select, node/leaf/walk) and counts itself in 63 when its
    ray pool was exhausted (renderer.hip, the iteration-cap check): scripts/hangcheck.py
    prints them, which is how the state-7 livelock of round 4 was found."""
    P = pt_mod
    monkeypatch.setenv("PT_TRACE_ITER_CAP", "3")
    s = _scene(P, synth_dir)
    r = P.Renderer(P.RenderConfig(width=64, height=48, iterations=1, max_bounces=4, accel=P.ACCEL_GRID_FAST,
                                  pipelines=2))
    r.allocateOnGPU(s)
    r.renderLoop(0, 2, sync=False)
    with pytest.raises(P.PathTracerError, match="gave up"):
        r.synchronize()
    faults = r.trace_faults()
    v = r.segments_per_bounce(128)
    lanes = [v[63 + slot] for slot in range(59, 63)]
    assert faults > 0
    assert sum(lanes) == 64 * faults, (lanes, faults)
    assert 0 <= v[63 + 63] <= faults
    r.free()


@pytest.mark.parametrize("accel", [1, 2])
def test_no_trace_faults_in_a_normal_run(gpu, pt_mod, synth_dir, accel):
    P = pt_mod
    s = _scene(P, synth_dir)
    r = P.Renderer(P.RenderConfig(width=96, height=64, iterations=3, max_bounces=8, accel=accel, pipelines=3))
    r.allocateOnGPU(s)
    r.renderLoop()
    assert r.trace_faults() == 0
    r.free()


@pytest.mark.parametrize("accel,pipes", [(2, 1), (1, 1), (2, 3)])
def test_graph_replay_rebind_image_between_loops(gpu, pt_mod, oracle_mod, synth_dir, monkeypatch, accel, pipes):
    """PT_GRAPH=1: bind_image between two renderLoop calls (graphs captured
    with the old accumulator in flight) waits for the enqueued work, drops the
    graphs and re-captures: each accumulator holds exactly its iterations."""
    import torch
    P, O = pt_mod, oracle_mod
    monkeypatch.setenv("PT_GRAPH", "1")
    s = _scene(P, synth_dir, seed=4)
    cfg = P.RenderConfig(width=81, height=47, iterations=5, max_bounces=6, accel=accel, pipelines=pipes)
    n = cfg.width * cfg.height * 3
    a = torch.zeros(n, dtype=torch.float32, device="cuda")
    b = torch.zeros(n, dtype=torch.float32, device="cuda")
    st = torch.cuda.Stream()
    r = P.Renderer(cfg)
    r.set_stream(st.cuda_stream)
    r.bind_image(a.data_ptr(), keepalive=a)
    r.allocateOnGPU(s)
    r.renderLoop(0, 2, sync=False)           # captured graphs write `a`
    r.bind_image(b.data_ptr(), keepalive=b)  # while those launches may still run
    r.renderLoop(2, 3, sync=False)
    r.synchronize()
    got_a = a.cpu().numpy().reshape(-1, 3)
    got_b = b.cpu().numpy().reshape(-1, 3)
    r.free()
    flat = flat_from_export(s.export())
    oc = oracle_cfg(cfg)
    oc.iterations, oc.first_iter = 2, 0
    want_a, _ = O.render(flat, oc)
    oc.iterations, oc.first_iter = 3, 2
    want_b, _ = O.render(flat, oc)
    assert_bitexact(got_a, want_a, "accumulator bound first")
    assert_bitexact(got_b, want_b, "accumulator bound second")


def test_trace_flags_checked_only_where_they_apply(gpu, pt_mod, oracle_mod, synth_dir, monkeypatch):
    """A leftover PT_GF_FLAGS / PT_TRACE_FLAGS value fails allocateOnGPU only for
    the trace that reads it: the reference grid mode renders as usual (and equals
    the oracle), while grid_fast refuses an invalid PT_GF_FLAGS and bvh an
    invalid PT_TRACE_FLAGS."""
    P, O = pt_mod, oracle_mod
    monkeypatch.setenv("PT_GF_FLAGS", "13")
    monkeypatch.setenv("PT_TRACE_FLAGS", "27")
    s = _scene(P, synth_dir)
    cfg = P.RenderConfig(width=40, height=32, iterations=1, max_bounces=4, accel=P.ACCEL_GRID)
    r = P.Renderer(cfg)
    r.allocateOnGPU(s)
    r.renderLoop()
    img = r.image()
    r.free()
    want, _ = O.render(flat_from_export(s.export()), oracle_cfg(cfg))
    assert_bitexact(img, want, "grid mode with leftover trace flags")
    for accel, flag in ((P.ACCEL_GRID_FAST, "PT_GF_FLAGS"), (P.ACCEL_BVH, "PT_TRACE_FLAGS")):
        r = P.Renderer(P.RenderConfig(width=40, height=32, iterations=1, max_bounces=4, accel=accel))
        with pytest.raises(P.PathTracerError, match=flag):
            r.allocateOnGPU(s)
        r.free()
