"""The sample-sharded multi-rank path on the HIP renderer (dist.render_sharded
with its default GPU branch): two gloo ranks share the one GPU, each renders
its iteration range (Renderer.cpp:582-644: iterations are independent) into its
own torch accumulator on the caller's stream, and the all-reduced image equals
the single-rank render up to fp32 summation order (rtol 1e-6).  bench.py's N>1
path uses the same split with RCCL over xGMI; on the 8-GPU node it is the
driver that runs it."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from helpers import flat_from_export, oracle_cfg

pytestmark = pytest.mark.gpu

WORKER = r"""
import os, sys
sys.path.insert(0, {root!r})
import numpy as np
import torch
import torch.distributed as dist
import pathtracerap_amd as P
from pathtracerap_amd.dist import render_sharded
rank = int(os.environ["RANK"])
dist.init_process_group("gloo")
torch.cuda.set_device(0)
s = P.Scene({scene_path!r})          # written once by the parent
s.build()
cfg = P.RenderConfig(width=96, height=72, iterations={iters}, max_bounces=8)
img = render_sharded(s, cfg, {iters})
assert img.is_cuda
if rank == 0:
    np.save({out!r}, img.cpu().numpy())
dist.barrier()
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_render_sharded_hip_two_ranks(gpu, pt_mod, oracle_mod, tmp_path):
    from pathtracerap_amd import synthetic
    P, O = pt_mod, oracle_mod
    iters = 7                                         # odd: the ranks get 4 and 3 iterations
    scene_dir = str(tmp_path / "scene")
    out = str(tmp_path / "img.npy")
    script = tmp_path / "worker.py"
    scene_path = synthetic.diffuse_scene(scene_dir, ntri=3000, seed=31, metallic=True)   # both ranks read it
    script.write_text(WORKER.format(root=ROOT, scene_path=scene_path, iters=iters, out=out))
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)
    got = np.load(out).reshape(-1, 3)

    s = P.Scene(scene_path)
    s.build()
    cfg = P.RenderConfig(width=96, height=72, iterations=iters, max_bounces=8)
    r = P.Renderer(cfg)
    r.allocateOnGPU(s)
    r.renderLoop()
    single = r.image()
    r.free()
    want, _ = O.render(flat_from_export(s.export()), oracle_cfg(cfg, threads=16))
    assert np.array_equal(single.view(np.uint32), want.view(np.uint32))
    assert np.abs(got).sum() > 0
    np.testing.assert_allclose(got, single, rtol=1e-6, atol=1e-6)


README_WORKER = r"""
import os, sys
sys.path.insert(0, {root!r})
import numpy as np
import torch
import torch.distributed as dist
import pathtracerap_amd as P
from pathtracerap_amd.dist import render_sharded
rank = int(os.environ["RANK"])
dist.init_process_group("gloo")
torch.cuda.set_device(0)
s = P.Scene({scene!r})
s.build()
cfg = s.apply_settings(P.RenderConfig())
cfg.width, cfg.height, cfg.pipelines = 2800, 2240, 2
img = render_sharded(s, cfg, 2)                 # 1 + 1 iterations
if rank == 0:
    np.save({out!r}, img.cpu().numpy())
dist.barrier()
dist.destroy_process_group()
"""


def _run_ranks(script, n=2, timeout=300):
    port = _free_port()
    procs = []
    for rank in range(n):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(n), LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=timeout)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)


def test_configs3_readme_scene_sharded_two_ranks(gpu, pt_mod, oracle_mod, tmp_path):
    """configs[3]'s workload: the README scene (Scene.cpp:3-224) at 2800x2240,
    its samples sharded over ranks (here 2 iterations split 1 + 1 over two gloo
    ranks sharing the GPU; RCCL over xGMI on the 8-GPU node) and the float3
    accumulators sum-reduced: equals the oracle's 2-iteration render."""
    from conftest import REF_SCENE
    P, O = pt_mod, oracle_mod
    out = str(tmp_path / "img.npy")
    script = tmp_path / "worker_readme.py"
    script.write_text(README_WORKER.format(root=ROOT, scene=REF_SCENE, out=out))
    _run_ranks(script)
    got = np.load(out).reshape(-1, 3)
    s = P.Scene(REF_SCENE)
    s.build()
    cfg = s.apply_settings(P.RenderConfig())
    cfg.width, cfg.height, cfg.iterations = 2800, 2240, 2
    want, _ = O.render(flat_from_export(s.export()), oracle_cfg(cfg, threads=16))
    assert np.abs(got).sum() > 0
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=0)


def test_bench_gpus_2_spawns_two_ranks(gpu):
    """bench.py --gpus 2 without a launcher starts both ranks itself (here gloo,
    two ranks on the one GPU) and reports the whole job: n_gpus == 2."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--steps", "2", "--warmup", "1", "--targets=", "--alt-accel=", "--no-cpu-baseline",
                        "--no-full-runs", "--no-profile"], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, p.stdout
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["trace_faults"] == 0
    assert d["config"]["parallelism"].startswith("samples sharded x2")


RCCL_WORKER = r"""
import os, sys
sys.path.insert(0, {root!r})
import numpy as np
import torch
import torch.distributed as dist
import pathtracerap_amd as P
from pathtracerap_amd.dist import render_sharded
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
s = P.Scene({scene_path!r})
s.build()
cfg = P.RenderConfig(width=96, height=72, iterations={iters}, max_bounces=8)
img = render_sharded(s, cfg, {iters})          # the all-reduce runs through RCCL even at world size 1
assert img.is_cuda
np.save({out!r}, img.cpu().numpy())
dist.destroy_process_group()
print("rccl ok")
"""


def test_rccl_one_rank_render_sharded_equals_oracle(gpu, pt_mod, oracle_mod, tmp_path):
    """RCCL loads, initialises (nccl backend, device_id=cuda:0) and orders its
    all-reduce after the renderer's launches on the torch stream: a one-rank
    group renders through render_sharded with the collective on the renderer's
    accumulator, and the image equals the oracle's bit for bit (a one-rank sum
    is exact)."""
    from pathtracerap_amd import synthetic
    P, O = pt_mod, oracle_mod
    iters = 3
    scene_path = synthetic.diffuse_scene(str(tmp_path / "scene"), ntri=3000, seed=37, metallic=True)
    out = str(tmp_path / "img.npy")
    script = tmp_path / "worker_rccl.py"
    script.write_text(RCCL_WORKER.format(root=ROOT, scene_path=scene_path, iters=iters, out=out))
    _run_ranks(script, n=1, timeout=240)
    got = np.load(out)
    s = P.Scene(scene_path)
    s.build()
    cfg = P.RenderConfig(width=96, height=72, iterations=iters, max_bounces=8)
    want, _ = O.render(flat_from_export(s.export()), oracle_cfg(cfg, threads=16))
    assert np.abs(got).sum() > 0
    assert np.array_equal(got.view(np.uint32), want.reshape(-1).view(np.uint32))


def test_bench_under_a_launcher_with_rccl_one_rank(gpu):
    """bench.py as the driver's N>1 launch runs it (WORLD_SIZE set, nccl), at one
    rank: the process group is RCCL, the accumulator all-reduce is inside the
    timed region, and the line reports it."""
    import json
    port = _free_port()
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist-backend", "nccl",
                        "--steps", "2", "--warmup", "1", "--targets=", "--alt-accel=", "--no-cpu-baseline",
                        "--no-full-runs", "--no-profile"], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, p.stdout
    d = json.loads(line[0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["config"]["trace_faults"] == 0
    assert "RCCL" in d["config"]["parallelism"]
