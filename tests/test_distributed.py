"""Multi-rank spp sharding on CPU (gloo, world_size 2): each rank renders its frame-id shard
(with the CPU oracle standing in for the GPU renderer), the accumulators are summed to
rank 0 with the same collective bench.py uses, and the result equals the single-process
render of all frames up to fp32 summation order."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total_spp, mode, out_dir):
    sys.path.insert(0, str(ROOT))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from optixpathtracer_amd import scenes, sharding
    from oracle.oracle import OracleScene

    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = scenes.tiny_scene("layered")
    o = OracleScene(sc)
    lp = o.launch(24, 16, 3)
    if mode == "strong":
        first, n = sharding.split_frames(total_spp, rank, world)
        img, _ = o.render(lp, first, n, threads=2)
    else:  # weak: two steps of total_spp frames per rank
        img = np.zeros((16, 24, 3), np.float32)
        for step in range(2):
            first, n = sharding.frame_range(step, rank, world, total_spp)
            img, _ = o.render(lp, first, n, sum_rgb=img, threads=2)
    t = torch.from_numpy(img)
    sharding.reduce_accumulator(t, dist)
    if rank == 0:
        np.save(os.path.join(out_dir, f"{mode}.npy"), t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["strong", "weak"])
def test_two_rank_spp_shard_equals_single(tmp_path, mode):
    import torch.multiprocessing as mp

    from optixpathtracer_amd import scenes
    from oracle.oracle import OracleScene

    world, spp = 2, 5
    mp.spawn(_worker, args=(world, _free_port(), spp, mode, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / f"{mode}.npy")
    sc = scenes.tiny_scene("layered")
    o = OracleScene(sc)
    lp = o.launch(24, 16, 3)
    total = spp if mode == "strong" else 2 * world * spp
    want, _ = o.render(lp, 1, total, threads=4)
    np.testing.assert_allclose(got, want, rtol=2e-6, atol=1e-7)


def test_shard_ranges_partition_the_frames():
    from optixpathtracer_amd import sharding

    for total in [1, 7, 1024, 4096]:
        for world in [1, 2, 3, 8]:
            ids = []
            for r in range(world):
                f, n = sharding.split_frames(total, r, world)
                ids += list(range(f, f + n))
            assert ids == list(range(1, total + 1))
    seen = set()
    for step in range(3):
        for r in range(4):
            f, n = sharding.frame_range(step, r, 4, 16)
            s = set(range(f, f + n))
            assert not (s & seen)
            seen |= s
    assert seen == set(range(1, 1 + 3 * 4 * 16))


def _gpu_worker(rank, world, port, total_spp, out_dir):
    sys.path.insert(0, str(ROOT))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from optixpathtracer_amd import scenes, sharding
    from optixpathtracer_amd.renderer import setup_renderer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = scenes.tiny_scene("conductor")
    r = setup_renderer(sc, 48, 32, 5, device=0)
    r.set_frames_per_launch(4)
    r.accum_clear()
    first, n = sharding.split_frames(total_spp, rank, world)
    r.render_frames(first, n)
    t = torch.from_numpy(r.accum())
    r.close()
    sharding.reduce_accumulator(t, dist)
    if rank == 0:
        np.save(os.path.join(out_dir, "gpu_strong.npy"), t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_process_gpu_shards_reduce_to_single_render(tmp_path):
    """The bench's multi-GPU path with two processes on one card: each renders its frame-id
    shard through libptamd, the host accumulators are summed over gloo (RCCL needs one GPU
    per rank), and the result equals one process rendering every frame, up to the fp32
    order of the cross-rank sum."""
    import torch.multiprocessing as mp

    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    world, spp = 2, 11
    mp.spawn(_gpu_worker, args=(world, _free_port(), spp, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "gpu_strong.npy")
    sc = scenes.tiny_scene("conductor")
    r = setup_renderer(sc, 48, 32, 5, device=0)
    r.accum_clear()
    r.render_frames(1, spp)
    want = r.accum()
    r.close()
    np.testing.assert_allclose(got, want, rtol=2e-6, atol=1e-7)


def _gpu_bench_worker(rank, world, port, spp, steps, out_dir):
    """bench.py's per-rank loop with a device accumulator: per step, sharding.render_step (clear
    -> render -> sync -> reduce -> sync); rank 0 keeps each step's reduced sum."""
    sys.path.insert(0, str(ROOT))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from optixpathtracer_amd import scenes, sharding
    from optixpathtracer_amd.renderer import setup_renderer

    # one GPU on the test box: RCCL needs a GPU per rank, so the collective runs over gloo on
    # host copies (sharding.reduce_accumulator); buffers, streams and step order are bench.py's
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    sc = scenes.tiny_scene("conductor")
    r = setup_renderer(sc, 48, 32, 5, device=0)
    r.set_frames_per_launch(3)  # several batches over both wavefront streams per step
    accum = torch.zeros((32, 48, 3), dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)
    r.set_accum_device_buffer(accum.data_ptr())
    red = []
    for s in range(steps):
        first, n = sharding.split_frames(spp, rank, world, base=1 + s * spp)
        red.append(sharding.render_step(r, accum, dist, first, n))
        if rank == 0:
            np.save(os.path.join(out_dir, f"step{s}.npy"), accum.cpu().numpy())
    rep = sharding.distributed_report(dist, red, accum)
    assert rep["backend"] == "gloo" and rep["world_size"] == world and rep["steps"] == steps
    dist.barrier()
    r.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_process_bench_steps_device_accumulators(tmp_path):
    """Two ranks on one GPU run three bench-style steps (strong split of 11 frames per step) on
    torch device accumulators.  Rank 0's sum after each step equals, bit for bit, the fp32 sum of
    the two ranks' shards rendered separately (the reduce adds two fp32 images), and the shards
    together hold every frame of the step: a clear overtaking the previous reduce, or a reduce
    reading a half-rendered sum, changes these bits."""
    import torch.multiprocessing as mp

    from optixpathtracer_amd import scenes, sharding
    from optixpathtracer_amd.renderer import setup_renderer

    world, spp, steps = 2, 11, 3
    mp.spawn(_gpu_bench_worker, args=(world, _free_port(), spp, steps, str(tmp_path)), nprocs=world, join=True)
    sc = scenes.tiny_scene("conductor")
    r = setup_renderer(sc, 48, 32, 5, device=0)
    for s in range(steps):
        got = np.load(tmp_path / f"step{s}.npy")
        shards = []
        for rank in range(world):
            first, n = sharding.split_frames(spp, rank, world, base=1 + s * spp)
            r.accum_clear()
            r.render_frames(first, n)
            shards.append(r.accum())
        np.testing.assert_array_equal(got, shards[0] + shards[1])
        r.accum_clear()
        r.render_frames(1 + s * spp, spp)
        np.testing.assert_allclose(got, r.accum(), rtol=2e-6, atol=1e-7)
    r.close()


class _NullRenderer:
    """bench.py's renderer calls, with nothing rendered (the reporting path only)."""

    def accum_clear(self):
        pass

    def render_frames(self, first, n):
        pass

    def synchronize(self):
        pass


def _report_worker(rank, world, port, out_dir):
    sys.path.insert(0, str(ROOT))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import json
    import time

    import torch
    import torch.distributed as dist

    from optixpathtracer_amd import sharding

    dist.init_process_group("gloo", rank=rank, world_size=world)
    accum = torch.full((8, 12, 3), float(rank + 1), dtype=torch.float32)
    red = [sharding.render_step(_NullRenderer(), accum, dist, 1 + s, 1) for s in range(3)]
    if rank == 1:
        time.sleep(0.05)  # rank 1's own mean must not decide the max-over-ranks alone
    red.append(0.02 * (rank + 1))
    rep = sharding.distributed_report(dist, red, accum)
    if rank == 0:
        (Path(out_dir) / "report.json").write_text(json.dumps({"rep": rep, "sum": accum[0, 0, 0].item()}))
    dist.barrier()
    dist.destroy_process_group()


def test_distributed_report_fields(tmp_path):
    """the bench JSON of an N > 1 run records the backend the process
    group ran (\"nccl\" = RCCL on the GPU node, gloo here), the rank count it saw and the mean reduce
    time per step, max over ranks; the step's reduce sums the ranks' accumulators on rank 0."""
    import json

    import torch.multiprocessing as mp

    from optixpathtracer_amd import sharding

    world = 2
    mp.spawn(_report_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    d = json.loads((tmp_path / "report.json").read_text())
    rep = d["rep"]
    assert rep["backend"] == "gloo"
    assert rep["world_size"] == world
    assert rep["steps"] == 4
    assert rep["reduce_ms_per_step"] >= 1e3 * 0.04 / 4  # rank 1's appended 40 ms, max over ranks
    assert rep["reduce_bytes"] == 8 * 12 * 3 * 4
    assert d["sum"] == 1.0 + 3 * 2.0  # three reduces onto rank 0 (1), each adding rank 1's 2
    one = sharding.distributed_report(None, [0.1])
    assert one["backend"] is None and one["world_size"] == 1
