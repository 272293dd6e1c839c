"""spp sharding across GPUs.

Every (pixel, frame id) sample is independent and seeded by tea<16>(W*y+x, frameId)
(devicePrograms.cu:631), so splitting the frame-id range across ranks reproduces the
single-GPU image exactly up to fp32 summation order.  The only exchange is one sum
reduce of the W*H*3 fp32 accumulator to rank 0 (RCCL over xGMI on the GPU box; any
torch.distributed backend works, gloo in the CPU tests).
"""
from __future__ import annotations


def frame_range(step: int, rank: int, world: int, spp: int, base: int = 1) -> tuple[int, int]:
    """Weak scaling (bench.py): each rank renders `spp` frames per step; ranges are
    disjoint over (step, rank) and contiguous in step-major, rank-minor order."""
    return base + (step * world + rank) * spp, spp


def split_frames(total_spp: int, rank: int, world: int, base: int = 1) -> tuple[int, int]:
    """Strong scaling (BASELINE config 4): frame ids base .. base+total_spp-1 split into
    `world` contiguous blocks (GPU g renders base + g*spp/N .. base + (g+1)*spp/N - 1)."""
    per, extra = divmod(total_spp, world)
    first = base + rank * per + min(rank, extra)
    return first, per + (1 if rank < extra else 0)


def reduce_accumulator(tensor, dist, dst: int = 0) -> None:
    """Sum every rank's accumulator into rank `dst` (one collective per image).

    With RCCL ("nccl") the device tensor is reduced in place over xGMI.  gloo (the CPU tests, or
    several ranks sharing one GPU, where RCCL cannot run) reduces host tensors: a device
    accumulator is then copied to the host, reduced, and copied back on rank `dst`."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() <= 1:
        return
    if tensor.is_cuda and dist.get_backend() == "gloo":
        host = tensor.cpu()
        dist.reduce(host, dst=dst, op=dist.ReduceOp.SUM)
        if dist.get_rank() == dst:
            tensor.copy_(host)
        return
    dist.reduce(tensor, dst=dst, op=dist.ReduceOp.SUM)


def render_step(renderer, accum, dist, first: int, n: int) -> float:
    """One bench.py step on one rank: clear -> render frames first .. first+n-1 into the device
    accumulator `accum` (a torch tensor registered with pt_set_accum_device_buffer) -> wait for
    libptamd's stream -> reduce to rank 0 -> wait for torch's stream.  The reduce runs on torch's
    stream and the next step's clear on libptamd's, so the step ends only after the reduce.
    Returns the seconds spent in the reduce (from the rendered sum being ready to the reduced sum
    being ready on this rank), which bench.py reports per step (`distributed.reduce_ms_per_step`)."""
    import time

    import torch

    renderer.accum_clear()
    renderer.render_frames(first, n)
    renderer.synchronize()
    t0 = time.perf_counter()
    reduce_accumulator(accum, dist)
    if accum.is_cuda:
        torch.cuda.current_stream(accum.device).synchronize()
    return time.perf_counter() - t0


def distributed_report(dist, reduce_s: list, accum=None) -> dict:
    """What the multi-rank run actually ran, for the bench JSON: the
    torch.distributed backend (\"nccl\" is RCCL on ROCm), the rank count the process group saw, and
    the mean reduce time per step, max over ranks (a collective; every rank must call it).  At one
    rank, or without a process group: backend None, world_size 1."""
    import torch

    if dist is None or not dist.is_initialized():
        return {"backend": None, "world_size": 1, "reduce_ms_per_step": None, "steps": len(reduce_s)}
    ms = 1e3 * sum(reduce_s) / max(1, len(reduce_s))
    backend = str(dist.get_backend())
    dev = accum.device if (accum is not None and accum.is_cuda and backend != "gloo") else torch.device("cpu")
    t = torch.tensor([ms], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {
        "backend": backend,
        "world_size": int(dist.get_world_size()),
        "reduce_ms_per_step": round(float(t.item()), 4),
        "reduce_bytes": int(accum.numel() * accum.element_size()) if accum is not None else None,
        "collective": "reduce (sum, fp32) of the W*H*3 accumulator to rank 0, once per step",
        "steps": len(reduce_s),
    }
