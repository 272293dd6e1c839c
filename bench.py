#!/usr/bin/env python3
"""Benchmark: Msamples/s of the MI355X path tracer on BASELINE.json configs[1].

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

Workload (configs[1]): the synthetic Diffuse sphere-in-box scene (34,570 triangles,
Lambert mode, Scene1 camera and 4 point lights), 1920x1080, depth 8.  One STEP = one
1024-spp render of the full frame: the 1024 frame ids are split over the ranks (spp
sharding), every rank renders its share into a device fp32 accumulator, and
the accumulators are summed to rank 0 with one RCCL reduce (torch.distributed "nccl" = RCCL
over xGMI).  The image is fixed as N grows ("strong" scaling, north_star's 1 -> 8 GPU scaling
of the 1024-spp image); value = the step's samples / max-over-ranks wall time.  At N > 1 one
more step with 1024 frames per rank reports the weak-scaling rate as `value_weak`.

`--config 3|4d|4l|5` runs BASELINE.json's other configs through the same harness (4d/4l: 4096
spp per step); the driver's default run is configs[1].

Extra fields: `roofline` (HBM roofline of the mode's dominant kernel, measured with one HIP event
pair per launch on the stream it runs on, per kernel: in the Lambert / Conductor / Dielectric modes
k_trace_pair (the shadow rays of bounce b and the extension rays of b+1 of a batch of --frames-per-launch frames, 128 by default), 48
algorithmic bytes per traced ray (an extension ray's 32-B record read and 16-B hit record written,
a shadow ray's three 16-B records read) plus 32 B (radiance read and write) per unoccluded shadow
ray, whose share comes from the untimed traversal-statistics render; in the Default / Layered modes
k_shade_nee, the layered NEE eval, 216 algorithmic bytes per item.  `window` says the timed
region's launch windows are concurrent with the other wavefront stream's kernels (`single_stream`
repeats the kernel alone); `binding` names the unit the PMC counters show binds the kernel -- the
vector memory path for k_trace_pair (`vmem`: 16-B lane loads per second against one line per
CU-cycle, with TA/TD busy from a committed PMC summary), VALU issue x lane utilisation for
k_shade_nee (`valu`); `pipeline_gbps` is SURVEY.md §8(d)'s whole-path 396 B/segment + 12 B/sample
over the render time; `traffic` is the PMC HBM bytes per launch from profiles/traffic.json),
`cpu_baseline` (the CPU oracle, oracle/, timed on a bounded band of the same workload on the host
cores, rank 0 at N=1 only) and `distributed` (the process group's backend and rank count and the
reduce time per step).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
BYTES_PER_SEGMENT = 396  # compulsory SoA queue + gather traffic per path segment
BYTES_PER_SAMPLE = 12  # final fp32 RGB accumulate
BYTES_PER_TRACE = 48  # trace-kernel share per ray: ray record read 32 B + hit / result write 16 B
# k_shade_nee per NEE item: queue entry 4 + hit record 16 + ray direction 16 + triangle gathers
# (isect v0 16 + shade 64) + material 32 + throughput|seed 16 + light index 4 + radiance RMW 32 +
# seed write-back 16 (pt_wavefront.hip k_shade_nee)
BYTES_PER_NEE_ITEM = 4 + 16 + 16 + 80 + 32 + 16 + 4 + 32 + 16
NEE_ADD_BYTES = 32  # k_trace_pair: radiance read + write of an unoccluded shadow ray (W.L[path], 16 B each)
CLOCK_HZ = 2.4e9  # MI355X shader clock (MI355X_MICROARCH.md; tools/td_probe.hip measured at 2400 MHz)
N_CUS, N_SIMDS = 256, 1024
# tools/td_probe.hip (profiles/r03s_td_probe.json): a 16-B-per-lane load costs the CU's texture
# data path about one cycle per distinct cache line its lanes touch (64 lines: 65 cycles), so the
# vector-memory ceiling for scattered 16-B loads is one lane load per CU-cycle
VMEM_LOADS_PER_S = N_CUS * CLOCK_HZ
NODE_LOADS = 7  # 16-B loads per global BVH4 node visit (6 sign-selected planes + child links)
TRI_LOADS = 3   # per triangle test (v0 | index, e1 | material, e2)


# BASELINE.json configs by index: scene, spp per step, scaling, workload label.  The default
# (configs[1]) is the headline; the others are reported in DESIGN.md from the same harness.
CONFIGS = {
    "2": ("sphere_box_diffuse", 1024, "strong",
          "BASELINE configs[1]: Diffuse sphere-in-box 1920x1080, 1024 spp, depth 8"),
    "3": ("sphere_box_conductor", 1024, "strong",
          "BASELINE configs[2]: Conductor (Trowbridge-Reitz) spheres + Layered walls (Default mode), "
          "1920x1080, 1024 spp, depth 8"),
    "4d": ("sphere_box_dielectric20", 4096, "strong",
           "BASELINE configs[3] (i): Dielectric-bright 1920x1080, 4096 spp split over the GPUs + RCCL reduce"),
    "4l": ("sphere_box_layered", 4096, "strong",
           "BASELINE configs[3] (ii): Layered 1920x1080, 4096 spp split over the GPUs + RCCL reduce"),
    "5": ("sponza_class", 1024, "strong",
          "BASELINE configs[4]: Sponza-class procedural atrium (~250k tris, mixed BRDFs) 1920x1080, 1024 spp"),
    "5t": ("sponza_textured", 1024, "strong",
           "BASELINE configs[4], textured: the atrium with albedo / normal / metal-rough maps and alpha-cut-out "
           "foliage (~250k tris, mixed BRDFs) 1920x1080, 1024 spp"),
}
# configs whose scene enters the renderer the way the reference's models do: written as .glb and
# read by the C++ glTF loader (pt_model_load_gltf, ModelLoader::LoadModel's counterpart)
GLB_CONFIGS = ("5", "5t")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_record(path: Path, sources_sha: str):
    """A committed PMC summary (profiles/*.json) and whether it belongs to these kernel sources.
    Returns (data, current): figures measured on other sources are never reported as this tree's."""
    if not path.exists():
        return None, False
    try:
        d = json.loads(path.read_text())
    except Exception:
        return None, False
    return d, d.get("sources_sha") == sources_sha


def device_identity(torch, dev: int) -> dict:
    """Which GPU the numbers came from (name, gfx arch, CUs, memory), for attributing outliers."""
    p = torch.cuda.get_device_properties(dev)
    return {"name": p.name, "gcn_arch": getattr(p, "gcnArchName", None), "cus": p.multi_processor_count,
            "memory_gb": round(p.total_memory / 2**30, 1),
            "visible": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="2", choices=sorted(CONFIGS),
                    help="BASELINE.json config: 2 = configs[1] (default, the headline), 3, 4d, 4l, 5, 5t")
    ap.add_argument("--scene-source", choices=["auto", "procedural", "glb"], default="auto",
                    help="auto: configs 5 / 5t through a .glb and the C++ glTF loader, the others in memory")
    ap.add_argument("--scene", default=None, help="override the config's scene")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=None,
                    help="samples per pixel per step: per GPU (weak configs) or in total (strong configs)")
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--kernel", type=int, default=2, help="0 = megakernel, 1 = wavefront, 2 = auto")
    ap.add_argument("--frames-per-launch", type=int, default=128)
    ap.add_argument("--no-dedup-check", action="store_true",
                    help="skip the extra step timed with pt_set_primary_dedup(0)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "traffic.json"),
                    help="PMC traffic per launch measured by tools/profile.sh (optional)")
    ap.add_argument("--queue-budget", type=int, default=0,
                    help="pt_set_queue_budget: bytes for all streams' wavefront queues (0 = the library's "
                         "default, a quarter of the device memory; -1 = none)")
    ap.add_argument("--wavefront-streams", type=int, default=0,
                    help="streams the wavefront batches alternate between (pt_set_wavefront_streams; "
                         "0 = the library's auto: two for Conductor and Dielectric, one otherwise)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="override the config's scaling (all configs: strong = the step's spp in total, split "
                         "over the ranks; weak = the step's spp per rank)")
    ap.add_argument("--reference-loops", type=int, default=1024,
                    help="pt_render calls (1 spp each, frame.id++, 24.9 MB download per call: the reference's "
                         "OptixView::DrawOptix -> OptixRenderer::Render loop, here the 1024 samples of the "
                         "configs[1] image) timed for value_reference_loop; 0 = off")
    a = ap.parse_args()
    scene, spp, scaling, a.workload = CONFIGS[a.config]
    a.scaling = a.scaling or scaling
    a.scene = a.scene or scene
    a.spp = a.spp or spp
    return a


def cpu_baseline(scene, args, budget_s: float):
    """The CPU oracle (oracle/liboracle.so, test/baseline infrastructure) on a band of the
    same workload, on this host's cores; sized to ~budget_s of CPU work.  Returns the band's
    radiance sum (rows, W, 3), its spp and the baseline record."""
    from oracle.oracle import OracleScene

    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    o = OracleScene(scene)
    lp = o.launch(args.width, args.height, args.depth)
    y0 = args.height // 2
    rows = args.height - y0  # the lower half of the frame, 1 spp, as the calibration pass
    t = time.perf_counter()
    o.render(lp, 1, 1, rect=(0, y0, args.width, y0 + rows), threads=threads)
    per_spp = max(time.perf_counter() - t, 1e-3)
    spp = int(max(1, min(args.spp, budget_s / per_spp)))
    t = time.perf_counter()
    band, segs = o.render(lp, 1, spp, rect=(0, y0, args.width, y0 + rows), threads=threads)
    band = band[y0:y0 + rows]
    dt = time.perf_counter() - t
    samples = rows * args.width * spp
    o.close()
    return band, spp, {
        "value": round(samples / dt / 1e6, 4),
        "unit": "Msamples/sec",
        "cores": threads,
        "kind": "port",
        "sample": f"{rows} rows x {args.width} px x {spp} spp (frame ids 1..{spp}) of the same scene/depth, "
                  f"rows {y0}..{y0 + rows - 1}, "
                  f"{dt:.1f} s, {segs} segments",
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    import numpy as np
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl", init_method="env://")
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import setup_renderer

    scene = scenes.make_scene(args.scene)
    source = {"kind": "procedural (in memory)"}
    if args.scene_source == "glb" or (args.scene_source == "auto" and args.config in GLB_CONFIGS):
        # the reference's scenes enter through ModelLoader::LoadModel (ModelLoader.cpp:11-43): the
        # procedural scene is written as one .glb (untimed) and read back by pt_model_load_gltf
        import shutil
        import tempfile

        from optixpathtracer_amd import gltf

        tmp = tempfile.mkdtemp(prefix="ptamd_glb_")
        try:
            scene, load_ms, glb_bytes = gltf.load_scene_glb(scene, tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        source = {"kind": "glb via pt_model_load_gltf (C++ glTF 2.0 loader)", "load_ms": round(load_ms, 1),
                  "glb_bytes": glb_bytes, "meshes": len(scene.meshes), "textures": len(scene.textures)}
    t0 = time.perf_counter()
    r = setup_renderer(scene, args.width, args.height, args.depth, device=local_rank, kernel=args.kernel)
    r.set_frames_per_launch(args.frames_per_launch)
    r.set_wavefront_streams(args.wavefront_streams)
    r.set_queue_budget(args.queue_budget)
    # the streams the timed region runs on: 0 is the library's auto (one for Lambert, two otherwise)
    eff_streams = args.wavefront_streams or (2 if scene.material_mode in (2, 3) else 1)
    if args.kernel != 0:  # wavefront (auto resolves to it): time every k_extend launch
        r.set_kernel_timing(True)
    setup_s = time.perf_counter() - t0
    bvh_ms = r.stats()["bvh_build_ms"]
    dev = torch.device("cuda", local_rank)
    accum = torch.zeros((args.height, args.width, 3), dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)
    r.set_accum_device_buffer(accum.data_ptr())
    if rank == 0:
        log(f"[bench] scene={args.scene} tris={scene.n_triangles} {args.width}x{args.height} spp/step/gpu={args.spp} "
            f"depth={args.depth} world={world} setup={setup_s:.2f}s lbvh={bvh_ms:.3f}ms")

    from optixpathtracer_amd import sharding

    reduce_s = []  # per timed step (sharding.render_step)

    def step(s: int, scaling: str | None = None):
        if (scaling or args.scaling) == "strong":  # args.spp frames per step in total, split over the ranks
            first, n = sharding.split_frames(args.spp, rank, world, base=1 + s * args.spp)
        else:  # args.spp frames per rank per step; disjoint frame ids per (step, rank)
            first, n = sharding.frame_range(s, rank, world, args.spp)
        # clear -> render -> sync -> RCCL reduce over xGMI -> sync torch's stream (the next
        # step's clear runs on libptamd's stream and must not overtake the reduce)
        return sharding.render_step(r, accum, dist, first, n)

    for s in range(args.warmup):
        step(s)
        if rank == 0:
            log(f"[bench] warmup {s + 1}/{args.warmup} done")
    torch.cuda.synchronize(dev)
    r.stats_reset()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        reduce_s.append(step(args.warmup + s))
        if rank == 0:
            log(f"[bench] step {s + 1}/{args.steps} {time.perf_counter() - t0:.2f}s")
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    st = r.stats()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    distributed = sharding.distributed_report(dist, reduce_s, accum)  # a collective at N > 1
    per_step_spp = args.spp if args.scaling == "strong" else args.spp * world
    samples_total = args.width * args.height * per_step_spp * args.steps
    value = samples_total / elapsed / 1e6
    # Transparency: the same step with every frame's (identical) camera ray traced again
    # instead of once per pixel per batch (pt_set_primary_dedup; bit-identical images).
    img = accum.cpu().numpy() if rank == 0 else None  # the timed steps' image
    value_nodedup = None
    if args.kernel != 0 and not args.no_dedup_check:
        r.set_primary_dedup(False)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        step(args.warmup + args.steps)
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        e1 = time.perf_counter() - t1
        if dist is not None:
            t = torch.tensor([e1], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e1 = float(t.item())
        value_nodedup = args.width * args.height * per_step_spp / e1 / 1e6
        r.set_primary_dedup(True)
    # Transparency at N > 1: the other scaling mode's rate from one more step (weak: every rank
    # renders the step's full spp; strong: the ranks split it)
    value_other = None
    if world > 1:
        other = "weak" if args.scaling == "strong" else "strong"
        dist.barrier()
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        step(args.warmup + args.steps + 2, scaling=other)
        torch.cuda.synchronize(dev)
        dist.barrier()
        e3 = time.perf_counter() - t3
        t = torch.tensor([e3], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        e3 = float(t.item())
        value_other = (other, args.width * args.height * (args.spp * world if other == "weak" else args.spp) / e3 / 1e6)
    # One more untimed render of two batches with the traversal counters on (a separate
    # kernel instance): node visits (global / from LDS), triangle tests and rays per trace launch,
    # for the vector-memory roofline of the trace kernels (roofline.vmem).  Its time is not used.
    trav = None
    if args.kernel != 0:
        r.set_traversal_stats(True)
        r.stats_reset()
        r.accum_clear()
        r.render_frames(1, min(args.spp, 2 * args.frames_per_launch))
        trav = r.stats()
        r.set_traversal_stats(False)
    # share of k_trace_pair's shadow rays that found their light unoccluded (each adds its
    # contribution to the path radiance: NEE_ADD_BYTES more algorithmic bytes)
    unocc_share = trav["nee_unoccluded"] / trav["pair_kernel_shadow_rays"] if trav and trav["pair_kernel_shadow_rays"] else 0.0
    # Transparency: with two streams the timed steps alternate the wavefront batches between them
    # (pt_set_wavefront_streams; auto takes two for Conductor and Dielectric), so a launch shares
    # the GPU with the other batch's kernels and its event window is longer than its solo run.
    # One more step on a single stream gives the trace kernels' solo launch time
    # (roofline.single_stream); on one stream the timed region is that run.
    single = None
    s1_all_ms = None  # single-stream mean over all trace launches (vmem rate)
    if args.kernel != 0 and not args.no_dedup_check and eff_streams > 1:
        r.set_wavefront_streams(1)
        r.stats_reset()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        step(args.warmup + args.steps + 1)
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        e2 = time.perf_counter() - t2
        s1 = r.stats()
        if s1["trace_kernel_launches"] > 0:
            # the dominant trace kernel alone: k_trace_pair in the fused modes, k_extend otherwise
            pair1 = s1["pair_kernel_launches"] > 0
            l1 = int(s1["pair_kernel_launches"] if pair1 else s1["trace_kernel_launches"])
            ms1 = (s1["pair_kernel_ms"] if pair1 else s1["trace_kernel_ms"]) / l1
            b1 = (s1["pair_kernel_bytes"] + NEE_ADD_BYTES * unocc_share * s1["pair_kernel_shadow_rays"]
                  if pair1 else s1["trace_kernel_bytes"])
            ach1 = b1 / l1 / (ms1 / 1e3) / 1e9
            s1_all_ms = s1["trace_kernel_ms"] / max(1, s1["trace_kernel_launches"])
            single = {"value": round(args.width * args.height * per_step_spp / e2 / 1e6, 3),
                      "kernel": "k_trace_pair" if pair1 else "k_extend",
                      "avg_launch_ms": round(ms1, 4), "achieved": round(ach1, 2),
                      "frac": round(ach1 / HBM_PEAK_GBPS, 5), "launches": l1,
                      "shade_avg_launch_ms": round(s1["shade_kernel_ms"] / max(1, s1["shade_kernel_launches"]), 4),
                      "shade_items_per_launch": s1["shade_kernel_items"] / max(1, s1["shade_kernel_launches"])}
        r.set_wavefront_streams(args.wavefront_streams)
    if rank == 0:
        nan_px = int(np.isnan(img).any(axis=-1).sum())
        kernel_s = st["total_render_ms"] / 1e3
        alg_bytes = st["segments"] * BYTES_PER_SEGMENT + st["samples"] * BYTES_PER_SAMPLE
        fused = scene.material_mode in (1, 2, 3)
        vmem_line = valu_line = trace_line = None
        if st["trace_kernel_launches"] > 0:
            # per kernel: k_trace_pair's own launches in the fused modes
            # (the batch's one k_extend is excluded), k_extend in Default / Layered
            pair = fused and st["pair_kernel_launches"] > 0
            launches = int(st["pair_kernel_launches"] if pair else st["trace_kernel_launches"])
            t_bytes = (st["pair_kernel_bytes"] + NEE_ADD_BYTES * unocc_share * st["pair_kernel_shadow_rays"]
                       if pair else st["trace_kernel_bytes"]) / launches
            t_s = (st["pair_kernel_ms"] if pair else st["trace_kernel_ms"]) / 1e3 / launches
            # all trace launches (k_extend + k_trace_pair): the denominator of the lane-load rate below
            all_s = st["trace_kernel_ms"] / 1e3 / int(st["trace_kernel_launches"])
            trace_line = {"kernel": "k_trace_pair" if pair else "k_extend", "launches": launches,
                          "avg_launch_ms": round(t_s * 1e3, 4), "bytes_per_launch": int(t_bytes),
                          "achieved": round(t_bytes / t_s / 1e9, 2), "frac": round(t_bytes / t_s / 1e9 / HBM_PEAK_GBPS, 5)}
            if trav and trav["trace_kernel_launches"] > 0:
                # 16-B lane loads of global memory per trace launch, counted like trace_kernel_bytes:
                # 7 per global node visit, 3 per triangle test, 2 per extension-ray record and 3 per
                # shadow-ray record (record loads are coalesced, 8 lanes per line, so as line touches
                # they count up to 8x; they are 6 % of the loads)
                tl = int(trav["trace_kernel_launches"])
                g_nodes = trav["nodes_visited"] - trav["lds_nodes_visited"]
                ext_rays = trav["rays"] - trav["shadow_rays"]
                loads = (NODE_LOADS * g_nodes + TRI_LOADS * trav["tri_tests"] + 2 * ext_rays
                         + 3 * trav["shadow_rays"]) / tl
                ach_v = loads / all_s  # lane loads of all trace launches over their summed time
                vmem_line = {
                    "unit": "16-B lane loads/s", "kernels": "k_extend + k_trace_pair (aggregate rate)",
                    "lane_loads_per_launch": round(loads),
                    "achieved": round(ach_v / 1e9, 2), "ceiling": round(VMEM_LOADS_PER_S / 1e9, 1),
                    "frac": round(ach_v / VMEM_LOADS_PER_S, 4),
                    "ceiling_def": "1 line per CU-cycle x 256 CUs x 2.4 GHz (tools/td_probe.hip)",
                    "node_visits_per_ray": round(trav["nodes_visited"] / max(1, trav["rays"]), 3),
                    "lds_node_share": round(trav["lds_nodes_visited"] / max(1, trav["nodes_visited"]), 4),
                    "tri_tests_per_ray": round(trav["tri_tests"] / max(1, trav["rays"]), 3),
                    "node_lane_utilisation": round(trav["nodes_visited"] / max(1, 64 * trav["wave_node_steps"]), 4),
                }
                if single and s1_all_ms:
                    sv = loads / (s1_all_ms / 1e3)
                    vmem_line["single_stream"] = {"achieved": round(sv / 1e9, 2), "frac": round(sv / VMEM_LOADS_PER_S, 4)}
        if fused and trace_line:
            # Lambert / Conductor / Dielectric: the trace kernels are the dominant kernels (k_extend
            # at bounce 0, k_trace_pair = shadow rays of bounce b + extension rays of b+1), each
            # launch bracketed by its own HIP event pair on the stream it runs on
            dom = trace_line["kernel"]
            launches = trace_line["launches"]
            per_launch_bytes = trace_line["bytes_per_launch"]
            avg_launch_s = trace_line["avg_launch_ms"] / 1e3
            bytes_def = ("48 B per traced ray of one k_trace_pair launch (the shadow rays of bounce b and the "
                         "extension rays of bounce b+1 of one batch): an extension ray's 32-B record read "
                         "and 16-B hit record written, a shadow ray's direction, contribution and origin records "
                         f"read; plus {NEE_ADD_BYTES} B (radiance read + write) per unoccluded shadow ray "
                         f"({unocc_share:.4f} of the shadow rays, traversal-statistics render)")
        elif st["shade_kernel_launches"] > 0:
            # Default / Layered: k_shade_nee (the stochastic layered NEE eval) takes 53-60 % of a frame
            # (DESIGN.md §8); its bound is VALU issue (roofline.valu), its HBM figure is reported too
            dom = "k_shade_nee"
            launches = int(st["shade_kernel_launches"])
            per_launch_bytes = st["shade_kernel_items"] * BYTES_PER_NEE_ITEM / launches
            avg_launch_s = st["shade_kernel_ms"] / 1e3 / launches
            bytes_def = (f"{BYTES_PER_NEE_ITEM} B per NEE item: queue entry, hit record, ray direction, triangle "
                         "gathers (v0 + shading record), material, throughput|seed, light index, radiance "
                         "read-modify-write, seed write-back")
        else:
            dom = "k_render_mega"
            launches = max(1, int(st["kernel_launches"]))
            per_launch_bytes = alg_bytes / launches
            avg_launch_s = kernel_s / launches
            bytes_def = "396 B per segment + 12 B per sample"
        achieved = per_launch_bytes / avg_launch_s / 1e9
        if single is None and eff_streams == 1 and fused and trace_line:
            # one stream: the timed region is the solo run
            single = {"value": round(value, 3), "kernel": dom, "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                      "achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBPS, 5),
                      "launches": launches, "note": "the timed region runs on one stream"}
        # PMC figures come from separate rocprofv3 passes committed under profiles/ (tools/profile.sh,
        # tools/pmc.sh); each carries the kernel-source hash it was measured on.  Only figures of
        # these sources fill the contract fields; older ones are listed under pmc_stale.
        from optixpathtracer_amd.provenance import kernel_sources_sha
        sha = kernel_sources_sha()
        pmc_stale = {}
        traffic = traffic_low = rd_sizes = None
        tjd, cur = pmc_record(Path(args.traffic_json), sha)
        if tjd and tjd.get("kernel") == dom and tjd.get("config", "2") == args.config:
            fig = {"hbm_bytes_per_launch": tjd.get("hbm_bytes_per_launch"),
                   "hbm_bytes_per_launch_low": tjd.get("hbm_bytes_per_launch_low")}
            if cur:
                traffic, traffic_low = fig["hbm_bytes_per_launch"], fig["hbm_bytes_per_launch_low"]
                rd_sizes = tjd.get("read_request_sizes")
            else:
                pmc_stale["traffic"] = {**fig, "sources_sha": tjd.get("sources_sha"), "stale": True}
        valu = None  # the VALU fraction beside the HBM roofline, from PMC passes
        vd, cur = pmc_record(ROOT / "profiles" / "valu.json", sha)
        if vd and fused and args.config == "2":
            fig = {k: vd.get(k) for k in ("kernel", "valu_busy", "valu_issue_slots", "lane_utilisation", "wait_per_wave_cycle")}
            if cur:
                valu = {**fig, "sources_sha": sha}
            else:
                pmc_stale["valu_pmc"] = {**fig, "sources_sha": vd.get("sources_sha"), "stale": True}
        vmem = None  # the vector memory path (TA / TD busy), what the trace kernel waits on
        md, cur = pmc_record(ROOT / "profiles" / "vmem.json", sha)
        if md and fused and args.config == "2":
            fig = {k: md.get(k) for k in ("kernel", "ta_busy", "td_busy", "td_tc_stall", "l2_read_latency_cycles")}
            if cur:
                vmem = {**fig, "sources_sha": sha}
            else:
                pmc_stale["vmem_pmc"] = {**fig, "sources_sha": md.get("sources_sha"), "stale": True}
        shade = None  # the memory-bound kernel of a Lambert frame, PMC HBM GB/s (tools/shade_pmc.py)
        sd, cur = pmc_record(ROOT / "profiles" / "shade_pmc.json", sha)
        if sd and fused and args.config == "2":
            ks = sd.get("kernels", {})
            # bounces >= 1 (the bounce-0 instance derives its path state, shade0)
            sk = ks.get("k_shade_fused<1, false, false>") or ks.get("k_shade_fused<1, false>")
            if sk:
                fig = {"kernel": "k_shade_fused<Lambert>", **{k: sk[k] for k in ("hbm_gbps", "frac", "avg_launch_ms")}}
                if cur:
                    shade = {**fig, "sources_sha": sha}
                else:
                    pmc_stale["shade_pmc"] = {**fig, "sources_sha": sd.get("sources_sha"), "stale": True}
        if dom == "k_shade_nee":
            # VALU issue of k_shade_nee (tools/pmc.sh + tools/pmc_summary.py --shade-json, per config):
            # wave64 VALU instructions x 2 cycles (MI355X_MICROARCH.md: a SIMD issues one every 2
            # cycles with several waves) over 1024 SIMDs x clock x the single-stream launch time
            nd, cur = pmc_record(ROOT / "profiles" / f"shade_valu_config{args.config}.json", sha)
            if nd:
                t_launch = (single or {}).get("shade_avg_launch_ms") or avg_launch_s * 1e3
                insts = nd.get("valu_insts_per_dispatch")
                fig = {"kernel": nd.get("kernel"), "valu_insts_per_dispatch": insts,
                       "lane_utilisation": nd.get("lane_utilisation"), "launch_ms": round(t_launch, 4),
                       "issue_frac": round(insts * 2 / (N_SIMDS * CLOCK_HZ * t_launch / 1e3), 4) if insts else None,
                       "issue_def": "wave64 VALU insts x 2 cycles / (1024 SIMDs x 2.4 GHz x single-stream launch time)"}
                if cur:
                    valu_line = {**fig, "sources_sha": sha}
                else:
                    pmc_stale["valu"] = {**fig, "sources_sha": nd.get("sources_sha"), "stale": True}
        # The unit that binds the dominant kernel.  `bound` stays "hbm": the
        # contract's roofline (achieved / peak in GB/s) is HBM; this names what the counters show.
        if dom == "k_trace_pair":
            binding = {"unit": "vector memory path (TA/TD): latency of each step's dependent load chain",
                       "frac": (vmem_line or {}).get("single_stream", {}).get("frac") or (vmem_line or {}).get("frac"),
                       "frac_def": "16-B lane loads/s of the trace launches (single stream) over one line per CU-cycle "
                                   "(roofline.vmem)",
                       "td_busy": (vmem or {}).get("td_busy"), "ta_busy": (vmem or {}).get("ta_busy"),
                       "hbm_frac_single_stream": (single or {}).get("frac")}
        elif dom == "k_shade_nee":
            vl = valu_line or {}
            ef = (round(vl["issue_frac"] * vl["lane_utilisation"], 4)
                  if vl.get("issue_frac") and vl.get("lane_utilisation") else None)
            binding = {"unit": "VALU", "frac": ef,
                       "frac_def": "VALU issue fraction x lane utilisation (roofline.valu, PMC)",
                       "issue_frac": vl.get("issue_frac"), "lane_utilisation": vl.get("lane_utilisation")}
        else:
            binding = None
        out = {
            "metric": "Msamples/sec at 1920x1080, max-depth 8; MSE vs reference",
            "value": round(value, 3),
            "unit": "Msamples/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (procedural {args.scene} scene; the reference's glTF assets are not in its repo)",
            "config": {
                "workload": args.workload + (f", {world}xMI355X" if args.scaling == "strong" or world == 1
                                             else f" per GPU, spp-sharded over {world} GPUs + RCCL reduce"),
                "scene": args.scene,
                "triangles": scene.n_triangles,
                "width": args.width,
                "height": args.height,
                "spp_per_step": args.spp,
                "spp_per_gpu_per_step": args.spp if args.scaling == "weak" else round(args.spp / world, 2),
                "max_depth": args.depth,
                "material_mode": {0: "default", 1: "lambert", 2: "conductor", 3: "dielectric",
                                  4: "layered"}.get(scene.material_mode, str(scene.material_mode)),
                "kernel": {0: "megakernel", 1: "wavefront", 2: "auto (wavefront)"}[args.kernel],
                "frames_per_launch": args.frames_per_launch,
                "wavefront_streams": eff_streams,
                "parallelism": f"spp-shard x{world}",
                "scene_source": source,
                # the batches the timed region ran (pt_stats): frames per batch after the queue
                # budget (pt_set_queue_budget, default a quarter of the device memory) and the
                # device memory the wavefront queues held
                "batch_frames": st["last_batch_frames"],
                "queue_bytes": st["queue_bytes"],
                "queue_budget_bytes": st["queue_budget"],
                "bvh_build_ms": round(bvh_ms, 3),  # the first build in the process (code loading included)
                # pt_options.bvh_builder = PT_BVH_AUTO: the binned-SAH binary tree built on the GPU
                # (pt_sah_gpu.hip) and collapsed to BVH4 on the GPU; the time above covers both
                "bvh_builder": "auto (GPU binned SAH + GPU SAH-optimal BVH4 collapse)",
                "primary_dedup": args.kernel != 0,
            },
            # one extra step with pt_set_primary_dedup(0): each frame traces its own copy of the
            # (identical, unjittered) camera rays; same image bit for bit
            "value_primary_per_frame": None if value_nodedup is None else round(value_nodedup, 3),
            # N > 1: the other scaling mode's rate from one extra step (value_weak / value_strong)
            **({f"value_{value_other[0]}": round(value_other[1], 3)} if value_other else {}),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 5),
                "traffic": traffic,
                "traffic_low": traffic_low,
                # the read requests by size (one more PMC pass): k_trace_pair reads whole 128-B lines,
                # so `traffic` (2 x FETCH_SIZE + WRITE_SIZE) is the exact figure; its split into the
                # queue records, BVH refetch, hit records and radiance adds: DESIGN.md §5
                "traffic_read_requests": rd_sizes,
                "kernel": dom,
                "bytes_per_launch": int(per_launch_bytes),
                "bytes_def": bytes_def,
                "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                "launches": launches,
                # the timed region alternates batches over two streams: a launch's event window
                # includes time it shares the GPU with the other stream's kernels (single_stream
                # gives the same kernel alone)
                "window": ("timed region, two wavefront streams (concurrent launch windows)"
                           if eff_streams > 1 else "timed region, one stream"),
                "binding": binding,
                "segments_per_sample": round(st["segments"] / max(1, st["samples"]), 4),
                # SURVEY.md §8(d) whole-path figure: (segments*396 + samples*12) / render time
                "pipeline_gbps": round(alg_bytes / max(kernel_s, 1e-9) / 1e9, 2),
                # what limits the trace kernel: the latency of each step's dependent
                # memory chain over the rays a CU holds in flight; VALU issue (valu_pmc) and the
                # vector memory units (vmem_pmc) are reported beside it
                "valu_pmc": valu,
                "vmem_pmc": vmem,
                # 16-B lane loads through the CU's vector memory path against one line per CU-cycle
                # (VERDICT round 3 item 2a).  Not the binding unit: round 4 cut the line touches per
                # node visit 3.3x (four lanes per ray) and TD stayed 93 % busy
                "vmem": vmem_line,
                # k_shade_nee (Default / Layered): VALU issue fraction
                "valu": valu_line,
                # the trace kernels' own line when they are not the dominant kernel (Default / Layered)
                "trace": trace_line if not fused else None,
                # PMC HBM bandwidth of the shading kernel (2 x FETCH_SIZE + WRITE_SIZE per launch)
                "shade_pmc": shade,
                "single_stream": single,
                # the kernel sources of this run; PMC figures measured on other sources (never
                # reported in the fields above)
                "sources_sha": sha,
                "pmc_stale": pmc_stale or None,
            },
            "image": {"mean": float(np.nanmean(img) / per_step_spp), "nan_pixels": nan_px},
            # what the process group ran: backend ("nccl" = RCCL), ranks, reduce time per step
            "distributed": distributed,
            "device": device_identity(torch, local_rank),
        }
        if world == 1 and args.reference_loops > 0 and args.kernel != 0:
            # The reference's own call pattern (OptixView::DrawOptix -> OptixRenderer::Render,
            # OptixView.cpp:201-210, OptixRenderer.cpp:617-647): one pt_render per spp (frame.id++,
            # one 1-frame wavefront batch) and a download of the 24.9 MB frame into a freshly
            # allocated host array every call; the GL upload and blend are not part of it.
            # pt_render renders ahead (pt_set_render_ahead, default 64 frames: while the render state
            # is unchanged, a call that misses renders the next 1, 2, 4, ... 64 frame ids in one batch
            # and later calls download theirs; once at 64, the first call served from a batch also
            # enqueues the next 64 frame ids, rendered while the caller downloads), so the loop is
            # timed from a state change on, ramp included, and up to the end of the last look-ahead
            # batch (frames no call asked for count as time, not as samples); the same loop with
            # render-ahead off is reported beside it.
            # the caller's loop runs without the per-launch event pairs of the roofline fields
            # (pt_set_kernel_timing is a diagnostic the reference's viewer does not have)
            r.set_kernel_timing(False)

            def ref_loop(calls):
                r.frame_id = 0
                r.Render()  # the first call after a change renders its own frame only
                t = time.perf_counter()
                for _ in range(calls):
                    r.Render(np.empty((args.height, args.width, 3), np.float32))
                r.synchronize()
                return time.perf_counter() - t

            fid = r.frame_id
            e4 = ref_loop(args.reference_loops)
            # Latency of a state change in the steady state:
            # after 200 sequential calls (a look-ahead batch in flight), the camera moves and one call
            # is timed.  pt_set_camera cancels the speculative batch (pt_capi.cpp cancel_look_ahead:
            # its kernels stop at their next poll), so the call waits for little more than its own
            # frame's render and download.  Median of 3.
            import statistics

            lat = []
            canc0 = r.stats()["look_ahead_cancelled"]
            for k in range(3):
                r.SetCameraBlender(scene.camera_blender_pos, scene.camera_blender_rot, scene.fov_deg)
                r.frame_id = 0
                for _ in range(200):
                    r.Render(np.empty((args.height, args.width, 3), np.float32))
                pos = np.asarray(scene.camera_blender_pos, np.float32) + np.float32(1e-3 * (k + 1))
                r.SetCameraBlender(pos, scene.camera_blender_rot, scene.fov_deg)
                t = time.perf_counter()
                r.Render(np.empty((args.height, args.width, 3), np.float32))
                lat.append(time.perf_counter() - t)
            r.SetCameraBlender(scene.camera_blender_pos, scene.camera_blender_rot, scene.fov_deg)
            r.synchronize()
            n_cancelled = r.stats()["look_ahead_cancelled"] - canc0
            r.set_render_ahead(1)
            n_off = min(args.reference_loops, 64)
            e5 = ref_loop(n_off)
            r.set_render_ahead(64)
            r.frame_id = fid
            out["value_reference_loop"] = round(args.width * args.height * args.reference_loops / e4 / 1e6, 3)
            out["reference_loop"] = {"calls": args.reference_loops, "ms_per_call": round(e4 / args.reference_loops * 1e3, 3),
                                     "what": "pt_render: 1 spp per call, frame.id++, D2H download of the 24.9 MB "
                                             "frame per call (the reference's DrawOptix loop), render-ahead on, "
                                             "kernel timing off",
                                     "first_call_after_change_ms": round(1e3 * statistics.median(lat), 3),
                                     "look_ahead_cancelled": n_cancelled,
                                     "render_ahead_budget_ms": 50.0,
                                     # one frame per call: two row bands on the two streams (pt_set_band_split)
                                     "no_render_ahead": {"calls": n_off, "ms_per_call": round(e5 / n_off * 1e3, 3),
                                                         "value": round(args.width * args.height * n_off / e5 / 1e6, 3)}}
        if world == 1 and not args.no_cpu_baseline:
            log("[bench] cpu baseline (oracle) ...")
            band, spp_cpu, out["cpu_baseline"] = cpu_baseline(scene, args, args.cpu_baseline_seconds)
            # "MSE vs reference" of the metric: the GPU renders the same frame ids (1..spp_cpu)
            # untimed, and its band is compared with the oracle's per-pixel mean radiance.  The
            # render runs the timed configuration's machinery: batches of a third of the frames
            # (so at least two batches, alternating over the wavefront streams, and a ragged tail
            # when spp_cpu is not a multiple of three).
            fpl_check = max(1, -(-spp_cpu // 3))
            r.set_frames_per_launch(fpl_check)
            r.accum_clear()
            r.render_frames(1, spp_cpu)
            r.synchronize()
            r.set_frames_per_launch(args.frames_per_launch)
            n_batches = -(-spp_cpu // fpl_check)
            gpu = accum.cpu().numpy()[args.height - band.shape[0]:].astype(np.float64) / spp_cpu
            ref = band.astype(np.float64) / spp_cpu
            diff = np.nan_to_num(gpu, nan=0.0) - np.nan_to_num(ref, nan=0.0)  # NaN -> 0 (WriteImage.cpp:52-55)
            if os.environ.get("PT_BENCH_DUMP"):  # debug aid: both band sums for offline comparison
                np.savez(os.environ["PT_BENCH_DUMP"], gpu=accum.cpu().numpy()[args.height - band.shape[0]:], ref=band)
            out["mse_vs_oracle"] = {
                "mse": float(np.mean(diff * diff)),
                "max_abs": float(np.max(np.abs(diff))),
                "bar": 1e-5,
                "sample": out["cpu_baseline"]["sample"].split(",")[0] + " (GPU render of the same frame ids)",
                "gpu_batches": n_batches,
                "gpu_frames_per_batch": fpl_check,
                "gpu_streams": min(n_batches, eff_streams),
            }
        print(json.dumps(out), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
