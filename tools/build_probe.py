#!/usr/bin/env python3
"""BVH build time per builder (pt_stats.bvh_build_ms), cold and warm, for the GPU SAH build bar
(<= 25 ms at 250k triangles).
    python tools/build_probe.py [--scene sponza_class | --soup N] [--builders 4,2,3] [--repeat 3]"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sponza_class")
    ap.add_argument("--builders", default="4,2,3")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--soup", type=int, default=0, help="a random soup of N triangles instead of --scene")
    a = ap.parse_args()
    import torch  # noqa: F401
    from optixpathtracer_amd import scenes
    from optixpathtracer_amd.renderer import OptixRenderer

    if a.soup:
        import numpy as np

        rng = np.random.default_rng(1)
        c = rng.uniform(-50, 50, size=(a.soup, 1, 3)).astype(np.float32)
        v = (c + rng.normal(size=(a.soup, 3, 3)).astype(np.float32) * np.float32(0.3)).reshape(-1, 3)
        mesh = scenes.Mesh(vertices=v, indices=np.arange(len(v), dtype=np.int32).reshape(-1, 3),
                           normals=np.tile(np.float32([0, 0, 1]), (len(v), 1)))
        sc = scenes.Scene(meshes=[mesh], lights=np.zeros((0, 6), np.float32), camera_blender_pos=(0, 0, 0),
                          camera_blender_rot=(0, 0, 0))
        a.scene = f"soup{a.soup}"
    else:
        sc = scenes.make_scene(a.scene)
    for b in [int(x) for x in a.builders.split(",")]:
        ms, wall = [], []
        for _ in range(a.repeat):
            t = time.perf_counter()
            r = OptixRenderer(None, sc, bvh_builder=b)
            wall.append(round((time.perf_counter() - t) * 1e3, 2))
            st = r.stats()
            ms.append(round(st["bvh_build_ms"], 3))
            r.close()
        print(json.dumps({"scene": a.scene, "tris": sc.n_triangles, "builder": b, "bvh_build_ms": ms,
                          "pt_create_wall_ms": wall, "bvh_nodes": st["bvh_nodes"], "bvh_depth": st["bvh_depth"]}),
              flush=True)


if __name__ == "__main__":
    main()
