#!/usr/bin/env python3
"""Compare two renders (EXR or PFM): MSE and LDR-FLIP, the two metrics of the reference README.

    python tools/imgdiff.py a.exr b.exr
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from optixpathtracer_amd import imageio

    a, b = imageio.read_image(sys.argv[1]), imageio.read_image(sys.argv[2])
    print(json.dumps({"a": sys.argv[1], "b": sys.argv[2], "width": a.shape[1], "height": a.shape[0],
                      "mse": imageio.mse(a, b), "flip": imageio.flip(a, b)}))


if __name__ == "__main__":
    main()
