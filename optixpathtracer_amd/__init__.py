"""MI355X-native replacement for the OptiX render path of Damo12320/OptixPathtracer.

Product = libptamd.so (HIP kernels for gfx950 + C ABI, include/ptamd.h) and this thin
host mirror of the reference's OptixRenderer interface.  See DESIGN.md.
"""
from . import capi, scenes
from .capi import MATERIAL_MODES, PTError
from .renderer import OptixRenderer, camera_from_blender, setup_renderer

__all__ = ["capi", "scenes", "OptixRenderer", "camera_from_blender", "setup_renderer", "PTError",
           "MATERIAL_MODES"]
