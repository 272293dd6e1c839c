"""Image output and the parity metric over the C ABI.

Mirrors Renderer/Images/WriteImage.cpp of the reference: EXR (float B,G,R, uncompressed,
rows flipped, NaN pixels -> 0), BMP (clamp * 255, truncated) and PFM.  Images are
float32 arrays of shape (H, W, 3) with row 0 = bottom, the colorBuffer / accumulator layout.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .capi import PTError, load


def _arr(img: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(img, dtype=np.float32)
    if a.ndim != 3 or a.shape[2] != 3:
        raise PTError(f"expected an (H, W, 3) image, got {a.shape}")
    return a


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _check(status: int, what: str) -> None:
    if status != 0:
        msg = load().pt_image_last_error()
        raise PTError(f"{what} failed ({status}): {msg.decode() if msg else ''}")


def write_exr(path: str, img: np.ndarray) -> None:
    a = _arr(img)
    _check(load().pt_image_write_exr(str(path).encode(), _ptr(a), a.shape[1], a.shape[0]), "pt_image_write_exr")


def write_pfm(path: str, img: np.ndarray) -> None:
    a = _arr(img)
    _check(load().pt_image_write_pfm(str(path).encode(), _ptr(a), a.shape[1], a.shape[0]), "pt_image_write_pfm")


def write_bmp(path: str, img: np.ndarray) -> None:
    a = _arr(img)
    _check(load().pt_image_write_bmp(str(path).encode(), _ptr(a), a.shape[1], a.shape[0]), "pt_image_write_bmp")


def read_image(path: str) -> np.ndarray:
    lib = load()
    w, h = C.c_int32(0), C.c_int32(0)
    _check(lib.pt_image_read(str(path).encode(), None, C.byref(w), C.byref(h)), "pt_image_read")
    out = np.empty((h.value, w.value, 3), dtype=np.float32)
    _check(lib.pt_image_read(str(path).encode(), _ptr(out), C.byref(w), C.byref(h)), "pt_image_read")
    return out


def mse(a: np.ndarray, b: np.ndarray) -> float:
    """SURVEY.md §8(c) parity metric: mean over pixels x channels, NaN pixels as 0."""
    x, y = _arr(a), _arr(b)
    if x.shape != y.shape:
        raise PTError(f"shape mismatch {x.shape} vs {y.shape}")
    return float(load().pt_image_mse(_ptr(x), _ptr(y), x.shape[0] * x.shape[1]))


def flip(reference: np.ndarray, test: np.ndarray, pixels_per_degree: float = 67.0, error_map: bool = False):
    """LDR-FLIP of two linear images (clamped, sRGB-encoded); mean, and optionally the map."""
    x, y = _arr(reference), _arr(test)
    if x.shape != y.shape:
        raise PTError(f"shape mismatch {x.shape} vs {y.shape}")
    emap = np.zeros(x.shape[:2], np.float32) if error_map else None
    v = float(load().pt_image_flip(_ptr(x), _ptr(y), x.shape[1], x.shape[0], float(pixels_per_degree),
                                   emap.ctypes.data_as(C.POINTER(C.c_float)) if emap is not None else None))
    if v < 0:
        raise PTError("pt_image_flip: invalid arguments")
    return (v, emap) if error_map else v
