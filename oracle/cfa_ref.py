"""TEST INFRASTRUCTURE ONLY -- literal Python restatements of Siril's
frame-level data movement around the stack (checked against the HIP kernels
in tests/test_cfa_ops.py).  Only tests/ import this module.

* shift_fit_from_reg      registration/registration.c:322-370
* apply_reg_shifts        cvTransfH (opencv/opencv.cpp:385-396) for
                          translations + translation_from_H (registration.c:301-304)
* extract_CFA_buffer      algos/demosaicing.c:936-975
* split_cfa               algos/extraction.c:982-1013
* merge_cfa               algos/demosaicing.c:757-820
"""
from __future__ import annotations

import numpy as np


def round_to_int(x: float) -> int:                      # core/proto.h:208-213
    x = min(x, 2147483647.0 - 0.5)
    x = max(x, -2147483648.0 + 0.5)
    return int(x + (0.5 if x >= 0.0 else -0.5))


def apply_reg_shifts(Hs, ref_index):
    Href = np.asarray(Hs[ref_index], np.float64)
    sx, sy = [], []
    for H in Hs:
        Hr = np.linalg.inv(Href) @ np.asarray(H, np.float64)   # H1.inv() * H0 with H0 = Himg, H1 = Htransf
        dx, dy = Hr[0, 2], -Hr[1, 2]
        sx.append(round_to_int(dx))
        sy.append(round_to_int(dy))
    return np.array(sx, np.int32), np.array(sy, np.int32)


def shift_fit_from_reg(img, shiftx, shifty):
    ry, rx = img.shape
    out = np.zeros_like(img)
    for y in range(ry):
        for x in range(rx):
            nx, ny = x + shiftx, y + shifty
            if 0 <= nx < rx and 0 <= ny < ry:
                out[ny, nx] = img[y, x]
    return out


def extract_CFA_buffer(img, pattern, pattern_size, layer):
    ry, rx = img.shape
    flat = img.ravel()
    buf = []
    i = 0
    pattern_y = 0
    for y in range(ry):
        idx_y = pattern_y * pattern_size
        for x in range(rx):
            if pattern[idx_y + x % pattern_size] == layer:
                buf.append(flat[i])
            i += 1
        pattern_y = (pattern_y + 1) % pattern_size
    return np.array(buf, img.dtype)


def split_cfa(img):
    ry, rx = img.shape
    w, h = rx // 2, ry // 2
    out = np.zeros((4, h * w), img.dtype)
    flat = img.ravel()
    j = 0
    for row in range(0, ry - 1, 2):
        for col in range(0, rx - 1, 2):
            out[0, j] = flat[col + row * rx]
            out[1, j] = flat[1 + col + row * rx]
            out[2, j] = flat[col + (1 + row) * rx]
            out[3, j] = flat[1 + col + (1 + row) * rx]
            j += 1
    return out.reshape(4, h, w)


def merge_cfa(planes):
    _, h, w = planes.shape
    out = np.zeros((2 * h, 2 * w), planes.dtype)
    for outx in range(0, 2 * w, 2):
        for outy in range(0, 2 * h, 2):
            cx, cy = outx >> 1, outy >> 1
            out[outy, outx] = planes[0, cy, cx]
            out[outy, outx + 1] = planes[1, cy, cx]
            out[outy + 1, outx] = planes[2, cy, cx]
            out[outy + 1, outx + 1] = planes[3, cy, cx]
    return out
