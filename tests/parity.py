"""Parity criterion between the HIP path and the CPU oracle:
per channel |gpu - oracle| <= 1e-4 on >= 99.95 % of pixels; NaN positions
must agree except on the (counted) pixels outside tolerance."""
from __future__ import annotations

import numpy as np

TOL = 1e-4
MAX_BAD_FRAC = 5e-4


def compare(gpu: np.ndarray, ref: np.ndarray) -> dict:
    assert gpu.shape == ref.shape, (gpu.shape, ref.shape)
    ng, nr = np.isnan(gpu), np.isnan(ref)
    d = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
    d[ng & nr] = 0.0
    d[ng ^ nr] = np.inf
    d = np.nan_to_num(d, nan=np.inf)
    px_bad = (d > TOL).any(axis=-1)
    px_exact = (d == 0).all(axis=-1)
    npx = px_bad.size
    return dict(pixels=npx, bad=int(px_bad.sum()), bad_frac=float(px_bad.sum()) / npx,
                exact_frac=float(px_exact.sum()) / npx, max_abs=float(np.max(d[np.isfinite(d)], initial=0.0)),
                nan_mismatch=int((ng ^ nr).any(axis=-1).sum()), nan_px=int(nr.any(axis=-1).sum()))


def assert_parity(gpu: np.ndarray, ref: np.ndarray, label: str = "") -> dict:
    c = compare(gpu, ref)
    assert c["bad_frac"] <= MAX_BAD_FRAC, f"{label}: {c}"
    return c
