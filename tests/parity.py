"""Parity criterion between the HIP path and its references (SURVEY.md §8c,
BASELINE.json north_star): per channel |gpu - ref| <= 1e-4 on EVERY pixel, and
NaN positions identical (a NaN on one side only is a mismatch).  No exception
budget: a single pixel outside the tolerance fails.

The quantised 8-bit values (`(int)(c * 255.0f)`, main.cpp:760-762) may differ
from the reference's only where the float lies within the tolerance of a
quantisation boundary: `quantized_flips` counts those values and checks that
each one is that kind of flip (one level apart, float within 255 * TOL of the
boundary between the two levels)."""
from __future__ import annotations

import numpy as np

TOL = 1e-4


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
    assert c["bad"] == 0 and c["nan_mismatch"] == 0, f"{label}: {c}"
    return c


def quantized_flips(gpu_f: np.ndarray, gpu_q: np.ndarray, ref_q: np.ndarray, label: str = "") -> dict:
    """8-bit values that differ from the reference's.  Every one must be a
    rounding flip: |q - q_ref| == 1 and the GPU float within 255 * TOL of the
    level boundary max(q, q_ref) / 255.  NaN pixels must quantise identically."""
    gq = np.asarray(gpu_q, dtype=np.int64)
    rq = np.asarray(ref_q, dtype=np.int64)
    assert gq.shape == rq.shape == gpu_f.shape, (gq.shape, rq.shape, gpu_f.shape)
    diff = gq != rq
    n = int(diff.sum())
    out = dict(values=int(gq.size), flipped=n, flipped_px=int(diff.any(axis=-1).sum()))
    if n:
        assert not np.isnan(gpu_f[diff]).any(), f"{label}: a NaN value quantised differently"
        step = np.abs(gq[diff] - rq[diff])
        assert step.max() == 1, f"{label}: a value is {int(step.max())} levels off"
        edge = np.maximum(gq[diff], rq[diff]).astype(np.float64)
        dist = np.abs(gpu_f[diff].astype(np.float64) * 255.0 - edge)
        out["max_dist_to_edge"] = float(dist.max())
        assert dist.max() <= 255.0 * TOL, f"{label}: flipped value {dist.max() / 255.0:.3g} from its edge"
    return out
