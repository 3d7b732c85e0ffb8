"""Row-strip sharding of one image across ranks (one process per GPU).

Every pixel is independent, so the image's rows are cut into
one contiguous strip per rank, padded to equal height so the strips can be
gathered with one fixed-count collective.  Each rank renders its strip into
HBM; rank 0 receives all strips (RCCL over xGMI when the backend is "nccl",
gloo on CPU in tests) and drops the padding rows.
"""
from __future__ import annotations


def strip_rows(H: int, world: int, rank: int) -> tuple[int, int, int]:
    """(y0, y1, rows_per): rank's rows [y0, y1) and the padded strip height."""
    rows_per = (H + world - 1) // world
    y0 = min(H, rank * rows_per)
    y1 = min(H, y0 + rows_per)
    return y0, y1, rows_per


def alloc_strips(H: int, W: int, world: int, rank: int, device, torch):
    """This rank's padded strip buffer and, on rank 0, the gather targets."""
    _, _, rows_per = strip_rows(H, world, rank)
    strip = torch.zeros((rows_per, W, 3), dtype=torch.float32, device=device)
    targets = None
    if world > 1 and rank == 0:
        targets = [torch.empty_like(strip) for _ in range(world)]
    return strip, targets


def gather_strips(strip, targets, world: int, rank: int, H: int, dist, torch):
    """Collect every rank's strip on rank 0; returns the H x W x 3 image there
    (None elsewhere).  One gather of world equal-size strips."""
    if world == 1:
        return strip[:H]
    dist.gather(strip, targets, dst=0)
    if rank != 0:
        return None
    return torch.cat(targets, dim=0)[:H]
