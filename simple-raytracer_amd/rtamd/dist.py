"""Row sharding of one image across ranks (one process per GPU).

Every pixel is independent.  Rows are dealt to ranks in
blocks of BLOCK rows, round robin (rank r gets row blocks r, r+N, r+2N, ...),
so every rank gets the same mix of cheap sky rows and expensive glass rows
(contiguous strips measured 82 % balanced at N = 8 on C3).  Each rank renders
its rows into an HBM buffer padded to the largest rank's row count; rank 0
gathers the N buffers with one fixed-count collective (RCCL over xGMI with the
"nccl" backend, gloo on CPU in tests) and scatters rows back to image order.
"""
from __future__ import annotations

BLOCK = 8


def row_set(H: int, world: int, rank: int, block: int = BLOCK) -> tuple[int, int, int, int, int]:
    """(y0, block, step, nrows, rows_per) for rt_render_row_blocks_async:
    local row k is image row y0 + (k // block) * step + k % block."""
    nblocks = (H + block - 1) // block
    mine = list(range(rank, nblocks, world))
    nrows = sum(min(block, H - b * block) for b in mine)
    rows_per = max(sum(min(block, H - b * block) for b in range(r, nblocks, world)) for r in range(world))
    return rank * block, block, block * world, nrows, max(rows_per, 1)


def image_rows(H: int, world: int, rank: int, block: int = BLOCK) -> list[int]:
    y0, b, step, nrows, _ = row_set(H, world, rank, block)
    return [y0 + (k // b) * step + k % b for k in range(nrows)]


class ImageGather:
    """One frame's row buffer on this rank plus, on rank 0, the gather targets,
    the full image and the image-order row indices (built once, reused every
    frame: no host->device index copies in the frame loop).

    fmt "f32" gathers the float rows (12 B per pixel); "u8" gathers the P3
    writer's pixel values as bytes (3 B per pixel; rt_quantize_u8 on the
    device, exact for values 0..255).  A value outside 0..255 (NaN, a
    background above 1) sets `self.flag` on the device: the u8 image is then
    not the writer's, and the caller must use "f32" (bench.py decides from its
    warm-up frame and checks the flag after the timed ones)."""

    def __init__(self, H: int, W: int, world: int, rank: int, device, torch, fmt: str = "f32"):
        *_, rows_per = row_set(H, world, rank)
        self.H, self.world, self.rank, self.torch, self.fmt = H, world, rank, torch, fmt
        self.strip = torch.zeros((rows_per, W, 3), dtype=torch.float32, device=device)
        self.send = self.strip
        self.flag = None
        if fmt == "u8":
            self.send = torch.zeros((rows_per, W, 3), dtype=torch.uint8, device=device)
            self.flag = torch.zeros(1, dtype=torch.int32, device=device)
        elif fmt != "f32":
            raise ValueError(f"gather format {fmt!r}")
        self.targets = self.image = None
        self.index = []
        self.W, self.rows_per = W, rows_per
        if world > 1 and rank == 0:
            # the N gathered row sets in one buffer (rank r's at [r]): one
            # device kernel puts them in image order (rt_deinterleave_rows
            # / _u8; N index_copy_ on CPU tensors)
            self.gathered = torch.empty((world,) + tuple(self.send.shape), dtype=self.send.dtype, device=device)
            self.targets = list(self.gathered.unbind(0))
            self.image = torch.empty((H, W, 3), dtype=self.send.dtype, device=device)
            if not self.send.is_cuda:
                for r in range(world):
                    rows = image_rows(H, world, r)
                    self.index.append(torch.tensor(rows, dtype=torch.long, device=device) if rows else None)

    def gather(self, dist):
        """Collect every rank's rows on rank 0 (one fixed-count collective) and
        put them in image order; returns the H x W x 3 image there (None
        elsewhere)."""
        if self.fmt == "u8":
            import rtamd
            quantize_u8_device(rtamd, self.torch, self.strip, self.send, self.flag)
        if self.world == 1:
            return self.send[: self.H]
        if self.send.is_cuda and dist.get_backend() == "gloo":
            # gloo (rehearsal of the multi-rank path on one GPU): host staging
            cpu = self.send.cpu()
            tg = [self.torch.empty_like(cpu) for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(cpu, tg, dst=0)
            if self.rank == 0:
                for r in range(self.world):
                    self.targets[r].copy_(tg[r])
        else:
            dist.gather(self.send, self.targets, dst=0)
        if self.rank != 0:
            return None
        if self.image.is_cuda:
            import rtamd
            rtamd.deinterleave_rows_device(self.gathered.data_ptr(), self.world, self.rows_per, self.W, self.H,
                                           BLOCK, self.image.data_ptr(), self.fmt == "u8",
                                           self.torch.cuda.current_stream().cuda_stream)
            return self.image
        for r, idx in enumerate(self.index):
            if idx is not None:
                self.image.index_copy_(0, idx, self.targets[r][: idx.numel()])
        return self.image



def quantize_u8_device(rtamd, torch, rgb, out, flag) -> None:
    """rt_quantize_u8 of a float32 device tensor into a uint8 one of the same
    shape, on the current stream (bit 0 of flag: a value outside 0..255)."""
    assert rgb.is_cuda and rgb.dtype == torch.float32 and out.dtype == torch.uint8
    assert rgb.is_contiguous() and out.is_contiguous() and rgb.numel() == out.numel()
    rtamd.quantize_u8_device(rgb.data_ptr(), rgb.numel(), out.data_ptr(), flag.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
