"""Multi-GPU partitioning of the MM motion-compensation path.

Given the reference pictures, PUs are independent: MC reads only the references plus the PU's
own descriptor.  A picture therefore shards by contiguous CTU-row stripes (PU -> rank owning
the CTU row of its top-left sample); the references stay replicated on every GPU because MM
motion can fetch anywhere in the picture (it wraps across the ERP seam).  After MC, one
all-gather of the predicted stripes (RCCL over xGMI with the "nccl" backend; gloo on CPU)
gives every rank the whole picture again, as a decoder needs for the next reference.

The bench's default multi-GPU mode does not use this: every rank predicts its own picture
(independent pictures, no data-path collective, weak scaling).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def stripe_rows(height: int, world: int, rank: int, ctu: int = 128) -> Tuple[int, int]:
    """Luma row range [y0, y1) of `rank`'s CTU-row stripe."""
    n_ctu = (height + ctu - 1) // ctu
    a = (n_ctu * rank) // world
    b = (n_ctu * (rank + 1)) // world
    return min(a * ctu, height), min(b * ctu, height)


def shard_pus(pus: np.ndarray, height: int, world: int, rank: int, ctu: int = 128) -> np.ndarray:
    """PUs whose top-left CTU row falls into `rank`'s stripe (PUs never cross CTU rows)."""
    y0, y1 = stripe_rows(height, world, rank, ctu)
    sel = (pus["y"] >= y0) & (pus["y"] < y1)
    return pus[sel]


def max_stripe_rows(height: int, world: int, ctu: int = 128) -> int:
    return max(b - a for a, b in (stripe_rows(height, world, r, ctu) for r in range(world)))


def allgather_stripes(planes: List, height: int, world: int, group=None, ctu: int = 128) -> None:
    """In place: every rank contributes its stripe of each plane (torch tensors [H_c, W_c]) and
    receives all the others.  Chroma planes (half height) use the halved stripe bounds."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    smax = max_stripe_rows(height, world, ctu)
    for p in planes:
        scale = height // p.shape[0]  # 1 luma, 2 chroma 4:2:0
        y0, y1 = stripe_rows(height, world, rank, ctu)
        rows = smax // scale
        send = torch.zeros((rows, p.shape[1]), dtype=p.dtype, device=p.device)
        send[: (y1 - y0) // scale] = p[y0 // scale: y1 // scale]
        # int16 samples travel bit-exactly as uint8 (NCCL/RCCL and gloo have no int16 type)
        send_b = send.view(torch.uint8)
        recv = [torch.empty_like(send_b) for _ in range(world)]
        dist.all_gather(recv, send_b, group=group)
        for r in range(world):
            a, b = stripe_rows(height, world, r, ctu)
            p[a // scale: b // scale] = recv[r].view(p.dtype)[: (b - a) // scale]
