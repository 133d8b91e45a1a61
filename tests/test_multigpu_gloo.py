"""CTU-row sharding + the one packed stripe all-gather on CPU with the
gloo backend, world sizes 2 and 3 (unequal stripes).

Each rank predicts its stripe's PUs with the CPU twin of the device pipeline, packs its stripe
into its segment of the stripe-major picture (mm360.parallel.StripeLayout), runs the single
in-place all-gather, and must end with exactly the unsharded full-picture prediction."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import mm360
from mm360 import parallel as P
from mm360 import workload as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg_name, out_dir):
    import sys
    for p in (os.path.join(ROOT, "vvc-extension-mm_amd"), ROOT, os.path.join(ROOT, "tests", "native")):
        sys.path.insert(0, p)
    import twin
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = W.CONFIGS[cfg_name]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg)
    mine = P.shard_pus(pus, cfg.height, world, rank)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    epi = [(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)]
    planes = twin.predict(params, W.CUR_POC, mine, refs, cfg.width, cfg.height, epi)
    layout = P.StripeLayout(cfg.width, cfg.height, world)
    buf = np.full(layout.total, -5, dtype=np.int16)
    layout.pack(planes, rank, buf)
    t = torch.from_numpy(buf)
    P.allgather_packed(t, layout)
    y, cb, cr = layout.unpack(t.numpy())
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), y=y, cb=cb, cr=cr, n=len(mine))
    dist.barrier()
    dist.destroy_process_group()


def test_stripe_layout_pointers_and_unpack():
    """The destination pointers of every rank land each stripe row in its own segment, and
    pack/unpack invert each other (C3 at 1, 2, 3, 4, 8 ranks)."""
    cfg = W.CONFIGS["C3"]
    rng = np.random.default_rng(3)
    planes = [rng.integers(-512, 1024, size=(cfg.height, cfg.width)).astype(np.int16),
              rng.integers(-512, 1024, size=(cfg.height // 2, cfg.width // 2)).astype(np.int16),
              rng.integers(-512, 1024, size=(cfg.height // 2, cfg.width // 2)).astype(np.int16)]
    for world in (1, 2, 3, 4, 8):
        lay = P.StripeLayout(cfg.width, cfg.height, world)
        buf = np.zeros(lay.total, dtype=np.int16)
        for r in range(world):
            lay.pack(planes, r, buf)
            y0, y1 = P.stripe_rows(cfg.height, world, r)
            py, sy, pcb, pcr, sc = lay.dst_pointers(0, r)
            # picture sample (y, x) of the stripe -> element (py + 2 (y sy + x)) / 2 of the buffer
            for (y, x) in ((y0, 0), (y1 - 1, cfg.width - 1)):
                assert buf[(py + 2 * (y * sy + x)) // 2] == planes[0][y, x]
            for (y, x) in ((y0 // 2, 0), (y1 // 2 - 1, cfg.width // 2 - 1)):
                assert buf[(pcb + 2 * (y * sc + x)) // 2] == planes[1][y, x]
                assert buf[(pcr + 2 * (y * sc + x)) // 2] == planes[2][y, x]
        for a, b in zip(lay.unpack(buf), planes):
            assert np.array_equal(a, b)


def test_stripes_partition_pus():
    cfg = W.CONFIGS["C3"]
    pus = W.pu_list(cfg)
    for world in (1, 2, 4, 8):
        parts = [P.shard_pus(pus, cfg.height, world, r) for r in range(world)]
        assert sum(len(p) for p in parts) == len(pus)
        assert sum(W.luma_area(p) for p in parts) == cfg.width * cfg.height
        rows = [P.stripe_rows(cfg.height, world, r) for r in range(world)]
        assert rows[0][0] == 0 and rows[-1][1] == cfg.height
        assert all(rows[i][1] == rows[i + 1][0] for i in range(world - 1))


@pytest.mark.parametrize("cfg_name,world", [("C1", 2), ("C2", 2), ("C2", 3)])
def test_gloo_sharded_equals_full(tmp_path, cfg_name, world):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, cfg_name, str(tmp_path)), nprocs=world, join=True)
    import twin
    cfg = W.CONFIGS[cfg_name]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    full = twin.predict(params, W.CUR_POC, W.pu_list(cfg), refs, cfg.width, cfg.height,
                        [(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)])
    counts = []
    for r in range(world):
        z = np.load(os.path.join(tmp_path, f"rank{r}.npz"))
        counts.append(int(z["n"]))
        for k, ref in zip(("y", "cb", "cr"), full):
            assert np.array_equal(z[k], ref), (r, k)
    assert sum(counts) == len(W.pu_list(cfg))
    n_ctu_rows = (cfg.height + 127) // 128
    assert all(c > 0 for c in counts) or n_ctu_rows < world  # C1 is a single CTU row
