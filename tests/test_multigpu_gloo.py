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
from mm360 import gop as G
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


@pytest.mark.parametrize("bd", [8, 10, 12])
def test_packed_transport_roundtrip(bd):
    """The stripe-packed C4 transport (include/mm360.h): K = 32 // bd samples per word, every
    bd-bit sample survives pack -> unpack, and a packed picture of every world size unpacks to the
    planes (C3 geometry at 1, 2, 3, 8 ranks; 10 bits: 2/3 of the int16 bytes)."""
    rng = np.random.default_rng(bd)
    v = rng.integers(0, 1 << bd, size=1001).astype(np.int16)
    w = P.pack_samples(v, bd)
    assert len(w) == -(-1001 // (32 // bd)) and w.dtype == np.uint32
    assert np.array_equal(P.unpack_samples(w, 1001, bd), v)
    cfg = W.CONFIGS["C3"]
    planes = [rng.integers(0, 1 << bd, size=(cfg.height, cfg.width)).astype(np.int16),
              rng.integers(0, 1 << bd, size=(cfg.height // 2, cfg.width // 2)).astype(np.int16),
              rng.integers(0, 1 << bd, size=(cfg.height // 2, cfg.width // 2)).astype(np.int16)]
    for world in (1, 2, 3, 8):
        lay = P.StripeLayout(cfg.width, cfg.height, world)
        buf = np.zeros(lay.total, dtype=np.int16)
        words = np.zeros(world * P.packed_words(lay, bd), dtype=np.uint32)
        for r in range(world):
            lay.pack(planes, r, buf)
            P.pack_segment(buf, lay, r, bd, words)
        for a, b in zip(P.unpack_picture(words, lay, bd), planes):
            assert np.array_equal(a, b)
        if bd == 10:
            assert abs(words.nbytes / buf.nbytes - 2 / 3) < 1e-3


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


GOP_CFG = W.Config("GOP", 512, 384, W.MPA3 + (mm360.GEODESIC_CAMPOSE, mm360.ROTATIONAL), 6,
                   "512x384 ERP, three CTU rows (decode-order chain)")


def _chain_pus(k, poc, refs):
    """Picture k's PU list with its two workload references (0, 16) mapped onto the picture's
    decode-order references: list 0 -> the nearest past one, list 1 -> the nearest future one
    (the other side when one side is empty)."""
    pus = W.pu_list(GOP_CFG, frame=k)
    past = [r for r in refs if r < poc]
    fut = [r for r in refs if r > poc]
    r0 = max(past) if past else min(fut)
    r1 = min(fut) if fut else max(past)
    rp = pus["ref_poc"]
    pus["ref_poc"] = np.where(rp == W.REF_POCS[0], r0, np.where(rp == W.REF_POCS[1], r1, -1))
    return pus


def _chain_worker(rank, world, port, n_pictures, out_dir, batch=1, packed=False):
    """One rank of the C4 decode-order loop (mm360.gop.DependencyLoop) on CPU: every picture is
    predicted FROM the gathered pictures it references, so a missing or early reference wait
    would show up as a wrong picture.  packed: the all-gather carries the stripe-packed picture
    (10-bit samples, three per word: mm360.parallel.pack_segment / unpack_picture, the host
    definition of mm_pack_samples / mm_upload_ref_packed)."""
    import sys
    for p in (os.path.join(ROOT, "vvc-extension-mm_amd"), ROOT, os.path.join(ROOT, "tests", "native")):
        sys.path.insert(0, p)
    import twin
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = GOP_CFG
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    seq = G.decode_sequence(n_pictures, "ra8")
    epi = [(poc, -1, W.GED_EPIPOLE_Q24) for poc, _, _ in seq]
    lay = P.StripeLayout(cfg.width, cfg.height, world)
    bufs = [np.full(lay.total, -5, dtype=np.int16) for _ in range(2)]
    decoded = {0: W.ref_planes(cfg.width, cfg.height, 0)}
    cur = {}

    def predict(k, poc, refs, b):
        mine = P.shard_pus(_chain_pus(k, poc, refs), cfg.height, world, rank)
        planes = twin.predict(params, poc, mine, {r: decoded[r] for r in refs}, cfg.width, cfg.height, epi)
        lay.pack(planes, rank, bufs[b])
        decoded[poc] = planes  # this rank's stripe only, until (and unless) the picture is all-gathered
        cur["poc"] = poc

    buf_poc = {}

    def predict_batch(items):
        """the batch's pictures (independent) in one mm_pred_device_multi-style call (CPU twin)"""
        pics = [(poc, P.shard_pus(_chain_pus(k, poc, refs), cfg.height, world, rank)) for k, poc, refs, _ in items]
        rr = {r: decoded[r] for _, _, refs, _ in items for r in refs}
        outs = twin.predict_multi(params, pics, rr, cfg.width, cfg.height, epi)
        for (k, poc, refs, b), planes in zip(items, outs):
            lay.pack(planes, rank, bufs[b])
            decoded[poc] = planes
            buf_poc[b] = poc

    def gather(b):
        poc = buf_poc.get(b, cur.get("poc")) if batch > 1 else cur["poc"]
        if packed:
            words = np.zeros(world * P.packed_words(lay, 10), dtype=np.uint32)
            P.pack_segment(bufs[b], lay, rank, 10, words)
            t = torch.from_numpy(words.view(np.int32))
            P.allgather_packed(t, lay)
            decoded[poc] = P.unpack_picture(t.numpy().view(np.uint32), lay, 10)
        else:
            t = torch.from_numpy(bufs[b])
            P.allgather_packed(t, lay)
            decoded[poc] = lay.unpack(t.numpy())
        return ("gathered", poc)

    waits = []
    loop = G.DependencyLoop("ra8", 2, predict, gather, waits.append)
    if batch > 1:
        while loop.k < n_pictures:
            loop.step_batch(min(batch, n_pictures - loop.k), predict_batch)
    else:
        for _ in range(n_pictures):
            loop.step()
    with open(os.path.join(out_dir, f"batches{rank}.txt"), "w") as f:
        f.write(str(loop.k))
    out = {f"poc{poc}_{c}": decoded[poc][i] for poc, _, _ in seq for i, c in enumerate(("y", "cb", "cr"))}
    np.savez(os.path.join(out_dir, f"chain{rank}.npz"), **out)
    with open(os.path.join(out_dir, f"trace{rank}.txt"), "w") as f:
        for poc, waited in loop.trace:
            f.write(f"{poc}:{','.join(map(str, waited))}\n")
    with open(os.path.join(out_dir, f"gathered{rank}.txt"), "w") as f:
        f.write(",".join(map(str, loop.gathered)))
    dist.barrier()
    dist.destroy_process_group()


def test_decode_sequences():
    """The reference's RA GOP-32 (cfg/encoder_randomaccess_vtm.cfg:20-51) and the dyadic GOP-8:
    every POC of a GOP decoded once, every reference decoded earlier (or before the sequence)."""
    for name, size in (("ra32", 32), ("ra8", 8)):
        seq = G.decode_sequence(3 * size, name)
        assert sorted(p for p, _, _ in seq) == list(range(1, 3 * size + 1))
        done = set()
        for poc, tid, refs in seq:
            assert poc not in refs and all(r in done or r <= 0 for r in refs), (name, poc, refs)
            done.add(poc)
        assert [p for p, _, _ in seq[:size]][:4] == [size, size // 2, size // 4, size // 8]
        leaves = [p for p, t, _ in seq if t == max(tt for _, tt, _ in seq)]
        assert all(p % 2 == 1 for p in leaves) and len(leaves) == len(seq) // 2
    assert G.decode_sequence(1, "ra32", 22)[0] == (22, 4, [0, 16, 18, 20, 24, 32])


def test_schedule_model():
    """The dependency-aware model: with every all-gather shorter than the MC, each picture that
    the next one references stalls the GPUs by one all-gather; half the pictures are referenced
    in both GOPs, so gathering only those halves a link-bound loop.  Without all-gathers it is the
    MC time."""
    for g in ("ra32", "ra8"):
        assert sum(G.is_referenced(p, g) for p in range(1, 65)) == 32
        assert G.schedule(64, 1.0, 0.0, g)["ms_per_picture"] == 1.0
        r = G.schedule(64, 1.0, 0.3, g)
        assert 1.0 < r["ms_per_picture"] < 1.3 and r["stall_ms_per_picture"] > 0
        slow_all = G.schedule(64, 0.1, 1.0, g, gather_all=True)  # all-gather bound
        slow_ref = G.schedule(64, 0.1, 1.0, g)
        assert slow_all["ms_per_picture"] >= 1.0 and 0.5 <= slow_ref["ms_per_picture"] <= 0.61
        # batched leaves (the same grouping as DependencyLoop.next_batch): with a batch of two at the
        # single-picture cost per picture nothing changes; cheaper batches cut only the leaves' MC
        same = G.schedule(64, 1.0, 0.0, g, batch_ms={2: 1.0})
        assert abs(same["ms_per_picture"] - 1.0) < 1e-9
        cheap = G.schedule(64, 1.0, 0.0, g, batch_ms={2: 0.5})["ms_per_picture"]
        loop = G.DependencyLoop(g, 4, None, None, None)
        n_batched = 0
        while loop.k < 64:
            b = loop.next_batch(2)
            n_batched += len(b) if len(b) == 2 else 0
            loop.k += len(b)
        assert n_batched > 0
        assert abs(cheap - (64 - 0.5 * n_batched) / 64) < 1e-9, (cheap, n_batched)


@pytest.mark.parametrize("batch,packed", [(1, False), (2, False), (1, True), (2, True)])
def test_gloo_decode_order_chain(tmp_path, batch, packed):
    """C4 decode-order loop, world 2: each picture of an RA GOP-8 sequence is predicted from its
    gathered references; only referenced pictures are all-gathered (every rank then holds exactly
    the unsharded picture), unreferenced ones stay sharded (each rank holds its stripe of it), and
    each picture waited for the all-gathers of all its references decoded in the sequence.
    batch 2: independent consecutive pictures (the leaves 1 and 3) are predicted together in one
    multi-picture call (DependencyLoop.step_batch, mm_pred_device_multi's CPU twin).
    packed: the all-gathers carry the stripe-packed pictures (2/3 of the int16 bytes)."""
    n = 6
    port = _free_port()
    mp.spawn(_chain_worker, args=(2, port, n, str(tmp_path), batch, packed), nprocs=2, join=True)
    if batch > 1:
        seq_b = G.decode_sequence(n, "ra8")
        loop = G.DependencyLoop("ra8", 2, None, None, None)
        loop.k = 3
        assert [p for p, _, _ in loop.next_batch(2)] == [1, 3]  # the leaves after 8 4 2 go together
        assert [p for p, _, _ in seq_b][3:5] == [1, 3]
    import twin
    cfg = GOP_CFG
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    seq = G.decode_sequence(n, "ra8")
    epi = [(poc, -1, W.GED_EPIPOLE_Q24) for poc, _, _ in seq]
    decoded = {0: W.ref_planes(cfg.width, cfg.height, 0)}
    for k, (poc, _, refs) in enumerate(seq):
        decoded[poc] = twin.predict(params, poc, _chain_pus(k, poc, refs), {r: decoded[r] for r in refs},
                                    cfg.width, cfg.height, epi)
    referenced = [poc for poc, _, _ in seq if G.is_referenced(poc, "ra8")]
    assert referenced == [8, 4, 2, 6]  # the GOP-8 leaves 1, 3 (and 5, 7) are never referenced
    for r in range(2):
        z = np.load(os.path.join(tmp_path, f"chain{r}.npz"))
        y0, y1 = P.stripe_rows(cfg.height, 2, r)
        for poc, _, _ in seq:
            for i, c in enumerate(("y", "cb", "cr")):
                got, want = z[f"poc{poc}_{c}"], decoded[poc][i]
                if poc in referenced:  # rebuilt on every rank by the all-gather
                    assert np.array_equal(got, want), (r, poc, c)
                else:  # stays sharded: this rank's stripe
                    a, b = (y0, y1) if i == 0 else (y0 // 2, y1 // 2)
                    assert np.array_equal(got[a:b], want[a:b]), (r, poc, c)
        assert open(os.path.join(tmp_path, f"gathered{r}.txt")).read() == ",".join(map(str, referenced))
        trace = open(os.path.join(tmp_path, f"trace{r}.txt")).read().split()
        for (poc, _, refs), line in zip(seq, trace):
            p, w = line.split(":")
            assert int(p) == poc
            assert sorted(int(x) for x in w.split(",") if x) == [x for x in refs if x > 0]
