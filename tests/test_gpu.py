"""Parity of the HIP path (through the C-ABI) with the CPU oracle and the golden vectors.

Bit-exact everywhere: fixed-point reprojection results, filter outputs and predicted samples are
integers.  Size-independent properties at the full 6144x3072 size: full-frame equality with the
oracle, determinism, prepare/run == one-shot, uni/bi consistency."""
import os

import numpy as np
import pytest

import mm360
from helpers import EPI, GOLDEN, describe_mismatch, dmvr_zero_mv_pus, load_blocks, load_pus
from mm360 import workload as W
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    mm360.load_library()  # raises if the HIP library is missing -- no fallback


def plane_mismatch(name, got, want):
    bad = np.argwhere(got != want)
    if not len(bad):
        return f"{name}: equal"
    y, x = bad[0]
    return f"{name}: {len(bad)} samples differ, first at (y={y}, x={x}): {got[y, x]} vs {want[y, x]}"


def _ctx(params, epipoles=EPI):
    ctx = mm360.MMContext(params, device=0)
    for (cur, ref, q) in epipoles:
        ctx.set_epipole(cur, ref, q)
    return ctx


def _gpu_predict(ctx, params, cur_poc, pus, refs):
    W_, H_ = params.width, params.height
    for poc, (y, cb, cr) in refs.items():
        ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
    dy = torch.zeros((H_, W_), dtype=torch.int16, device="cuda")
    dcb = torch.zeros((H_ // 2, W_ // 2), dtype=torch.int16, device="cuda")
    dcr = torch.zeros_like(dcb)
    ctx.predict(cur_poc, pus, dy, dcb, dcr)
    torch.cuda.synchronize()
    return dy.cpu().numpy(), dcb.cpu().numpy(), dcr.cpu().numpy()


@pytest.mark.parametrize("name", ["reproject_c1_all_models.npz", "reproject_c2_all_models.npz",
                                  "reproject_c1_offset15_original.npz"])
def test_reproject_golden(name):
    z = np.load(os.path.join(GOLDEN, name))
    blocks = load_blocks(z)
    off, flav = [int(v) for v in z["params"]]
    params = mm360.seq_params(int(z["width"]), int(z["height"]), [int(m) for m in z["models"]], mm_offset4x4=off,
                              ged_flavor=flav)
    with _ctx(params) as ctx:
        got = ctx.reproject(blocks)
    assert np.array_equal(got, z["result"]), describe_mismatch(blocks, got, z["result"])


@pytest.mark.parametrize("w,h,seed,off,flav", [(256, 128, 11, 1, 1), (2048, 1024, 12, 0, 1), (6144, 3072, 13, 1, 1),
                                             (1024, 512, 14, 4, 0), (4096, 2048, 15, 3, 1)])
def test_reproject_random_vs_oracle(w, h, seed, off, flav):
    models = W.ALL_MODELS + (7, 8, 9)
    params = mm360.seq_params(w, h, models, mm_offset4x4=off, ged_flavor=flav)
    blocks = W.random_blocks(w, h, models, 4000, seed, sizes=(4, 8, 16, 32, 64, 128))
    want = Oracle(params, EPI).reproject(blocks)
    with _ctx(params) as ctx:
        got = ctx.reproject(blocks)
    assert np.array_equal(got, want), describe_mismatch(blocks, got, want)


def test_reproject_single_call_shape():
    params = mm360.seq_params(256, 128, W.ALL_MODELS)
    with _ctx(params) as ctx:
        X, Y = ctx.reproject_motion_vector_subblocks((32, 16), (16, 8), (37, -5), mm360.ROTATIONAL, 0)
        assert X.shape == (2, 4) and Y.shape == (2, 4)
        # zero motion with the ROT shortcut returns the grid: (4*i + off - off) * 16
        X0, Y0 = ctx.reproject_motion_vector_subblocks((32, 16), (16, 8), (0, 0), mm360.ROTATIONAL, 0)
        assert np.array_equal(X0[0], (32 + 4 * np.arange(4)) * 16) and np.array_equal(Y0[:, 0], (16 + 4 * np.arange(2)) * 16)


def test_pred_golden_c1():
    z = np.load(os.path.join(GOLDEN, "pred_c1.npz"))
    cfg = W.CONFIGS["C1"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    with _ctx(params) as ctx:
        y, cb, cr = _gpu_predict(ctx, params, W.CUR_POC, load_pus(z), refs)
    assert np.array_equal(y, z["y"]) and np.array_equal(cb, z["cb"]) and np.array_equal(cr, z["cr"])


@pytest.mark.parametrize("cfg_name,frame", [("C1", 3), ("C2", 0), ("C2", 5), ("C3", 0)])
def test_pred_full_frame_vs_oracle(cfg_name, frame):
    cfg = W.CONFIGS[cfg_name]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=frame)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        got = _gpu_predict(ctx, params, W.CUR_POC, pus, refs)
    for name, g, w in zip("Y Cb Cr".split(), got, want):
        assert np.array_equal(g, w), f"{name}: {(g != w).sum()} samples differ"


@pytest.mark.parametrize("model", W.ALL_MODELS)
def test_pred_uniform_per_model(model):
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, W.ALL_MODELS)
    pus = W.pu_list(cfg, uniform=True, uniform_model=model)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        got = _gpu_predict(ctx, params, W.CUR_POC, pus, refs)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("w,h,bd,off,flav,frame", [(264, 136, 10, 1, 1, 1), (1032, 520, 8, 4, 0, 2),
                                                  (520, 264, 12, 0, 1, 3), (2056, 1032, 10, 3, 1, 4)])
def test_pred_ragged_size_and_seq_variants(w, h, bd, off, flav, frame):
    """Picture sizes that are multiples of 8 but not of the CTU or 16 (partial CTUs on the right
    and bottom, 8-wide / 8-high leaves there), 8/10/12-bit samples, every mm_offset4x4 code
    (MVReprojection.cpp:10), both GED flavors, and the axis geodesic models GEODESIC_X/Y/Z
    besides the seven of ALL_MODELS."""
    models = W.ALL_MODELS + (mm360.GEODESIC_X, mm360.GEODESIC_Y, mm360.GEODESIC_Z)
    cfg = W.Config("ragged", w, h, models, 1, "ragged")
    params = mm360.seq_params(w, h, models, bit_depth=bd, mm_offset4x4=off, ged_flavor=flav)
    pus = W.pu_list(cfg, frame=frame)
    assert (pus["x"] + pus["w"]).max() == w and (pus["y"] + pus["h"]).max() == h
    refs = {poc: W.ref_planes(w, h, poc, bit_depth=bd) for poc in W.REF_POCS}
    if bd == 12:  # spread the 10-bit content over the 12-bit range
        refs = {poc: tuple(np.clip(a.astype(np.int32) * 4 + 3, 0, 4095).astype(np.int16) for a in planes)
                for poc, planes in refs.items()}
    want = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, w, h)
    with _ctx(params) as ctx:
        got = _gpu_predict(ctx, params, W.CUR_POC, pus, refs)
        # the same list already resident in HBM (mm_pred_device), planned in 3 stripes
        ctx.set_stripes(3)
        dst = _planes(cfg, -7)
        ctx.predict_device(W.CUR_POC, mm360.pus_to_device(pus), *dst)
        assert ctx.status() == (mm360.MM_OK, -1)
        got_dev = [t.cpu().numpy() for t in dst]
    for name, g, gd, wv in zip("Y Cb Cr".split(), got, got_dev, want):
        assert np.array_equal(g, wv), f"{name}: {(g != wv).sum()} samples differ"
        assert np.array_equal(gd, wv), f"{name} (device plan): {(gd != wv).sum()} samples differ"
    assert int(want[0].max()) <= (1 << bd) - 1 and int(want[0].max()) > (1 << bd) // 2


def test_pred_extreme_motion_zeroing():
    cfg = W.CONFIGS["C1"]
    params = mm360.seq_params(cfg.width, cfg.height, W.ALL_MODELS)
    pus = W.pu_list(cfg, frame=2)
    rng = np.random.default_rng(9)
    pus["model"] = rng.choice(np.array(W.ALL_MODELS), size=pus["model"].shape)
    pus["mv"] = rng.integers(-(1 << 14), 1 << 14, size=pus["mv"].shape)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        got = _gpu_predict(ctx, params, W.CUR_POC, pus, refs)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    # EquirectangularProjection::fromSphere maps every direction into [0, W] x [0, H], so the
    # out-of-range zeroing rule (InterPrediction.cpp:780) cannot trigger for ERP reprojections;
    # large motions wrap around the sphere instead.


@pytest.mark.parametrize("world", [1, 3, 8])
def test_c4_packed_transport_uploads_the_same_reference(world):
    """C4 transport (mm360.h, stripe-packed pictures): every rank's int16 segment packed by
    mm_pack_samples == the host definition (mm360.parallel.pack_segment), and the packed picture
    made a reference by mm_upload_ref_packed (unpacked straight into the padded pool copy) -- or the
    int16 stripe-major picture by mm_upload_ref_stripes -- predicts what the oracle predicts from the
    same planes, with large motion, so windows reach the margins the unpack fills."""
    from mm360 import parallel as P
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    pus = W.pu_list(cfg, frame=4)
    rng = np.random.default_rng(17)
    pus["mv"] = rng.integers(-(1 << 13), 1 << 13, size=pus["mv"].shape)
    lay = P.StripeLayout(cfg.width, cfg.height, world)
    buf = np.zeros(lay.total, dtype=np.int16)
    for r in range(world):
        lay.pack(refs[W.REF_POCS[1]], r, buf)
    nw = P.packed_words(lay, 10)
    want_words = np.zeros(world * nw, dtype=np.uint32)
    for r in range(world):
        P.pack_segment(buf, lay, r, 10, want_words)
    want = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        assert ctx.stripe_packed_dwords(world) == nw
        d_buf = torch.from_numpy(buf).cuda()
        packed = torch.full((world * nw,), -1, dtype=torch.int32, device="cuda")
        for r in range(world):
            ctx.pack_samples(d_buf[r * lay.seg:(r + 1) * lay.seg], packed[r * nw:(r + 1) * nw])
        torch.cuda.synchronize()
        assert np.array_equal(packed.cpu().numpy().view(np.uint32), want_words)
        y, cb, cr = refs[W.REF_POCS[0]]
        ctx.upload_ref(W.REF_POCS[0], torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_pus = mm360.pus_to_device(pus)
        for transport in ("packed", "int16"):  # mm_upload_ref_packed, then mm_upload_ref_stripes
            if transport == "packed":
                ctx.upload_ref_packed(W.REF_POCS[1], packed, world)
            else:
                ctx.release_ref(W.REF_POCS[1])
                ctx.upload_ref_stripes(W.REF_POCS[1], d_buf, world)
            out = _planes(cfg, -1)
            ctx.predict_device(W.CUR_POC, d_pus, *out)
            ctx.synchronize()
            for name, t, x in zip(("y", "cb", "cr"), out, want):
                got = t.cpu().numpy()
                assert np.array_equal(got, x), (transport, plane_mismatch(name, got, x))


@pytest.mark.parametrize("max_cu", [8, 32, 64])
def test_pred_small_max_cu_padded_margins(max_cu):
    """The reference pool's edge-replicated margins are sized from maxCU (mm_kernels.hip
    plane_layout: maxCU + filter reach + 8, rounded to 64 columns; maxCU + reach + 8 rows), and the
    out-of-range rule zeroes with +-maxCU (InterPrediction.cpp:780).  Small maxCU gives the
    narrowest margins; random large motions put windows on every picture edge."""
    cfg = W.CONFIGS["C1"]
    params = mm360.seq_params(cfg.width, cfg.height, W.ALL_MODELS, max_cu=max_cu)
    pus = W.pu_list(cfg, frame=5)
    rng = np.random.default_rng(max_cu)
    pus["model"] = rng.choice(np.array(W.ALL_MODELS), size=pus["model"].shape)
    pus["mv"] = rng.integers(-(1 << 12), 1 << 12, size=pus["mv"].shape)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        got = _gpu_predict(ctx, params, W.CUR_POC, pus, refs)
    for name, g, w in zip("Y Cb Cr".split(), got, want):
        assert np.array_equal(g, w), f"{name}: {(g != w).sum()} samples differ"


def test_pred_deterministic_and_split_api():
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=7)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    with _ctx(params) as ctx:
        a = _gpu_predict(ctx, params, W.CUR_POC, pus, refs)
        dy = torch.full((cfg.height, cfg.width), -1, dtype=torch.int16, device="cuda")
        dcb = torch.full((cfg.height // 2, cfg.width // 2), -1, dtype=torch.int16, device="cuda")
        dcr = torch.full_like(dcb, -1)
        ctx.prepare(W.CUR_POC, pus)
        for _ in range(3):
            ctx.run(dy, dcb, dcr)
        ctx.synchronize()
        assert ctx.last_timing_ms() > 0
        ctx.set_call_timing(False)  # no events around the call: nothing to read
        ctx.run(dy, dcb, dcr)
        ctx.synchronize()
        with pytest.raises(mm360.MMError):
            ctx.last_timing_ms()
        ctx.set_call_timing(True)
    for x, t in zip(a, (dy, dcb, dcr)):
        assert np.array_equal(x, t.cpu().numpy())


def _filter_cases():
    rng = np.random.default_rng(5)
    src = rng.integers(0, 1024, size=(40, 40)).astype(np.int16)
    src[5:9, :] = 1023
    src[20:24, :] = 0
    return src


@pytest.mark.parametrize("comp", [0, 1])
def test_filter_all_phases_vs_oracle(comp):
    src = _filter_cases()
    params = mm360.seq_params(256, 128, [1])
    orc = Oracle(params)
    phases = 16 if comp == 0 else 32
    with _ctx(params, []) as ctx:
        for frac in range(phases):
            for (w, h) in ((4, 4), (2, 2), (8, 4), (16, 16)):
                for last in (False, True):
                    got = ctx.filter_hor(comp, src, 8, 8, w, h, frac, last)
                    want = orc.filter(comp, 0, 10, src, 8, 8, w, h, frac, True, last)
                    assert np.array_equal(got, want), (comp, frac, w, h, last)
                for first in (False, True):
                    for last in (False, True):
                        s = src if first else (src.astype(np.int32) * 16 - 8192).astype(np.int16)
                        got = ctx.filter_ver(comp, s, 8, 8, w, h, frac, first, last)
                        want = orc.filter(comp, 1, 10, s, 8, 8, w, h, frac, first, last)
                        assert np.array_equal(got, want), (comp, frac, w, h, first, last)


def test_error_paths():
    cfg = W.CONFIGS["C1"]
    params = mm360.seq_params(cfg.width, cfg.height, W.MPA3 + (mm360.GEODESIC_CAMPOSE,))
    pus = W.pu_list(cfg)
    with mm360.MMContext(params) as ctx:
        dy = torch.zeros((cfg.height, cfg.width), dtype=torch.int16, device="cuda")
        dc = torch.zeros((cfg.height // 2, cfg.width // 2), dtype=torch.int16, device="cuda")
        with pytest.raises(mm360.MMError) as e:
            ctx.predict(W.CUR_POC, pus, dy, dc, dc.clone())  # no references uploaded
        assert e.value.code == mm360.MM_ERR_NOREF
        blk = np.array([(0, 0, 16, 16, 16, 16, mm360.GEODESIC_CAMPOSE, 0, 8, 0)], dtype=mm360.BLOCK_DTYPE)
        with pytest.raises(mm360.MMError) as e:
            ctx.reproject(blk)  # no epipole
        assert e.value.code == mm360.MM_ERR_NOEPIPOLE
        for bad_model in (mm360.CLASSIC, mm360.TANGENTIAL):
            blk = np.array([(0, 0, 16, 16, 16, 16, bad_model, 0, 8, 0)], dtype=mm360.BLOCK_DTYPE)
            with pytest.raises(mm360.MMError) as e:
                ctx.reproject(blk)
            assert e.value.code == mm360.MM_ERR_MODEL
        blk = np.array([(250, 0, 16, 16, 16, 16, 1, 0, 8, 0)], dtype=mm360.BLOCK_DTYPE)
        with pytest.raises(mm360.MMError) as e:
            ctx.reproject(blk)  # outside the picture
        assert e.value.code == mm360.MM_ERR_ARG
        blk = np.array([(0, 0, 256, 128, 16, 16, 1, 0, 8, 0)], dtype=mm360.BLOCK_DTYPE)
        with pytest.raises(mm360.MMError) as e:
            ctx.reproject(blk)  # wider than one CTU (JobDev's 8-bit block sizes)
        assert e.value.code == mm360.MM_ERR_ARG


def test_pu_descriptor_guards():
    """Unknown flag bits, nonzero reserved words and MM_PUF_DMVR without mm_set_dmvr are rejected
    (a stale 48-byte layout fails loudly); a clean descriptor still predicts."""
    cfg = W.CONFIGS["C1"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    with mm360.MMContext(params) as ctx:
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, y, cb, cr)
        dst = _planes(cfg)
        for field, val in (("flags", 0x2), ("flags", mm360.PUF_DMVR), ("reserved", 1)):
            bad = pus.copy()
            if field == "reserved":
                bad["reserved"][7, 1] = val
            else:
                bad[field][7] = val
            with pytest.raises(mm360.MMError) as e:
                ctx.predict(W.CUR_POC, bad, *dst)
            assert e.value.code == mm360.MM_ERR_ARG and "PU 7" in str(e.value), (field, str(e.value))
        ctx.predict(W.CUR_POC, pus, *dst)


def _planes(cfg, fill=0):
    dy = torch.full((cfg.height, cfg.width), fill, dtype=torch.int16, device="cuda")
    dcb = torch.full((cfg.height // 2, cfg.width // 2), fill, dtype=torch.int16, device="cuda")
    return dy, dcb, torch.full_like(dcb, fill)


@pytest.mark.parametrize("cfg_name", ["C2", "C3"])
def test_pred_device_resident_list_vs_oracle(cfg_name):
    """mm_pred_device on a PU list already in HBM (device planning) == the oracle, bit-exact."""
    cfg = W.CONFIGS[cfg_name]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=3)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    orc = Oracle(params, EPI)
    want = orc.predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_pus = mm360.pus_to_device(pus)
        dst = _planes(cfg, -7)
        ctx.predict_device(W.CUR_POC, d_pus, *dst)
        assert ctx.status() == (mm360.MM_OK, -1)
    for x, t, name in zip(want, dst, ("y", "cb", "cr")):
        got = t.cpu().numpy()
        assert np.array_equal(got, x), plane_mismatch(name, got, x)


def test_pred_stripes_do_not_change_results():
    """mm_set_stripes: the PU list cut into 1..7 stripes over two streams predicts the same picture
    (== the oracle), and the lowest failing PU is reported whichever stripe holds it (first, a
    middle or the last stripe: every stripe reports into the picture's one status word)."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=7)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_pus = mm360.pus_to_device(pus)
        for stripes in (1, 2, 3, 7):
            ctx.set_stripes(stripes)
            dst = _planes(cfg, -3)
            ctx.predict_device(W.CUR_POC, d_pus, *dst)
            assert ctx.status() == (mm360.MM_OK, -1)
            for x, t, name in zip(want, dst, ("y", "cb", "cr")):
                got = t.cpu().numpy()
                assert np.array_equal(got, x), (stripes, plane_mismatch(name, got, x))
            for k_bad in (3, len(pus) // 2, len(pus) - 5):  # first / middle / last stripe
                bad = pus.copy()
                bad[k_bad]["x"] = 2
                ctx.predict_device(W.CUR_POC, mm360.pus_to_device(bad), *_planes(cfg))
                assert ctx.status() == (mm360.MM_ERR_ARG, k_bad), (stripes, k_bad)
            # a clean picture after a failing one reports OK (the word was reset)
            ctx.predict_device(W.CUR_POC, d_pus, *_planes(cfg))
            assert ctx.status() == (mm360.MM_OK, -1), stripes
        with pytest.raises(mm360.MMError):
            ctx.set_stripes(0)


def test_pred_contexts_in_flight_together():
    """Independent pictures predicted by two contexts at once (INTEGRATION.md 'in flight together'):
    each context on its own stream with plan-ahead off, calls interleaved without synchronisation,
    every output == the oracle (the contexts share no mutable device state).  Context 0 starts with
    a third of its list, so its buffers grow mid-sequence while context 1's pictures are in flight:
    growth frees the old buffers in the growing context's own stream order (DevBuf::ensure)."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    full = [W.pu_list(cfg, frame=f) for f in (7, 8)]
    short = full[0][: len(full[0]) // 3]
    lists = [[short, full[0], full[0]], [full[1]] * 3]  # [context][round]
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    orc = Oracle(params, EPI)
    want = {id(p): orc.predict(W.CUR_POC, p, refs, cfg.width, cfg.height) for p in (short, full[0], full[1])}
    streams = [torch.cuda.Stream() for _ in range(2)]
    with _ctx(params) as c0, _ctx(params) as c1:
        ctxs = [c0, c1]
        for ctx, s in zip(ctxs, streams):
            ctx.set_stream(s.cuda_stream)
            ctx.set_plan_ahead(False)
            for poc, (y, cb, cr) in refs.items():
                ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_lists = {id(p): mm360.pus_to_device(p) for p in (short, full[0], full[1])}
        torch.cuda.synchronize()
        outs = [[_planes(cfg, 0) for _ in range(3)] for _ in range(2)]  # the short list leaves zeros, as the oracle
        for r in range(3):
            for k, ctx in enumerate(ctxs):
                ctx.predict_device(W.CUR_POC, d_lists[id(lists[k][r])], *outs[k][r])
        torch.cuda.synchronize()
        for k, ctx in enumerate(ctxs):
            assert ctx.status() == (mm360.MM_OK, -1)
            for r in range(3):
                for x, t, name in zip(want[id(lists[k][r])], outs[k][r], ("y", "cb", "cr")):
                    got = t.cpu().numpy()
                    assert np.array_equal(got, x), (k, r, plane_mismatch(name, got, x))


def test_growth_and_destroy_do_not_wait_for_other_streams():
    """A context that grows its buffers, synchronises and is destroyed while unrelated work runs on
    another stream (here ~0.3 s of matrix products on a torch stream) never waits for that work:
    its buffers come from the stream-ordered pool and are freed in its own stream's order
    (dev_alloc / dev_free; hipFree would wait for every queue of the device,
    tools/ubench/free_sync.hip).  The picture it predicts == the oracle."""
    import time
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    full = W.pu_list(cfg, frame=7)
    short = full[: len(full) // 4]
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict(W.CUR_POC, full, refs, cfg.width, cfg.height)
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.float32)
    busy = torch.cuda.Stream()

    def run_busy(n):
        with torch.cuda.stream(busy):
            x = a
            for _ in range(n):
                x = torch.mm(x, a) * 1e-3
        return x

    # calibrate the unrelated work (after a warm-up call, which selects the GEMM kernel): ~0.3 s
    run_busy(2)
    busy.synchronize()
    t0 = time.perf_counter()
    run_busy(20)
    busy.synchronize()
    per = (time.perf_counter() - t0) / 20
    n_busy = min(20000, max(20, int(0.3 / max(per, 1e-5))))
    ctx = _ctx(params)
    try:
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_short, d_full = mm360.pus_to_device(short), mm360.pus_to_device(full)
        out = _planes(cfg, 0)
        ctx.predict_device(W.CUR_POC, d_short, *out)
        ctx.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_busy(n_busy)  # queued, ~0.3 s
        ctx.predict_device(W.CUR_POC, d_full, *out)  # grows every plan buffer
        ctx.synchronize()
        t_ctx = time.perf_counter() - t0
        got = [t.cpu().numpy() for t in out]
    finally:
        t1 = time.perf_counter()
        ctx.close()
        t_destroy = time.perf_counter() - t1
    busy.synchronize()
    t_busy = time.perf_counter() - t0
    assert t_busy > 0.2, t_busy
    assert t_ctx < 0.5 * t_busy, (t_ctx, t_busy)
    assert t_destroy < 0.5 * t_busy, (t_destroy, t_busy)
    for name, g, x in zip(("y", "cb", "cr"), got, want):
        assert np.array_equal(g, x), plane_mismatch(name, g, x)


@pytest.mark.parametrize("plan_ahead", [False, True])
def test_pred_device_multi_pictures_vs_oracle(plan_ahead):
    """mm_pred_device_multi: three independent C2 pictures (own current POC, camera-pose epipole,
    PU list and planes) in ONE launch chain == the oracle picture by picture; twice, so plan-ahead
    reuses its slots; then a failing PU in the third picture is reported with its index counted
    through the pictures' lists."""
    from test_multi_picture import _pictures
    cfg = W.CONFIGS["C2"]
    models = tuple(cfg.models) + (mm360.GEODESIC_CAMPOSE,)
    params = mm360.seq_params(cfg.width, cfg.height, models)
    pics, refs, epis = _pictures(cfg, 3)
    for _, pus in pics:
        pus["model"][::7] = mm360.GEODESIC_CAMPOSE
    orc = Oracle(params, epis)
    want = [orc.predict(cur, pus, refs, cfg.width, cfg.height) for cur, pus in pics]
    with _ctx(params, epis) as ctx:
        ctx.set_plan_ahead(plan_ahead)
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_lists = [mm360.pus_to_device(p) for _, p in pics]
        torch.cuda.synchronize()
        for rnd in range(2):
            outs = [_planes(cfg, -3) for _ in pics]
            ctx.predict_device_multi([(cur, d, *o) for (cur, _), d, o in zip(pics, d_lists, outs)])
            assert ctx.status() == (mm360.MM_OK, -1)
            for q, (o, w) in enumerate(zip(outs, want)):
                for name, t, x in zip(("y", "cb", "cr"), o, w):
                    got = t.cpu().numpy()
                    assert np.array_equal(got, x), (rnd, q, plane_mismatch(name, got, x))
        bad = pics[2][1].copy()
        bad["x"][5] = 3  # not 4x4 aligned
        d_bad = mm360.pus_to_device(bad)
        outs = [_planes(cfg, 0) for _ in pics]
        ctx.predict_device_multi([(pics[0][0], d_lists[0], *outs[0]), (pics[1][0], d_lists[1], *outs[1]),
                                  (pics[2][0], d_bad, *outs[2])])
        code, first = ctx.status()
        assert code == mm360.MM_ERR_ARG and first == len(pics[0][1]) + len(pics[1][1]) + 5, (code, first)


def test_pred_plan_ahead_rotating_pictures():
    """mm_set_plan_ahead: three different PU lists predicted back to back (twice round, so each
    plan slot is reused while the other picture's kernels may still run; a smaller list first, so
    the slot buffers grow mid-sequence), every output == the oracle; a failing PU in the last
    call is reported, and switching plan-ahead off and on again keeps the results."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    lists = [W.pu_list(cfg, frame=f) for f in (7, 8, 9)]
    lists.insert(0, lists[0][: len(lists[0]) // 3])
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = [Oracle(params, EPI).predict(W.CUR_POC, p, refs, cfg.width, cfg.height) for p in lists]
    with _ctx(params) as ctx:
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_lists = [mm360.pus_to_device(p) for p in lists]
        torch.cuda.synchronize()
        for mode in (1, 0, 1):
            ctx.set_plan_ahead(bool(mode))
            order = [0, 1, 2, 3, 1, 2, 3]
            outs = [_planes(cfg, 0) for _ in order]  # the short list leaves samples at 0, as the oracle
            for k, o in zip(order, outs):
                ctx.predict_device(W.CUR_POC, d_lists[k], *o)
            assert ctx.status() == (mm360.MM_OK, -1)
            for k, o in zip(order, outs):
                for x, t, name in zip(want[k], o, ("y", "cb", "cr")):
                    got = t.cpu().numpy()
                    assert np.array_equal(got, x), (mode, k, plane_mismatch(name, got, x))
        bad = lists[2].copy()
        k_bad = len(bad) // 2
        bad[k_bad]["x"] = 2
        d_bad = mm360.pus_to_device(bad)
        torch.cuda.synchronize()
        ctx.predict_device(W.CUR_POC, d_lists[1], *_planes(cfg))
        ctx.predict_device(W.CUR_POC, d_bad, *_planes(cfg))
        assert ctx.status() == (mm360.MM_ERR_ARG, k_bad)
        ctx.predict_device(W.CUR_POC, d_lists[3], *_planes(cfg))
        assert ctx.status() == (mm360.MM_OK, -1)


def test_pred_plan_ahead_lists_written_on_the_context_stream():
    """Plan-ahead contract (mm360.h mm_set_plan_ahead): the planning of call N waits for the
    interpolation of call N-2, so a device list written by work on the context stream is ordered
    before call N's planning when that work was enqueued before call N-2 was issued.  Each list is
    copied into its device buffer (hipMemcpyAsync on the context stream, from pinned host memory)
    just before the call two ahead of it; a buffer is rewritten only after its previous picture's
    call completed.  Every output == the oracle."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    lists = [W.pu_list(cfg, frame=f) for f in (11, 12, 13, 14, 15)]
    n_max = max(len(p) for p in lists)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    orc = Oracle(params, EPI)
    want = [orc.predict(W.CUR_POC, p, refs, cfg.width, cfg.height) for p in lists]
    stream = torch.cuda.current_stream()
    with _ctx(params) as ctx:
        ctx.set_stream(stream.cuda_stream)
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        ctx.set_plan_ahead(True)
        host = [torch.from_numpy(p.view(np.uint8)).pin_memory() for p in lists]
        bufs = [torch.zeros(n_max * mm360.PU_DTYPE.itemsize, dtype=torch.uint8, device="cuda") for _ in range(3)]
        outs = [_planes(cfg, -1) for _ in lists]
        torch.cuda.synchronize()
        order = list(range(len(lists))) * 2
        for i, k in enumerate(order):
            if i == 0:  # lists 0 and 1 ahead of the first call
                for j in (0, 1):
                    bufs[j][: host[order[j]].numel()].copy_(host[order[j]], non_blocking=True)
            if i + 2 < len(order):  # list i + 2 now: before call i, two calls ahead of its own
                b = bufs[(i + 2) % 3]
                b[: host[order[i + 2]].numel()].copy_(host[order[i + 2]], non_blocking=True)
            buf = bufs[i % 3]
            ctx.predict_device(W.CUR_POC, buf[: host[k].numel()].view(torch.int32), *outs[k])
        assert ctx.status() == (mm360.MM_OK, -1)
        for k, o in enumerate(outs):
            for x, t, name in zip(want[k], o, ("y", "cb", "cr")):
                got = t.cpu().numpy()
                assert np.array_equal(got, x), (k, plane_mismatch(name, got, x))


def test_pred_plan_ahead_interleaved_call_kinds():
    """Plan-ahead stays on while other call kinds use the plan slots in between: a 2-stripe call
    (both slots, context and auxiliary streams), a per-list call (mm_pred_list) and a host-list
    call (mm_pred), each followed by plan-ahead device calls that reuse the slots.  The slot gates
    (events bound to the k_mc_dev of each slot's last user) must order every reuse; every output
    == the oracle."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    lists = [W.pu_list(cfg, frame=f) for f in (11, 12, 13)]
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    orc = Oracle(params, EPI)
    want = [orc.predict(W.CUR_POC, p, refs, cfg.width, cfg.height) for p in lists]
    l0 = lists[0][lists[0]["ref_poc"][:, 0] >= 0]
    want_l0 = orc.predict_list(W.CUR_POC, l0, 0, False, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        _upload(ctx, refs)
        d_lists = [mm360.pus_to_device(p) for p in lists]
        torch.cuda.synchronize()
        ctx.set_plan_ahead(True)
        checks = []

        def dev(k):
            o = _planes(cfg)
            ctx.predict_device(W.CUR_POC, d_lists[k], *o)
            checks.append((o, want[k], f"device list {k}"))

        dev(0)
        dev(1)
        ctx.set_stripes(2)
        o = _planes(cfg)
        ctx.predict(W.CUR_POC, lists[2], *o)  # host list, two stripes on both streams
        checks.append((o, want[2], "2-stripe host call"))
        ctx.set_stripes(1)
        dev(1)
        dev(2)
        o = _planes(cfg)
        ctx.predict_list(W.CUR_POC, l0, 0, False, *o)
        checks.append((o, want_l0, "per-list call"))
        dev(0)
        dev(2)
        dev(1)
        assert ctx.status() == (mm360.MM_OK, -1)
        torch.cuda.synchronize()
        for o, w, what in checks:
            for x, t, name in zip(w, o, ("y", "cb", "cr")):
                got = t.cpu().numpy()
                assert np.array_equal(got, x), (what, plane_mismatch(name, got, x))


def test_c4_stripe_sublists_into_packed_picture():
    """C4 on one GPU: each of the 8 CTU-row stripe sub-lists of the C3 PU list (one per rank of an
    8-GPU node) is predicted through the C-ABI straight into its segment of the stripe-major packed
    picture (the buffer the one all-gather moves); the unpacked picture == the oracle's full C3
    prediction.  Also 3 unequal stripes."""
    from mm360 import parallel as P
    cfg = W.CONFIGS["C3"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=0)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        _upload(ctx, refs)
        for world in (8, 3):
            lay = P.StripeLayout(cfg.width, cfg.height, world)
            buf = torch.full((lay.total,), -11, dtype=torch.int16, device="cuda")
            for rank in range(world):
                mine = P.shard_pus(pus, cfg.height, world, rank)
                ctx.prepare(W.CUR_POC, mine)
                ctx.run_raw(*lay.dst_pointers(buf.data_ptr(), rank))
                ctx.synchronize()
            got = lay.unpack(buf.cpu().numpy())
            for name, g, w in zip(("y", "cb", "cr"), got, want):
                assert np.array_equal(g, w), (world, plane_mismatch(name, g, w))


def _upload(ctx, refs):
    for poc, (y, cb, cr) in refs.items():
        ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())


def test_pred_bcw_every_index_vs_oracle():
    """Bi PUs with every BCW index (addWeightedAvg, Buffer.cpp:398-424, chosen at
    InterPrediction.cpp:1596-1600) at C2 == the oracle; an index outside 0..4 is rejected."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=4)
    pus["bcw_idx"] = np.random.default_rng(4).integers(0, 5, len(pus))
    bi = (pus["ref_poc"] >= 0).all(axis=1)
    assert set(pus["bcw_idx"][bi].tolist()) == {0, 1, 2, 3, 4}
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        got = _gpu_predict(ctx, params, W.CUR_POC, pus, refs)
        bad = pus.copy()
        k = int(np.nonzero(bi)[0][10])
        bad[k]["bcw_idx"] = 5
        dst = _planes(cfg)
        ctx.predict_device(W.CUR_POC, mm360.pus_to_device(bad), *dst)
        assert ctx.status() == (mm360.MM_ERR_ARG, k)
    for name, g, w in zip(("y", "cb", "cr"), got, want):
        assert np.array_equal(g, w), plane_mismatch(name, g, w)


@pytest.mark.parametrize("list_,hp", [(0, 1), (1, 1), (0, 0), (1, 0)])
def test_pred_list_vs_oracle(list_, hp):
    """mm_pred_list == xPredInterBlkMM 1:1 per list (InterPrediction.h:151-154): the 14-bit
    bi=true intermediate (hp) or the clipped prediction of one list, at C2, bit-exact vs the
    oracle; per-component calls (a NULL plane) predict the other component alone."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=5)
    pus = pus[pus["ref_poc"][:, list_] >= 0]
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict_list(W.CUR_POC, pus, list_, hp, refs, cfg.width, cfg.height)
    with _ctx(params) as ctx:
        _upload(ctx, refs)
        dst = _planes(cfg)
        ctx.predict_list(W.CUR_POC, pus, list_, hp, *dst)
        for name, t, w in zip(("y", "cb", "cr"), dst, want):
            got = t.cpu().numpy()
            assert np.array_equal(got, w), plane_mismatch(name, got, w)
        luma_only = _planes(cfg)
        ctx.predict_list(W.CUR_POC, pus, list_, hp, luma_only[0])
        assert np.array_equal(luma_only[0].cpu().numpy(), want[0])
        chroma_only = _planes(cfg)  # no luma plane at all: only chroma is predicted
        ctx.predict_list(W.CUR_POC, pus, list_, hp, None, chroma_only[1], chroma_only[2])
        assert np.array_equal(chroma_only[1].cpu().numpy(), want[1])
        assert np.array_equal(chroma_only[2].cpu().numpy(), want[2])
        other = W.pu_list(cfg, frame=5)
        miss = np.nonzero(other["ref_poc"][:, list_] < 0)[0]
        with pytest.raises(mm360.MMError):  # a PU without the requested list
            ctx.predict_list(W.CUR_POC, other[: miss[0] + 1], list_, hp, *_planes(cfg))


def test_device_validation_reports_lowest_failing_pu():
    """Device-side CHECKs: a bad PU is skipped and reported (lowest index first); the rest of the
    picture is still predicted exactly."""
    cfg = W.CONFIGS["C1"]
    params = mm360.seq_params(cfg.width, cfg.height, W.MPA3 + (mm360.GEODESIC_CAMPOSE,))
    pus = W.pu_list(cfg)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    orc = Oracle(params, EPI)
    want = orc.predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)

    def broken(k, field, value, ctx_epi=True):
        bad = pus.copy()
        if field == "x":
            bad[k]["x"] = value
        elif field == "model":
            bad[k]["model"][0] = value
            bad[k]["ref_poc"][0] = 0
        elif field == "ref_poc":
            bad[k]["ref_poc"][0] = value
            bad[k]["model"][0] = 1
        elif field == "nolist":
            bad[k]["ref_poc"][:] = -1
        return bad

    cases = [(37, "x", 2, mm360.MM_ERR_ARG), (11, "model", mm360.CLASSIC, mm360.MM_ERR_MODEL),
             (5, "model", mm360.TANGENTIAL, mm360.MM_ERR_MODEL), (20, "ref_poc", 99, mm360.MM_ERR_NOREF),
             (3, "nolist", 0, mm360.MM_ERR_ARG)]
    with _ctx(params) as ctx:
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        for k, field, value, code in cases:
            bad = broken(k, field, value)
            bad2 = broken(k + 40, field, value) if k + 40 < len(pus) else bad
            both = bad.copy()
            both[k + 40:k + 41] = bad2[k + 40:k + 41]
            dst = _planes(cfg)
            ctx.predict_device(W.CUR_POC, mm360.pus_to_device(both), *dst)
            rc, first = ctx.status()
            assert (rc, first) == (code, k), (field, rc, first)
            # every PU except the broken ones is predicted exactly
            got = dst[0].cpu().numpy()
            mask = np.ones_like(got, dtype=bool)
            for j in (k, k + 40):
                u = pus[j]
                mask[u["y"]:u["y"] + u["h"], u["x"]:u["x"] + u["w"]] = False
            assert np.array_equal(got[mask], want[0][mask])
        # GED camera pose without an epipole for (8, 0)
        g = pus.copy()
        g[9]["model"][:] = mm360.GEODESIC_CAMPOSE
    with mm360.MMContext(params) as ctx:  # no epipoles set
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, y, cb, cr)
        dst = _planes(cfg)
        ctx.predict_device(W.CUR_POC, mm360.pus_to_device(g), *dst)
        assert ctx.status() == (mm360.MM_ERR_NOEPIPOLE, 9)
        # over capacity: the same list three times covers the picture 3x
        ctx.predict_device(W.CUR_POC, mm360.pus_to_device(np.concatenate([pus] * 3)), *dst)
        rc, _ = ctx.status()
        assert rc == mm360.MM_ERR_ARG
        # empty list is a no-op
        ctx.predict_device(W.CUR_POC, mm360.pus_to_device(pus[:0]), *dst)
        assert ctx.status() == (mm360.MM_OK, -1)


def test_cpp_shim_example_on_gpu():
    """C++ host shim end to end on the GPU: MVReprojection-shaped call, host and device PU lists
    predict identical pictures."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vvc-extension-mm_amd", "lib",
                       "example_decode")
    assert os.path.exists(exe), "build with __graft_entry__.build() / make -C vvc-extension-mm_amd example"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


ME_ALL = W.MPA3 + (mm360.TANGENTIAL, mm360.THREE_D_TRANSLATIONAL, mm360.ROTATIONAL, mm360.GEODESIC_CAMPOSE)


def _me_ctx(params, w, h):
    ctx = _ctx(params)
    for poc in W.REF_POCS:
        y, cb, cr = W.ref_planes(w, h, poc)
        ctx.upload_ref(poc, y, cb, cr)
    ctx.upload_org(W.CUR_POC, W.org_plane(w, h))
    return ctx


@pytest.mark.parametrize("step,sub_shift", [(16, 0), (4, 1)])
def test_sad_window_vs_oracle(step, sub_shift):
    """mm_sad_window (encoder candidate SADs) == the oracle, bit-exact, all models, edge blocks."""
    from test_me import _case
    w, h = 256, 128
    params = mm360.seq_params(w, h, ME_ALL)
    blocks, refs, org = _case(w, h, ME_ALL, 60, seed=3 + step, sub_shift=sub_shift)
    want = Oracle(params, EPI).sad_window(W.CUR_POC, blocks, 3, step, refs, org)
    with _me_ctx(params, w, h) as ctx:
        got = ctx.sad_window(W.CUR_POC, blocks, 3, step).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]


def test_sad_window_c5_full_window_vs_oracle():
    """C5 geometry (2048x1024, all models, 33x33 integer window) on a seeded subset of the PU
    grid: the GPU equals the oracle (96 blocks x 1089 candidates, ~2 s of oracle time)."""
    w, h = 2048, 1024
    params = mm360.seq_params(w, h, ME_ALL)
    blocks = W.me_blocks(w, h, ME_ALL, grid=16, seed=11, max_blocks=96)
    refs = {poc: W.ref_planes(w, h, poc)[0] for poc in W.REF_POCS}
    org = W.org_plane(w, h)
    want = Oracle(params, EPI).sad_window(W.CUR_POC, blocks, 16, 16, refs, org)
    with _me_ctx(params, w, h) as ctx:
        got = ctx.sad_window(W.CUR_POC, blocks, 16, 16).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    # the search picks the same best candidate per block
    assert np.array_equal(got.argmin(axis=1), want.argmin(axis=1))


TZ_SQUARE = [(-1, -1), (0, -1), (1, -1), (-1, 0), (1, 0), (-1, 1), (0, 1), (1, 1)]  # InterSearch.cpp:492-526
TZ_DIAMOND = [(0, -2), (-1, -1), (1, -1), (-2, 0), (2, 0), (-1, 1), (1, 1), (0, 2)]


@pytest.mark.parametrize("pattern", ["square1", "square8", "diamond4", "refine_half", "star32", "ragged"])
def test_sad_pattern_vs_oracle(pattern):
    """mm_sad_pattern (one call per TZ / refinement step, the block's setup and each sub-block's
    model head shared by its k candidates) == the oracle's range-0 SAD of every (block, offset),
    bit-exact, all models, edge blocks, 16x16 and ragged block sizes."""
    from test_me import _case
    w, h = 256, 128
    params = mm360.seq_params(w, h, ME_ALL)
    if pattern.startswith("square"):
        d = int(pattern[6:])
        off = [(16 * d * x, 16 * d * y) for x, y in TZ_SQUARE]
    elif pattern == "diamond4":
        off = [(32 * x, 32 * y) for x, y in TZ_DIAMOND]
    elif pattern == "refine_half":  # xPatternRefinementProjected: 9 points, half-pel
        off = [(8 * x, 8 * y) for y in (-1, 0, 1) for x in (-1, 0, 1)]
    elif pattern == "star32":
        off = [(16 * d * x, 16 * d * y) for d in (1, 2, 4, 8, 16, 32) for x, y in TZ_DIAMOND]
    else:
        off = [(5, -3), (0, 0), (-37, 12), (64, 64), (-1, 100), (3, 3), (-128, -7)]
    blocks, refs, org = _case(w, h, ME_ALL, 40, seed=21 + len(off), sub_shift=1 if pattern == "ragged" else 0)
    if pattern == "ragged":
        blocks = blocks.copy()
        blocks["w"] = np.minimum(blocks["w"], 8)
    k = len(off)
    rep = np.repeat(blocks, k)
    o = np.tile(np.asarray(off, np.int32), (len(blocks), 1))
    rep["mv_hor"] += o[:, 0]
    rep["mv_ver"] += o[:, 1]
    want = Oracle(params, EPI).sad_window(W.CUR_POC, rep, 0, 16, refs, org).reshape(len(blocks), k)
    with _me_ctx(params, w, h) as ctx:
        got = ctx.sad_pattern(W.CUR_POC, blocks, off).cpu().numpy().view(np.uint32)
        got0 = ctx.sad_window(W.CUR_POC, rep, 0, 16).cpu().numpy().view(np.uint32).reshape(len(blocks), k)
        with pytest.raises(mm360.MMError):
            ctx.sad_pattern(W.CUR_POC, blocks, off + [off[0]])  # repeated offset
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    assert np.array_equal(got0, want)


@pytest.mark.parametrize("step", [16, 4])
def test_sad_pattern_grid_equals_window_at_c5_size(step):
    """At the C5 geometry (2048x1024, every model, the whole 16x16 PU grid = 57,344 blocks): the
    pattern entry point with the 5x5 grid pattern equals the range-2 window (same candidate order),
    and the TZ square at distance 2 equals that window's corner / edge-centre candidates."""
    w, h = 2048, 1024
    params = mm360.seq_params(w, h, ME_ALL)
    blocks = W.me_blocks(w, h, ME_ALL, grid=16, seed=13)
    grid = [(step * i, step * j) for j in range(-2, 3) for i in range(-2, 3)]
    sq = [(2 * step * x, 2 * step * y) for x, y in TZ_SQUARE]
    with _me_ctx(params, w, h) as ctx:
        win = ctx.sad_window(W.CUR_POC, blocks, 2, step).cpu().numpy().view(np.uint32)
        pat = ctx.sad_pattern(W.CUR_POC, blocks, grid).cpu().numpy().view(np.uint32)
        sqr = ctx.sad_pattern(W.CUR_POC, blocks, sq).cpu().numpy().view(np.uint32)
    assert np.array_equal(pat, win)
    idx = [(y + 2) * 5 + (x + 2) for x, y in [(2 * a, 2 * b) for a, b in TZ_SQUARE]]
    assert np.array_equal(sqr, win[:, idx])


@pytest.mark.parametrize("w,h", [(256, 128), (1024, 512)])
def test_pred_dmvr_vs_oracle(w, h):
    """MM-DMVR on the GPU == the oracle: refined per-sub-PU deltas and predicted planes."""
    models = ME_ALL
    cfg = W.Config("T", w, h, tuple(models), 1, "test")
    params = mm360.seq_params(w, h, models)
    pus = W.dmvr_pu_list(cfg, frame=2)
    refs = {poc: W.ref_planes(w, h, poc) for poc in W.REF_POCS}
    want, want_mvd = Oracle(params, EPI).predict_dmvr(W.CUR_POC, pus, refs, w, h)
    with _ctx(params) as ctx:
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, y, cb, cr)
        dst = _planes(cfg)
        mvd = ctx.predict_dmvr(W.CUR_POC, pus, *dst)
    assert np.array_equal(mvd, want_mvd), np.argwhere(mvd != want_mvd)[:5]
    for name, t, x in zip(("y", "cb", "cr"), dst, want):
        got = t.cpu().numpy()
        assert np.array_equal(got, x), plane_mismatch(name, got, x)


def test_pred_dmvr_zero_mv_offsets_vs_oracle():
    """MM-DMVR where search offsets land on a zero MV (the models' identity setups, block_setup's
    zero-MV shortcut) and where the merge MV itself is zero (the centre setup is the identity, the
    offsets' setups still need the centre terms): the search derives each offset's setup from the
    sub-PU's centre terms (mm_models.h setup_from_centre); deltas and planes == the oracle's full
    block setups, every model, 16x16 and 16x8 / 8x16 sub-PUs."""
    w, h = 512, 256
    models = ME_ALL
    cfg = W.Config("T", w, h, tuple(models), 1, "test")
    params = mm360.seq_params(w, h, models)
    pus = dmvr_zero_mv_pus(cfg, models)
    assert len(pus) >= 4 * len(models)  # every (aim, model) pair
    refs = {poc: W.ref_planes(w, h, poc) for poc in W.REF_POCS}
    want, want_mvd = Oracle(params, EPI).predict_dmvr(W.CUR_POC, pus, refs, w, h)
    with _ctx(params) as ctx:
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, y, cb, cr)
        dst = _planes(cfg)
        mvd = ctx.predict_dmvr(W.CUR_POC, pus, *dst)
    assert np.array_equal(mvd, want_mvd), np.argwhere(mvd != want_mvd)[:5]
    for name, t, x in zip(("y", "cb", "cr"), dst, want):
        got = t.cpu().numpy()
        assert np.array_equal(got, x), plane_mismatch(name, got, x)


def test_pred_dmvr_every_branch_vs_oracle():
    """MM-DMVR on the GPU over the branch fixture (tests/golden/dmvr_branches.npz): early exits,
    border bests, division and half-pel tie cases on both axes and sides, a zero denominator
    (InterPrediction.cpp:2516-2531, :2162-2163, :1996-2048).  mm_pred_dmvr's deltas == the
    fixture's (the oracle's), its planes == the oracle's; then the same PUs with every other one
    flagged MM_PUF_DMVR in ONE mm_pred_device picture (plan-ahead on) == predict_mixed."""
    from oracle.oracle import dmvr_branches
    from test_dmvr import branch_fixture
    params, w, h, fams = branch_fixture()
    cfg = W.Config("T", w, h, tuple(int(m) for m in W.ALL_MODELS), 1, "test")
    orc = Oracle(params, EPI)
    tot = {}
    for fam, refs, pus, mvd, tr in fams:
        for k, v in dmvr_branches(tr).items():
            tot[k] = tot.get(k, 0) + v
        want, _ = orc.predict_dmvr(W.CUR_POC, pus, refs, w, h)
        mixed = pus.copy()
        mixed["flags"][::2] |= mm360.PUF_DMVR
        want_mixed = orc.predict_mixed(W.CUR_POC, mixed, refs, w, h)
        with _ctx(params) as ctx:
            for poc, (y, cb, cr) in refs.items():
                ctx.upload_ref(poc, y, cb, cr)
            dst = _planes(cfg)
            got_mvd = ctx.predict_dmvr(W.CUR_POC, pus, *dst)
            assert np.array_equal(got_mvd, mvd), (fam, np.argwhere(got_mvd != mvd)[:5])
            for name, t, x in zip(("y", "cb", "cr"), dst, want):
                got = t.cpu().numpy()
                assert np.array_equal(got, x), plane_mismatch(f"{fam} {name}", got, x)
            ctx.set_dmvr(True)
            ctx.set_plan_ahead(True)
            d_list = mm360.pus_to_device(mixed)
            out = _planes(cfg)  # 16x8 / 8x16 PUs leave part of their cell unpredicted (zero in both)
            torch.cuda.synchronize()
            ctx.predict_device(W.CUR_POC, d_list, *out)
            ctx.synchronize()
            for name, t, x in zip(("y", "cb", "cr"), out, want_mixed):
                got = t.cpu().numpy()
                assert np.array_equal(got, x), plane_mismatch(f"{fam} mixed {name}", got, x)
    for k in ("early_exit", "border_best", "h_tie_minus", "h_tie_plus", "v_tie_minus", "v_tie_plus", "v_den0"):
        assert tot[k] > 0, (k, tot)


@pytest.mark.parametrize("n", [20000, 40000])
def test_mvp_convert_vs_oracle(n):
    """Batched MM-MVP on the GPU == the oracle for every model pair (incl. CLASSIC), both epipoles;
    40 K queries take the model-sorted path (MVP_SORT_MIN = 32768), where the status of bad
    queries must still name the lowest failing input index."""
    from test_mvp import ALL as MVP_ALL, EPI2
    params = mm360.seq_params(2048, 1024, MVP_ALL)
    q = W.mvp_queries(2048, 1024, MVP_ALL, n, seed=21)
    want = Oracle(params, EPI2).mvp(q)
    with _ctx(params, EPI2) as ctx:
        got = ctx.mvp_convert(q)
        # device-resident form: same results, stream-ordered, no host buffers
        d_q = mm360.queries_to_device(q)
        d_out = torch.full((len(q), 2), -7, dtype=torch.int32, device="cuda")
        ctx.mvp_convert_device(d_q, d_out)
        ctx.mvp_status()
        got_dev = d_out.cpu().numpy()
    assert np.array_equal(got, want), np.argwhere((got != want).any(axis=1))[:5]
    assert np.array_equal(got_dev, want), np.argwhere((got_dev != want).any(axis=1))[:5]
    if n >= 32768:
        bad = q.copy()
        bad["model_desired"][n - 5] = 99  # sorted into key 0, ahead of most queries
        bad["shift_hor"][n - 900] = 9
        with _ctx(params, EPI2) as ctx:
            d_out = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
            ctx.mvp_convert_device(mm360.queries_to_device(bad), d_out)
            with pytest.raises(mm360.MMError) as e:
                ctx.mvp_status()
            assert e.value.code == mm360.MM_ERR_ARG and f"MVP query {n - 900}:" in str(e.value), str(e.value)
            ok = np.ones(n, bool)
            ok[[n - 5, n - 900]] = False
            assert np.array_equal(d_out.cpu().numpy()[ok], want[ok])


def test_mvp_device_errors_and_epipole_refresh():
    """mm_mvp_convert_device: the lowest failing query's code is deferred to mvp_status; the device
    epipole table follows later mm_set_epipole calls."""
    from test_mvp import ALL as MVP_ALL, EPI2
    params = mm360.seq_params(256, 128, MVP_ALL)
    q = W.mvp_queries(256, 128, MVP_ALL, 700, seed=4)
    q["model_orig"][300:] = mm360.GEODESIC_CAMPOSE
    q["mv_hor"][300:] |= 1
    with _ctx(params, []) as ctx:  # no epipoles yet
        d_q = mm360.queries_to_device(q)
        d_out = torch.zeros((len(q), 2), dtype=torch.int32, device="cuda")
        ctx.mvp_convert_device(d_q, d_out)
        with pytest.raises(mm360.MMError) as e:
            ctx.mvp_status()
        assert e.value.code == mm360.MM_ERR_NOEPIPOLE
        cam = (q["model_orig"] == mm360.GEODESIC_CAMPOSE) | (q["model_desired"] == mm360.GEODESIC_CAMPOSE)
        first = int(np.argmax(cam & ~((q["mv_hor"] == 0) & (q["mv_ver"] == 0))))
        assert f"MVP query {first}:" in str(e.value), str(e.value)
        for (cur, ref, qq) in EPI2:
            ctx.set_epipole(cur, ref, qq)
        ctx.mvp_convert_device(d_q, d_out)
        ctx.mvp_status()
        want = Oracle(params, EPI2).mvp(q)
        assert np.array_equal(d_out.cpu().numpy(), want)
        bad = q.copy()
        bad["shift_hor"][123] = 9
        bad["model_desired"][456] = 99
        ctx.mvp_convert_device(mm360.queries_to_device(bad), d_out)
        with pytest.raises(mm360.MMError) as e:
            ctx.synchronize()
        assert e.value.code == mm360.MM_ERR_ARG and "MVP query 123" in str(e.value)


def test_mvp_device_error_in_later_waves_is_reported():
    """A failing query only in waves 1-3 of its 256-query workgroup (lanes 64-255) still reaches the
    status word: k_mvp_dev zeroes its workgroup's status before any wave records a failure.  Many
    workgroups, each with its one bad query at a different lane >= 64; repeated launches."""
    from test_mvp import ALL as MVP_ALL, EPI2
    params = mm360.seq_params(256, 128, MVP_ALL)
    q = W.mvp_queries(256, 128, MVP_ALL, 256 * 64, seed=9)
    rng = np.random.default_rng(3)
    lanes = rng.integers(64, 256, size=64)
    bad = q.copy()
    for b, lane in enumerate(lanes):
        bad["shift_hor"][256 * b + int(lane)] = 9  # invalid shift: MM_ERR_ARG for that query only
    first = int(256 * 0 + lanes[0])
    with _ctx(params, EPI2) as ctx:
        d_q = mm360.queries_to_device(bad)
        d_out = torch.zeros((len(q), 2), dtype=torch.int32, device="cuda")
        for _ in range(20):
            ctx.mvp_convert_device(d_q, d_out)
            with pytest.raises(mm360.MMError) as e:
                ctx.mvp_status()
            assert e.value.code == mm360.MM_ERR_ARG and f"MVP query {first}:" in str(e.value), str(e.value)
        # the valid queries are still converted
        ok = np.ones(len(q), dtype=bool)
        ok[[256 * b + int(l) for b, l in enumerate(lanes)]] = False
        want = Oracle(params, EPI2).mvp(q[ok])
        assert np.array_equal(d_out.cpu().numpy()[ok], want)


def test_mvp_c3_size_vs_oracle():
    """MM-MVP at the C3 size (6144x3072, all models of the C3 config, the bench's 2 queries per PU
    of a C3 picture: the model-sorted device path) == the oracle, and the host per-query form
    (mm_mvp_convert_host, used at the spatial candidates) gives the same MVs."""
    from test_mvp import EPI2
    cfg = W.CONFIGS["C3"]
    models = tuple(cfg.models) + (mm360.GEODESIC_CAMPOSE,)
    params = mm360.seq_params(cfg.width, cfg.height, models)
    q = W.mvp_queries(cfg.width, cfg.height, models, 2 * 77947, seed=5)
    want = Oracle(params, EPI2).mvp(q)
    with _ctx(params, EPI2) as ctx:
        d_out = torch.full((len(q), 2), -7, dtype=torch.int32, device="cuda")
        ctx.mvp_convert_device(mm360.queries_to_device(q), d_out)
        ctx.mvp_status()
        got = d_out.cpu().numpy()
        host = mm360.mvp_convert_host(params, q[:20000], ctx.epipole_list())
    assert np.array_equal(got, want), np.argwhere((got != want).any(axis=1))[:5]
    assert np.array_equal(host, want[:20000])


def test_mvp_epipole_refresh_behind_side_stream_conversions():
    """Conversions on their own MVP stream, then EpipoleList changes that sort new entries BEFORE the
    existing ones (an earlier POC, random-access order) with no synchronisation in between: every
    batch converts against the list as it was when the batch was issued.  Three versions, so the
    first table is reused by the third refresh (which must wait for the first batch)."""
    from test_mvp import ALL as MVP_ALL
    params = mm360.seq_params(2048, 1024, MVP_ALL)
    q = W.mvp_queries(2048, 1024, MVP_ALL, 120000, seed=8)
    cam = (q["model_orig"] == mm360.GEODESIC_CAMPOSE) | (q["model_desired"] == mm360.GEODESIC_CAMPOSE)
    q["cur_poc_orig"][cam] = W.CUR_POC
    q["cur_poc_desired"][cam] = W.CUR_POC
    versions = [[(W.CUR_POC, -1, (0, 11863283, 11863283))],
                [(W.CUR_POC, -1, (0, 11863283, 11863283)), (2, 0, (1 << 24, 0, 0))],
                [(W.CUR_POC, -1, (0, 11863283, 11863283)), (2, 0, (1 << 24, 0, 0)), (W.CUR_POC, 0, (0, 1 << 24, 0))]]
    wants = [Oracle(params, v).mvp(q) for v in versions]
    side = torch.cuda.Stream()
    with _ctx(params, versions[0]) as ctx:
        ctx.set_mvp_stream(side.cuda_stream)
        d_q = mm360.queries_to_device(q)
        torch.cuda.synchronize()
        outs = [torch.zeros((len(q), 2), dtype=torch.int32, device="cuda") for _ in versions]
        for k, v in enumerate(versions):
            if k:
                cur, ref, qq = v[-1]
                ctx.set_epipole(cur, ref, qq)  # sorts before (W.CUR_POC, -1)
            ctx.mvp_convert_device(d_q, outs[k])
        ctx.mvp_status()
        for k in range(len(versions)):
            got = outs[k].cpu().numpy()
            assert np.array_equal(got, wants[k]), (k, np.argwhere((got != wants[k]).any(axis=1))[:5])
    assert not np.array_equal(wants[0], wants[2])  # the versions convert differently


def test_mvp_status_sticky_over_calls():
    """A failing conversion followed by a clean one, with no status read in between: the next
    mm_mvp_status still reports the failure (the status word accumulates until it is read)."""
    from test_mvp import ALL as MVP_ALL, EPI2
    params = mm360.seq_params(256, 128, MVP_ALL)
    q = W.mvp_queries(256, 128, MVP_ALL, 3000, seed=12)
    bad = q.copy()
    bad["shift_ver"][1234] = 9
    with _ctx(params, EPI2) as ctx:
        d_out = torch.zeros((len(q), 2), dtype=torch.int32, device="cuda")
        ctx.mvp_convert_device(mm360.queries_to_device(bad), d_out)
        ctx.mvp_convert_device(mm360.queries_to_device(q), d_out)
        ctx.mvp_convert_device(mm360.queries_to_device(q), d_out)
        with pytest.raises(mm360.MMError) as e:
            ctx.mvp_status()
        assert e.value.code == mm360.MM_ERR_ARG and "MVP query 1234" in str(e.value), str(e.value)
        ctx.mvp_convert_device(mm360.queries_to_device(q), d_out)
        ctx.mvp_status()  # read and cleared: clean again
        assert np.array_equal(d_out.cpu().numpy(), Oracle(params, EPI2).mvp(q))


@pytest.mark.parametrize("plan_ahead", [False, True])
def test_pred_device_mixed_dmvr_picture_vs_oracle(plan_ahead):
    """A full C2 picture mixing MM_PUF_DMVR PUs (30 % of the DMVR-eligible bi leaves) with ordinary
    PUs, predicted by ONE asynchronous mm_pred_device launch sequence with mm_set_dmvr on (search,
    decision and refined prediction inside the picture's plan; InterPrediction.cpp:591-592,
    2442-2634), == the oracle's predict + predict_dmvr.  Twice in a row, with and without
    plan-ahead (the search runs on the context stream after the planning on the auxiliary one)."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    lists = [W.pu_list(cfg, frame=f, dmvr_share=0.3) for f in (0, 1)]
    orc = Oracle(params, EPI)
    with _ctx(params) as ctx:
        ctx.set_dmvr(True)
        ctx.set_plan_ahead(plan_ahead)
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_lists = [mm360.pus_to_device(p) for p in lists]
        outs = [_planes(cfg, fill=-1) for _ in lists]
        torch.cuda.synchronize()  # plan-ahead contract: the lists are complete before the calls
        for d, o in zip(d_lists, outs):
            ctx.predict_device(W.CUR_POC, d, *o)
        ctx.synchronize()
        got = [[t.cpu().numpy() for t in o] for o in outs]
    for pus, g in zip(lists, got):
        assert W.dmvr_flagged(pus).sum() > 100
        want = orc.predict_mixed(W.CUR_POC, pus, refs, cfg.width, cfg.height)
        for name, a, b in zip(("y", "cb", "cr"), g, want):
            assert np.array_equal(a, b), plane_mismatch(name, a, b)


@pytest.mark.parametrize("plan_ahead", [False, True])
def test_pred_device_multi_with_dmvr_vs_oracle(plan_ahead):
    """mm_pred_device_multi with mm_set_dmvr on: three C2 pictures, each with its own current POC,
    references and camera-pose epipole, mixing MM_PUF_DMVR PUs (30 % of the DMVR-eligible bi leaves)
    with ordinary PUs in ONE launch chain -- every picture's sub-PUs searched, decided and predicted
    into its own planes -- == the oracle's predict_mixed picture by picture; twice, so the plan slots
    and DMVR buffers are reused."""
    from test_multi_picture import _pictures
    cfg = W.CONFIGS["C2"]
    models = tuple(cfg.models) + (mm360.GEODESIC_CAMPOSE,)
    params = mm360.seq_params(cfg.width, cfg.height, models)
    pics, refs, epis = _pictures(cfg, 3, dmvr_share=0.3)
    for _, pus in pics:
        pus["model"][::7] = mm360.GEODESIC_CAMPOSE
        assert W.dmvr_flagged(pus).sum() > 100
    orc = Oracle(params, epis)
    want = [orc.predict_mixed(cur, pus, refs, cfg.width, cfg.height) for cur, pus in pics]
    with _ctx(params, epis) as ctx:
        ctx.set_dmvr(True)
        ctx.set_plan_ahead(plan_ahead)
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_lists = [mm360.pus_to_device(p) for _, p in pics]
        torch.cuda.synchronize()  # plan-ahead contract: the lists are complete before the calls
        for rnd in range(2):
            outs = [_planes(cfg, fill=-1) for _ in pics]
            ctx.predict_device_multi([(cur, d, *o) for (cur, _), d, o in zip(pics, d_lists, outs)])
            assert ctx.status() == (mm360.MM_OK, -1)
            for q, (o, w) in enumerate(zip(outs, want)):
                for name, t, x in zip(("y", "cb", "cr"), o, w):
                    got = t.cpu().numpy()
                    assert np.array_equal(got, x), (rnd, q, plane_mismatch(name, got, x))


def test_pred_plan_ahead_dmvr_on_off_growing_lists():
    """Plan-ahead with MM-DMVR switched on and off between calls while the lists grow (round-5
    advisor): a small DMVR list, a larger plain list, a medium DMVR list -- the third call's
    DMVR-derived capacities (jobs, sub-PU records) exceed what the first sized, so its buffers must
    grow through the synchronised branch, not under the auxiliary stream's planning.  Every output
    == the oracle (predict_mixed), twice round."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    full_d = W.pu_list(cfg, frame=3, dmvr_share=0.5)
    plain = W.pu_list(cfg, frame=4)
    small_d = full_d[W.dmvr_flagged(full_d)][:40]
    medium_d = full_d[: 2 * len(full_d) // 3]
    calls = [(True, small_d), (False, plain), (True, medium_d)]
    orc = Oracle(params, EPI)
    want = [orc.predict_mixed(W.CUR_POC, p, refs, cfg.width, cfg.height) for _, p in calls]
    with _ctx(params) as ctx:
        ctx.set_plan_ahead(True)
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_lists = [mm360.pus_to_device(p) for _, p in calls]
        torch.cuda.synchronize()  # plan-ahead contract: the lists are complete before the calls
        for rnd in range(2):
            outs = [_planes(cfg, fill=0) for _ in calls]
            for (dm, _), d, o in zip(calls, d_lists, outs):
                ctx.set_dmvr(dm)
                ctx.predict_device(W.CUR_POC, d, *o)
            ctx.synchronize()
            for k, (o, w) in enumerate(zip(outs, want)):
                for name, t, x in zip(("y", "cb", "cr"), o, w):
                    got = t.cpu().numpy()
                    assert np.array_equal(got, x), (rnd, k, plane_mismatch(name, got, x))


@pytest.mark.parametrize("plan_ahead", [False, True])
def test_pred_device_multi_more_epipoles_than_one_chain_holds(plan_ahead):
    """mm_pred_device_multi over four C1 pictures with six resident references and one distinct
    camera-pose epipole per (cur, ref) pair: 24 epipoles, more than one launch chain's 16
    (PicTables::ged), so the call is cut into runs (round-5 advisor) -- every picture == the oracle,
    and a failing PU in the last picture is reported with its index counted through all four lists."""
    cfg = W.CONFIGS["C1"]
    params = mm360.seq_params(cfg.width, cfg.height, tuple(cfg.models) + (mm360.GEODESIC_CAMPOSE,))
    ref_pocs = [0, 16, 32, 48, 64, 80]
    refs = {p: W.ref_planes(cfg.width, cfg.height, p) for p in ref_pocs}
    rng = np.random.default_rng(91)
    pics, epis = [], []
    for q in range(4):
        cur = 8 + 16 * q
        for r in ref_pocs:
            v = rng.normal(size=3)
            v = v / np.linalg.norm(v)
            epis.append((cur, r, tuple(int(round(c * (1 << 24))) for c in v)))
        pus = W.pu_list(cfg, frame=q)
        pus["ref_poc"] = np.where(pus["ref_poc"] >= 0, np.array(ref_pocs)[rng.integers(0, 6, size=pus["ref_poc"].shape)], -1)
        pus["model"][::3] = mm360.GEODESIC_CAMPOSE
        pics.append((cur, pus))
    orc = Oracle(params, epis)
    want = [orc.predict(cur, pus, refs, cfg.width, cfg.height) for cur, pus in pics]
    with _ctx(params, epis) as ctx:
        ctx.set_plan_ahead(plan_ahead)
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        d_lists = [mm360.pus_to_device(p) for _, p in pics]
        torch.cuda.synchronize()
        outs = [_planes(cfg, -3) for _ in pics]
        ctx.predict_device_multi([(cur, d, *o) for (cur, _), d, o in zip(pics, d_lists, outs)])
        assert ctx.status() == (mm360.MM_OK, -1)
        for q, (o, w) in enumerate(zip(outs, want)):
            for name, t, x in zip(("y", "cb", "cr"), o, w):
                got = t.cpu().numpy()
                assert np.array_equal(got, x), (q, plane_mismatch(name, got, x))
        bad = pics[3][1].copy()
        bad["x"][2] = 3  # not 4x4 aligned
        d_bad = mm360.pus_to_device(bad)
        torch.cuda.synchronize()
        ctx.predict_device_multi([(pics[0][0], d_lists[0], *outs[0]), (pics[1][0], d_lists[1], *outs[1]),
                                  (pics[2][0], d_lists[2], *outs[2]), (pics[3][0], d_bad, *outs[3])])
        code, first = ctx.status()
        assert code == mm360.MM_ERR_ARG and first == sum(len(p) for _, p in pics[:3]) + 2, (code, first)


def test_effective_blocks_end_to_end_vs_oracle():
    """a2 wired end to end: decoded PUs of a C2 picture (merge / mvRefine DMVR PUs, SbTMVP PUs with
    8x8 motion fields, BDOF-split bi PUs) -> the product's mm_derive_effective_blocks -> one
    mm_pred_device list (DMVR PUs flagged) on the GPU, against the oracle's own derivation
    (motionCompensation restated) + predict + predict_dmvr."""
    from oracle.oracle import effective_blocks
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    dec, tools = W.decoded_pus(cfg, frame=5, dmvr_share=0.3)
    rng = np.random.default_rng(77)
    fields, n_sub = [], 0
    for p in dec:
        u = p["pu"]
        if p["flags"] or u["w"] < 16 or u["h"] < 16 or rng.random() > 0.2:
            continue
        cols, rows = int(u["w"]) // 8, int(u["h"]) // 8
        base = mm360.new_pus(3)
        for b in base:
            bi = rng.random() < 0.6
            lst = int(rng.integers(0, 2))
            b["ref_poc"] = [W.REF_POCS[0] if (bi or lst == 0) else -1, W.REF_POCS[1] if (bi or lst == 1) else -1]
            b["mv"] = rng.integers(-400, 400, size=(2, 2))
            b["model"] = [int(rng.choice(cfg.models)), int(rng.choice(cfg.models))]
        field = mm360.new_pus(cols * rows)
        for k in range(cols * rows):  # runs of equal motion, merged into strips by xSubPuMC
            field[k] = base[int(rng.integers(0, 3))] if (k == 0 or rng.random() < 0.4) else field[k - 1]
        field["mv"][field["ref_poc"] < 0] = 0
        p["flags"] = mm360.PU_SUBPU | mm360.PU_MERGE
        p["sub_motion"] = n_sub
        fields.append(field)
        n_sub += len(field)
    sub = np.concatenate(fields)
    mc, dm = mm360.derive_effective_blocks(tools, dec, sub)
    omc, odm = effective_blocks(tools, dec, sub, mm360.PU_DTYPE)
    assert mc.tobytes() == omc.tobytes() and dm.tobytes() == odm.tobytes()
    assert len(dm) > 50 and len(fields) > 50
    flagged = dm.copy()
    flagged["flags"] |= mm360.PUF_DMVR
    pus = np.concatenate([mc, flagged])
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    orc = Oracle(params, EPI)
    want = orc.predict(W.CUR_POC, omc, refs, cfg.width, cfg.height)
    orc.predict_dmvr(W.CUR_POC, odm, refs, cfg.width, cfg.height, out=want)
    with _ctx(params) as ctx:
        ctx.set_dmvr(True)
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
        out = _planes(cfg, fill=-1)
        ctx.predict_device(W.CUR_POC, mm360.pus_to_device(pus), *out)
        ctx.synchronize()
        got = [t.cpu().numpy() for t in out]
    for name, a, b in zip(("y", "cb", "cr"), got, want):
        assert np.array_equal(a, b), plane_mismatch(name, a, b)
