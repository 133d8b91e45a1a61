"""Bitstream side: SPS / PH MM syntax and the CABAC motion_model() element.

The product (csrc/mm_syntax.h through the C-ABI, host code -- no GPU) against the oracle
(oracle/mm_syntax.py: the H.266 spec's bit-serial arithmetic coder and Exp-Golomb definitions).
Parity UNPINNED: no reference-produced MM bitstream exists (the reference ships none and its coder
needs Eigen), so the oracle pins by independent formulation, not by reference bits.
"""
import random

import numpy as np
import pytest

from mm360 import MM_ERR_ARG, MM_ERR_BITSTREAM, MMError
from mm360 import syntax as S
from oracle import mm_syntax as O


def rand_sps(rng, multi=None):
    d = {k: int(rng.random() < 0.5) for k in ("mpa", "t3d", "tan", "rot", "ged", "geda")}
    if multi is False:
        d = {k: 0 for k in d}
    elif multi is True and not any(d.values()):
        d["ged"] = 1
    d.update(ged_flavor=rng.randint(0, 1), mmmvp=rng.randint(0, 1), mm_offset_4x4=rng.randint(0, 4),
             projection_fct=rng.randint(0, 2), focal_length_px=rng.randint(0, 5000),
             optical_center_x_px=rng.randint(0, 2 ** 32 - 2), optical_center_y_px=rng.randint(0, 9000))
    n = rng.randint(0, 16)
    d["num_calibrated_coeffs"] = n
    d["calibrated_coeffs"] = [rng.randint(-2 ** 31 + 1, 2 ** 31 - 1) for _ in range(n)]
    d["global_epipole"] = [rng.randint(-2 ** 31 + 1, 2 ** 31 - 1) if rng.random() < 0.2 else rng.randint(-4096, 4096)
                           for _ in range(3)]
    return d


def coded_view(d):
    """The fields the bitstream carries (the rest read back as MMConfig defaults)."""
    s = O.parse_sps(O.Bits(O.sps_bits(d)))
    return s


# ------------------------------------------------------------------------------ Exp-Golomb
def test_exp_golomb_definition():
    # H.266 Table 9-2 / 9-3 (the oracle's codes are the spec's bit strings)
    assert [O.ue_bits(v) for v in range(5)] == ["1", "010", "011", "00100", "00101"]
    assert [O.se_bits(v) for v in (0, 1, -1, 2, -2)] == ["1", "010", "011", "00100", "00101"]
    assert O.ue_bits(0xFFFFFFFE) == "0" * 31 + "1" + "1" * 31


@pytest.mark.parametrize("seed", range(4))
def test_sps_fragment_matches_oracle_and_round_trips(seed):
    rng = random.Random(seed)
    for _ in range(150):
        d = rand_sps(rng)
        s = S.sps_mm(**d)
        # at an unaligned offset inside a larger RBSP, surrounding bits untouched
        off = rng.randint(0, 40)
        buf = np.full(300, 0xA5, np.uint8)
        buf, end = S.write_sps_mm(s, buf, off)
        bits = O.bytes_to_bits(buf.tobytes())
        assert bits[off:end] == O.sps_bits(d)
        assert bits[:off] == O.bytes_to_bits(bytes([0xA5] * 300))[:off]
        assert bits[end:] == O.bytes_to_bits(bytes([0xA5] * 300))[end:]
        r, pos = S.read_sps_mm(buf, end, off)
        assert pos == end
        want = coded_view(d)
        got = r.as_dict()
        for k in O.SPS_FIELDS:
            assert got[k] == want[k], k


def test_sps_no_multi_model_is_six_flags():
    s = S.sps_mm(ged_flavor=1, mm_offset_4x4=3, global_epipole=[1, 2, 3])
    buf, end = S.write_sps_mm(s)
    assert end == 6 and O.bytes_to_bits(buf.tobytes())[:6] == "000000"
    r, pos = S.read_sps_mm(buf, 6)
    assert pos == 6 and r.mm_offset_4x4 == 0 and list(r.global_epipole) == [0, 0, 0]


@pytest.mark.parametrize("field,value", [("mm_offset_4x4", 5), ("projection_fct", 3), ("num_calibrated_coeffs", 17),
                                         ("mm_offset_4x4", -1), ("ged_flavor", -1)])
def test_sps_write_rejects_what_the_reader_rejects(field, value):
    d = dict(ged=1, projection_fct=O.CALIBRATED)
    d[field] = value
    with pytest.raises(MMError) as e:
        S.write_sps_mm(S.sps_mm(**d))
    assert e.value.code == MM_ERR_ARG


@pytest.mark.parametrize("case", ["offset", "projection", "calib", "truncated", "long_prefix"])
def test_sps_read_rejects_malformed(case):
    # hand-built fragments: tan only -> mmmvp, offset, projection ...
    if case == "offset":
        bits = "001000" + "0" + O.ue_bits(5) + O.ue_bits(2)  # VLCReader.cpp:1948 CHECK
    elif case == "projection":
        bits = "001000" + "0" + O.ue_bits(1) + O.ue_bits(3)  # :1952 CHECK
    elif case == "calib":
        bits = "001000" + "0" + O.ue_bits(1) + O.ue_bits(1) + O.ue_bits(7) * 3 + O.ue_bits(17)
    elif case == "truncated":
        bits = "000010" + O.ue_bits(1) + "1" + O.ue_bits(0) + O.ue_bits(2) + O.se_bits(5)[:-1]
    else:
        bits = "001000" + "0" + "0" * 33 + "1"
    data = O.bits_to_bytes(bits)
    with pytest.raises(MMError) as e:
        S.read_sps_mm(np.frombuffer(data, np.uint8).copy(), len(bits))
    assert e.value.code == MM_ERR_BITSTREAM


def test_ph_epipole_delta():
    rng = random.Random(7)
    for _ in range(200):
        d = rand_sps(rng)
        s = S.sps_mm(**d)
        delta = [0, 0, 0] if rng.random() < 0.3 else [rng.randint(-70000, 70000) for _ in range(3)]
        off = rng.randint(0, 20)
        buf, end = S.write_ph_epipole(s, delta, np.zeros(64, np.uint8), off)
        want = O.ph_bits(d, delta)
        assert O.bytes_to_bits(buf.tobytes())[off:end] == want
        got, pos = S.read_ph_epipole(s, buf, end, off)
        assert pos == end
        assert got == (delta if (O.multi_model(d) and d["ged"]) else [0, 0, 0])
    with pytest.raises(MMError):
        S.write_ph_epipole(S.sps_mm(ged=1), [-2 ** 31, 0, 0])


# ------------------------------------------------------------------------------- candidates
def rand_col(rng, gw, gh, models):
    pool = models + [O.INVALID]
    base = rng.choice(pool)
    col = np.empty((gh, gw, 2), np.int8)
    for y in range(gh):
        for x in range(gw):
            for lst in range(2):
                col[y, x, lst] = base if rng.random() < 0.4 else rng.choice(pool + [m for m in range(11)])
    return col


@pytest.mark.parametrize("pred_type", [0, 1, 2, 3])
def test_candidate_order_matches_oracle(pred_type):
    rng = random.Random(100 + pred_type)
    for _ in range(120):
        d = rand_sps(rng, multi=True)
        s = S.sps_mm(**d)
        W, H = rng.choice([(64, 32), (128, 64), (96, 48)])
        col = rand_col(rng, W // 4, H // 4, O.active_models(d))
        w, h = rng.choice([4, 8, 16, 32, 64]), rng.choice([4, 8, 16, 32])
        w, h = min(w, W), min(h, H)
        x, y = rng.randrange(0, W - w + 1, 4), rng.randrange(0, H - h + 1, 4)
        lst = rng.randint(0, 1)
        got = S.motion_model_candidates(s, pred_type, col, W, H, lst, x, y, w, h)
        want = O.candidates(d, pred_type, col.tolist(), W, H, lst, x, y, w, h)
        assert got == want
        assert sorted(got) == sorted(O.active_models(d))


def test_candidate_order_rules():
    d = dict(mpa=1, tan=1, ged=1, geda=1)
    s = S.sps_mm(**d)
    act = [0, 1, 2, 3, 4, 10, 7, 8, 9]  # getActiveMotionModels order (MMConfig.cpp:7-39), not id order
    assert S.motion_model_candidates(s) == act
    col = np.full((8, 8, 2), -1, np.int8)
    col[..., 0] = 4  # TAN everywhere in list 0
    assert S.motion_model_candidates(s, 1, col, 32, 32, 0, 8, 8, 8, 8)[0] == 4
    # a predicted model that is not active leaves the order (undefined erase(end()) in the reference)
    col[..., 0] = 5
    assert S.motion_model_candidates(s, 1, col, 32, 32, 0, 8, 8, 8, 8) == act
    # voted: INVALID in the chosen list falls back to the other list
    col[..., 0] = -1
    col[..., 1] = 9
    assert S.motion_model_candidates(s, 2, col, 32, 32, 0, 0, 0, 16, 16)[0] == 9
    # sorted: vote-descending, ties in list order
    col[:, :4, 0] = 10
    col[:, 4:, 0] = 2
    got = S.motion_model_candidates(s, 3, col, 32, 32, 0, 0, 0, 32, 32)
    assert got[:2] == [2, 10] and got[2:] == [0, 1, 3, 4, 7, 8, 9]
    with pytest.raises(MMError):
        S.motion_model_candidates(s, 2, col, 32, 32, 0, 24, 24, 16, 16)  # PU outside the picture
    bad = col.copy()
    bad[0, 0, 0] = 11
    with pytest.raises(MMError):
        S.motion_model_candidates(s, 2, bad, 32, 32, 0, 0, 0, 8, 8)


# ---------------------------------------------------------------------------------- CABAC
def rand_stream(rng, d, npu):
    act = O.active_models(d)
    cands, models = [], []
    skew = rng.random()
    for _ in range(npu):
        c = act[:]
        if rng.random() < 0.5:
            rng.shuffle(c)
        cands.append(c)
        models.append(c[0] if rng.random() < skew else rng.choice(c))
    aff = [int(rng.random() < 0.1) for _ in range(npu)]
    if O.multi_model(d):
        models = [0 if a else m for a, m in zip(aff, models)]
    else:
        models = [0] * npu
    return cands, models, aff


@pytest.mark.parametrize("seed", range(6))
def test_motion_model_cabac_matches_spec_coder(seed):
    rng = random.Random(seed)
    for _ in range(60):
        d = rand_sps(rng, multi=None if seed else True)
        s = S.sps_mm(**d)
        npu = rng.choice([0, 1, 2, rng.randint(3, 400)])
        depth = rng.choice([0, 1, 2, 3, S.APP_CODING_DEPTH, rng.randint(0, 12)])
        qp = rng.randint(-6, 70)
        init_type = rng.randint(0, 2)
        cands, models, aff = rand_stream(rng, d, npu)
        mine = S.encode_motion_models(s, models, cands, qp, init_type, depth, aff)
        assert mine == O.encode_models(d, models, cands, qp, depth, aff)
        assert S.decode_motion_models(s, mine, cands, qp, init_type, depth, aff) == models
        assert O.decode_models(d, mine, cands, qp, depth, aff) == models


def test_motion_model_cabac_long_skewed_stream():
    # 20k PUs of a skewed source: long runs of MPS bins, carries through 0xff runs (bitsOutstanding)
    rng = random.Random(11)
    d = dict(mpa=1, t3d=1, tan=1, rot=1, ged=1, geda=1)
    s = S.sps_mm(**d)
    act = O.active_models(d)
    cands = [act] * 20000
    models = [act[0] if rng.random() < 0.97 else rng.choice(act) for _ in range(20000)]
    for depth in (9, 0):
        mine = S.encode_motion_models(s, models, cands, 37, 0, depth)
        assert mine == O.encode_models(d, models, cands, 37, depth)
        assert S.decode_motion_models(s, mine, cands, 37, 0, depth) == models


def test_motion_model_cabac_errors():
    d = dict(tan=1, rot=1)
    s = S.sps_mm(**d)
    act = O.active_models(d)
    with pytest.raises(MMError) as e:  # a model outside the PU's list
        S.encode_motion_models(s, [5], [act])
    assert e.value.code == MM_ERR_ARG
    with pytest.raises(MMError):  # affine PUs must be CLASSIC (CABACWriter.cpp:1860)
        S.encode_motion_models(s, [4], [act], affine=[1])
    with pytest.raises(MMError):  # a candidate row that is not a permutation of the active models
        S.encode_motion_models(s, [0], [[0, 4, 4]])
    models = [4, 6, 0, 6, 6, 4] * 20
    stream = S.encode_motion_models(s, models, [act] * len(models))
    for bad in (stream[:-1], stream + b"\0", stream[:-1] + bytes([stream[-1] ^ 0x01]), b""):
        with pytest.raises(MMError) as e:
            S.decode_motion_models(s, bad, [act] * len(models))
        assert e.value.code in (MM_ERR_BITSTREAM, MM_ERR_ARG)
    # bypass index past the list: depth 0 over 3 candidates codes a 3-bin index, values 3..7 are
    # not candidates (the reference would index past its vector)
    e3 = O.SpecEncoder()
    for b in (1, 1, 1):
        e3.bypass(b)
    e3.terminate(1)
    with pytest.raises(MMError) as e:
        S.decode_motion_models(s, e3.data(), [act], coding_depth=0)
    assert e.value.code == MM_ERR_BITSTREAM


def test_motion_model_no_multi_model_codes_nothing():
    s = S.sps_mm()
    stream = S.encode_motion_models(s, [0] * 50, [[0]] * 50)
    assert stream == O.encode_models({}, [0] * 50, [[0]] * 50)
    assert stream == b"\xfe\x80"  # end_of_slice + flush + stop bit only
    assert S.decode_motion_models(s, stream, [[0]] * 50) == [0] * 50


def test_malformed_input_never_crashes():
    """Random bytes into the readers: a status, never a crash or an out-of-range model (the
    reference would read past its buffers or vectors on some of these)."""
    rng = random.Random(99)
    d = dict(mpa=1, t3d=1, tan=1, rot=1, ged=1, geda=1)
    s = S.sps_mm(**d)
    act = O.active_models(d)
    for _ in range(300):
        data = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 40)))
        arr = np.frombuffer(data or b"\0", np.uint8).copy()
        try:
            S.read_sps_mm(arr, 8 * len(data))
        except MMError as e:
            assert e.code == MM_ERR_BITSTREAM
        try:
            S.read_ph_epipole(s, arr, 8 * len(data))
        except MMError as e:
            assert e.code == MM_ERR_BITSTREAM
        n = rng.randint(0, 30)
        try:
            got = S.decode_motion_models(s, data, [act] * n, coding_depth=rng.choice([0, 2, 9]))
            assert all(m in act for m in got)
        except MMError as e:
            assert e.code == MM_ERR_BITSTREAM
