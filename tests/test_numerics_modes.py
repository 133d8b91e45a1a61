"""Numerics-mode switches: every unverifiable Eigen 3.3.7 belief is a
compile-time flag in both the product headers (CPU twin builds) and the oracle.  In each
alternative mode the twin and the oracle must still agree bit for bit (the switch means the same
thing on both sides), and the mode must be wired (it changes something on a workload that
exercises it, except ROUND (exact-half cases are rare) and TAN_CENTRE (glibc sinf/cosf are
correctly rounded almost everywhere, so float and double-then-float centre terms rarely differ)
-- DESIGN 2 counts them at C3)."""
import numpy as np
import pytest

import mm360
import twin
from helpers import EPI
from mm360 import workload as W
from oracle.oracle import Oracle


@pytest.fixture(autouse=True)
def _restore_default():
    yield
    twin.use_variant(None)


@pytest.mark.parametrize("mode", ["round", "prod3", "tanc", "psqrt"])
def test_mode_twin_equals_oracle(mode):
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, W.ALL_MODELS)
    blocks = W.random_blocks(cfg.width, cfg.height, W.ALL_MODELS, 1500, seed=77)
    twin.use_variant(mode)
    t = twin.reproject(params, blocks, EPI)
    o = Oracle(params, EPI, variant=mode).reproject(blocks)
    assert np.array_equal(t, o)
    twin.use_variant(None)
    d = twin.reproject(params, blocks, EPI)
    changed = int(np.any(d != t, axis=1).sum())
    if mode not in ("round", "tanc"):
        assert changed > 0, f"{mode}: switch changes nothing on 1500 random blocks"
