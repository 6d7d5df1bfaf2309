"""The oracle against its committed golden frames (tests/golden, build-authored:
the reference has none).  Any change to the oracle's arithmetic shows up here."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden  # noqa: E402
import oracle  # noqa: E402

GOLD = np.load(os.path.join(HERE, "golden", "frames.npz"), allow_pickle=False)
COUNTS = json.load(open(os.path.join(HERE, "golden", "counters.json")))


@pytest.mark.parametrize("name", list(make_golden.GOLDEN))
def test_oracle_matches_golden(name):
    sc = make_golden.build(name)
    rgb, c = oracle.render(sc, seed=COUNTS["seed"])
    assert np.array_equal(rgb, GOLD[name])
    assert c == COUNTS["counters"][name]


def test_oracle_is_thread_count_invariant():
    sc = make_golden.build("C4")
    a, ca = oracle.render(sc, seed=3, threads=1)
    b, cb = oracle.render(sc, seed=3, threads=7)
    assert np.array_equal(a, b) and ca == cb


def test_oracle_subset_equals_full_frame_pixels():
    sc = make_golden.build("C5")
    full, _ = oracle.render(sc, seed=1)
    ids = np.array([0, 5, 77, sc.width * sc.height - 1], np.int32)
    sub, _ = oracle.render(sc, seed=1, subset=ids)
    assert np.array_equal(sub, full.reshape(-1, 3)[ids])


def test_fixed_spp_through_adaptive_sampler():
    """SampleSettings{tol 0, batch spp, max spp-1} runs exactly one batch (camera.rs:137-164)."""
    sc = make_golden.build("C1")
    _, c = oracle.render(sc, seed=1)
    assert c["paths"] == sc.width * sc.height * sc.settings.batch_size
    assert c["pixels"] == sc.width * sc.height
