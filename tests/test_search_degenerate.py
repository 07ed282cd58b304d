"""Degenerate texts (homopolymers of each letter, two and three letters, short
periods, runs at the end, texts of a few bases) with any read length --
m % K != 0 through the remainder table -- and a random ftab, against
brute-force suffix ranks: the first worlds of scripts/diag/search_degenerate.py
as a fixed test (CPU suite: the host search; GPU suite: every plain backend
the geometry takes, K 1-4)."""
import sys

import pytest

from util import REPO

sys.path.insert(0, str(REPO / "scripts" / "diag"))
import search_degenerate as S  # noqa: E402

WORLDS = 80


@pytest.mark.parametrize("w", range(WORLDS))
def test_search_degenerate_host(w):
    bad = [(b, what) for b, what in S.run_world(w, False) if what]
    assert not bad, (w, bad)


@pytest.mark.gpu
@pytest.mark.parametrize("w", range(WORLDS))
def test_search_degenerate_gpu(kfmi_mod, w):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_device(0)
    bad = [(b, what) for b, what in S.run_world(w, True) if what]
    assert not bad, (w, bad)
