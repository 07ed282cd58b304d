"""Degenerate worlds through the reference's own driver and searchers: the
first worlds of scripts/diag/dropin_degenerate.py (homopolymers of each
letter, two- and three-letter texts, short periods, runs at the end, texts of
a few bases, reads longer than the text) as a fixed test -- every result file
the reference defines must be byte-identical (CPU suite: the library's host
search; GPU suite: a GPU backend per tag).  The script runs the same
generator for as long as it is given (profiles/r05/dropin_degenerate_*)."""
import sys

import pytest

from util import REPO

sys.path.insert(0, str(REPO / "scripts" / "diag"))
import dropin_degenerate as D  # noqa: E402

WORLDS = 60


def _check(w, gpu):
    if not (D.REF / "cpu_1_64").exists() or not (D.REF / "searchQueries_cpu_dropin").exists():
        if gpu:
            pytest.fail("oracle/_ref missing on the GPU box")
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    k, d, n, kind, m, checked = D.run_world(w, gpu)
    bad = [(tag, b) for tag, b, same in checked if not same]
    assert not bad, dict(world=w, k=k, d=d, n=n, kind=kind, m=m, bad=bad)


@pytest.mark.parametrize("w", range(WORLDS))
def test_dropin_degenerate_cpu(w):
    _check(w, False)


@pytest.mark.gpu
@pytest.mark.parametrize("w", range(WORLDS))
def test_dropin_degenerate_gpu(kfmi_mod, w):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_device(0)
    _check(w, True)
