"""The host C layer under AddressSanitizer + UBSan (CPU only): csrc/host/*.c
compiled with gcc -fsanitize=address,undefined together with
tests/asan/host_asan.c (HIP layer stubbed) and driven over the golden
fixtures, error paths included.  Any out-of-bounds access, use-after-free,
leak or UB report fails the test."""
import os
import shutil
import subprocess

import pytest

from util import GOLDEN, PKG, REPO

HARNESS = REPO / "tests" / "asan" / "host_asan.c"


@pytest.fixture(scope="module")
def binary(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    out = tmp_path_factory.mktemp("asan") / "host_asan"
    srcs = sorted(str(p) for p in (PKG / "csrc" / "host").glob("*.c"))
    cmd = ["gcc", "-g", "-O1", "-std=gnu11", "-fopenmp", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-o", str(out), str(HARNESS)] + srcs
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


@pytest.mark.parametrize("case,k,d,m,num", [("textA", 2, 64, 100, 360), ("textA", 1, 192, 12, 0),
                                            ("textB", 2, 192, 100, 0), ("textD", 1, 64, 2, 0),
                                            ("textE", 2, 64, 12, 0), ("textC", 1, 192, 4, 0)])
def test_host_layer_clean_under_asan(binary, tmp_path, case, k, d, m, num):
    import json
    man = json.loads((GOLDEN / "manifest.json").read_text())
    if case not in man or f"k{k}_d{d}" not in man[case]["indexes"] or str(m) not in man[case]["queries"]:
        pytest.skip("fixture not present")
    num = num or man[case]["queries"][str(m)]["num"]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([str(binary), str(GOLDEN), str(tmp_path), case, str(k), str(d), str(m), str(num)],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0 and p.stdout.startswith("OK"), p.stdout[-2000:] + p.stderr[-4000:]
