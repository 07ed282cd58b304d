"""Seeded random real-FASTA worlds for the 'ref' alphabet mode, against the
reference's own builder (oracle/_ref/gfmi_K_d, genFMindex.c:457-543, with its
readRef, common/common.c:42-76).

Each world writes a multi-FASTA file -- several records, line widths from 30
to 400 bytes (so some lines reach the reference loader in 255-byte fgets
pieces, each of which loses its last byte), N runs, soft-masked stretches,
IUPAC letters -- and builds it with the reference tool and with this build's
host builder (and GPU builder in the GPU suite) in 'ref' mode; the index files
must be byte-identical.  For K >= 2 the reference leaves rows of BWT_1..
uninitialised on such texts (tests/test_alphabet.py), so it runs under glibc's
MALLOC_PERTURB_=p and the product's image (whose builder writes a defined
byte there) is patched by tests/ref_fill.py with p ^ 0xff, the byte the
fresh allocation then holds (tests/golden/make_golden_alpha.py) -- with the
thread cache off (GLIBC_TUNABLES=glibc.malloc.tcache_count=0): a small chunk
the cache hands back is not perturbed and holds what its last owner left
there (3 of 80 worlds differed that way; with the cache off, all agree)."""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

import ref_fill
from util import REPO

REF = REPO / "oracle" / "_ref"
GEOMS = [(1, 64), (1, 192), (2, 64), (2, 192), (3, 64), (4, 64)]
WORLDS = 80


class _Ref(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint64), ("p", ctypes.c_void_p)]


def _readref_len(fasta: bytes) -> int:
    """Bytes the reference's readRef yields from the whole file: after the
    first fgets piece, strlen - 1 bytes of every piece of at most 255."""
    total, first = 0, True
    for line in fasta.split(b"\n")[:-1]:
        raw = line + b"\n"
        while raw:
            piece, raw = raw[:255], raw[255:]
            if first:
                first = False
                continue
            total += len(piece) - 1
    return total


def world(i):
    rng = np.random.default_rng(55_000 + i)
    k, d = GEOMS[int(rng.integers(0, len(GEOMS)))]
    recs = []
    for r in range(int(rng.integers(1, 4))):
        parts = []

        def pick(alpha, size):
            return np.frombuffer(alpha, np.uint8)[rng.integers(0, len(alpha), size=size)].tobytes()

        for _ in range(int(rng.integers(2, 8))):
            kind = int(rng.integers(0, 5))
            n = int(rng.integers(20, 1500))
            if kind == 0:
                parts.append(pick(b"ACGT", n))
            elif kind == 1:
                parts.append(pick(b"acgt", n))
            elif kind == 2:
                parts.append((b"N" if rng.random() < 0.7 else b"n") * int(rng.integers(1, 400)))
            elif kind == 3:
                parts.append(pick(b"RYKMSWBDHVN", int(rng.integers(1, 60))))
            else:
                parts.append(pick(b"ACGT", n))
        seq = b"".join(parts)
        w = int(rng.choice([30, 60, 70, 80, 254, 255, 256, 300, 400]))
        recs.append(b">rec%d random world %d\n" % (r, i) + b"\n".join(seq[j:j + w] for j in range(0, len(seq), w)))
    fasta = b"\n".join(recs) + b"\n"
    avail = _readref_len(fasta)
    n = int(rng.integers(max(2 * k + 2, avail // 2), avail + 1))
    pert = int(rng.integers(1, 256)) if k >= 2 else None
    return k, d, fasta, n, pert


def _reference_md5(tmp_path, k, d, fasta, n, pert):
    gfmi = REF / f"gfmi_{k}_{d}"
    if not gfmi.exists():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    (tmp_path / "ref.fa").write_bytes(fasta)
    env = {x: v for x, v in os.environ.items() if x != "MALLOC_PERTURB_"}
    if pert is not None:
        env["MALLOC_PERTURB_"] = str(pert)
        env["GLIBC_TUNABLES"] = "glibc.malloc.tcache_count=0"
    subprocess.run([str(gfmi), "ref.fa", str(n)], cwd=tmp_path, check=True, capture_output=True, timeout=120,
                   env=env)
    return hashlib.md5((tmp_path / f"ref.fa.{n}.{d}fmi{k}steps.fmi").read_bytes()).hexdigest()


def _ours(K, tmp_path, k, d, n, pert, gpu):
    L = K.load()
    ref = ctypes.c_void_p()
    assert L.loadRef(str(tmp_path / "ref.fa").encode(), n, ctypes.byref(ref)) == 0
    r = _Ref.from_address(ref.value)
    text = ctypes.string_at(r.p, r.size)
    L.freeReference(ctypes.byref(ref), None)
    idx = K.Index.build(text, k=k, d=d, gpu=gpu)
    img = idx.image()
    if pert is not None:   # the reference's unvisited rows under MALLOC_PERTURB_ (tests/ref_fill.py)
        img = ref_fill.patch(img, text, ref_fill.full_sa(K, text, k, d), pert ^ 0xFF)
    h = hashlib.md5(img.tobytes()).hexdigest()
    idx.close()
    return h


@pytest.fixture
def ref_mode(kfmi_mod):
    kfmi_mod.set_alphabet("ref")
    yield kfmi_mod
    kfmi_mod.set_alphabet(None)


@pytest.mark.parametrize("i", range(WORLDS))
def test_alphabet_world_host(ref_mode, tmp_path, i):
    k, d, fasta, n, pert = world(i)
    want = _reference_md5(tmp_path, k, d, fasta, n, pert)
    assert _ours(ref_mode, tmp_path, k, d, n, pert, False) == want, dict(world=i, k=k, d=d, n=n, p=pert)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(WORLDS))
def test_alphabet_world_gpu(ref_mode, tmp_path, i):
    K = ref_mode
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    k, d, fasta, n, pert = world(i)
    want = _reference_md5(tmp_path, k, d, fasta, n, pert)
    assert _ours(K, tmp_path, k, d, n, pert, True) == want, dict(world=i, k=k, d=d, n=n, p=pert)
