"""Test harness: the reference builder's uninitialised rows, applied after the
build.

For K >= 2 and a text with bytes other than A/C/G/T, genFMindex.c's LF walk
(generateOthersBWTs, genFMindex.c:347-391) is not a permutation of the rows:
rows it never visits keep, in every BWT_s (s >= 1), whatever malloc returned
(:342).  glibc's MALLOC_PERTURB_=p makes that byte p ^ 0xff, which is how the
golden files under tests/golden/alpha were pinned.  The product builder
('ref' mode, csrc/host/fmi_build.c kfmi_index_ref_walk) writes a defined
byte there (0, base2index -> A); this module turns such a product image into
the one the reference writes for a given fill byte:

  1. the rows the walk never visits, from the walk restated here on the raw
     text and its raw-byte suffix array (:347-391, chunk-32 counters of
     precalculateBasesPreviousBWT :262-325, exact 'A'/'C'/'G'/'T' only);
  2. those rows' codes for s >= 1 set to base2index(fill) in the bit planes;
  3. every counter recomputed from the rows' K-mer codes: cnt_b[c] = C'[c] +
     rows below b*d with code c, '$' rows (D_s) left out (precalculateBases
     KSteps :184-260, dollar2BaseBWT :246-250).

Test infrastructure only: nothing under k-step_fm-index_amd/ imports it.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle


def base2index(x: int) -> int:
    """genFMindex.c:71-84: code = (bit2 << 1) | (bit1 ^ bit2) of the byte."""
    b2 = (x >> 2) & 1
    return (b2 << 1) | (((x >> 1) & 1) ^ b2)


def visited_rows(text: bytes, sa: np.ndarray) -> np.ndarray:
    """Rows of T$ the reference's LF walk writes (bool[n + 1])."""
    n = len(text)
    rows = n + 1
    t = np.frombuffer(text, dtype=np.uint8)
    sa = np.asarray(sa, dtype=np.int64)
    prev = sa - 1
    bwt0 = np.where(sa == 0, ord("$"), t[np.where(prev < 0, 0, prev)]).astype(np.uint8)
    dpos0 = int(np.flatnonzero(sa == 0)[0])
    acgt = b"ACGT"
    # occ[c][r]: exact-letter rows below r; chunk counters at r % 32 == 0 plus the C offsets
    occ = np.zeros((4, rows + 1), dtype=np.int64)
    for c in range(4):
        occ[c, 1:] = np.cumsum(bwt0 == acgt[c])
    tot = occ[:, rows]
    acc = [1, 1 + tot[0], 1 + tot[0] + tot[1], 1 + tot[0] + tot[1] + tot[2]]
    seen = np.zeros(rows, dtype=bool)
    pos = dpos0
    for _ in range(rows):          # refpos = rows-1 .. 0: each visits `pos`, then steps
        seen[pos] = True
        base = int(bwt0[pos])
        posb = pos - pos % 32
        if base in acgt:
            c = acgt.index(base)
            pos = int(acc[c] + occ[c, posb] + (occ[c, pos] - occ[c, posb]))
        else:                      # any other byte: row 0 plus its own in-chunk count
            pos = int(np.count_nonzero(bwt0[posb:pos] == base))
    return seen


def patch(image, text: bytes, sa: np.ndarray, fill: int) -> np.ndarray:
    """The tag-100 image the reference writes with `fill` in its unvisited
    rows, from the product's (fill 0) image of the same text."""
    img = np.array(image, dtype=np.uint8, copy=True)
    h = oracle.header(img)
    k, d, rows, ne = h["steps"], h["chunk"], h["bwtsize"], h["nentries"]
    assert h["tag"] == 100 and k >= 2
    nb, nc = d // 32, 1 << (2 * k)
    ew = 2 * nb * k + nc
    ent = img[img.size - 4 * ew * ne:].view(np.uint32).reshape(ne, ew)
    # per-row K-mer codes from the planes (plane index s*2*nb + t*nb + w, MSB = first row)
    r = np.arange(rows)
    b, w, p = r // d, (r % d) // 32, 31 - (r % 32)
    code = np.zeros(rows, dtype=np.int64)
    for s in range(k):
        for tb in range(2):
            bit = (ent[b, s * 2 * nb + tb * nb + w] >> p.astype(np.uint32)) & 1
            code |= bit.astype(np.int64) << (2 * s + tb)
    isd = np.isin(r, h["dollar_pos"])

    def counters(cd):
        onehot = np.zeros((ne * d, nc), dtype=np.int64)
        keep = ~isd
        onehot[r[keep], cd[keep]] = 1
        run = np.cumsum(onehot.reshape(ne, d, nc).sum(axis=1), axis=0)
        run = np.vstack([np.zeros((1, nc), dtype=np.int64), run[:-1]])
        t2 = np.bincount(cd[keep], minlength=nc)
        c2 = np.zeros(nc, dtype=np.int64)
        c2[1:] = np.cumsum(t2)[:-1]
        for s, db in enumerate(h["dollar_base"]):
            c2[db & (0xFFFFFFFF << (2 * s)):] += 1
        return (run + c2[None, :]).astype(np.uint32)

    # self-check: the restated counters are the image's own before any patch
    assert np.array_equal(counters(code), ent[:, 2 * nb * k:]), "counter restatement disagrees with the build"
    unseen = ~visited_rows(text, sa)
    f = base2index(fill)
    new = code.copy()
    for s in range(1, k):
        new[unseen] = (new[unseen] & ~(3 << (2 * s))) | (f << (2 * s))
    if np.array_equal(new, code):
        return img
    for s in range(1, k):
        for tb in range(2):
            col = s * 2 * nb + tb * nb
            words = ent[:, col:col + nb].copy()
            words[:] = 0
            bits = ((new >> (2 * s + tb)) & 1).astype(np.uint64) << p.astype(np.uint64)
            np.add.at(words, (b, w), bits.astype(np.uint32))
            ent[:, col:col + nb] = words
    ent[:, 2 * nb * k:] = counters(new)
    return img


def full_sa(K, text: bytes, k: int, d: int) -> np.ndarray:
    """The raw-byte suffix array of text$ the 'ref'-mode builder sorts (every
    row sampled), from a host build with sa_rate 1."""
    idx = K.Index.build(text, k=k, d=d, gpu=False, sa_rate=1)
    rate, sa = idx.sa()
    assert rate == 1 and sa.size == len(text) + 1
    out = np.array(sa, dtype=np.int64)
    idx.close()
    return out
