#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Every index and result file here is produced by the REFERENCE's own tools,
compiled from /root/reference sources by oracle/Makefile into oracle/_ref/:
  gfmi_<K>_<d>    = common/generateIndex.c + src/genFMindex.c  (tag 100 .fmi)
  tfmiBMP_<K>_<d> = src/transformIndexBitmaps.c                 (tag 101 .interleaving)
  tfmiAC_<K>_<d>  = src/transformIndexAlternateCounters.c       (tags 200/201 .ac/.interleaving.ac)
  cpu_<K>_<d>     = common/searchQueries.c + src/fmIndexCPUBaseline.c
  cpuac_<K>_<d>   = common/searchQueries.c + src/fmIndexCPUBaseline-AltCounters.c
The inputs (texts, reads) come from our own seeded generator below.  The
outputs are data (inputs + expected outputs); no reference source is stored.

Run (in the dev container, where /root/reference exists):
    make -C oracle ref && python3 tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import random
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = REPO / "oracle" / "_ref"

KD = [(1, 64), (2, 64), (1, 192), (2, 192)]


def fasta(name: str, seq: str) -> bytes:
    lines = [seq[i:i + 70] for i in range(0, len(seq), 70)]
    return (">" + name + "\n" + "\n".join(lines) + "\n").encode()


def qry(reads: list[str]) -> bytes:
    return b"".join(b">r%d\n%s\n" % (i, r.encode()) for i, r in enumerate(reads))


def dollar_edge_reads(t: str, m: int) -> list[str]:
    """Reads that straddle the end of T (where '$' sits) -- the $-row
    correction (fmIndexCPUBaseline.c:252-256) only matters for these."""
    n = len(t)
    out = []
    for k in range(0, m, max(1, m // 12)):
        if k <= n and m - k - 1 <= n:
            out.append(t[n - k:] + "A" + t[:m - k - 1])   # '$' read as A
            out.append(t[n - k:] + "T" + t[:m - k - 1])
    if m <= n:
        out += [t[:m], t[n - m:], "A" + t[:m - 1], t[n - m + 1:] + "A", "T" + t[:m - 1],
                t[1:m + 1] if m + 1 <= n else t[:m]]
    return [r for r in out if len(r) == m]


def reads_for(t: str, m: int, rng: random.Random, nsamp: int, nrand: int) -> list[str]:
    n = len(t)
    out = []
    if m <= n:
        for _ in range(nsamp):
            s = rng.randint(0, n - m)
            out.append(t[s:s + m])
    out += ["".join(rng.choice("ACGT") for _ in range(m)) for _ in range(nrand)]
    out += dollar_edge_reads(t, m)
    out += ["N" * m, "A" * m, "C" * m, "G" * m, "T" * m]
    if out:
        out.append(out[0].lower())                         # lowercase == uppercase
        r = list(out[1]); r[m // 2] = "N"; out.append("".join(r))   # N -> G (code 2)
        out.append("".join(rng.choice("acgtnACGTN") for _ in range(m)))
    return out


def run(cmd, cwd):
    p = subprocess.run([str(c) for c in cmd], cwd=cwd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"{cmd} failed: {p.stdout[-400:]} {p.stderr[-400:]}")
    return p.stdout


def md5(p: Path) -> str:
    return hashlib.md5(p.read_bytes()).hexdigest()


def make_case(name: str, text: str, qsets: dict[int, list[str]], manifest: dict) -> None:
    out = HERE / name
    if out.exists():
        shutil.rmtree(out)
    out.mkdir(parents=True)
    n = len(text)
    (out / "ref.fa").write_bytes(fasta(name, text))
    case = {"n": n, "text_md5": hashlib.md5(text.encode()).hexdigest(), "indexes": {}, "queries": {}}
    for m, reads in qsets.items():
        (out / f"q{m}.qry").write_bytes(qry(reads))
        case["queries"][str(m)] = {"file": f"q{m}.qry", "num": len(reads)}
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        shutil.copy(out / "ref.fa", td / "ref.fa")
        for k, d in KD:
            if (n + 1) % d == 0:
                continue  # reference UB; not a fixture
            run([REF / f"gfmi_{k}_{d}", "ref.fa", n], td)
            base = f"ref.fa.{n}.{d}fmi{k}steps.fmi"
            run([REF / f"tfmiBMP_{k}_{d}", base], td)
            run([REF / f"tfmiAC_{k}_{d}", base], td)
            files = {100: base, 101: base + ".interleaving", 200: base + ".ac",
                     201: base + ".interleaving.ac"}
            key = f"k{k}_d{d}"
            ent = {"k": k, "d": d, "files": {}, "results": {}}
            for tag, fn in files.items():
                dst = f"{key}.{tag}.fmi"
                shutil.copy(td / fn, out / dst)
                ent["files"][str(tag)] = {"file": dst, "md5": md5(out / dst)}
            for m, reads in qsets.items():
                if m % k or not reads:
                    continue
                shutil.copy(out / f"q{m}.qry", td / f"q{m}.qry")
                for tool, tag in (("cpu", 100), ("cpuac", 200)):
                    run([REF / f"{tool}_{k}_{d}", files[tag], f"q{m}.qry", m, len(reads)], td)
                    resname = f"{key}.q{m}.{tool}.res"
                    shutil.copy(td / (files[tag] + ".res.cpu"), out / resname)
                    ent["results"][f"{m}.{tag}"] = {"file": resname, "md5": md5(out / resname)}
            case["indexes"][key] = ent
    manifest[name] = case


def main() -> int:
    if not (REF / "gfmi_2_64").exists():
        print("build the reference tools first: make -C oracle ref", file=sys.stderr)
        return 1
    manifest: dict = {}
    rng = random.Random(20261015)

    # A: 50,000 uniform ACGT bases ((n+1) % 64 = 17, % 192 = 81).
    tA = "".join(rng.choice("ACGT") for _ in range(50_000))
    make_case("textA", tA, {
        100: reads_for(tA, 100, rng, 256, 64),
        150: reads_for(tA, 150, rng, 48, 16),
        12: reads_for(tA, 12, rng, 200, 56) + [a + b + "ACGTACGTAC" for a in "ACGT" for b in "ACGT"],
        2: [a + b for a in "ACGTN" for b in "ACGTN"],
        1: list("ACGTNacgtn"),
    }, manifest)

    # B: a long T run at the start puts the '$' rows D_0, D_1 in the LAST
    # d-block, the only place the AltCounters sentinel entry
    # (transformIndexAlternateCounters.c:420-431) makes the AC oracle differ
    # from the plain one.
    tB = "T" * 80 + "".join(rng.choice("ACGT") for _ in range(4_000))
    make_case("textB", tB, {
        100: reads_for(tB, 100, rng, 96, 16),
        12: reads_for(tB, 12, rng, 96, 16) + ["T" * 12, "T" * 11 + "A", "A" + "T" * 11],
        2: [a + b for a in "ACGT" for b in "ACGT"],
    }, manifest)

    # C: tiny / repetitive texts.
    tC = "ACGT" * 40 + "A"                       # periodic
    make_case("textC", tC, {
        4: reads_for(tC, 4, rng, 32, 8),
        2: [a + b for a in "ACGT" for b in "ACGT"],
    }, manifest)
    tD = "GATTACA"
    make_case("textD", tD, {
        2: [a + b for a in "ACGT" for b in "ACGT"] + ["CA", "AT", "TT"],
        4: ["GATT", "ATTA", "TACA", "ACAG", "AAAA", "CAGA"],
    }, manifest)
    tE = "A" * 300 + "C" + "A" * 200             # long repeats, many 32-mer ties
    make_case("textE", tE, {
        12: ["A" * 12, "A" * 11 + "C", "C" + "A" * 11, "AAAACAAAAAAA", "CCCCCCCCCCCC"],
        100: ["A" * 100, "A" * 99 + "C", "C" + "A" * 99, "A" * 50 + "C" + "A" * 49],
    }, manifest)

    (HERE / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=True) + "\n")
    print("wrote", HERE / "manifest.json")
    return 0


if __name__ == "__main__":
    sys.exit(main())
