#!/usr/bin/env python3
"""Golden fixtures for the builders' "ref" alphabet mode (tests/golden/alpha/).

A multi-FASTA reference with what real genomes hold -- N runs, soft-masked
(lowercase) stretches, IUPAC codes, a second record's header line, a line
longer than the reference loader's 255-byte fgets pieces -- indexed by the
REFERENCE's own builder (oracle/_ref/gfmi_<K>_<d>, compiled from
/root/reference sources by oracle/Makefile), transformed by its tfmiBMP /
tfmiAC, and searched by its CPU searchers (cpu_/cpuac_).  Outputs are data;
no reference source is stored.

K = 1 output is a function of the file.  For K >= 2 the reference's LF walk
(genFMindex.c:327-400) never writes some rows of BWT_1.. when the text has
bytes other than A/C/G/T, so those rows hold uninitialised malloc memory; the
builder is therefore run under glibc's MALLOC_PERTURB_=p, which fills fresh
allocations with p ^ 0xff -- the byte our builders take as KFMI_REF_FILL.
Two perturb values are recorded to show the dependence.

Run in the dev container (needs /root/reference for make -C oracle ref):
    make -C oracle ref && python3 tests/golden/make_golden_alpha.py
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = REPO / "oracle" / "_ref"
OUT = HERE / "alpha"

# (K, d, MALLOC_PERTURB_ value or None); files are committed for the first
# perturb value of each (K, d), md5s only for the others
BUILDS = [(1, 64, None), (1, 192, None), (2, 64, 85), (2, 64, 170), (2, 192, 85), (4, 64, 85)]
COMMIT = {(1, 64, None), (1, 192, None), (2, 64, 85), (2, 192, 85)}


def read_ref_exact(fasta: bytes, refsize: int) -> bytes:
    """The reference's readRef (common/common.c:42-76): fgets pieces of at most
    255 bytes; after the first line every piece gives strlen - 1 bytes."""
    pieces = []
    for line in fasta.split(b"\n")[:-1] if fasta.endswith(b"\n") else fasta.split(b"\n"):
        raw = line + b"\n"
        while raw:
            pieces.append(raw[:255])
            raw = raw[255:]
    # the first piece is the header line's first piece; the header is < 255 bytes here
    out = bytearray()
    for p in pieces[1:]:
        s = p.split(b"\0")[0]
        take = s[:len(s) - 1] if s else b""
        out += take[:refsize - len(out)]
        if len(out) >= refsize:
            break
    return bytes(out)


def make_fasta(rng: random.Random) -> bytes:
    def acgt(n):
        return "".join(rng.choice("ACGT") for _ in range(n))
    rec1 = (acgt(8000) + "N" * 300 + acgt(5000) + acgt(1500).lower() + "n" * 50 + acgt(1450).lower()
            + "".join(rng.choice("RYKMSWBDHV") for _ in range(200)) + acgt(3000))
    rec2 = acgt(6000) + "N" * 77 + acgt(4000)
    lines = [">chr1 synthetic record with N runs, soft-masked and IUPAC letters"]
    lines += [rec1[i:i + 60] for i in range(0, 6000, 60)]
    lines.append(rec1[6000:6300])              # one 300-byte line: two fgets pieces
    lines += [rec1[i:i + 60] for i in range(6300, len(rec1), 60)]
    lines.append(">chr2 second record")        # readRef copies header lines into the text
    lines += [rec2[i:i + 60] for i in range(0, len(rec2), 60)]
    return ("\n".join(lines) + "\n").encode()


def reads(text: bytes, m: int, rng: random.Random) -> list[bytes]:
    n = len(text)
    out = []
    for _ in range(300):
        s = rng.randint(0, n - m)
        out.append(text[s:s + m])
    # windows over the N run, the lowercase stretch, the IUPAC letters, the header bytes
    for anchor in (b"NNNN", b"nnnn", b"chr2", b"RY", b"YK", b"acg"):
        i = text.find(anchor)
        if i >= 0:
            for off in range(-m + 4, 1, max(1, m // 6)):
                s = min(max(0, i + off), n - m)
                out.append(text[s:s + m])
    out += [bytes(rng.choice(b"ACGT") for _ in range(m)) for _ in range(40)]
    out += [b"N" * m, b"A" * m, bytes(rng.choice(b"ACGTNacgtnRY") for _ in range(m))]
    out += [text[:m], text[n - m:]]
    return [r for r in out if len(r) == m]


def run(cmd, cwd, env=None):
    p = subprocess.run([str(c) for c in cmd], cwd=cwd, capture_output=True, text=True, env=env)
    if p.returncode != 0:
        raise RuntimeError(f"{cmd} failed: {p.stdout[-400:]} {p.stderr[-400:]}")
    return p.stdout


def md5(p: Path) -> str:
    return hashlib.md5(p.read_bytes()).hexdigest()


def main() -> int:
    if not (REF / "gfmi_2_64").exists():
        print("build the reference tools first: make -C oracle ref", file=sys.stderr)
        return 1
    rng = random.Random(20261017)
    fa = make_fasta(rng)
    text = read_ref_exact(fa, 1 << 40)
    n = len(text)
    assert (n + 1) % 64 and (n + 1) % 192, n
    if OUT.exists():
        shutil.rmtree(OUT)
    OUT.mkdir(parents=True)
    (OUT / "ref.fa").write_bytes(fa)
    qsets = {100: reads(text, 100, rng), 12: reads(text, 12, rng)}
    man = {"n": n, "text_md5": hashlib.md5(text).hexdigest(), "queries": {}, "indexes": {}}
    for m, rs in qsets.items():
        (OUT / f"q{m}.qry").write_bytes(b"".join(b">r%d\n%s\n" % (i, r) for i, r in enumerate(rs)))
        man["queries"][str(m)] = {"file": f"q{m}.qry", "num": len(rs)}
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        shutil.copy(OUT / "ref.fa", td / "ref.fa")
        for m in qsets:
            shutil.copy(OUT / f"q{m}.qry", td / f"q{m}.qry")
        for k, d, pert in BUILDS:
            env = dict(os.environ)
            env.pop("MALLOC_PERTURB_", None)
            if pert is not None:
                env["MALLOC_PERTURB_"] = str(pert)
            for f in td.glob("ref.fa.*"):
                f.unlink()
            run([REF / f"gfmi_{k}_{d}", "ref.fa", n], td, env)
            base = f"ref.fa.{n}.{d}fmi{k}steps.fmi"
            key = f"k{k}_d{d}" + (f"_p{pert}" if pert is not None else "")
            ent = {"k": k, "d": d, "perturb": pert, "fill": (pert ^ 0xFF) if pert is not None else None,
                   "md5": {"100": md5(td / base)}, "files": {}, "results": {}}
            keep = (k, d, pert) in COMMIT
            if keep:
                tools = [(REF / f"tfmiBMP_{k}_{d}", [(101, base + ".interleaving")]),
                         (REF / f"tfmiAC_{k}_{d}", [(200, base + ".ac"), (201, base + ".interleaving.ac")])]
                files = {100: base}
                for tool, outs in tools:
                    if tool.exists():
                        run([tool, base], td)
                        files.update(dict(outs))
                for tag, fn in files.items():
                    dst = f"{key}.{tag}.fmi"
                    shutil.copy(td / fn, OUT / dst)
                    ent["files"][str(tag)] = {"file": dst, "md5": md5(OUT / dst)}
                    ent["md5"][str(tag)] = md5(OUT / dst)
            for m, rs in qsets.items():
                if m % k:
                    continue
                for tool, tag in (("cpu", 100), ("cpuac", 200)):
                    exe = REF / f"{tool}_{k}_{d}"
                    if not exe.exists() or (tag == 200 and 200 not in {int(t) for t in ent["files"]}):
                        continue
                    fn = base if tag == 100 else base + ".ac"
                    run([exe, fn, f"q{m}.qry", m, len(rs)], td)
                    resname = f"{key}.q{m}.{tool}.res"
                    shutil.copy(td / (fn + ".res.cpu"), OUT / resname)
                    ent["results"][f"{m}.{tag}"] = {"file": resname, "md5": md5(OUT / resname)}
            man["indexes"][key] = ent
    (OUT / "alpha.json").write_text(json.dumps(man, indent=1, sort_keys=True) + "\n")
    print("wrote", OUT / "alpha.json", "n =", n)
    return 0


if __name__ == "__main__":
    sys.exit(main())
