"""Damaged query files through the device parser (kfmi_load_queries_gpu)
against the host's mapped loadQueries: valid files with random bytes flipped
or cut, and files of junk bytes mostly from ">\\n\\rACGTNacgt", 0-300 KB (so
they cross the parser's 64 KiB tiles), random read lengths and limits.  The
device must return what the host returns: the same error code, or reads whose
search results equal the host reads'.

usage: python3 scripts/diag/ingest_junk.py SECONDS"""
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "k-step_fm-index_amd"))
sys.path.insert(0, str(REPO / "tests"))
import kstep_fmi as K  # noqa: E402
from test_ingest import load, search_loaded  # noqa: E402

ALPHA = np.frombuffer(b">\n\r\nACGTNacgt", np.uint8)


def junk(rng):
    kind = int(rng.integers(0, 3))
    m = int(rng.choice([1, 2, 3, 4, 17, 64, 100, 150, 255]))
    limit = int(rng.integers(1, 3000))
    if kind == 0:
        size = int(rng.integers(0, 300_000))
        body = ALPHA[rng.integers(0, ALPHA.size, size=size)]
        sel = rng.random(size) < 0.01
        body[sel] = rng.integers(0, 256, size=int(sel.sum()))
        return m, limit, body.tobytes(), kind
    nreads = int(rng.integers(1, 4000))
    reads = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, size=(nreads, m))]
    lines = []
    for j in range(nreads):
        if rng.random() < 0.5:
            lines.append(b">r%d" % j)
        lines.append(reads[j].tobytes())
    body = bytearray(b"\n".join(lines) + b"\n")
    if kind == 1:   # flips
        for p in rng.integers(0, len(body), size=int(rng.integers(1, 20))):
            body[p] = int(rng.choice(ALPHA))
    else:           # a cut, maybe mid-line
        body = body[:int(rng.integers(0, len(body) + 1))]
    return m, limit, bytes(body), kind


def main():
    limit_s = float(sys.argv[1]) if len(sys.argv) > 1 else 120
    K.set_device(0)
    rng0 = np.random.default_rng(17)
    text = rng0.choice(np.frombuffer(b"ACGT", np.uint8), size=100_001).tobytes()
    idx = K.Index.build(text, k=2, d=64, gpu=True)
    t0 = time.time()
    w = bad = loaded = 0
    with tempfile.TemporaryDirectory() as td:
        path = Path(td) / "q.fa"
        while time.time() - t0 < limit_s:
            rng = np.random.default_rng(930_000 + w)
            m, limit, body, kind = junk(rng)
            path.write_bytes(body)
            try:
                host = load(K, path, m, limit)
            except K.KfmiError as e:
                host = e.code
            try:
                dev = K.Queries.load_gpu(path, m, limit)
            except K.KfmiError as e:
                dev = e.code
            if isinstance(host, int) or isinstance(dev, int):
                if host != dev:
                    bad += 1
                    print(f"MISMATCH file {w} kind={kind} m={m} limit={limit} bytes={len(body)}: "
                          f"host {host if isinstance(host, int) else 'reads'} device "
                          f"{dev if isinstance(dev, int) else 'reads'}", flush=True)
                if not isinstance(dev, int):
                    dev.close()
            else:
                loaded += 1
                got = search_loaded(K, idx, dev)
                dev.close()
                want = K.search_array(idx, host, "task-mid") if host.shape[0] else np.zeros(0, np.uint32)
                if not np.array_equal(got, want):
                    bad += 1
                    print(f"MISMATCH file {w} kind={kind} m={m} limit={limit}: reads differ", flush=True)
            w += 1
            if w % 100 == 0:
                print(f"{w} files, {loaded} loaded, {bad} bad, {time.time() - t0:.0f}s", flush=True)
    idx.close()
    print(f"done: {w} files, {loaded} loaded, {bad} bad", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
