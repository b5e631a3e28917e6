"""Generate tests/golden/*.json (run in the build container only).

Inputs: the reference's own fuzz corpora (/root/reference/testdata/fuzz,
Go "go test fuzz v1" files — data, parsed here) and seeded synthetic streams.
Expected outputs: computed with tests/pyoracle.py, the independent Python
restatement of writer.go / reader.go.  The committed fixtures are then
checked against the C oracle (tests/test_oracle_kat.py) and the GPU path
(tests/test_gpu_*.py); neither needs /root/reference at run time.

    python tests/golden/make_golden.py
"""

from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

import pyoracle as P  # noqa: E402

REF = "/root/reference/testdata/fuzz"


def _unquote_go(s: str) -> bytes:
    """Decode the body of a Go %q string literal (UTF-8 text + escapes)."""
    out = bytearray()
    i = 0
    simple = {"a": 7, "b": 8, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11, "\\": 92, '"': 34, "'": 39}
    while i < len(s):
        c = s[i]
        if c != "\\":
            out += c.encode()
            i += 1
            continue
        e = s[i + 1]
        if e in simple:
            out.append(simple[e])
            i += 2
        elif e == "x":
            out.append(int(s[i + 2 : i + 4], 16))
            i += 4
        elif e in "01234567":
            out.append(int(s[i + 1 : i + 4], 8))
            i += 4
        elif e == "u":
            out += chr(int(s[i + 2 : i + 6], 16)).encode()
            i += 6
        elif e == "U":
            out += chr(int(s[i + 2 : i + 10], 16)).encode()
            i += 10
        else:
            raise ValueError(f"escape \\{e}")
    return bytes(out)


def parse_corpus(path: str) -> list[bytes]:
    lines = open(path, encoding="utf-8").read().splitlines()
    assert lines[0] == "go test fuzz v1", path
    vals = []
    for ln in lines[1:]:
        if not ln.strip():
            continue
        assert ln.startswith('[]byte("') and ln.endswith('")'), ln
        vals.append(_unquote_go(ln[len('[]byte("') : -2]))
    return vals


def read_all(b: bytes, buf: int, limit: int = 1 << 16):
    """NewReader(BufReader{b}) (BlockSizeLimit 16 MiB, as FuzzReader uses,
    eazy_test.go:1375-1376) read with a `buf`-byte buffer until a terminal
    error or `limit` output bytes -> {"out": hex, "errs": [err per Read]}."""
    r = P.Reader(src=b)
    out, errs = bytearray(), []
    while len(out) < limit:
        got, err = r.read(buf)
        out += got
        errs.append(err)
        if err not in (P.OK, P.EBREAK):
            break
    return {"out": bytes(out[:limit]).hex(), "errs": errs}


def main():
    fixtures = {}
    # FuzzWriter corpus (eazy_test.go:1295-1362): 3 Writes into NewWriter(512, 32)
    fw = []
    for name in sorted(os.listdir(os.path.join(REF, "FuzzWriter"))):
        writes = parse_corpus(os.path.join(REF, "FuzzWriter", name))
        ent = {"name": name, "writes": [w.hex() for w in writes]}
        for block, ht in ((512, 32), (1 << 20, 1024)):
            ent[f"stream_{block}_{ht}"] = P.compress(block, ht, writes).hex()
            ent[f"single_{block}_{ht}"] = [P.compress(block, ht, [w]).hex() for w in writes]
        fw.append(ent)
    fixtures["fuzz_writer"] = fw
    # FuzzReader corpus (eazy_test.go:1364-1385): decoding must not crash; pin
    # the bytes and errors of NewReader(p) read with 16- and 4096-byte buffers.
    fr = []
    for name in sorted(os.listdir(os.path.join(REF, "FuzzReader"))):
        (p,) = parse_corpus(os.path.join(REF, "FuzzReader", name))
        fr.append({"name": name, "input": p.hex(), "read16": read_all(p, 16), "read4096": read_all(p, 4096)})
    # the FuzzReader seeds themselves (eazy_test.go:1367-1372)
    seeds = [
        bytes([0x03, 97, 98, 99]),
        bytes([0x03, 97, 98, 99, 0x83, 0]),
        bytes([0x80, 0x08, 1]),
        bytes([0x80, 0x10, 6]),
        bytes([0x80, 0x08, 1, 0x80, 0x10, 6, 0x03, 97, 98, 99]),
        bytes([0x80, 0x08, 1, 0x80, 0x10, 6, 0x03, 97, 98, 99, 0x83, 0]),
        bytes([0x80, 0x10, 6, 0x03, 97, 98, 99, 0x83, 0]),
        bytes([0x80, 0x10, 6, 0x03, 97, 98, 99, 0x80, 0x1F, 0x83, 2]),
    ]
    for k, p in enumerate(seeds):
        fr.append({"name": f"seed{k}", "input": p.hex(), "read16": read_all(p, 16), "read4096": read_all(p, 4096)})
    fixtures["fuzz_reader"] = fr
    # seeded synthetic log-like streams (one Write each) at the BASELINE block/table
    from eazy_amd import synth

    d = synth.logs(42, 6 * 4096 + 3 * 16384).tobytes()
    bufs = [d[k * 4096 : (k + 1) * 4096] for k in range(6)]
    bufs += [d[6 * 4096 + k * 16384 : 6 * 4096 + (k + 1) * 16384] for k in range(3)]
    syn = []
    for k, b in enumerate(bufs):
        ent = {"input": b.hex()}
        for block, ht in ((1 << 20, 1024), (1 << 17, 1024), (1024, 32)):
            ent[f"stream_{block}_{ht}"] = P.compress(block, ht, [b]).hex()
        syn.append(ent)
    fixtures["synthetic_logs"] = syn
    # a multi-Write stream (k = 4, carried window) for the Writer handle
    fixtures["multi_write"] = {
        "writes": [b.hex() for b in bufs[:4]],
        "stream_1048576_1024": P.compress(1 << 20, 1024, bufs[:4]).hex(),
        "stream_2048_64": P.compress(2048, 64, bufs[:4]).hex(),
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(fixtures, f, indent=0, sort_keys=True)
    print("wrote", os.path.join(HERE, "golden.json"), os.path.getsize(os.path.join(HERE, "golden.json")), "bytes")


if __name__ == "__main__":
    main()
