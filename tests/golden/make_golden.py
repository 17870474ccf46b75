#!/usr/bin/env python3
"""Generate tests/golden/* from the reference's OWN test data (run in the build container only;
the GPU box has no /root/reference and only reads the committed outputs).

What is extracted (paths relative to bearcove/loona @ 2025-05-09, read as text/data):
  huffman_table.json   the 257 (code, len) pairs        crates/loona-hpack/src/huffman.rs:222-480
  static_table.json    HPACK static table (61 entries)  crates/loona-hpack/src/lib.rs:293-355
  kat.json             huffman.rs unit-test vectors      crates/loona-hpack/src/huffman.rs:523-707
  rfc7541_blocks.json  App. C.3-C.6 header-block sequences and block-level error cases
                                                         crates/loona-hpack/src/decoder.rs:957-1508
  interop.json.gz      every http2jp interop story (wire hex + decoded header list)
                                                         crates/loona-hpack/fixtures/hpack/interop/*
  interop_digest.json  literal counts, byte totals and sha256 of the concatenated Huffman
                       literals (encoded and decoded) over the whole corpus
  error_vectors.json   seeded random byte strings labelled by the pure-Python restatement
                       (oracle/hpack_ref.py) — checked against the C oracle by the tests

Nothing here copies reference source: only the vectors and tables its tests hold.
Every vector is re-verified against oracle/hpack_ref.py before it is written.
"""

import gzip
import hashlib
import json
import os
import random
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference/crates/loona-hpack"
sys.path.insert(0, os.path.join(REPO, "oracle"))


def write_json(name, obj, gz=False):
    path = os.path.join(HERE, name)
    data = json.dumps(obj, indent=None if gz else 1, sort_keys=False).encode()
    if gz:
        with gzip.GzipFile(path, "wb", compresslevel=9, mtime=0) as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data + b"\n")
    print("wrote", name, os.path.getsize(path), "bytes")


def extract_table():
    src = open(os.path.join(REF, "src/huffman.rs")).read()
    start = src.index("static HUFFMAN_CODE_TABLE")
    ents = re.findall(r"\((0x[0-9a-f]+),\s*(\d+)\)", src[start : start + 20000])[:257]
    return [[int(c, 16), int(n)] for c, n in ents]


def extract_static_table():
    src = open(os.path.join(REF, "src/lib.rs")).read()
    start = src.index("static STATIC_TABLE")
    body = src[start : src.index("];", start)]
    pairs = re.findall(r'\(b"([^"]*)",\s*b"([^"]*)"\)', body)
    assert len(pairs) == 61, len(pairs)
    return [list(p) for p in pairs]


# huffman.rs unit tests (input bytes -> expected). status: 0 ok, 1 PaddingTooLarge,
# 2 InvalidPadding, 3 EOSInString (hpk.h / huffman.rs:28-41).
KATS = [
    ([(0x7 << 3) + 7], b"o", 0, "huffman.rs:529-537"),
    ([0x0 + 7], b"0", 0, "huffman.rs:538-546"),
    ([(0x21 << 2) + 3], b"A", 0, "huffman.rs:547-555"),
    ([255, 160 + 15], b"#", 0, "huffman.rs:566-573"),
    ([255, 200 + 7], b"$", 0, "huffman.rs:574-581"),
    ([255, 255, 255, 240 + 3], bytes([10]), 0, "huffman.rs:582-589"),
    ([254, 1], b"!0", 0, "huffman.rs:595-602"),
    ([(0x14 << 2) | 0x3, 248], b" !", 0, "huffman.rs:603-610"),
    ([0xFF, 0xFF, 0xFF, 0xFF], None, 3, "huffman.rs:618-630"),
    ([0x3F, 0xFF, 0xFF, 0xFF, 0xFF], None, 3, "huffman.rs:631-644"),
    ([0x3F], b"o", 0, "huffman.rs:649-657"),
    ([0x3F, 0xFF], None, 1, "huffman.rs:660-674"),
    ([0x3E], None, 2, "huffman.rs:681-692"),
    ([254, 0], None, 2, "huffman.rs:693-706"),
]


def extract_rfc_blocks():
    """The four App. C sequence tests: each block's hex_dump + expected header list."""
    src = open(os.path.join(REF, "src/decoder.rs")).read()
    seqs = []
    for fn, line in [
        ("fn test_request_sequence_no_huffman", 957),
        ("fn response_sequence_no_huffman", 1045),
        ("fn request_sequence_huffman", 1217),
        ("fn response_sequence_huffman", 1304),
    ]:
        start = src.index(fn)
        end = src.index("\n    }\n", start)
        body = src[start:end]
        max_size = None
        m = re.search(r"set_max_table_size\((\d+)\)", body)
        if m:
            max_size = int(m.group(1))
        blocks = []
        for hm in re.finditer(r"let hex_dump = \[(.*?)\];", body, re.S):
            hexes = re.findall(r"0x([0-9a-fA-F]{2})", hm.group(1))
            wire = bytes(int(h, 16) for h in hexes)
            after = body[hm.end() :]
            am = re.search(r"assert_eq!\(\s*header_list,\s*\[(.*?)\]\s*\);", after, re.S)
            if am is None or "let hex_dump" in after[: am.start()]:
                am = re.search(r"let expected_header_list = \[(.*?)\];", after, re.S)
            hdrs = re.findall(r'\(\s*b"([^"]*)"\.to_vec\(\),\s*b"([^"]*)"\.to_vec\(\),?\s*\)', am.group(1))
            blocks.append({"wire": wire.hex(), "headers": [list(h) for h in hdrs]})
        seqs.append({"ref": "decoder.rs:%d" % line, "name": fn.split()[-1], "max_table_size": max_size, "blocks": blocks})
    # block-level error cases (decoder.rs:1417-1508)
    errors = [
        {"ref": "decoder.rs:1451-1465", "wire": bytes([0x82, 0x86, 0x84, 0x41, 0x8C, 0xF1, 0xE3, 0xC2, 0xE5, 0xF2, 0x3A, 0x6B,
                                                       0xA0, 0xAB, 0x90, 0xF4, 0xFE]).hex(),
         "error": ["StringDecodingError", "HuffmanDecoderError", 2]},
        {"ref": "decoder.rs:1425", "wire": "80", "error": ["HeaderIndexOutOfBounds"]},
        {"ref": "decoder.rs:1430", "wire": "be", "error": ["HeaderIndexOutOfBounds"]},
        {"ref": "decoder.rs:1433", "wire": bytes([126, 1, 65]).hex(), "error": ["HeaderIndexOutOfBounds"]},
        {"ref": "decoder.rs:1470-1488", "wire": (bytes([0x40, 0x0A]) + b"custom-ke").hex(),
         "error": ["StringDecodingError", "NotEnoughOctets"]},
        {"ref": "decoder.rs:1491-1507", "wire": (bytes([0x40, 0x0A]) + b"custom-key").hex(),
         "error": ["IntegerDecodingError", "NotEnoughOctets"]},
    ]
    return seqs, errors


def load_interop():
    base = os.path.join(REF, "fixtures/hpack/interop")
    out = {}
    for enc in sorted(os.listdir(base)):
        stories = []
        for fn in sorted(os.listdir(os.path.join(base, enc))):
            j = json.load(open(os.path.join(base, enc, fn)))
            cases = []
            for c in j["cases"]:
                hs = [[k, v] for h in c["headers"] for k, v in h.items()]
                cases.append({"wire": c["wire"], "headers": hs})
            stories.append({"file": "%s/%s" % (enc, fn), "cases": cases})
        out[enc] = stories
    return out


def main():
    import hpack_ref as R

    table = extract_table()
    assert [list(t) for t in R.TABLE] == table, "oracle table != reference table"
    write_json("huffman_table.json", {"ref": "crates/loona-hpack/src/huffman.rs:222-480", "table": table})

    static = extract_static_table()
    write_json("static_table.json", static)

    kats = []
    for inp, exp, st, ref in KATS:
        got_st, got = R.huffman_decode(bytes(inp))
        assert got_st == st, (inp, got_st, st)
        if st == 0:
            assert got == exp, (inp, got, exp)
        kats.append({"in": bytes(inp).hex(), "status": st, "out": None if exp is None else exp.hex(),
                     "ref": "crates/loona-hpack/src/" + ref})
    write_json("kat.json", kats)

    seqs, errors = extract_rfc_blocks()
    for seq in seqs:
        d = R.Decoder()
        if seq["max_table_size"] is not None:
            d.dynamic.set_max_table_size(seq["max_table_size"])
        for b in seq["blocks"]:
            got = [[n.decode(), v.decode()] for n, v in d.decode(bytes.fromhex(b["wire"]))]
            assert got == b["headers"], (seq["name"], got, b["headers"])
    for e in errors:
        try:
            R.Decoder().decode(bytes.fromhex(e["wire"]))
            raise AssertionError("expected error")
        except R.DecoderError as err:
            kind = [err.kind]
            if err.detail is not None:
                kind += list(err.detail) if isinstance(err.detail, tuple) else [err.detail]
            assert kind == e["error"], (kind, e)
    # the 12 Huffman literals of App. C.4/C.6
    lits = []
    for seq in seqs:
        if "huffman" not in seq["name"]:
            continue
        for b in seq["blocks"]:
            w = bytes.fromhex(b["wire"])
            for s, e in R.huffman_literal_spans(w):
                st, out = R.huffman_decode(w[s:e])
                assert st == 0
                lits.append({"in": w[s:e].hex(), "out": out.hex(), "ref": seq["ref"]})
    write_json("rfc7541_blocks.json", {"sequences": seqs, "errors": errors, "huffman_literals": lits})

    inter = load_interop()
    n_lit = enc_b = dec_b = 0
    h_enc, h_dec = hashlib.sha256(), hashlib.sha256()
    per_enc = {}
    for enc, stories in inter.items():
        cnt = 0
        for story in stories:
            d = R.Decoder()
            for c in story["cases"]:
                w = bytes.fromhex(c["wire"])
                got = [[n.decode("utf-8"), v.decode("utf-8")] for n, v in d.decode(w)]
                assert got == c["headers"], story["file"]
                for s, e in R.huffman_literal_spans(w):
                    st, out = R.huffman_decode(w[s:e])
                    assert st == 0
                    # canonical re-encode reproduces the wire literal (encode parity)
                    assert R.huffman_encode(out) == w[s:e], story["file"]
                    n_lit += 1
                    cnt += 1
                    enc_b += e - s
                    dec_b += len(out)
                    h_enc.update(w[s:e])
                    h_dec.update(out)
        per_enc[enc] = cnt
    write_json("interop.json.gz", inter, gz=True)
    write_json("interop_digest.json", {
        "ref": "crates/loona-hpack/fixtures/hpack/interop (decoder.rs:1661-1717)",
        "huffman_literals": n_lit, "encoded_bytes": enc_b, "decoded_bytes": dec_b,
        "per_encoder_literals": per_enc,
        "sha256_encoded": h_enc.hexdigest(), "sha256_decoded": h_dec.hexdigest(),
    })

    # error-path vectors: seeded random byte strings, labelled by the restatement
    rng = random.Random(7541)
    vecs = []
    for i in range(3000):
        n = rng.choice([0, 1, 1, 2, 2, 3, 3, 4, 5, 6, 7, 8, 12, 16, 31, 64])
        mode = rng.random()
        if mode < 0.3:
            b = bytes(rng.getrandbits(8) for _ in range(n))
        elif mode < 0.6:  # valid literal with the tail perturbed
            txt = bytes(rng.getrandbits(8) if rng.random() < 0.2 else rng.choice(b"abcdefghijklmnop0123456789-/.=")
                        for _ in range(n))
            b = bytearray(R.huffman_encode(txt))
            if b:
                b[-1] ^= 1 << rng.randrange(8)
            b = bytes(b)
        elif mode < 0.8:  # long runs of ones (EOS / padding edge cases)
            b = bytes([0xFF] * n) + bytes([rng.choice([0xFF, 0xFE, 0x7F, 0x3F, 0x00])])
        else:
            txt = bytes(rng.getrandbits(8) for _ in range(n))
            b = R.huffman_encode(txt) + bytes([0xFF] * rng.randrange(0, 5))
        st, out = R.huffman_decode(b)
        vecs.append({"in": b.hex(), "status": st, "out": out.hex()})
    write_json("error_vectors.json", {"seed": 7541, "labelled_by": "oracle/hpack_ref.py", "vectors": vecs})


if __name__ == "__main__":
    main()
