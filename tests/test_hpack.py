"""HPACK header blocks through the two-pass decoder (hpk_hdec_*) on the CPU batch
path: the reference's own block vectors (RFC 7541 App. C sequences and error cases,
decoder.rs:957-1507; the interop stories, decoder.rs:1661-1717 — every story through one
decoder, all stories in ONE batch call) and seeded corruptions checked against the Python
restatement of decoder.rs (oracle/hpack_ref.py). GPU variants live in test_gpu.py."""

import random

import pytest

from hpk_util import hpack_ref, load

from loona_amd import hpack


def _ref_decode(dec, wire):
    try:
        return dec.decode(wire)
    except hpack_ref.DecoderError as e:
        return hpack.DecoderError(e.kind, e.detail)


def test_static_table_matches_reference():
    g = load("static_table.json")
    d = hpack.Decoder()
    got = d.decode(bytes(0x80 | i for i in range(1, 62)))
    assert [[n.decode(), v.decode()] for n, v in got] == g
    with pytest.raises(hpack.DecoderError) as ei:
        hpack.Decoder().decode(bytes([0x80 | 62]))
    assert ei.value.kind == "HeaderIndexOutOfBounds"


def test_rfc7541_sequences_and_errors():
    g = load("rfc7541_blocks.json")
    for seq in g["sequences"]:
        d = hpack.Decoder()
        if seq["max_table_size"] is not None:
            d.set_max_table_size(seq["max_table_size"])
        for b in seq["blocks"]:
            got = [[n.decode(), v.decode()] for n, v in d.decode(bytes.fromhex(b["wire"]))]
            assert got == b["headers"], seq["name"]
    for e in g["errors"]:
        with pytest.raises(hpack.DecoderError) as ei:
            hpack.Decoder().decode(bytes.fromhex(e["wire"]))
        det = ei.value.detail
        kind = [ei.value.kind] + ([] if det is None else list(det) if isinstance(det, tuple) else [det])
        assert kind == e["error"], e["ref"]


def _stories():
    inter = load("interop.json.gz")
    for enc in sorted(inter):
        for story in inter[enc]:
            yield enc, story


def test_interop_stories_one_batch():
    """All 5 encoders' stories, one decoder per story, every block of every story in one call."""
    pairs, want = [], []
    for enc, story in _stories():
        d = hpack.Decoder()
        for c in story["cases"]:
            pairs.append((d, bytes.fromhex(c["wire"])))
            want.append([(n.encode(), v.encode()) for n, v in c["headers"]])
    got = hpack.decode_blocks(pairs)
    assert len(got) == len(want) > 16000
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, i


def test_interop_stories_any_thread_count(monkeypatch):
    """The same batch on 1, 3 and 16 host threads: decoders are placed on the apply threads by hash
    buckets balanced on the scanned work (hpk_hpack.cpp), each decoder's blocks in order on one
    thread, so every count gives the reference's headers."""
    pairs, want = [], []
    stories = list(_stories())
    for nth in ("1", "3", "16"):
        monkeypatch.setenv("HPK_HDEC_THREADS", nth)
        pairs, want = [], []
        for enc, story in stories:
            d = hpack.Decoder()
            for c in story["cases"]:
                pairs.append((d, bytes.fromhex(c["wire"])))
                want.append([(n.encode(), v.encode()) for n, v in c["headers"]])
        got = hpack.decode_blocks(pairs)
        assert got == want, nth


def test_table_size_update_and_eviction():
    d = hpack.Decoder()
    # literal with incremental indexing, new name: 'custom-key: custom-header' (RFC 7541 C.2.1)
    blk = bytes.fromhex("400a637573746f6d2d6b65790d637573746f6d2d686561646572")
    assert d.decode(blk) == [(b"custom-key", b"custom-header")]
    assert d.table_size() == (55, 1, 4096)
    assert d.decode(bytes([0x80 | 62])) == [(b"custom-key", b"custom-header")]
    # size update to 0 then an indexed static field: evicts everything
    assert d.decode(bytes([0x20, 0x82])) == [(b":method", b"GET")]
    assert d.table_size() == (0, 0, 0)
    with pytest.raises(hpack.DecoderError) as ei:
        d.decode(bytes([0x3F, 0xE1, 0x1F]))  # size update 4096 at the end of the block
    assert ei.value.kind == "SizeUpdateAtEnd"
    d2 = hpack.Decoder()
    d2.set_max_allowed_table_size(100)
    with pytest.raises(hpack.DecoderError) as ei:
        d2.decode(bytes([0x3F, 0xE1, 0x1F, 0x82]))
    assert ei.value.kind == "InvalidMaxDynamicSize"


def _mutate(rng, w):
    w = bytearray(w)
    op = rng.randrange(4)
    if op == 0 and w:
        w[rng.randrange(len(w))] ^= 1 << rng.randrange(8)
    elif op == 1 and w:
        del w[rng.randrange(len(w)) :]
    elif op == 2:
        w[rng.randrange(len(w) + 1) : 0] = bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 6)))
    else:
        for _ in range(rng.randrange(1, 4)):
            if w:
                w[rng.randrange(len(w))] = rng.getrandbits(8)
    return bytes(w)


def test_corrupted_stories_match_restatement():
    """Seeded corruptions of interop stories (bit flips, truncations, insertions, random bytes):
    per block, headers or the first error equal decoder.rs's restatement, with the dynamic table
    carried across the blocks of a story exactly as the reference's decoder carries it."""
    rng = random.Random(7541)
    stories = [s for _, s in _stories()]
    pairs, want = [], []
    for story in rng.sample(stories, 40):
        d, r = hpack.Decoder(), hpack_ref.Decoder()
        for c in story["cases"][:12]:
            w = bytes.fromhex(c["wire"])
            if rng.random() < 0.5:
                w = _mutate(rng, w)
            pairs.append((d, w))
            want.append(_ref_decode(r, w))
    got = hpack.decode_blocks(pairs)
    errs = sum(isinstance(x, hpack.DecoderError) for x in want)
    assert errs > 20
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, pairs[i][1].hex())


def test_random_blocks_match_restatement():
    rng = random.Random(11)
    pairs, want = [], []
    for _ in range(3000):
        w = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 24)))
        pairs.append((hpack.Decoder(), w))
        want.append(_ref_decode(hpack_ref.Decoder(), w))
    got = hpack.decode_blocks(pairs)
    kinds = {(x.kind, x.detail if not isinstance(x.detail, tuple) else x.detail[0]) for x in want
             if isinstance(x, hpack.DecoderError)}
    assert len(kinds) >= 5
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, pairs[i][1].hex())


def test_httpwg_invalid_header_block_fragment():
    """httpwg's `invalid_header_block_fragment` (crates/httpwg/src/rfc9113/_4_http_frames.rs:153-170)
    sends the block b"\\x40" (literal with incremental indexing, no name length) and expects
    COMPRESSION_ERROR, which loona raises for any DecoderError (h2/server.rs:1621-1634,
    h2/types.rs:366-367). The error itself must equal decoder.rs's."""
    want = _ref_decode(hpack_ref.Decoder(), b"\x40")
    assert isinstance(want, hpack.DecoderError)
    with pytest.raises(hpack.DecoderError) as ei:
        hpack.Decoder().decode(b"\x40")
    assert ei.value == want
    assert hpack.decode_blocks([(hpack.Decoder(), b"\x40")]) == [want]


def test_every_truncation_of_rfc_blocks():
    """Every proper prefix of every RFC 7541 App. C block, decoded with the table state the
    sequence had built so far: headers or the first error equal the restatement's."""
    g = load("rfc7541_blocks.json")
    pairs, want = [], []
    for seq in g["sequences"]:
        for k, b in enumerate(seq["blocks"]):
            w = bytes.fromhex(b["wire"])
            for cut in range(len(w)):
                d, r = hpack.Decoder(), hpack_ref.Decoder()
                if seq["max_table_size"] is not None:
                    d.set_max_table_size(seq["max_table_size"])
                    r.set_max_table_size(seq["max_table_size"])
                for prev in seq["blocks"][:k]:
                    d.decode(bytes.fromhex(prev["wire"]))
                    r.decode(bytes.fromhex(prev["wire"]))
                pairs.append((d, w[:cut]))
                want.append(_ref_decode(r, w[:cut]))
    got = hpack.decode_blocks(pairs)
    assert sum(isinstance(x, hpack.DecoderError) for x in want) > 50
    for i, (gg, ww) in enumerate(zip(got, want)):
        assert gg == ww, (i, pairs[i][1].hex())


def test_dynamic_table_churn_matches_restatement():
    """Long runs of insertions, lookups, evictions and size updates through one decoder per stream,
    all blocks in one call: the table's entry ring grows past its first 64 slots and its byte buffer
    is compacted many times (hpk_hdec's allocation-free table); every block's headers or first error
    equal decoder.rs's restatement (oracle/hpack_ref.py)."""
    rng = random.Random(4096)
    pairs, want = [], []
    for stream in range(6):
        d, r = hpack.Decoder(), hpack_ref.Decoder()
        entries = 0
        for _ in range(120):
            blk = bytearray()
            if rng.random() < 0.15:  # dynamic table size update (decoder.rs:538-554)
                blk += hpack_ref.encode_integer(rng.choice([0, 100, 4096, 20000, 60000]), 5, 0x20)
            for _ in range(rng.randrange(1, 24)):
                op = rng.random()
                if op < 0.55:  # literal with incremental indexing, new name
                    nl = rng.choice([0, 1, 5, 12, 40, rng.randrange(0, 300)])
                    vl = rng.choice([0, 3, 20, 100, rng.randrange(0, 5000)])
                    blk += b"\x40" + hpack_ref.encode_integer(nl, 7, 0) + bytes(rng.randrange(97, 123) for _ in range(nl))
                    blk += hpack_ref.encode_integer(vl, 7, 0) + bytes(rng.randrange(32, 127) for _ in range(vl))
                    entries += 1
                elif op < 0.75:  # literal with incremental indexing, indexed name
                    idx = rng.randrange(1, 62) if rng.random() < 0.7 else rng.randrange(62, 65)
                    vl = rng.randrange(0, 60)
                    blk += hpack_ref.encode_integer(idx, 6, 0x40)
                    blk += hpack_ref.encode_integer(vl, 7, 0) + bytes(rng.randrange(32, 127) for _ in range(vl))
                    entries += 1
                else:  # indexed field, sometimes past the table
                    hi = 62 + min(entries, 400) + 3 if rng.random() < 0.05 else 65
                    blk += hpack_ref.encode_integer(rng.randrange(1, hi), 7, 0x80)
            w = bytes(blk)
            pairs.append((d, w))
            want.append(_ref_decode(r, w))
    got = hpack.decode_blocks(pairs)
    assert sum(isinstance(x, hpack.DecoderError) for x in want) > 10
    assert sum(not isinstance(x, hpack.DecoderError) for x in want) > 300
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, pairs[i][1][:64].hex())


def test_block_decoder_after_fork(monkeypatch):
    """the block decoder's process-wide worker pool survives a fork. The parent decodes
    on 16 threads (the pool's threads start), forks, and the child decodes the same batch again: it
    must get a fresh pool (the parent's threads do not exist in the child) instead of waiting forever
    for them. The child runs under a time limit; its exit code says whether its headers matched."""
    import os
    import signal
    import time

    monkeypatch.setenv("HPK_HDEC_THREADS", "16")

    def batch():
        pairs, want = [], []
        for enc, story in _stories():
            d = hpack.Decoder()
            for c in story["cases"]:
                pairs.append((d, bytes.fromhex(c["wire"])))
                want.append([(n.encode(), v.encode()) for n, v in c["headers"]])
        return pairs, want

    pairs, want = batch()
    assert hpack.decode_blocks(pairs) == want
    pairs, want = batch()
    pid = os.fork()
    if pid == 0:  # child: no pytest machinery, just the decode and an exit code
        code = 1
        try:
            code = 0 if hpack.decode_blocks(pairs) == want else 2
        finally:
            os._exit(code)
    deadline = time.time() + 120
    while True:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            break
        if time.time() > deadline:
            os.kill(pid, signal.SIGKILL)
            os.waitpid(pid, 0)
            pytest.fail("the child's block decode hung after fork")
        time.sleep(0.05)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
    assert hpack.decode_blocks(pairs) == want  # the parent's pool still works
