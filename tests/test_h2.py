"""HTTP/2 frame layer (hpk_h2_read_frames) on the CPU batch path: the interop stories
sent as HEADERS + CONTINUATION frames (random fragment sizes, padding, priority blocks, other frame
types between blocks, bytes arriving in random chunks over several calls, many connections per call)
decode to the fixtures' header lists; every connection error the reference's deframer / frame loop
/ read_headers raises (crates/loona/src/h2/server.rs:290-390, 895-911, 1299-1303, 1349-1417) and the
httpwg cases for §4.3 (crates/httpwg/src/rfc9113/_4_http_frames.rs:153-260) give the reference's
error and GOAWAY code. tests/test_gpu.py runs the replay with the Huffman batch on the device."""

import random

import pytest

from hpk_util import load

from loona_amd import h2

HEADERS, CONTINUATION, DATA, PRIORITY, SETTINGS, PING = 0x1, 0x9, 0x0, 0x2, 0x4, 0x6
END_STREAM, END_HEADERS, PADDED, PRIO = 0x1, 0x4, 0x8, 0x20


def header_frames(rng, sid, block, end_stream, max_frame=16384):
    """One header block as HEADERS (+ CONTINUATION) frames: random split, padding, priority."""
    cuts = sorted(rng.sample(range(1, len(block)), min(len(block) - 1, rng.randrange(0, 4)))) if len(block) > 1 else []
    frags = [block[a:b] for a, b in zip([0] + cuts, cuts + [len(block)])]
    out = []
    flags = END_STREAM if end_stream else 0
    first = frags[0]
    if rng.random() < 0.3:  # priority block: 31-bit dependency (never itself) + weight
        first = (sid + 2).to_bytes(4, "big") + bytes([rng.randrange(256)]) + first
        flags |= PRIO
    if rng.random() < 0.3:  # padding: length byte + zeros at the end
        pad = rng.randrange(0, 20)
        first = bytes([pad]) + first + b"\0" * pad
        flags |= PADDED
    assert len(first) <= max_frame
    out.append(h2.frame(HEADERS, flags | (END_HEADERS if len(frags) == 1 else 0), sid, first))
    for i, f in enumerate(frags[1:], 1):
        out.append(h2.frame(CONTINUATION, END_HEADERS if i == len(frags) - 1 else 0, sid, f))
    return out


def other_frame(rng, sid):
    k = rng.randrange(3)
    if k == 0:
        return h2.frame(SETTINGS, 0, 0, b"\0\x03\0\0\0\x64")
    if k == 1:
        return h2.frame(PING, 0, 0, b"12345678")
    body = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 30)))
    return h2.frame(DATA, PADDED, sid, bytes([3]) + body + b"\0\0\0")


def interop_connections(seed=0):
    """(wire bytes per connection, expected [(stream, end_stream, headers)] per connection)."""
    rng = random.Random(seed)
    inter = load("interop.json.gz")
    wires, wants = [], []
    for enc in sorted(inter):
        for story in inter[enc]:
            frames, want = [], []
            for i, c in enumerate(story["cases"]):
                sid = 2 * i + 1
                es = rng.random() < 0.5
                block = bytes.fromhex(c["wire"])
                if not block:
                    continue  # an empty header block is legal but carries nothing to check
                if rng.random() < 0.2:
                    frames.append(other_frame(rng, sid))
                frames += header_frames(rng, sid, block, es)
                want.append((sid, es, [(n.encode(), v.encode()) for n, v in c["headers"]]))
            wires.append(b"".join(frames))
            wants.append(want)
    return wires, wants


def replay(codec, seed=0, calls=4):
    """Every interop story on its own connection, all connections' bytes in `calls` random cuts."""
    rng = random.Random(seed + 1)
    wires, wants = interop_connections(seed)
    conns = [h2.Connection() for _ in wires]
    cuts = [sorted(rng.sample(range(len(w) + 1), calls - 1)) + [len(w)] for w in wires]
    pos = [0] * len(wires)
    got = [[] for _ in wires]
    for k in range(calls):
        chunks = [wires[c][pos[c] : cuts[c][k]] for c in range(len(wires))]
        res = h2.read_frames(conns, chunks, codec)
        assert res.errors == [None] * len(wires)
        for c in range(len(wires)):
            pos[c] += res.consumed[c]  # an incomplete frame is sent again with the next bytes
        for conn, sid, es, val in res.blocks:
            got[conn].append((sid, es, val))
    assert pos == [len(w) for w in wires]
    assert got == wants
    return sum(len(w) for w in wants)


def test_interop_replay_frames_cpu():
    assert replay(None) > 10000


def test_single_call_many_connections():
    wires, wants = interop_connections(7)
    conns = [h2.Connection() for _ in wires]
    res = h2.read_frames(conns, wires, None)
    assert res.errors == [None] * len(wires) and res.consumed == [len(w) for w in wires]
    got = [[] for _ in wires]
    for conn, sid, es, val in res.blocks:
        got[conn].append((sid, es, val))
    assert got == wants


def one(frames, conn=None):
    c = conn or h2.Connection()
    r = h2.read_frames([c], [b"".join(frames)], None)
    return r, c


BLOCK = bytes.fromhex("828684418cf1e3c2e5f23a6ba0ab90f4ff")  # RFC 7541 C.4.1 (Huffman)
C41 = [(b":method", b"GET"), (b":scheme", b"http"), (b":path", b"/"), (b":authority", b"www.example.com")]


def test_httpwg_invalid_header_block_fragment():
    """_4_http_frames.rs:153-169: HEADERS(END_STREAM|END_HEADERS) b"\\x40" -> COMPRESSION_ERROR."""
    r, c = one([h2.frame(HEADERS, END_STREAM | END_HEADERS, 1, b"\x40")])
    assert r.errors == ["HpackDecodingError"] and h2.error_code(r.errors[0]) == "COMPRESSION_ERROR"
    (blk,) = r.blocks
    assert blk[3].kind == "IntegerDecodingError"
    assert c.error == "HpackDecodingError"


def test_httpwg_priority_frame_while_sending_headers():
    """_4_http_frames.rs:176-210: HEADERS(END_HEADERS), PRIORITY, CONTINUATION -> PROTOCOL_ERROR
    (the CONTINUATION is unexpected: server.rs:1299-1303); the first block still decodes."""
    r, _ = one([h2.frame(HEADERS, END_HEADERS, 1, BLOCK), h2.frame(PRIORITY, 0, 1, b"\0\0\0\0\xff"),
                h2.frame(CONTINUATION, END_HEADERS, 1, BLOCK)])
    assert r.errors == ["UnexpectedContinuationFrame"] and h2.error_code(r.errors[0]) == "PROTOCOL_ERROR"
    assert r.blocks == [(0, 1, False, C41)]


def test_httpwg_headers_frame_to_another_stream():
    """_4_http_frames.rs:215-250: HEADERS without END_HEADERS, then HEADERS for another stream ->
    ExpectedContinuationForStream, PROTOCOL_ERROR. read_headers compares the stream id before the
    frame type (server.rs:1391-1397, then 1399-1408), so the other stream wins over the wrong type."""
    r, _ = one([h2.frame(HEADERS, 0, 1, BLOCK), h2.frame(HEADERS, END_HEADERS, 3, BLOCK)])
    assert r.errors == ["ExpectedContinuationForStream"] and h2.error_code(r.errors[0]) == "PROTOCOL_ERROR"
    assert r.blocks == []


@pytest.mark.parametrize("second,err", [
    # same stream, wrong type: only the type check fails (server.rs:1399-1408)
    (h2.frame(DATA, 0, 1, b"xyz"), "ExpectedContinuationFrame"),
    (h2.frame(HEADERS, END_HEADERS, 1, BLOCK), "ExpectedContinuationFrame"),
    # another stream, any type: the stream check comes first (server.rs:1391-1397)
    (h2.frame(DATA, 0, 3, b"xyz"), "ExpectedContinuationForStream"),
    (h2.frame(CONTINUATION, END_HEADERS, 3, BLOCK[5:]), "ExpectedContinuationForStream"),
    (h2.frame(PING, 0, 0, b"12345678"), "ExpectedContinuationForStream"),
])
def test_continuation_check_order(second, err):
    r, c = one([h2.frame(HEADERS, 0, 1, BLOCK[:5]), second])
    assert r.errors == [err] and h2.error_code(err) == "PROTOCOL_ERROR" and c.error == err
    assert r.blocks == []


@pytest.mark.parametrize("frames,err,code", [
    ([h2.frame(HEADERS, 0, 1, BLOCK[:5]), h2.frame(CONTINUATION, END_HEADERS, 3, BLOCK[5:])],
     "ExpectedContinuationForStream", "PROTOCOL_ERROR"),
    ([h2.frame(HEADERS, END_HEADERS | PADDED, 1, b"")], "PaddedFrameEmpty", "FRAME_SIZE_ERROR"),
    ([h2.frame(HEADERS, END_HEADERS | PADDED, 1, bytes([40]) + BLOCK)], "PaddedFrameTooShort", "PROTOCOL_ERROR"),
    ([h2.frame(DATA, PADDED, 1, b"")], "PaddedFrameEmpty", "FRAME_SIZE_ERROR"),
    ([h2.frame(HEADERS, END_HEADERS | PRIO, 1, b"\0\0\0\x01\x10" + BLOCK)], "HeadersInvalidPriority", "PROTOCOL_ERROR"),
    ([h2.frame(HEADERS, END_HEADERS | PRIO, 1, b"\0\0")], "ReadAndParse(PrioritySpec)", "PROTOCOL_ERROR"),
    ([h2.frame(CONTINUATION, END_HEADERS, 1, BLOCK)], "UnexpectedContinuationFrame", "PROTOCOL_ERROR"),
    ([h2.frame(DATA, 0, 1, b"x" * 16385)], "FrameTooLarge", "FRAME_SIZE_ERROR"),
])
def test_connection_errors(frames, err, code):
    r, c = one(frames)
    assert r.errors == [err] and h2.error_code(err) == code and c.error == err


def test_padding_priority_and_continuations_decode():
    r, _ = one([h2.frame(HEADERS, PADDED | PRIO | END_STREAM, 5, bytes([4]) + b"\0\0\0\x07\x20" + BLOCK[:3] + b"\0" * 4),
                h2.frame(CONTINUATION, 0, 5, BLOCK[3:9]), h2.frame(CONTINUATION, END_HEADERS, 5, BLOCK[9:])])
    assert r.errors == [None] and r.blocks == [(0, 5, True, C41)]


def test_compression_error_stops_the_connection():
    """After a decoding error the connection's later blocks are not decoded (skipped) and the
    connection stays in error on later calls; other connections are unaffected."""
    bad = h2.frame(HEADERS, END_HEADERS, 1, b"\x40")
    good = h2.frame(HEADERS, END_HEADERS, 3, BLOCK)
    a, b = h2.Connection(), h2.Connection()
    r = h2.read_frames([a, b], [bad + good, good], None)
    assert r.errors == ["HpackDecodingError", None]
    assert [(x[0], x[1], x[3] is None) for x in r.blocks] == [(0, 1, False), (0, 3, True), (1, 3, False)]
    assert r.blocks[2][3] == C41
    r = h2.read_frames([a, b], [good, h2.frame(HEADERS, END_HEADERS, 5, bytes.fromhex("828684be"))], None)
    assert r.errors == ["HpackDecodingError", None] and r.consumed[0] == 0
    assert r.blocks == [(1, 5, False, C41)]  # dynamic-table entry 62 (C.4.1's authority) reused


def test_incomplete_frames_and_pending_continuation_across_calls():
    frames = h2.frame(HEADERS, 0, 1, BLOCK[:4]) + h2.frame(CONTINUATION, END_HEADERS, 1, BLOCK[4:])
    c = h2.Connection()
    got, pos = [], 0
    for cut in (3, 9, 15, len(frames)):  # mid-header, mid-payload, between frames, the end
        r = h2.read_frames([c], [frames[pos:cut]], None)
        assert r.errors == [None]
        pos += r.consumed[0]
        got += r.blocks
    assert pos == len(frames) and got == [(0, 1, False, C41)]


def replay_in_arena(codec, pin):
    """The interop connections' frames received into a buffet-shaped arena (64Ki x 4 KiB buffers in
    one anonymous mapping; the connections' bytes back to back) and decoded in place, all
    connections in one call."""
    wires, wants = interop_connections(3)
    arena = h2.Arena(65536, 4096, pin=pin)
    try:
        offs = [0]
        for w in wires:
            arena.view[offs[-1] : offs[-1] + len(w)] = memoryview(w)
            offs.append(offs[-1] + len(w))
        conns = [h2.Connection() for _ in wires]
        res = h2.read_frames_in(conns, arena, offs, codec)
        assert res.errors == [None] * len(wires) and res.consumed == [len(w) for w in wires]
        got = [[] for _ in wires]
        for conn, sid, es, val in res.blocks:
            got[conn].append((sid, es, val))
        assert got == wants
    finally:
        arena.close()


def test_replay_in_unpinned_arena_cpu():
    replay_in_arena(None, pin=False)
