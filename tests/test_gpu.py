"""GPU parity: the gfx950 kernels through the C ABI vs the oracle, bit for bit.

Covers the reference's own vectors (KATs with every error variant, RFC 7541 App. C, the whole
interop corpus), seeded random/error literals, edge cases (empty batch, empty literals, all-ones
runs, unaligned blob base, tiny capacities) and, at the bench's full size, size-independent
properties (encode -> decode round trip == input, per-literal lengths)."""

import numpy as np
import pytest

from hpk_util import compare_batches, interop_literals, load, oracle_decode_batch, oracle_encode_batch, pack

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", params=["fill", "wave", "compact", "compact_wave", "small"])
def codec(request):
    """A device codec; every test runs with each decode kernel (hpk_ctx_set_decode_kernel: the
    workgroup fills and the wave fills), in the compacted-output form (hpk_decode_batch_compact,
    through gpu_decode / _device_decode) under each kernel (tests that pass their own output regions
    run the region form of that kernel there), and in the small-call mode (hpk_ctx_set_small_mode:
    synchronous device calls of up to 64k literals answered by the persistent kernel), which must all
    give identical results."""
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a GPU (run with -m 'not gpu' on CPU)")
    from loona_amd import HuffmanCodec, _lib

    c = HuffmanCodec(0, stream=torch.cuda.current_stream())
    c.set_decode_kernel({"compact": "fill", "compact_wave": "wave", "small": "auto"}.get(request.param, request.param))
    c.compact = request.param.startswith("compact")
    c.variant = request.param
    if request.param == "small":
        c.set_small_mode(65536, 4, 200)
    yield c
    if request.param == "small":
        assert _lib.lib().hpk_test_small_calls(c._h) > 0, "the small-call mode answered no call"
        c.set_small_mode(0)
    c.close()


def to_dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def gpu_decode(codec, blob, off, shift=0):
    blob = np.ascontiguousarray(blob, np.uint8)
    n = len(off) - 1
    if shift:
        pad = np.zeros(blob.size + shift + 1, np.uint8)
        pad[shift : shift + blob.size] = blob
        dblob = to_dev(pad)[shift:]
    else:
        dblob = to_dev(blob if blob.size else np.zeros(1, np.uint8))
    doff = to_dev(np.asarray(off, np.int64).astype(np.int32))
    if getattr(codec, "compact", False):
        out, oo, ol, st = codec.decode_compact(dblob, doff, sync=True)
        _check_compact(out, oo, ol, n)
    else:
        out, oo, ol, st = codec.decode_device(dblob, doff, sync=True)
    torch.cuda.synchronize()
    return (out.cpu().numpy(), oo.cpu().numpy().astype(np.uint32), ol[:n].cpu().numpy().astype(np.uint32),
            st[:n].cpu().numpy())


def _check_compact(out, oo, ol, n):
    """The compacted form's layout: literals' byte ranges disjoint and inside out_off[n], which is at
    most the output capacity."""
    if n == 0:
        assert int(oo[0].item()) == 0
        return
    o = oo.to(torch.int64) & 0xFFFFFFFF
    ln = ol[:n].to(torch.int64)
    end = int(o[n].item())
    assert end <= out.numel()
    assert bool(((o[:n] + ln) <= end).all().item())
    nz = ln > 0  # (an empty literal may share its start with its neighbour)
    s, e = o[:n][nz], (o[:n] + ln)[nz]
    order = torch.argsort(s)
    s, e = s[order], e[order]
    assert bool((s[1:] >= e[:-1]).all().item()), "compacted literals overlap"


def gpu_encode(codec, blob, off):
    n = len(off) - 1
    dblob = to_dev(blob if blob.size else np.zeros(1, np.uint8))
    doff = to_dev(np.asarray(off, np.int64).astype(np.int32))
    out, oo, ol, st = codec.encode_device(dblob, doff, sync=True)
    torch.cuda.synchronize()
    return (out.cpu().numpy(), oo.cpu().numpy().astype(np.uint32), ol[:n].cpu().numpy().astype(np.uint32),
            st[:n].cpu().numpy())


def test_kats_and_rfc(codec):
    lits = [bytes.fromhex(k["in"]) for k in load("kat.json")]
    lits += [bytes.fromhex(x["in"]) for x in load("rfc7541_blocks.json")["huffman_literals"]]
    blob, off = pack(lits)
    got = gpu_decode(codec, blob, off)
    compare_batches(got, oracle_decode_batch(blob, off), "kat+rfc")
    kats = load("kat.json")
    for i, k in enumerate(kats):
        assert got[3][i] == k["status"]


def test_error_vectors(codec):
    vecs = load("error_vectors.json")["vectors"]
    lits = [bytes.fromhex(v["in"]) for v in vecs]
    blob, off = pack(lits)
    got = gpu_decode(codec, blob, off)
    compare_batches(got, oracle_decode_batch(blob, off), "error vectors")
    assert [int(s) for s in got[3]] == [v["status"] for v in vecs]


@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_interop_corpus(codec, shift):
    blob, off = pack(interop_literals())
    compare_batches(gpu_decode(codec, blob, off, shift), oracle_decode_batch(blob, off), f"interop shift={shift}")


def test_random_and_edge_literals(codec):
    rng = np.random.default_rng(99)
    lens = rng.integers(0, 70, size=50000)
    lits = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    lits += [b"", b"", b"\xff", b"\xff" * 3, b"\xff" * 4, b"\xff" * 5, b"\xff" * 40, b"\x00" * 9]
    lits += [b""] * 70
    blob, off = pack(lits)
    compare_batches(gpu_decode(codec, blob, off), oracle_decode_batch(blob, off), "random")


def test_long_literals(codec):
    """Long literals (v16: the wave-cooperative path; v19: the long-literal phase, here mostly whole
    ranges handed over): valid
    ones of every code length, random bytes (padding errors), an EOS in the middle at every bit
    offset class, bad padding after a long valid run, and long runs of 30-bit codes and of ones
    (where speculative starts synchronise late). Bit-exact against the oracle, with short literals
    interleaved so both paths run in the same fills."""
    from loona_amd import huffman_encode

    rng = np.random.default_rng(2025)
    lits = []
    for n in rng.integers(224, 4000, size=300):  # valid, mixed alphabets
        s = rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() if rng.random() < 0.5 else \
            rng.choice(np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_=;, ", np.uint8), int(n)).tobytes()
        lits.append(huffman_encode(s))
        lits.append(rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8).tobytes())
    for n in rng.integers(224, 3000, size=200):  # random bytes
        lits.append(rng.integers(0, 256, int(n), dtype=np.uint8).tobytes())
    eos = (1 << 30) - 1
    for k in range(64):  # EOS after a long valid prefix, at every offset mod 64 bits
        body = huffman_encode(b"x" * (300 + k))
        bits = int.from_bytes(body, "big") >> (len(body) * 8 - (300 + k) * 7)  # 'x' is 7 bits
        nb = (300 + k) * 7
        tail = int(rng.integers(0, 1 << 20))
        v = (((bits << 30) | eos) << 20) | tail
        tot = nb + 50
        pad = (-tot) % 8
        lits.append(((v << pad) | ((1 << pad) - 1)).to_bytes((tot + pad) // 8, "big"))
    for k in range(32):  # long valid run then a bad padding / too much padding
        body = bytearray(huffman_encode(b"accept-encoding: gzip, deflate" * (10 + k)))
        body[-1] &= 0xF0
        lits.append(bytes(body))
        lits.append(huffman_encode(b"y" * (400 + k)) + b"\xff")
    lits.append(b"\xff" * 3000)  # ones only: EOS at once
    lits.append(huffman_encode(bytes([1]) * 800))  # 23-bit codes back to back
    lits.append(huffman_encode(bytes(range(256)) * 12))  # every code length
    blob, off = pack(lits)
    compare_batches(gpu_decode(codec, blob, off), oracle_decode_batch(blob, off), "long literals")


def test_split_long_literals(codec):
    """Literals of 1.5-6 KiB encoded (left to the long-literal phase, one lane each, hpk_long.h):
    text and random bytes (long codes), an EOS before, near and after the middle byte at every
    offset class mod 64 bits, bad and too-long padding, a run of ones from the middle on, literals
    just below and above that size range, at exact-bound regions on an unaligned base with guard
    bytes. Bit-exact (lengths, statuses, bytes) against the oracle. (Written for the v22 experiment
    that split such literals into two pieces joined where their walks met; that split measured
    slower and was reverted, the cases stay as long-literal coverage.)"""
    from loona_amd import huffman_encode

    rng = np.random.default_rng(2207)
    text = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_=;,/.:ABCDEFGHIJ ", np.uint8)
    lits = []
    for n in rng.integers(1800, 8200, size=40):  # text: 1.3-6 KB encoded
        lits.append(huffman_encode(rng.choice(text, int(n)).tobytes()))
    for n in rng.integers(700, 2600, size=40):  # uniform bytes: ~2.3x, 1.6-6 KB encoded
        lits.append(huffman_encode(rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()))
    for n in rng.integers(1536, 6200, size=20):  # random bits: padding errors, false codes
        lits.append(rng.integers(0, 256, int(n), dtype=np.uint8).tobytes())
    eos = (1 << 30) - 1
    for frac in (0.1, 0.45, 0.49, 0.5, 0.51, 0.55, 0.9):
        for k in range(0, 64, 7):  # EOS at a fraction of a ~2.4 KB literal, offset classes mod 64
            m = int(2800 * frac) + k
            body = huffman_encode(b"x" * m)
            bits = int.from_bytes(body, "big") >> (len(body) * 8 - m * 7)  # 'x' is 7 bits
            after = huffman_encode(b"y" * (2800 - m))
            abits = int.from_bytes(after, "big")
            tot = m * 7 + 30 + len(after) * 8
            v = (((bits << 30) | eos) << (len(after) * 8)) | abits
            pad = (-tot) % 8
            lits.append(((v << pad) | ((1 << pad) - 1)).to_bytes((tot + pad) // 8, "big"))
    for k in range(16):  # bad padding / too much padding at the end
        body = bytearray(huffman_encode(b"content-security-policy: default-src 'self'" * (60 + k)))
        body[-1] &= 0xF0
        lits.append(bytes(body))
        lits.append(huffman_encode(b"z" * (2000 + 37 * k)) + b"\xff")
    half = huffman_encode(rng.choice(text, 2500).tobytes())
    lits.append(half + b"\xff" * len(half))  # ones from the middle on: EOS where the text ends
    lits.append(b"\xff" * 2000)
    for n in (1535, 1536, 1537, 6144, 6145):  # the split range's edges (encoded bytes)
        s = huffman_encode(rng.choice(text, n * 2).tobytes())[:n]
        lits.append(s)
        lits.append(rng.integers(0, 256, 40, dtype=np.uint8).tobytes())  # short ones between
    blob, off = pack(lits)
    ref = oracle_decode_batch(blob, off)
    compare_batches(gpu_decode(codec, blob, off), ref, "split literals")
    bound = [int(off[i + 1] - off[i]) * 8 // 5 for i in range(len(off) - 1)]
    got, guard = _decode_regions(codec, blob, off, bound, shift=3)
    compare_batches(got, ref, "split literals, exact-bound regions at +3")
    assert (guard == 0xAB).all()


def _decode_regions(codec, blob, off, caps, shift=0, guard=64):
    """Decode into caller-chosen region sizes `caps` (back to back), the output buffer surrounded
    by guard bytes; returns (out, out_off, out_len, status) over the regions and the guard bytes."""
    blob = np.ascontiguousarray(blob, np.uint8)
    n = len(off) - 1
    oo = np.zeros(n + 1, np.int64)
    np.cumsum(np.asarray(caps, np.int64), out=oo[1:])
    pad = np.zeros(blob.size + shift + 1, np.uint8)
    pad[shift : shift + blob.size] = blob
    dblob = to_dev(pad)[shift:]
    doff = to_dev(np.asarray(off, np.int64).astype(np.int32))
    big = torch.full((int(oo[-1]) + 2 * guard + shift,), 0xAB, dtype=torch.uint8, device="cuda")
    out = big[guard + shift : guard + shift + int(oo[-1]) + 1]
    ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    codec.decode_into(dblob, doff, out, to_dev(oo.astype(np.int32)), ol, st, device=True, sync=True)
    g = big.cpu().numpy()
    return (out.cpu().numpy(), oo.astype(np.uint32), ol.cpu().numpy().astype(np.uint32), st.cpu().numpy()), \
        np.concatenate([g[: guard + shift], g[guard + shift + int(oo[-1]) :]])


def test_long_literals_sprinkled_in_short_fills(codec):
    """v19: literals of >= 64 encoded bytes inside ranges of short ones are left by the fills and
    decoded after them, one lane each from HBM (hpk_long.h); 1 % of the literals, 64 B - 4 KiB, at
    random positions, every kind the oracle distinguishes, base pointers at 4 alignments."""
    from loona_amd import huffman_encode

    rng = np.random.default_rng(77)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_=;,/: ", np.uint8)
    lits = []
    for i in range(60000):
        if rng.random() < 0.01:
            n = int(rng.integers(80, 4000))
            k = rng.random()
            if k < 0.6:
                lits.append(huffman_encode(rng.choice(alpha, n).tobytes()))
            elif k < 0.8:
                lits.append(huffman_encode(rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
            elif k < 0.9:
                body = bytearray(huffman_encode(rng.choice(alpha, n).tobytes()))
                body[-1] &= 0xF0  # bad padding (or a truncated code)
                lits.append(bytes(body))
            else:
                lits.append(rng.integers(0, 256, n // 2, dtype=np.uint8).tobytes())  # random bits
        else:
            lits.append(huffman_encode(rng.choice(alpha, int(rng.integers(0, 60))).tobytes()))
    blob, off = pack(lits)
    want = oracle_decode_batch(blob, off)
    for shift in (0, 5):
        compare_batches(gpu_decode(codec, blob, off, shift), want, f"sprinkled long literals, shift {shift}")


@pytest.mark.parametrize("shift", [0, 3])
def test_long_literals_exact_bound_regions(codec, shift):
    """Long literals made only of 5-bit codes fill their region's decoded bound exactly, regions
    back to back with unrounded capacities and unaligned bases: the long-literal phase's 16-byte
    group stores and bytewise first/last groups must not touch a neighbour's bytes or the guard."""
    from loona_amd import huffman_encode

    rng = np.random.default_rng(5)
    five = np.frombuffer(b"012aceiost", np.uint8)
    lits = []
    for k in range(4000):
        if k % 3 == 0:
            lits.append(huffman_encode(rng.choice(five, 8 * int(rng.integers(13, 300))).tobytes()))  # >= 65 B
        elif k % 3 == 1:
            lits.append(huffman_encode(rng.choice(five, int(rng.integers(1, 40))).tobytes()))
        else:
            lits.append(b"")
    blob, off = pack(lits)
    bound = (np.diff(off.astype(np.int64)) * 8) // 5
    got, guard = _decode_regions(codec, blob, off, bound, shift)
    compare_batches(got, oracle_decode_batch(blob, off), "long exact-bound regions")
    assert (got[2].astype(np.int64)[0::3] == bound[0::3]).all()
    assert (guard == 0xAB).all()


def test_dense_range_falls_back_to_fills(codec):
    """A range dominated by long literals is handed to the long-literal phase whole, unless one of
    its literals has a region below the decoded bound: then the range is decoded by fills after
    all, and that literal stops at its capacity (HPK_OUTPUT_OVERFLOW) as on the short path."""
    from loona_amd import huffman_encode

    rng = np.random.default_rng(9)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", np.uint8)
    lits = [huffman_encode(rng.choice(alpha, int(rng.integers(300, 3000))).tobytes()) for _ in range(3000)]
    blob, off = pack(lits)
    enc = np.diff(off.astype(np.int64))
    caps = (enc * 8) // 5
    small = [7, 1500, 2999]
    caps[small] = 7
    got, guard = _decode_regions(codec, blob, off, caps)
    want = oracle_decode_batch(blob, off)
    keep = np.setdiff1d(np.arange(len(lits)), small)
    assert (got[3][small] == 4).all() and (got[2][small] == 7).all()
    assert (got[3][keep] == 0).all() and (got[2][keep] == want[2][keep]).all()
    for i in small:  # the first 7 bytes are the literal's first 7 decoded bytes
        assert bytes(got[0][got[1][i] : got[1][i] + 7]) == bytes(want[0][want[1][i] : want[1][i] + 7])
    for i in keep[::97]:
        assert bytes(got[0][got[1][i] : got[1][i] + got[2][i]]) == bytes(want[0][want[1][i] : want[1][i] + want[2][i]])
    assert (guard == 0xAB).all()


def test_empty_batch_and_empty_literals(codec):
    blob, off = pack([])
    got = gpu_decode(codec, blob, off)
    assert got[2].size == 0
    blob, off = pack([b""] * 1000)
    got = gpu_decode(codec, blob, off)
    assert not got[2].any() and not got[3].any()


def test_host_pointer_mode(codec):
    from loona_amd.batch import unpack

    lits = interop_literals()[:5000]
    blob, off = pack(lits)
    out, oo, ol, st = codec.decode_host(blob, off)
    compare_batches((out, oo, ol, st), oracle_decode_batch(blob, off), "host mode")
    dec = unpack(out, oo, ol)
    eb, eo = pack(dec)
    e_out, e_oo, e_ol, e_st = codec.encode_host(eb, eo)
    assert unpack(e_out, e_oo, e_ol) == lits


def test_small_capacity_overflow(codec):
    """Caller-provided capacity below the decoded size: status 4, no bytes past capacity."""
    from loona_amd import huffman_encode

    lits = [huffman_encode(b"abcdefghij" * k) for k in range(1, 30)]
    blob, off = pack(lits)
    n = len(lits)
    cap = np.full(n, 7, np.int64)
    oo = np.zeros(n + 1, np.int64)
    np.cumsum(cap, out=oo[1:])
    dblob, doff = to_dev(blob), to_dev(off.astype(np.int32))
    doo = to_dev(oo.astype(np.int32))
    out = torch.full((int(oo[-1]) + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    codec.decode_into(dblob, doff, out, doo, ol, st, device=True, sync=True)
    assert (st.cpu().numpy() == 4).all() and (ol.cpu().numpy() == 7).all()
    assert (out[int(oo[-1]) :].cpu().numpy() == 0xAB).all()


def test_exact_bound_regions(codec):
    """Literals made only of 5-bit codes decode to exactly floor(8n/5) bytes: their output fills
    the region's decoded bound, so a 16-bit store's second byte after the last symbol would fall
    on the next region (the kernel repairs it, pair_fixup). Exact-bound regions back to back, with
    exact (unrounded) capacities, empty literals and normal ones between them."""
    from loona_amd import huffman_encode

    rng = np.random.default_rng(17)
    five = b"012aceiost"  # the 5-bit codes
    lits = []
    for k in range(6000):
        r = k % 5
        if r == 0:
            lits.append(b"")
        elif r == 4:
            lits.append(huffman_encode(rng.choice(list(b"abcdefghij-/:"), int(rng.integers(1, 40))).astype(np.uint8).tobytes()))
        else:
            lits.append(huffman_encode(rng.choice(list(five), 8 * int(rng.integers(1, 12))).astype(np.uint8).tobytes()))
    blob, off = pack(lits)
    n = len(lits)
    bound = (np.diff(off.astype(np.int64)) * 8) // 5
    oo = np.zeros(n + 1, np.int64)
    np.cumsum(bound, out=oo[1:])
    dblob, doff = to_dev(blob), to_dev(off.astype(np.int32))
    doo = to_dev(oo.astype(np.int32))
    out = torch.full((int(oo[-1]) + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    codec.decode_into(dblob, doff, out, doo, ol, st, device=True, sync=True)
    got = (out.cpu().numpy(), oo.astype(np.uint32), ol.cpu().numpy().astype(np.uint32), st.cpu().numpy())
    compare_batches(got, oracle_decode_batch(blob, off), "exact-bound regions")
    assert (got[2].astype(np.int64)[1::5] == bound[1::5]).all()  # the 5-bit literals do fill their bound
    assert (got[0][int(oo[-1]) :] == 0xAB).all()


def test_encode_matches_oracle(codec):
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 200, size=20000)
    strs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    blob, off = pack(strs)
    compare_batches(gpu_encode(codec, blob, off), oracle_encode_batch(blob, off), "encode")


@pytest.mark.parametrize("shift", [1, 3, 13])
def test_encode_unaligned_bases(codec, shift):
    """Encode v2 reads 16-byte chunks from a rounded-down base and writes a tile's output span with
    16-byte stores: unaligned input and output bases, empty literals among them."""
    from hpk_util import oracle_encode

    rng = np.random.default_rng(11 + shift)
    lens = rng.integers(0, 90, size=3000)
    lens[::7] = 0
    strs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    blob, off = pack(strs)
    pad = np.zeros(blob.size + shift + 1, np.uint8)
    pad[shift : shift + blob.size] = blob
    dblob = to_dev(pad)[shift:]
    doff = to_dev(np.asarray(off, np.int64).astype(np.int32))
    from loona_amd.batch import encode_offsets_torch

    oo = encode_offsets_torch(doff)
    big = torch.full((int(oo[-1].item()) + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    out = big[shift:]
    n = len(strs)
    ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    codec.encode_into(dblob, doff, out, oo, ol, st, device=True, sync=True)
    o, oon, oln, stn = out.cpu().numpy(), oo.cpu().numpy(), ol.cpu().numpy(), st.cpu().numpy()
    assert not stn.any()
    for i in range(n):
        want = oracle_encode(strs[i])
        assert int(oln[i]) == len(want), i
        assert o[oon[i] : oon[i] + oln[i]].tobytes() == want, i
    assert (big[:shift].cpu().numpy() == 0x5A).all()  # nothing before the output base


def test_encode_small_capacity_and_huge_literal(codec):
    """Capacities below the encoded size: status HPK_OUTPUT_OVERFLOW, out_len = capacity, the bytes
    are the encoding's prefix and nothing is written past a region. A 70 KB literal (larger than a
    tile) takes the one-lane path."""
    from hpk_util import oracle_encode

    rng = np.random.default_rng(5)
    strs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 60, size=500)]
    strs.append(bytes(rng.integers(0, 256, 70000, dtype=np.uint8)))
    strs.append(b"www.example.com")
    blob, off = pack(strs)
    n = len(strs)
    want = [oracle_encode(s) for s in strs]
    cap = np.array([max(1, len(w) - (i % 3)) for i, w in enumerate(want)], np.int64)  # some short by 1 or 2
    oo = np.zeros(n + 1, np.int64)
    np.cumsum(cap, out=oo[1:])
    dblob, doff = to_dev(blob), to_dev(off.astype(np.int32))
    doo = to_dev(oo.astype(np.int32))
    out = torch.full((int(oo[-1]) + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    codec.encode_into(dblob, doff, out, doo, ol, st, device=True, sync=True)
    o, oln, stn = out.cpu().numpy(), ol.cpu().numpy(), st.cpu().numpy()
    for i in range(n):
        c = int(cap[i])
        if len(want[i]) <= c:
            assert stn[i] == 0 and int(oln[i]) == len(want[i]), i
        else:
            assert stn[i] == 4 and int(oln[i]) == c, i
        assert o[oo[i] : oo[i] + oln[i]].tobytes() == want[i][: int(oln[i])], i
    assert (o[int(oo[-1]) :] == 0xAB).all()


@pytest.mark.parametrize("seed", [0, 1])
def test_encode_mixed_regions_and_empty_runs(codec, seed):
    """Encode v5 finds a thread's literal starts in a per-tile start map and the literal holding its
    first byte by a max scan, and picks the checked pass 2 per tile: tiles mixing bound-sized and exact
    regions, runs of empty literals (several literals starting at one byte), 1-byte literals (up to 32
    starts in one thread's bytes) and literals crossing many threads."""
    from hpk_util import oracle_encode

    rng = np.random.default_rng(100 + seed)
    lens = rng.choice([0, 1, 2, 5, 31, 32, 33, 200, 1500], size=6000, p=[.2, .2, .1, .1, .1, .1, .1, .08, .02])
    lens[100:140] = 0
    lens[500:900] = 1
    strs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    want = [oracle_encode(x) for x in strs]
    blob, off = pack(strs)
    n = len(strs)
    # exact regions for every third literal after 2,000, bound regions (30 bits per byte) otherwise
    cap = np.array([len(w) if (i >= 2000 and i % 3 == 0) else (30 * len(s) + 7) // 8 for i, (s, w) in
                    enumerate(zip(strs, want))], np.int64)
    oo = np.zeros(n + 1, np.int64)
    np.cumsum(cap, out=oo[1:])
    dblob, doff = to_dev(blob), to_dev(off.astype(np.int32))
    doo = to_dev(oo.astype(np.int32))
    out = torch.full((int(oo[-1]) + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    codec.encode_into(dblob, doff, out, doo, ol, st, device=True, sync=True)
    o, oln, stn = out.cpu().numpy(), ol.cpu().numpy(), st.cpu().numpy()
    assert not stn.any()
    for i in range(n):
        assert int(oln[i]) == len(want[i]), i
        assert o[oo[i] : oo[i] + oln[i]].tobytes() == want[i], i
    assert (o[int(oo[-1]) :] == 0xAB).all()


def test_config2_full_roundtrip(codec):
    """BASELINE config 2 at full size (1M literals): GPU decode of the canonical encoding gives back
    the generated strings exactly (size-independent property); a 100k prefix is also compared to
    the oracle byte for byte."""
    from loona_amd import synth

    w = synth.config2()
    got = gpu_decode(codec, w.enc_blob, w.enc_off)
    out, oo, ol, st = got
    assert not st.any()
    assert np.array_equal(ol.astype(np.int64), np.diff(w.dec_off.astype(np.int64)))
    ln = ol.astype(np.int64)
    idx = np.repeat(oo[:-1].astype(np.int64) - (np.cumsum(ln) - ln), ln) + np.arange(int(ln.sum()))
    assert np.array_equal(out[idx], w.dec_blob)
    k = 100_000
    sub_off = w.enc_off[: k + 1]
    sub_blob = w.enc_blob[: int(sub_off[-1])]
    compare_batches(gpu_decode(codec, sub_blob, sub_off), oracle_decode_batch(sub_blob, sub_off), "config2 prefix")


def test_config3_roundtrip_sample(codec):
    """BASELINE config 3 distribution (Zipf lengths to 4 KiB, 5 % uniform bytes): device encode ->
    device decode == input; device encode == oracle encode on a 20k sample."""
    from loona_amd import synth

    w = synth.config3(n=20000)
    e = gpu_encode(codec, w.dec_blob, w.dec_off)
    compare_batches(e, oracle_encode_batch(w.dec_blob, w.dec_off), "config3 encode")
    eo, eoo, eol, est = e
    ln = eol.astype(np.int64)
    idx = np.repeat(eoo[:-1].astype(np.int64) - (np.cumsum(ln) - ln), ln) + np.arange(int(ln.sum()))
    enc_blob = eo[idx]
    enc_off = np.zeros(len(ln) + 1, np.int64)
    np.cumsum(ln, out=enc_off[1:])
    d = gpu_decode(codec, enc_blob, enc_off.astype(np.uint32))
    assert not d[3].any()
    dl = d[2].astype(np.int64)
    idx = np.repeat(d[1][:-1].astype(np.int64) - (np.cumsum(dl) - dl), dl) + np.arange(int(dl.sum()))
    assert np.array_equal(d[0][idx], w.dec_blob)


def test_host_pointer_mode_pipelined(codec):
    """HPK_PTR_HOST at a size that takes the chunked copy/decode pipeline (8 chunks), from
    pageable and from page-locked (hpk_host_register) buffers: identical to the device path."""
    from loona_amd import _lib, synth

    w = synth.config2(n=300_000, seed=99)
    ref = gpu_decode(codec, w.enc_blob, w.enc_off)
    got = codec.decode_host(w.enc_blob, w.enc_off)
    compare_batches(got, ref, "host pipelined vs device")
    L = _lib.lib()
    blob = np.ascontiguousarray(w.enc_blob)
    assert L.hpk_host_register(blob.ctypes.data, blob.nbytes) == 0
    try:
        got = codec.decode_host(blob, w.enc_off)
    finally:
        assert L.hpk_host_unregister(blob.ctypes.data) == 0
    compare_batches(got, ref, "host pipelined (pinned) vs device")
    # encode through the same pipeline round-trips
    e = codec.encode_host(w.dec_blob, w.dec_off)
    assert not e[3].any()
    assert np.array_equal(e[2].astype(np.int64), np.diff(w.enc_off.astype(np.int64)))


def test_hpack_blocks_on_device(codec):
    """Two-pass HPACK block decoding with the Huffman batch on the GPU: every interop story in one
    call (one decoder per story) and seeded corruptions vs the decoder.rs restatement."""
    import random

    from hpk_util import hpack_ref

    from loona_amd import hpack

    inter = load("interop.json.gz")
    pairs, want = [], []
    for enc in sorted(inter):
        for story in inter[enc]:
            d = hpack.Decoder()
            for c in story["cases"]:
                pairs.append((d, bytes.fromhex(c["wire"])))
                want.append([(n.encode(), v.encode()) for n, v in c["headers"]])
    assert hpack.decode_blocks(pairs, codec) == want
    rng = random.Random(3)
    pairs, want = [], []
    for _ in range(2000):
        w = bytearray(bytes.fromhex(rng.choice(rng.choice(inter[rng.choice(sorted(inter))])["cases"])["wire"]))
        if w:
            w[rng.randrange(len(w))] ^= 1 << rng.randrange(8)
        pairs.append((hpack.Decoder(), bytes(w)))
        r = hpack_ref.Decoder()
        try:
            want.append(r.decode(bytes(w)))
        except hpack_ref.DecoderError as e:
            want.append(hpack.DecoderError(e.kind, e.detail))
    assert hpack.decode_blocks(pairs, codec) == want


@pytest.mark.parametrize("kind", ["decreasing", "past_in_cap", "past_out_cap", "huge"])
def test_bad_device_offsets(codec, kind):
    """hpk.h device-pointer contract: offsets that decrease or pass a blob's capacity are caught by
    the kernels as they read them (the reference checks lengths before any Huffman work,
    decoder.rs:138-142): the offending literal gets HPK_BAD_OFFSETS, a synchronous call raises
    (HPK_E_INVAL), no byte outside the output buffer changes, nothing is read outside the input."""
    from loona_amd import _lib, synth
    from loona_amd.batch import decode_offsets_np, encode_offsets_np

    w = synth.config2(n=20000, seed=5)
    n = w.n
    io = w.enc_off.astype(np.int64).copy()
    oo = decode_offsets_np(w.enc_off).astype(np.int64)
    j = 12345
    if kind == "decreasing":
        io[j] = io[j + 1] + 3
    elif kind == "past_in_cap":
        io[j + 1 :] += 1 << 20
    elif kind == "past_out_cap":
        oo[-1] += 64
    else:
        io[j] = 0xFFFFFFF0
        oo[j] = 0xFFFFFFF0
    guard = 4096
    big = torch.full((guard + int(decode_offsets_np(w.enc_off)[-1]) + guard,), 0xAB, dtype=torch.uint8, device="cuda")
    out = big[guard:-guard]
    blob = to_dev(w.enc_blob)
    ol = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    dio = to_dev(io.astype(np.uint32).view(np.int32))
    doo = to_dev(oo.astype(np.uint32).view(np.int32))
    with pytest.raises(RuntimeError, match="hpk_decode_batch"):
        codec.decode_into(blob, dio, out, doo, ol, st, device=True, sync=True)
    stn = st.cpu().numpy()
    assert (stn == _lib.HPK_BAD_OFFSETS).any()
    assert set(np.unique(stn)) <= {0, _lib.HPK_BAD_OFFSETS}
    assert (ol.cpu().numpy()[stn == _lib.HPK_BAD_OFFSETS] == 0).all()
    g = big.cpu().numpy()
    assert (g[:guard] == 0xAB).all() and (g[-guard:] == 0xAB).all()
    codec.check()  # the sticky flag was cleared by the failing synchronous call
    # async: the call returns, the flag is reported by check()
    codec.decode_into(blob, dio, out, doo, ol, st, device=True, sync=False)
    with pytest.raises(RuntimeError, match="hpk_ctx_check"):
        codec.check()
    # the same buffers with good offsets decode normally afterwards
    codec.decode_into(blob, to_dev(w.enc_off.view(np.int32)), out, to_dev(decode_offsets_np(w.enc_off).view(np.int32)),
                      ol, st, device=True, sync=True)
    assert not st.cpu().numpy().any()
    # encode: the same checks
    eo = encode_offsets_np(w.dec_off).astype(np.int64)
    dio2 = w.dec_off.astype(np.int64).copy()
    dio2[j] = dio2[j + 1] + 1
    ebig = torch.full((guard + int(eo[-1]) + guard,), 0xAB, dtype=torch.uint8, device="cuda")
    with pytest.raises(RuntimeError, match="hpk_encode_batch"):
        codec.encode_into(to_dev(w.dec_blob), to_dev(dio2.astype(np.uint32).view(np.int32)), ebig[guard:-guard],
                          to_dev(eo.astype(np.uint32).view(np.int32)), ol, st, device=True, sync=True)
    assert (st.cpu().numpy() == _lib.HPK_BAD_OFFSETS).any()
    g = ebig.cpu().numpy()
    assert (g[:guard] == 0xAB).all() and (g[-guard:] == 0xAB).all()


def test_bad_offsets_with_long_literals_in_the_fill(codec):
    """A bad literal's fill also holds long literals (>= 64 encoded bytes, left to the long-literal
    phase): the whole rest of the workgroup's range gets HPK_BAD_OFFSETS with out_len 0, and the
    long-literal phase must not decode those long literals afterwards (hpk.h contract); long
    literals of valid ranges elsewhere still decode."""
    from loona_amd import _lib, huffman_encode
    from loona_amd.batch import decode_offsets_np

    rng = np.random.default_rng(3)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_=;,/: ", np.uint8)
    j = 12345
    lits = []
    for i in range(20000):
        long_ = (j < i <= j + 6) or i % 997 == 0
        n = int(rng.integers(120, 600)) if long_ else int(rng.integers(4, 50))
        lits.append(huffman_encode(rng.choice(alpha, n).tobytes()))
    blob, off = pack(lits)
    n = len(lits)
    io = np.asarray(off, np.int64).copy()
    oo = decode_offsets_np(np.asarray(off, np.uint32)).astype(np.int64)
    io[j] = io[j + 1] + 3  # decreasing: literal j is bad
    out = torch.full((int(oo[-1]) + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    ol = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    with pytest.raises(RuntimeError, match="hpk_decode_batch"):
        codec.decode_into(to_dev(blob), to_dev(io.astype(np.uint32).view(np.int32)), out,
                          to_dev(oo.astype(np.uint32).view(np.int32)), ol, st, device=True, sync=True)
    stn, oln = st.cpu().numpy(), ol.cpu().numpy()
    bad = stn == _lib.HPK_BAD_OFFSETS
    # the long literal after j in its fill included (j + 1 shares j's fill under both kernels: the
    # workgroup kernel voids its whole range from the bad fill on, the wave kernel its wave's range)
    assert bad[j : j + 2].all(), stn[j : j + 7]
    assert (oln[bad] == 0).all()
    assert set(np.unique(stn)) <= {0, _lib.HPK_BAD_OFFSETS}
    good_long = [i for i in range(0, n, 997) if not bad[i]]
    assert len(good_long) > 10 and all(stn[i] == 0 and oln[i] > 0 for i in good_long)


def _prefix_host(out, oo, ol, st, k):
    """The first k literals of a device decode as numpy (out_blob, out_off, out_len, status); their
    bytes gathered on the device first (the compacted form's offsets are not monotone)."""
    from loona_amd import synth

    got = synth.gather_output(out, oo, ol, 0, k)
    ln = ol[:k].cpu().numpy().view(np.uint32).astype(np.int64)
    offs = np.zeros(k + 1, np.int64)
    np.cumsum(ln, out=offs[1:])
    return (got.cpu().numpy() if got.numel() else np.zeros(1, np.uint8), offs.astype(np.uint32),
            ln.astype(np.uint32), st[:k].cpu().numpy())


def _device_decode(codec, w):
    from loona_amd.batch import decode_offsets_torch

    if getattr(codec, "compact", False):
        out, oo, ol, st = codec.decode_compact(w.enc_blob, w.enc_off, sync=True)
        _check_compact(out, oo, ol, w.n)
        return out, oo, ol, st

    oo = decode_offsets_torch(w.enc_off)
    out = torch.empty((int(oo[-1].item()) & 0xFFFFFFFF) + 16, dtype=torch.uint8, device="cuda")
    ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
    st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
    codec.decode_into(w.enc_blob, w.enc_off, out, oo, ol, st, device=True, sync=True)
    return out, oo, ol, st


def _check_encode_prefix(w, k):
    """Device encode (the workload's encoded literals) == oracle encode on the first k strings."""
    dec_off = w.dec_off[: k + 1].cpu().numpy().astype(np.uint32)
    dec_blob = w.dec_blob[: int(dec_off[-1])].cpu().numpy()
    want = oracle_encode_batch(dec_blob, dec_off)
    enc_off = w.enc_off[: k + 1].cpu().numpy().view(np.uint32)
    got = (w.enc_blob[: int(enc_off[-1])].cpu().numpy(), enc_off, np.diff(enc_off.astype(np.int64)).astype(np.uint32),
           np.zeros(k, np.uint8))
    compare_batches(got, want, "device encode vs oracle")


def test_config5_shard_full(codec):
    """One config-5 shard at full size: 32M distinct seeded literals (870 MB encoded), the unit of one
    bench launch. Every status, length and decoded byte against the generated strings; the first
    100k literals' decode and encode against the oracle."""
    from loona_amd import synth

    w = synth.device_config5_shard(codec, 0)
    assert w.n == 32_000_000 and w.enc_bytes > 800_000_000
    out, oo, ol, st = _device_decode(codec, w)
    synth.check_decoded(w, out, oo, ol, st)
    k = 100_000
    eo = w.enc_off[: k + 1].cpu().numpy().view(np.uint32)
    want = oracle_decode_batch(w.enc_blob[: int(eo[-1])].cpu().numpy(), eo)
    compare_batches(_prefix_host(out, oo, ol, st, k), want, "config5 shard prefix vs oracle")
    _check_encode_prefix(w, k)


def test_config3_full_roundtrip(codec):
    """BASELINE config 3 at full size (1M literals, Zipf lengths to 4 KiB, 5 % uniform bytes):
    device encode -> device decode gives back every generated byte; device encode == oracle encode
    and device decode == oracle decode on the first 100k literals."""
    from loona_amd import synth

    w = synth.device_config3(codec)
    assert w.n == 1_000_000 and w.dec_bytes > 300_000_000
    out, oo, ol, st = _device_decode(codec, w)
    synth.check_decoded(w, out, oo, ol, st)
    k = 100_000
    _check_encode_prefix(w, k)
    eo = w.enc_off[: k + 1].cpu().numpy().view(np.uint32)
    want = oracle_decode_batch(w.enc_blob[: int(eo[-1])].cpu().numpy(), eo)
    compare_batches(_prefix_host(out, oo, ol, st, k), want, "config3 prefix vs oracle")


def test_h2_frames_replay_on_device(codec):
    """SURVEY §8f-3/§8f-4 through the device: every interop story as HEADERS + CONTINUATION frames
    (random splits, padding, priority, other frames between blocks, bytes in random chunks over
    several calls, one connection per story) decodes to the fixtures' header lists with the
    Huffman batch on the GPU; httpwg's invalid_header_block_fragment
    (crates/httpwg/src/rfc9113/_4_http_frames.rs:153-169) gives COMPRESSION_ERROR."""
    from test_h2 import replay

    from loona_amd import h2

    assert replay(codec, seed=11) > 10000
    c = h2.Connection()
    r = h2.read_frames([c], [h2.frame(0x1, 0x5, 1, b"\x40")], codec)
    assert r.errors == ["HpackDecodingError"] and h2.error_code(r.errors[0]) == "COMPRESSION_ERROR"


def test_encode_blocks_on_device(codec):
    """SURVEY §8f-2 through the device: many responses' header blocks with every Huffman string in
    one device encode batch, compared block by block with the encoder.rs restatement
    (oracle/hpack_ref.Encoder(huffman=True): Encoder::encode, encoder.rs:210-234, with the H bit set
    where the Huffman form is strictly shorter than encode_string_literal's raw form,
    encoder.rs:296-307) on the same lists (interop headers plus random binary and numeric values),
    and with hpk_henc_encode block by block. A failed device call leaves the encoders unchanged."""
    from test_hpack_encoder import response_lists

    from hpk_util import hpack_ref
    from loona_amd import _lib, hpack

    lists = response_lists(seed=5)
    k = 5
    assert hpack.encode_blocks([], codec) == []
    encs_d = [hpack.Encoder(huffman=True) for _ in range(k)]
    encs_s = [hpack.Encoder(huffman=True) for _ in range(k)]
    refs = [hpack_ref.Encoder(huffman=True) for _ in range(k)]
    got = hpack.encode_blocks([(encs_d[i % k], hs) for i, hs in enumerate(lists)], codec)
    oracle = [refs[i % k].encode(hs) for i, hs in enumerate(lists)]
    assert got == oracle
    assert got == [encs_s[i % k].encode(hs) for i, hs in enumerate(lists)]
    # a call failing after the table pass commits nothing: the next one matches the oracle again
    more = response_lists(seed=6, n=200)
    L = _lib.lib()
    L.hpk_test_fail_batches(1)
    try:
        with pytest.raises(RuntimeError, match="injected"):
            hpack.encode_blocks([(encs_d[i % k], hs) for i, hs in enumerate(more)], codec)
    finally:
        L.hpk_test_fail_batches(0)
    got = hpack.encode_blocks([(encs_d[i % k], hs) for i, hs in enumerate(more)], codec)
    assert got == [refs[i % k].encode(hs) for i, hs in enumerate(more)]


def test_scatter_decode_gather_device_world1(codec):
    """shard.scatter_decode_gather on device tensors over RCCL ("nccl", world 1: the root keeps every
    shard): the device-resident path bench.py times at N > 1, results equal the oracle's."""
    import os
    import socket

    import torch.distributed as dist

    from loona_amd import shard, synth
    from loona_amd.batch import decode_offsets_torch

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        w = synth.config2(n=30000, seed=21)
        b = shard.balanced_ranges(w.enc_off, 3)
        shards = []
        for r in range(3):
            sb, so = shard.shard(w.enc_blob, w.enc_off, int(b[r]), int(b[r + 1]))
            shards.append((to_dev(sb if sb.size else np.zeros(1, np.uint8)), to_dev(so.view(np.int32))))

        def decode_fn(blob, off):
            if codec.compact:  # the compacted form: the owner's written span travels as it is
                return codec.decode_compact(blob, off, sync=False)
            oo = decode_offsets_torch(off)
            out = torch.empty((int(oo[-1].item()) & 0xFFFFFFFF) + 16, dtype=torch.uint8, device="cuda")
            ol = torch.empty(max(off.numel() - 1, 1), dtype=torch.int32, device="cuda")
            st = torch.empty(max(off.numel() - 1, 1), dtype=torch.uint8, device="cuda")
            codec.decode_into(blob, off, out, oo, ol, st, device=True, sync=False)
            return out, oo, ol, st

        res = shard.scatter_decode_gather(shards, decode_fn, device="cuda", compacted=codec.compact)
        torch.cuda.synchronize()
        for r, (cb, coff, ol, st) in enumerate(res):  # each shard's decoded bytes laid end to end
            lo, hi = int(b[r]), int(b[r + 1])
            sb, so = shard.shard(w.enc_blob, w.enc_off, lo, hi)
            cbh = cb.cpu().numpy() if cb.numel() else np.zeros(1, np.uint8)
            got = (cbh, coff.cpu().numpy().astype(np.uint32), ol.cpu().numpy().view(np.uint32), st.cpu().numpy())
            compare_batches(got, oracle_decode_batch(sb, so), f"world-1 shard {r}")
    finally:
        dist.destroy_process_group()


def test_h2_frames_in_pinned_arena_on_device(codec):
    """Frames in a page-locked buffet-shaped arena (hpk_arena_create, 64Ki x 4 KiB) decoded in place
    with the Huffman batch on the device."""
    from test_h2 import replay_in_arena

    replay_in_arena(codec, pin=True)


def _large_literals():
    """Literals of 16 KiB - 1 MiB encoded: the reference accepts string lengths up to
    ~2^28 (crates/loona-hpack/src/decoder.rs:96-99) and concatenates CONTINUATION payloads into one
    block (crates/loona/src/h2/server.rs:1625-1633), so one literal can be a whole large header."""
    from loona_amd import huffman_encode

    rng = np.random.default_rng(4096)
    text = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_=;,/.:ABCDEFGHIJ ", np.uint8)

    def text_enc(nbytes):  # a valid literal of exactly nbytes encoded bytes (text prefix, EOS padding)
        s = huffman_encode(rng.choice(text, nbytes * 2).tobytes())[:nbytes]
        return bytes(s)

    lits = []
    for nb in (16384, 65535, 65536, 65537, 262144, 1 << 20):
        lits.append(text_enc(nb))  # cut mid-code: padding error or a valid end, as the oracle says
        lits.append(huffman_encode(rng.choice(text, nb + nb // 3).tobytes()))  # valid text
        lits.append(rng.integers(0, 40, 17, dtype=np.uint8).tobytes())  # a short one between
    lits.append(huffman_encode(rng.integers(0, 256, 120000, dtype=np.uint8).tobytes()))  # ~270 KB, long codes
    eos = (1 << 30) - 1
    for m in (70000, 140001):  # EOS 40 bits before the end of a ~64/128 KB literal
        body = huffman_encode(b"x" * m)
        bits = int.from_bytes(body, "big") >> (len(body) * 8 - m * 7)  # 'x' is 7 bits
        v = (((bits << 30) | eos) << 10) | 0x3FF
        tot = m * 7 + 40
        pad = (-tot) % 8
        lits.append(((v << pad) | ((1 << pad) - 1)).to_bytes((tot + pad) // 8, "big"))
    body = bytearray(huffman_encode(b"content-security-policy: default-src 'self'" * 3000))
    body[-1] &= 0xF0  # bad padding after ~100 KB of valid codes
    lits.append(bytes(body))
    lits.append(huffman_encode(b"z" * 80000) + b"\xff")  # too much padding
    lits.append(b"\xff" * 70000)  # EOS at once
    return lits


def test_large_literals(codec):
    """16 KiB, 64 KiB +- 1, 256 KiB and 1 MiB encoded literals through both kernels (they exceed any
    fill window: the long-literal phase or the one-lane global path) against the oracle: valid, cut
    mid-code, long codes, EOS near the end, bad and too-long padding; then at exact-bound regions on
    an unaligned base (+3) with guard bytes around the output."""
    lits = _large_literals()
    blob, off = pack(lits)
    ref = oracle_decode_batch(blob, off)
    compare_batches(gpu_decode(codec, blob, off), ref, "large literals")
    compare_batches(gpu_decode(codec, blob, off, shift=5), ref, "large literals, input at +5")
    bound = [int(off[i + 1] - off[i]) * 8 // 5 for i in range(len(off) - 1)]
    got, guard = _decode_regions(codec, blob, off, bound, shift=3)
    compare_batches(got, ref, "large literals, exact-bound regions at +3")
    assert (guard == 0xAB).all()


@pytest.mark.parametrize("kind", ["decreasing", "past_in_cap"])
def test_compact_bad_offsets(codec, kind):
    """The compacted form under bad input offsets (the kernel checks them as it reads them, as in the
    region form): the offending literals get HPK_BAD_OFFSETS with out_len 0, a synchronous call raises,
    the literals that did decode match the oracle, and nothing is written past the span out_off[n]
    reports (guard bytes around the output buffer unchanged)."""
    from loona_amd import _lib, synth
    from loona_amd.batch import compact_capacity

    if not codec.compact:
        pytest.skip("the compacted form only")
    w = synth.config2(n=20000, seed=8)
    io = w.enc_off.astype(np.int64).copy()
    j = 7777
    if kind == "decreasing":
        io[j] = io[j + 1] + 3
    else:
        io[j + 1 :] += 1 << 20
    n = w.n
    guard = 4096
    need = compact_capacity(w.enc_blob.size, n)
    big = torch.full((guard + need + guard,), 0xAB, dtype=torch.uint8, device="cuda")
    out = big[guard:-guard]
    oo = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    ol = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    dio = to_dev(io.astype(np.uint32).view(np.int32))
    with pytest.raises(RuntimeError, match="hpk_decode_batch_compact"):
        codec.decode_compact(to_dev(w.enc_blob), dio, out, oo, ol, st, sync=True)
    stn, oln = st.cpu().numpy(), ol.cpu().numpy().view(np.uint32)
    bad = stn == _lib.HPK_BAD_OFFSETS
    assert bad[j] and (oln[bad] == 0).all()
    g = big.cpu().numpy()
    assert (g[:guard] == 0xAB).all() and (g[-guard:] == 0xAB).all()
    end = int(oo[n].item()) & 0xFFFFFFFF
    assert (g[guard + end : guard + need] == 0xAB).all(), "bytes written past the reported span"
    near = np.zeros(n, bool)
    near[max(0, j - 1) : j + 2] = True  # (literal j - 1 ends at the bad offset: its bytes are not the oracle's)
    ok = np.nonzero(~bad & ~near)[0]
    want = oracle_decode_batch(w.enc_blob, w.enc_off)
    oon = oo.cpu().numpy().view(np.uint32).astype(np.int64)
    outn = g[guard : guard + need]
    for i in ok[:: max(1, len(ok) // 2000)]:  # a sample of the literals that decoded
        assert stn[i] == want[3][i] and oln[i] == want[2][i]
        s0 = int(want[1][i])
        assert np.array_equal(outn[oon[i] : oon[i] + oln[i]], want[0][s0 : s0 + oln[i]])
    codec.check()


def test_many_huge_literals(codec):
    """The huge-literal phase (hpk_huge.h) with many huge literals in one workgroup's range: 64 of 8-20
    KiB first (text, random bytes, cut mid-code), then 64k short ones, so the first workgroup lists
    more than its 16 huge slots hold and the rest go to the long-literal phase; several huge literals
    share a round of pieces. Against the oracle, and at exact-bound regions with guard bytes."""
    from loona_amd import huffman_encode

    rng = np.random.default_rng(88)
    text = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_=;,/.:ABCDEFGHIJ ", np.uint8)
    lits = []
    for k in range(64):
        nb = int(rng.integers(8192, 20000))
        if k % 4 == 3:
            lits.append(rng.integers(0, 256, nb, dtype=np.uint8).tobytes())  # EOS / padding errors early
        else:
            lits.append(bytes(huffman_encode(rng.choice(text, nb * 2).tobytes())[:nb]))
    for _ in range(64000):
        lits.append(huffman_encode(rng.choice(text, int(rng.integers(4, 30))).tobytes()))
    blob, off = pack(lits)
    ref = oracle_decode_batch(blob, off)
    compare_batches(gpu_decode(codec, blob, off), ref, "many huge literals")
    bound = [int(off[i + 1] - off[i]) * 8 // 5 for i in range(len(off) - 1)]
    got, guard = _decode_regions(codec, blob, off, bound, shift=7)
    compare_batches(got, ref, "many huge literals, exact-bound regions at +7")
    assert (guard == 0xAB).all()


def test_stream_destroyed_then_another_stream(codec):
    """a context bound to a caller-created stream A (hpk_ctx_set_stream) that the caller
    then destroys must not touch A's handle when a second stream B first uses it (the switch to
    per-slot events). Every result checked against the oracle."""
    import ctypes

    from loona_amd import synth

    hip = ctypes.CDLL("libamdhip64.so")
    w = synth.config2(n=3000, seed=17)
    want = oracle_decode_batch(w.enc_blob, w.enc_off)
    streams = []
    try:
        for k in range(3):
            s = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(s)) == 0
            codec.set_stream(s.value)
            torch.cuda.synchronize()
            compare_batches(gpu_decode(codec, w.enc_blob, w.enc_off), want, f"stream {k}")
            assert hip.hipStreamSynchronize(s) == 0
            assert hip.hipStreamDestroy(s) == 0
            streams.append(s.value)
    finally:
        codec.set_stream(torch.cuda.current_stream())
    compare_batches(gpu_decode(codec, w.enc_blob, w.enc_off), want, "back on torch's stream")


def test_hpack_blocks_many_chunks_on_device(codec):
    """the block decoder's overlap of its apply threads with the device chunks (threads
    waiting on chunk j's copy-out while later chunks still copy) with enough bytes for the host
    pipeline to cut the batch into its 8 chunks: every interop story six times over under fresh
    decoders, every block compared with the fixture's header list."""
    from loona_amd import hpack

    inter = load("interop.json.gz")
    pairs, want = [], []
    for _ in range(6):
        for enc in sorted(inter):
            for story in inter[enc]:
                d = hpack.Decoder()
                for c in story["cases"]:
                    pairs.append((d, bytes.fromhex(c["wire"])))
                    want.append([(n.encode(), v.encode()) for n, v in c["headers"]])
    assert hpack.decode_blocks(pairs, codec) == want


def test_exact_bound_regions_short_literals(codec):
    """Short literals decoded in the fills into regions of exactly hpk_decoded_bound bytes, back to
    back, on an unaligned output base with guard bytes: all-5-bit-code text (the decoded length
    reaches the bound), mixed text, long codes, random bytes, EOS and bad padding. The v27 body steps
    store unconditionally past the decoded bytes; this pins that such bytes never leave a literal's
    own region (every neighbour is compared with the oracle, the guards must stay 0xAB)."""
    from loona_amd import huffman_encode

    rng = np.random.default_rng(5)
    five = np.frombuffer(b"012aceiost", np.uint8)
    text = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_=;,/.:ABC ", np.uint8)
    lits = []
    for i in range(40000):
        k = i % 5
        n = int(rng.integers(1, 70))
        if k == 0:
            lits.append(huffman_encode(rng.choice(five, n).tobytes()))
        elif k == 1:
            lits.append(huffman_encode(rng.choice(text, n).tobytes()))
        elif k == 2:
            lits.append(huffman_encode(rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
        elif k == 3:
            lits.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        else:
            s = bytearray(huffman_encode(rng.choice(five, n).tobytes()))
            s[-1] ^= 0x01 if s[-1] & 1 else 0  # bad padding when the last bit was padding
            lits.append(bytes(s))
    blob, off = pack(lits)
    ref = oracle_decode_batch(blob, off)
    bound = [int(off[i + 1] - off[i]) * 8 // 5 for i in range(len(off) - 1)]
    for shift in (0, 3):
        got, guard = _decode_regions(codec, blob, off, bound, shift=shift)
        compare_batches(got, ref, f"exact-bound short literals at +{shift}")
        assert (guard == 0xAB).all()


def test_compact_two_streams_overlap(codec):
    """two HPK_ASYNC compacted calls on two streams at once. Each call takes its stream's
    slot of the context (cursor, bound layout, scan scratch, long-literal list), so the second call's
    cursor reset and scan cannot reach the first call's kernel. A large batch on stream 1 is issued
    first, then a different small batch on stream 2; both are checked byte for byte against their
    generated strings, and the layouts must be disjoint and inside each call's capacity."""
    from loona_amd import HuffmanCodec, synth

    if codec.variant != "fill":
        pytest.skip("runs once (its own context, auto kernel selection): the fill variant's run")
    big = synth.device_config2(codec, n=2_000_000, seed=101)
    small = synth.device_config2(codec, n=20_000, seed=202)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with HuffmanCodec(0, stream="own") as c:
        for rep in range(3):
            c.set_stream(s1)
            r1 = c.decode_compact(big.enc_blob, big.enc_off, sync=False)
            c.set_stream(s2)
            r2 = c.decode_compact(small.enc_blob, small.enc_off, sync=False)
            torch.cuda.synchronize()
            c.check()
            for w, (out, oo, ol, st) in ((big, r1), (small, r2)):
                _check_compact(out, oo, ol, w.n)
                synth.check_decoded(w, out, oo, ol, st)


@pytest.mark.parametrize("kernel", ["fill", "wave"])
def test_first_call_on_foreign_stream_then_slot_reuse(codec, kernel):
    """a context whose FIRST call runs on a stream it does not own, followed by calls on 9
    more streams, so that the 8 per-stream slots (long-literal list, bound layout, cursor) are all taken
    and the oldest one -- the foreign stream's, still decoding a large batch -- is reused. The slot's
    recorded event must survive the switch to multi-stream mode, so the reuse waits for the large
    decode instead of resetting its cursor or list under it. Both compacted forms (the fill kernel's
    device cursor, the wave kernel's per-workgroup shares) and the region form; every output checked
    byte for byte against the generated strings."""
    from loona_amd import HuffmanCodec, synth

    if codec.variant != "fill":
        pytest.skip("runs once per kernel, on its own context")
    big = synth.device_config3(codec, n=300_000, seed=303)  # long literals: the long-literal list is used
    small = [synth.device_config2(codec, n=5_000 + 997 * k, seed=400 + k) for k in range(9)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(10)]
    with HuffmanCodec(0, stream="own") as c:
        c.set_decode_kernel(kernel)
        for compact in (True, False):
            c.set_stream(streams[0])
            if compact:
                r0 = c.decode_compact(big.enc_blob, big.enc_off, sync=False)
            else:
                r0 = c.decode_device(big.enc_blob, big.enc_off, sync=False)
            rs = []
            for k, w in enumerate(small):
                c.set_stream(streams[k + 1])
                rs.append(c.decode_compact(w.enc_blob, w.enc_off, sync=False) if compact
                          else c.decode_device(w.enc_blob, w.enc_off, sync=False))
            torch.cuda.synchronize()
            c.check()
            for w, (out, oo, ol, st) in [(big, r0)] + list(zip(small, rs)):
                if compact:
                    _check_compact(out, oo, ol, w.n)
                synth.check_decoded(w, out, oo, ol, st)
        c.set_stream(torch.cuda.current_stream())


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 300_001, 16_781_313])
def test_bound_scan(codec, n):
    """The compacted form's bound layout (hpk_bound_scan, two passes over in_off): the exclusive sum
    of the literals' 4-rounded decoded bounds mod 2^32 over n + 1 elements, across the tile boundaries
    (4,096 literals) and past one workgroup of tile sums (16,777,216 literals); decreasing offsets take
    the clamped bound 2^31 - 1 rounded as the library does."""
    import torch

    from loona_amd import _lib

    if codec.variant != "wave" and n > 4097:
        pytest.skip("one kernel variant is enough for the large sizes")
    g = np.random.default_rng(n + 11)
    ln = g.integers(0, 80, size=n, dtype=np.int64)
    if n > 100:
        ln[g.integers(0, n, size=8)] = g.integers(2000, 5000, size=8)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(ln, out=off[1:])
    off32 = off.astype(np.uint32)
    if n >= 4097:  # a decreasing pair: off[i + 1] - off[i] wraps in u32
        off32[4000] = off32[4001] + 7
    d = np.diff(off32.astype(np.int64)) % 2**32
    b = np.minimum(((d * 8) // 5 + 3) & ~3, 0x7FFFFFFF)
    want = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(b, out=want[1:])
    want %= 2**32
    din = torch.from_numpy(off32.view(np.int32)).to(codec.device)
    dout = torch.full((n + 1,), -1, dtype=torch.int32, device=codec.device)
    rc = _lib.lib().hpk_test_bound_scan(codec._h, din.data_ptr(), n, dout.data_ptr())
    assert rc == 0
    got = dout.cpu().numpy().view(np.uint32).astype(np.int64)
    assert (got == want).all(), np.nonzero(got != want)[0][:5]


@pytest.mark.parametrize("shift", [1, 3, 6])
def test_compact_unaligned_bases(codec, shift):
    """The compacted form on blobs whose bases are not 16-, 4- or 2-aligned (the wave kernel's lane
    stores are 16-byte pieces at any byte address, their last piece ending at the literal's last
    byte): literals of 0-3 decoded bytes (bytewise), 4-15 (dwords), 16-100 (pieces) and >= 64 encoded
    bytes (listed for the long-literal phase), two of >= 8 KiB (the huge phase), bad padding; bytes equal the oracle's,
    literals disjoint, nothing written outside [0, out_off[n]) of the output (guard bytes)."""
    from hpk_util import oracle_encode

    from loona_amd.batch import compact_capacity

    if not codec.compact:
        pytest.skip("the compacted form only")
    g = np.random.default_rng(40 + shift)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, ABCDEFGH", np.uint8)
    lits = []
    for i in range(3000):
        k = i % 10
        n = int(g.integers(0, 4)) if k == 0 else int(g.integers(4, 16)) if k < 4 else \
            int(g.integers(16, 101)) if k < 9 else int(g.integers(100, 400))
        if i in (1234, 2345):  # two huge literals (>= 8 KiB encoded: the huge-literal phase)
            n = 14000 + i
        s = bytes(alpha[g.integers(0, alpha.size, size=n)])
        if i % 97 == 5:
            s = bytes(g.integers(0, 256, size=n, dtype=np.uint8))
        e = oracle_encode(s)
        if i % 101 == 7 and e:
            e = e[:-1] + bytes([e[-1] & 0xF0])  # bad padding (or a changed last code)
        lits.append(e)
    blob, off = pack(lits)
    n = len(lits)
    want = oracle_decode_batch(blob, off)
    guard = 4096
    need = compact_capacity(blob.size, n)
    ibig = torch.zeros(blob.size + 64, dtype=torch.uint8, device="cuda")
    ibig[shift : shift + blob.size] = torch.from_numpy(blob).cuda()
    din = ibig[shift : shift + blob.size]
    big = torch.full((guard + need + guard + 16,), 0xAB, dtype=torch.uint8, device="cuda")
    out = big[guard + shift : guard + shift + need]
    oo = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
    ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    codec.decode_compact(din, to_dev(off.view(np.int32)), out, oo, ol, st, sync=True)
    _check_compact(out, oo, ol, n)
    gb = big.cpu().numpy()
    assert (gb[: guard + shift] == 0xAB).all(), "bytes written before the output"
    end = int(oo[n].item()) & 0xFFFFFFFF
    assert (gb[guard + shift + end :] == 0xAB).all(), "bytes written past the reported span"
    outn = gb[guard + shift : guard + shift + need]
    oon = oo.cpu().numpy().view(np.uint32).astype(np.int64)
    got = (outn, np.concatenate([oon[:n], [end]]), ol.cpu().numpy().view(np.uint32), st.cpu().numpy())
    stw, lw = want[3], want[2]
    assert (got[3] == stw).all(), np.nonzero(got[3] != stw)[0][:5]
    assert (got[2] == lw).all(), np.nonzero(got[2] != lw)[0][:5]
    wo = np.asarray(want[1], dtype=np.int64)
    for i in range(n):
        a, m = int(oon[i]), int(lw[i])
        assert bytes(outn[a : a + m]) == bytes(want[0][wo[i] : wo[i] + m]), f"literal {i}"


def test_small_mode_idle_restart_bad_offsets_and_off(codec):
    """The small-call mode (hpk_ctx_set_small_mode): calls answered by the persistent kernel give the
    oracle's bytes; after its idle exit the next call starts it again; a batch with bad offsets is handed
    to the launch path (the call fails as in the launch path, nothing is written outside the blobs);
    turned off, calls go to the launch path. Runs once (the fixture's small variant)."""
    if codec.variant != "small":
        pytest.skip("small-call mode case: once")
    import time

    from loona_amd import _lib
    from loona_amd.batch import decode_offsets_torch

    L = _lib.lib()
    rng = np.random.default_rng(41)
    strs = [bytes(rng.choice(list(b"abcdefghijklmnopqrstuvwxyz0123456789-/.:;="), int(k))) for k in rng.integers(0, 70, 1000)]
    from hpk_util import oracle_encode

    lits = [oracle_encode(x) for x in strs]
    lits += [bytes.fromhex(k["in"]) for k in load("kat.json")]
    blob, off = pack(lits)
    want = oracle_decode_batch(blob, off)

    def run(expect_small):
        before = L.hpk_test_small_calls(codec._h)
        got = gpu_decode(codec, blob, off)
        compare_batches(got, want, "small mode")
        assert (L.hpk_test_small_calls(codec._h) - before == 1) == expect_small

    codec.set_small_mode(4096, 2, 2)  # (2 ms idle)
    run(True)
    time.sleep(0.05)  # the kernel has exited
    run(True)
    run(True)
    # bad offsets: the launch path's result and error
    n = len(lits)
    dblob = to_dev(blob)
    bad = np.asarray(off, np.int64).copy()
    bad[n // 2] = bad[n // 2 + 1] + 1  # a decreasing pair
    doff = to_dev(bad.astype(np.int32))
    oo = decode_offsets_torch(to_dev(np.asarray(off, np.int64).astype(np.int32)))
    out = torch.full((int(oo[-1].item()) + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    before = L.hpk_test_small_calls(codec._h)
    with pytest.raises(Exception):
        codec.decode_into(dblob, doff, out, oo, ol, st, device=True, sync=True)
    assert L.hpk_test_small_calls(codec._h) == before
    assert (st.cpu().numpy() == 5).any()  # HPK_BAD_OFFSETS, from the launch path
    assert (out[int(oo[-1].item()):].cpu().numpy() == 0xAB).all()
    run(True)  # the mode still answers after a declined batch
    codec.set_small_mode(0)
    run(False)
    codec.set_small_mode(65536, 4, 200)
    run(True)
