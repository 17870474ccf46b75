#!/usr/bin/env python3
"""(round 6, development) Where a decode of config 3 differs from the generated strings: per bad literal its
status, length (got / want), encoded length and first differing byte. HPK_LIB selects the library."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from loona_amd import HuffmanCodec, synth  # noqa: E402
from loona_amd.batch import decode_offsets_torch  # noqa: E402

codec = HuffmanCodec(0)
if len(sys.argv) > 2:
    codec.set_decode_kernel(sys.argv[2])
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
w = synth.device_config3(codec, n=n)
doff = decode_offsets_torch(w.enc_off)
out = torch.empty(int(doff[-1].item()) + 16, dtype=torch.uint8, device="cuda")
ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
codec.decode_into(w.enc_blob, w.enc_off, out, doff, ol, st, device=True, sync=True)
want = (w.dec_off[1:] - w.dec_off[:-1]).to(torch.int64)
enc = (w.enc_off[1:].to(torch.int64) - w.enc_off[:-1].to(torch.int64))
bad = torch.nonzero((st[: w.n] != 0) | (ol[: w.n].to(torch.int64) != want)).flatten()
res = {"n": w.n, "bad": int(bad.numel()), "examples": []}
# byte mismatches on literals with the right length and status
okl = torch.nonzero((st[: w.n] == 0) & (ol[: w.n].to(torch.int64) == want)).flatten()
nb = 0
for i in okl[enc[okl] >= 128].tolist()[:200000]:
    a, b = int(doff[i].item()), int(w.dec_off[i].item())
    L = int(want[i].item())
    if not torch.equal(out[a:a + L], w.dec_blob[b:b + L]):
        nb += 1
        if nb <= 10:
            d = torch.nonzero(out[a:a + L] != w.dec_blob[b:b + L]).flatten()
            res["examples"].append({"i": i, "kind": "bytes", "enc": int(enc[i]), "len": L, "first_diff": int(d[0]),
                                    "ndiff": int(d.numel())})
res["byte_bad"] = nb
for i in bad.tolist()[:20]:
    res["examples"].append({"i": i, "status": int(st[i]), "len": int(ol[i]), "want": int(want[i]), "enc": int(enc[i])})
print(json.dumps(res))
