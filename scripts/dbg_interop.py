#!/usr/bin/env python3
"""Dev check: decode the interop corpus (and subsets) on the GPU, compare with the oracle."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from hpk_util import compare_batches, interop_literals, oracle_decode_batch, pack  # noqa: E402

import torch  # noqa: E402

from loona_amd import HuffmanCodec  # noqa: E402

lits = interop_literals()
print("literals", len(lits), "long", sum(len(x) >= 224 for x in lits), flush=True)
with HuffmanCodec(0, stream=torch.cuda.current_stream()) as c:
    for name, sel in [("short", [x for x in lits if len(x) < 224]), ("long", [x for x in lits if len(x) >= 224]),
                      ("all", lits)]:
        blob, off = pack(sel)
        t0 = time.time()
        out, oo, ol, st = c.decode_device(torch.from_numpy(blob).cuda(), torch.from_numpy(off.astype(np.int32)).cuda(),
                                          sync=True)
        torch.cuda.synchronize()
        n = len(sel)
        got = (out.cpu().numpy(), oo.cpu().numpy().astype(np.uint32), ol[:n].cpu().numpy().astype(np.uint32),
               st[:n].cpu().numpy())
        print(name, n, "decoded in", round(time.time() - t0, 3), "s", flush=True)
        compare_batches(got, oracle_decode_batch(blob, off), name)
        print(name, "OK", flush=True)
