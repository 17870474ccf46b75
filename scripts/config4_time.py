#!/usr/bin/env python3
"""Config 4 (captured HEADERS, hpk_hdec_decode_blocks) on the library HPK_LIB names: bench.py's
config4 block (device leg and library CPU batch leg, median of 5 alternating calls) plus the
per-pass times of 5 more calls per leg (HPK_HDEC_TIMING). One JSON line."""
import json
import os
import re
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    if os.environ.get("_C4_CHILD"):
        sys.path.insert(0, REPO)
        import torch  # noqa: F401

        import bench
        from loona_amd import HuffmanCodec

        codec = HuffmanCodec(0)
        r = bench.run_config4(codec, 16)
        r["lib"] = os.path.basename(os.environ.get("HPK_LIB", "libhpk.so"))
        print(json.dumps(r))
        return
    env = dict(os.environ, _C4_CHILD="1", HPK_HDEC_TIMING="1")
    p = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        sys.stderr.write(p.stderr[-3000:])
        raise SystemExit(p.returncode)
    line = json.loads(p.stdout.strip().splitlines()[-1])
    passes = {}
    for l in p.stderr.splitlines():
        m = re.search(r"scan (\d+) us, batch (\w+) (\d+) us, apply (\d+) us, join (\d+) us", l)
        if m:
            leg = "device" if m.group(2) == "issue" else "cpu_batch"
            passes.setdefault(leg, []).append([int(m.group(i)) for i in (1, 3, 4, 5)])
    line["pass_median_us"] = {leg: dict(zip(("scan", "batch", "apply", "join"),
                                            [statistics.median(x[i] for x in v) for i in range(4)]))
                              for leg, v in passes.items()}
    print(json.dumps({k: line[k] for k in ("lib", "device_ms", "cpu_batch_ms", "device_over_cpu", "calls_ms",
                                           "pass_median_us", "host_threads")}))


if __name__ == "__main__":
    main()
