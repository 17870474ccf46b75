#!/usr/bin/env python3
"""Extract the per-lane decode code of the product kernels (loona_amd/csrc) into a host-compilable
header (tests/emu/shim.h stands in for the HIP builtins), so tests/test_walk_emulation.py can run the
REAL lane-walk functions (lit12_body, lit12_step, the tails' end detection) and the huge-literal
phase's per-piece functions on the CPU against the oracle. Test infrastructure only."""
import re
import sys

csrc = sys.argv[1]
out_path = sys.argv[2]
k = open(f"{csrc}/hpk_decode_kernel.h").read()
kpart = k[k.index("namespace hpkdec {") : k.index("// v7: output staged in LDS")]
kpart = kpart.replace("__device__ unsigned long long g_chk[8];", "unsigned long long g_chk[8];")
kpart = re.sub(r"__device__ __forceinline__ void chk_report\(.*?\n}\n",
               "inline void chk_report(uint32_t, uint32_t, uint32_t, uint32_t) {}\n", kpart, flags=re.S)
d = open(f"{csrc}/hpk_decode12.h").read()
walk = d[d.index("namespace hpkdec {") : d.index('#include "hpk_long.h"')]
walk = re.sub(r"// LDS carve-up: Geo7.*?\n};\n", "", walk, flags=re.S)
h = open(f"{csrc}/hpk_huge.h").read()
huge = h[h.index("namespace hpkdec {") :]
hdr = ['#pragma once', '#include "shim.h"', f'#include "{csrc}/hpk_code.h"',
       "#define HPK_OK 0", "#define HPK_PADDING_TOO_LARGE 1", "#define HPK_INVALID_PADDING 2",
       "#define HPK_EOS_IN_STRING 3", "#define HPK_OUTPUT_OVERFLOW 4", "#define HPK_BAD_OFFSETS 5",
       "#define HPK_FLUSH_LOOP 1", "#define HPK_HUGE_HOST 1", kpart, "}  // namespace hpkdec", walk, huge]
open(out_path, "w").write("\n".join(hdr))
