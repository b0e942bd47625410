#!/usr/bin/env python3
"""Disassemble the gfx950 code object of a built library (development tool):
tools/dis_lib.py [lib] > out.dis  (same extraction as tests/test_tile_isa.py)."""
import os
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "spgemm_new_amd", "lib",
    "libmaxk_spgemm.so")
with tempfile.TemporaryDirectory() as d:
    fat = os.path.join(d, "fat.bin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", lib],
                   check=True)
    b = open(fat, "rb").read()
    i = b.find(b"__CLANG_OFFLOAD_BUNDLE__")
    n = struct.unpack_from("<Q", b, i + 24)[0]
    off = i + 32
    for _ in range(n):
        o, sz, tl = struct.unpack_from("<QQQ", b, off)
        off += 24
        triple = b[off:off + tl].decode()
        off += tl
        if "gfx950" in triple:
            co = os.path.join(d, "dev.co")
            open(co, "wb").write(b[i + o:i + o + sz])
            sys.stdout.write(subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co],
                                            check=True, capture_output=True, text=True).stdout)
