"""The TILE backward's counted-vmcnt invariant, checked on the compiled code
(CPU, no GPU): bwd_tile_kernel waits for its chunk with a COUNTED
`s_waitcnt vmcnt(N)` that assumes every step issues exactly kTilePieces DMA
loads + 1 header load + 1 record prefetch (csrc/maxk_spgemm.hip, `step`; a step
issuing a different number of VMEM operations makes a wave read a header still
in flight -> garbage record counts -> a memory-access fault).
The compiler could break that silently (a spill, a hoisted load), so this
disassembles the built library's gfx950 code object and checks every
specialisation: each step barrier is preceded by vmcnt(kTileVmcnt), the code
between consecutive step barriers issues exactly kTilePieces + 2 VMEM loads, no
scratch is used, and the barrier count is the unrolled ring.
Round 4: the kernel loops over the pieces of its workgroup range; the piece
loop must not push the ring loop into spills (checked: no scratch).
"""
import os
import re
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "spgemm_new_amd", "lib", "libmaxk_spgemm.so")
LLVM = "/opt/rocm/lib/llvm/bin"
PIECES, NBUF = 3, 3       # tile_format.h: kTilePieces, TILE_NBUF (the default build)
STEP_OPS = PIECES + 2
VMCNT = (STEP_OPS - PIECES) + STEP_OPS * (NBUF - 2)   # kTileVmcnt

LOAD = re.compile(r"\s(buffer_load\w*|global_load\w*|flat_load\w*|scratch_load\w*)\s")
SCRATCH = re.compile(r"\sscratch_\w+|\sbuffer_\w+.*\boffen\b.*s\[0:3\]")


def _code_object(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    objcopy, objdump = os.path.join(LLVM, "llvm-objcopy"), os.path.join(LLVM, "llvm-objdump")
    if not (shutil.which(objcopy) and shutil.which(objdump)):
        pytest.skip("llvm tools not available")
    fat = tmp_path / "fat.bin"
    subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fat}", LIB], check=True)
    b = fat.read_bytes()
    i = b.find(b"__CLANG_OFFLOAD_BUNDLE__")
    assert i >= 0
    n = struct.unpack_from("<Q", b, i + 24)[0]
    off = i + 32
    for _ in range(n):
        o, sz, tl = struct.unpack_from("<QQQ", b, off)
        off += 24
        triple = b[off:off + tl].decode()
        off += tl
        if "gfx950" in triple:
            co = tmp_path / "dev.co"
            co.write_bytes(b[i + o:i + o + sz])
            out = subprocess.run([objdump, "-d", str(co)], check=True, capture_output=True,
                                 text=True).stdout
            return out
    pytest.fail("no gfx950 code object in the library")


def _functions(dis, pat):
    """{symbol: [instruction lines]} of the functions whose name matches pat."""
    funcs, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1) if re.search(pat, m.group(1)) else None
            if cur:
                funcs[cur] = []
            continue
        if cur and line.strip():
            funcs[cur].append(line.split("//")[0])
    return funcs


def test_tile_step_vmem_count(tmp_path):
    dis = _code_object(tmp_path)
    funcs = _functions(dis, r"bwd_tile_kernel")
    assert len(funcs) == 4, list(funcs)          # K in {32, 64} x {buffer, global} DMA
    for name, lines in funcs.items():
        assert not any(SCRATCH.search(ln) for ln in lines), f"{name}: scratch in the TILE kernel"
        steps, barriers = [], []
        for i, ln in enumerate(lines):
            if "s_barrier" in ln and i > 0:
                barriers.append(i)
                # the step barrier's own wait (the record asm: a bare counted vmcnt);
                # the compiler's waits before __syncthreads name other counters too
                m = re.search(r"s_waitcnt vmcnt\((\d+)\)\s*$", lines[i - 1])
                if m:
                    assert int(m.group(1)) == VMCNT, (name, lines[i - 1])
                    steps.append(i)
        assert len(steps) == NBUF, (name, len(steps))   # the ring's steps, unrolled
        # a step's code runs to the next barrier (the last step's: to the piece's
        # closing barrier, or the end)
        ends = [next((j for j in barriers if j > a), len(lines)) for a in steps]
        for a, b_ in zip(steps, ends):
            loads = [ln.strip() for ln in lines[a:b_] if LOAD.search(" " + ln + " ")]
            assert len(loads) == STEP_OPS, (name, loads)
            dma = [ln for ln in loads if " lds" in ln or "load_lds" in ln]
            assert len(dma) == PIECES, (name, loads)
