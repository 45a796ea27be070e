"""Static check of the built code object (CPU): every buffer store of more
than 64 bits keeps its data VGPRs unwritten for two wait states.

hipcc (ROCm 7.2) pads this VMEM-store data hazard for global stores but not
for __builtin_amdgcn_raw_buffer_store_b128: a VALU write of a data register
in the next instruction can reach memory instead of the stored value.  In
round 5 that corrupted a few Adam second-moment entries of the streaming
update per launch (LDS-offset bit patterns in v), until every b128 buffer
store went through BSTORE128 (csrc/psvi_internal.hpp: the store, then an
``s_nop 1`` that reads the data).  This test disassembles
psvi/runtime/libpsvi_hip.so's gfx950 code objects and fails on any such store
whose data registers are redefined within two wait states -- a raw b128
buffer store added without the macro."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "blackbox-coresets-vi_amd", "psvi", "runtime", "libpsvi_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
WAIT_STATES = 2

STORE = re.compile(r"^\s*buffer_store_dwordx([34])\s+v\[(\d+):(\d+)\]")
# an instruction line of llvm-objdump -d: mnemonic, operands, // address: encoding
INST = re.compile(r"^\s*([a-z_][a-z0-9_]*)\s*(.*?)\s*//")
VREG = re.compile(r"^v\[(\d+):(\d+)\]|^v(\d+)\b")
# mnemonics whose first operand is not a VGPR destination
NO_VDST = ("s_", "buffer_store", "global_store", "flat_store", "scratch_store", "ds_write",
           "ds_store", "v_cmp", "v_cmpx", "v_readlane", "v_readfirstlane", "buffer_atomic",
           "global_atomic", "exp", "ds_add", "ds_max", "ds_min")


def _dst_vgprs(mnem, ops):
    if mnem.startswith(NO_VDST) or not ops:
        return set()
    m = VREG.match(ops.split(",")[0].strip())
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def _waits(mnem, ops):
    if mnem == "s_nop":
        return int(ops.split()[0], 0) + 1
    return 1


def check_listing(lines):
    """(stores checked, [violations]) over one disassembly."""
    n, bad = 0, []
    for i, line in enumerate(lines):
        m = STORE.match(line)
        if not m:
            continue
        n += 1
        data = set(range(int(m.group(2)), int(m.group(3)) + 1))
        ws = 0
        for nxt in lines[i + 1:i + 8]:
            im = INST.match(nxt)
            if not im:
                if nxt.strip().endswith(">:") or not nxt.strip():
                    break  # the next function / a label ends the straight line
                continue
            mnem, ops = im.group(1), im.group(2)
            if _dst_vgprs(mnem, ops) & data:
                bad.append((line.strip(), nxt.strip()))
                break
            ws += _waits(mnem, ops)
            if ws >= WAIT_STATES:
                break
    return n, bad


def test_checker_flags_an_unpadded_store():
    ok = ["\tbuffer_store_dwordx4 v[10:13], v48, s[40:43], 0 offen sc1 // 0: E0",
          "\ts_nop 1 // 8: BF",
          "\tv_or_b32_e32 v10, v1, v2 // c: 00"]
    hazard = [ok[0], "\tv_or_b32_e32 v10, v1, v2 // 8: 00"]
    mfma_between = [ok[0], "\tv_mfma_f32_32x32x2_f32 a[0:15], v54, v58, a[0:15] // 8: D3",
                    "\tv_mov_b32_e32 v12, 0 // 10: 7E"]
    assert check_listing(ok) == (1, [])
    assert check_listing(hazard)[1] and check_listing(mfma_between)[1]
    later = [ok[0], "\tv_add_u32_e32 v1, v2, v3 // 8: 00", "\tv_add_u32_e32 v4, v2, v3 // c: 00",
             "\tv_mov_b32_e32 v10, 0 // 10: 7E"]
    assert check_listing(later) == (1, [])   # two wait states passed


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump (ROCm) not installed")
def test_b128_buffer_stores_are_padded(tmp_path):
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} is not built (make -C blackbox-coresets-vi_amd)")
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], cwd=tmp_path, check=True,
                   capture_output=True)
    objs = sorted(p for p in os.listdir(tmp_path) if p.endswith("gfx950"))
    assert objs, "no gfx950 code object in the library"
    total, bad = 0, []
    for o in objs:
        out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(tmp_path / o)], check=True,
                             capture_output=True, text=True).stdout
        n, b = check_listing(out.splitlines())
        total += n
        bad += b
    assert total > 0, "no b128 buffer store found: the streaming update's state stores use them"
    assert not bad, f"{len(bad)} unpadded >64-bit buffer stores, first: {bad[:3]}"
