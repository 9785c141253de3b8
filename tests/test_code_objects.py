"""Resource checks on the built library's gfx950 code objects (CPU only: reads the .so).

The hot kernels run at two waves per SIMD with up to 256 VGPRs; a register spill there puts
scratch loads on the critical path (and a spilled address reload's vmcnt(0) drains the LDS-DMA
prefetch).  Round 2 shipped the causal forward and dQ with 64 and 92 bytes of scratch per lane
(VERDICT.md, weak 3-4); this test keeps every hot instantiation at zero.

How: the .so's `.hip_fatbin` section holds one clang offload bundle per translation unit; each
gfx950 entry is an ELF code object whose `<kernel>.kd` symbols point at 64-byte kernel
descriptors (AMDGPU ABI: group_segment_fixed_size u32 @0, private_segment_fixed_size u32 @4,
compute_pgm_rsrc1 u32 @48 with the VGPR granule in bits 0-5).  Pure-Python ELF parsing, no ROCm
tools needed.
"""
import os
import re
import struct

import pytest

from fa2_triton_amd import _lib

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf: bytes):
    """{name: (offset, size, addr)} of a 64-bit little-endian ELF."""
    assert elf[:4] == b"\x7fELF" and elf[4] == 2 and elf[5] == 1
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    heads = []
    for i in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, shoff + i * shentsize)
        heads.append((name, typ, addr, off, size, link, entsize))
    stroff = heads[shstrndx][3]

    def nm(o):
        return elf[stroff + o: elf.index(b"\0", stroff + o)].decode()

    return {nm(h[0]): h for h in heads}, heads


def _code_objects(lib_path):
    data = open(lib_path, "rb").read()
    secs, _ = _sections(data)
    _, _, _, off, size, _, _ = secs[".hip_fatbin"]
    fat = data[off: off + size]
    pos = 0
    while True:
        pos = fat.find(MAGIC, pos)
        if pos < 0:
            return
        n, = struct.unpack_from("<Q", fat, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24: p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and esize:
                yield fat[pos + eoff: pos + eoff + esize]
        pos += len(MAGIC)


def _kernel_descriptors(co: bytes):
    """{kernel symbol: (private_segment_fixed_size, vgprs, lds_bytes)} of one code object."""
    secs, heads = _sections(co)
    name, typ, addr, off, size, link, entsize = secs[".symtab"] if ".symtab" in secs else secs[".dynsym"]
    stroff = heads[link][3]
    out = {}
    for i in range(size // 24):
        st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", co, off + i * 24)
        sym = co[stroff + st_name: co.index(b"\0", stroff + st_name)].decode()
        if not sym.endswith(".kd") or st_shndx == 0:
            continue
        sh = heads[st_shndx]
        fo = sh[3] + (st_value - sh[2])
        lds, scratch = struct.unpack_from("<II", co, fo)
        rsrc1, = struct.unpack_from("<I", co, fo + 48)
        out[sym[:-3]] = (scratch, ((rsrc1 & 0x3F) + 1) * 8, lds)
    return out


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    kd = {}
    for co in _code_objects(_lib.LIB_PATH):
        kd.update(_kernel_descriptors(co))
    assert kd, "no gfx950 kernel descriptors found in the library"
    return kd


# hot instantiations: bf16 / fp16 (Lb1 / Lb0), D tiles 64 and 128, causal and not; the plain
# path (no bias, no dropout, aligned; dQ in the input dtype)
HOT = {
    "fwd_pipe": r"_ZN3fa215fwd_pipe_kernelILb[01]ELi(64|128)ELb[01]ELi4ELi0EEEv12fa2_fwd_args",
    "dq": r"_ZN3fa29dq_kernelILb[01]ELi(64|128)ELb[01]ELi0ELb0ELb1ELb0EEEv12fa2_bwd_args",
    "dkdv": r"_ZN3fa211dkdv_kernelILb[01]ELi(64|128)ELb[01]ELi0ELb0ELb1EEEv12fa2_bwd_argsi",
}


@pytest.mark.parametrize("kind", sorted(HOT))
def test_hot_kernels_have_no_scratch(kernels, kind):
    pat = re.compile(HOT[kind] + "$")
    found = {k: v for k, v in kernels.items() if pat.match(k)}
    assert len(found) == 8, (kind, sorted(found))  # 2 dtypes x 2 head-dim tiles x causal / not
    spilled = {k: v[0] for k, v in found.items() if v[0] != 0}
    assert not spilled, f"scratch bytes per lane: {spilled}"
    for k, (_, vgprs, lds) in found.items():
        assert vgprs <= 256, (k, vgprs)  # two waves per SIMD
        assert lds <= 80 * 1024, (k, lds)  # two workgroups per CU


def test_every_kernel_fits_the_cu(kernels):
    for k, (scratch, vgprs, lds) in kernels.items():
        assert vgprs <= 512 and lds <= 160 * 1024, (k, vgprs, lds)


# the hand-placed one-wave-per-SIMD kernels (hp_gen.py): whole register file, zero scratch
HP = {
    "fwd_hp": r"_ZN3fa213fwd_hp_kernelILb[01]ELb[01]ELb1ELi128ELb[01]EEEv12fa2_fwd_args",
    "dkdv_hp": r"_ZN3fa214dkdv_hp_kernelILb[01]ELb[01]ELb[01]EEEv12fa2_bwd_argsi",
    "dq_hp": r"_ZN3fa212dq_hp_kernelILb[01]ELb[01]ELb[01]EEEv12fa2_bwd_args",
}


@pytest.mark.parametrize("kind", sorted(HP))
def test_hand_placed_kernels_have_no_scratch(kernels, kind):
    pat = re.compile(HP[kind] + "$")
    found = {k: v for k, v in kernels.items() if pat.match(k)}
    # dtypes x causal x dropout (the pre-scaled-Q forward exists only in development builds,
    # FA2_HP_DEV)
    assert len(found) == 8, (kind, sorted(found))
    for k, (scratch, vgprs, lds) in found.items():
        assert scratch == 0, (k, scratch)
        assert vgprs <= 512 and lds <= 160 * 1024, (k, vgprs, lds)  # one workgroup of 4 waves per CU


# The accumulators of a hand-placed kernel live in fixed AGPRs from the end of its main statement
# until the read statements copy them out.  Nothing the compiler emits in between may write those
# registers (a "+a" operand moved there early overwrote dQ rows once).  Checked on the ISA: from
# the statement's closing `s_nop 15` pair to the last accumulator read, no AGPR write to them.
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
ACC_RANGE = {"fwd_hp": 128, "dq_hp": 128, "dkdv_hp": 256}


def _disassemble(co: bytes, tmp_path, n):
    import subprocess

    f = tmp_path / f"co{n}.o"
    f.write_bytes(co)
    res = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(f)], capture_output=True, text=True)
    return res.stdout


@pytest.mark.parametrize("kind", sorted(ACC_RANGE))
def test_accumulators_untouched_until_read(tmp_path, kind):
    if not os.path.exists(_lib.LIB_PATH) or not os.path.exists(OBJDUMP):
        pytest.skip("library or llvm-objdump missing")
    n_acc0 = ACC_RANGE[kind]
    sym = {"fwd_hp": "fwd_hp_kernel", "dq_hp": "dq_hp_kernel", "dkdv_hp": "dkdv_hp_kernel"}[kind]
    checked = 0
    for n, co in enumerate(_code_objects(_lib.LIB_PATH)):
        if sym.encode() not in co:
            continue
        text = _disassemble(co, tmp_path, n)
        for func in re.split(r"\n(?=[0-9a-f]+ <)", text):
            if sym not in func.split("\n", 1)[0]:
                continue
            n_acc = n_acc0
            lines = [ln.split("//")[0].strip() for ln in func.split("\n")[1:]]
            lines = [ln for ln in lines if ln]
            i = 0
            while i < len(lines):
                if lines[i].startswith("s_nop 15") and i + 1 < len(lines) and lines[i + 1].startswith("s_nop 15"):
                    # window: up to the read of the last accumulator register
                    last = f"a{n_acc - 1}"
                    j = i + 2
                    while j < len(lines) and not (lines[j].startswith("v_accvgpr_read_b32") and lines[j].endswith(last)):
                        m = re.match(r"(v_accvgpr_write_b32|v_accvgpr_mov_b32|\w*load\w*)\s+a\[?(\d+)", lines[j])
                        assert not (m and int(m.group(2)) < n_acc), (kind, lines[j])
                        j += 1
                    checked += 1
                    i = j
                i += 1
    assert checked > 0, f"no {kind} main statement found"


def test_bias_gradient_kernels_have_no_scratch(kernels):
    """dbias_kernel (round-4 restructure: the block's sums in registers over the broadcast group)
    in every instantiation -- dtypes, head-dim tiles, causal, dropout, alignment -- spills nothing."""
    found = {k: v for k, v in kernels.items() if "dbias_kernel" in k}
    assert len(found) == 64, sorted(found)
    assert not {k: v[0] for k, v in found.items() if v[0]}, "scratch bytes per lane"


# the kernels a D = 128 run with a 16-bit bias whose rows are 16-byte aligned dispatches to (the
# bench's --bias line; the reference's test_fwd_only always has a bias): the pipelined forward
# and dK/dV spill nothing; the bias dQ spills a few dwords at two waves per SIMD (one wave per SIMD
# removes it but measured 20 % slower), bounded here so that it cannot grow unnoticed
BIAS_LINE = {
    "fwd_pipe": (r"_ZN3fa215fwd_pipe_kernelILb[01]ELi128ELb[01]ELi4ELi1[67]EEEv12fa2_fwd_args", 0),
    "dkdv": (r"_ZN3fa211dkdv_kernelILb[01]ELi128ELb[01]ELi1[67]ELb0ELb1EEEv12fa2_bwd_argsi", 0),
    "dq": (r"_ZN3fa29dq_kernelILb[01]ELi128ELb[01]ELi1[67]ELb0ELb1ELb[01]EEEv12fa2_bwd_args", 48),
}


@pytest.mark.parametrize("kind", sorted(BIAS_LINE))
def test_bias_line_kernels_scratch(kernels, kind):
    pat, limit = BIAS_LINE[kind]
    found = {k: v for k, v in kernels.items() if re.match(pat + "$", k)}
    assert len(found) == (16 if kind == "dq" else 8), (kind, sorted(found))  # dtypes x causal x bias dtype (x dQ dtype)
    over = {k: v[0] for k, v in found.items() if v[0] > limit}
    assert not over, f"scratch bytes per lane over {limit}: {over}"


# The next unit's Q (forward) and Q / dO (dQ) fragments are loaded by the main statement's tail
# straight into its "+a" operand registers and stay in flight across the compiler's epilogue
# code: nothing may read, copy or overwrite those AGPRs before the wait (the
# spilling dropout dQ moved them early and computed with garbage).  Windows checked on the ISA:
# forward -- from the statement's closing `s_nop 15` pair to the function end, and from the loop
# head marker (`s_nop 13`) to the next statement's opening `s_nop 7` pair; dQ -- from the closing
# pair to the wait statement (`s_nop 14`).  The dropout dQ loads its next unit in a statement of
# its own (loads and wait together, opening with `s_nop 12`), so nothing is in flight there.
OPERANDS = {"fwd_hp": (128, 192), "dq_hp": (128, 256)}


def _agpr_refs(line):
    out = set()
    for m in re.finditer(r"\ba\[(\d+):(\d+)\]|\ba(\d+)\b", line):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


@pytest.mark.parametrize("kind", sorted(OPERANDS))
def test_in_flight_operands_untouched(tmp_path, kind):
    if not os.path.exists(_lib.LIB_PATH) or not os.path.exists(OBJDUMP):
        pytest.skip("library or llvm-objdump missing")
    lo, hi = OPERANDS[kind]
    sym = {"fwd_hp": "fwd_hp_kernel", "dq_hp": "dq_hp_kernel"}[kind]
    checked = 0
    for n, co in enumerate(_code_objects(_lib.LIB_PATH)):
        if sym.encode() not in co:
            continue
        text = _disassemble(co, tmp_path, n)
        for func in re.split(r"\n(?=[0-9a-f]+ <)", text):
            if sym not in func.split("\n", 1)[0]:
                continue
            lines = [ln.split("//")[0].strip() for ln in func.split("\n")[1:]]
            lines = [ln for ln in lines if ln]
            pairs = lambda op: [i for i in range(len(lines) - 1) if lines[i].startswith(op) and lines[i + 1].startswith(op)]
            ends, starts = pairs("s_nop 15"), pairs("s_nop 7")
            assert len(ends) == 1 and len(starts) == 1, (kind, len(ends), len(starts))
            windows = []
            if kind == "fwd_hp":
                head = [i for i, ln in enumerate(lines) if ln.startswith("s_nop 13")]
                assert len(head) == 1, head
                windows = [(ends[0] + 2, len(lines)), (head[0] + 1, starts[0])]
            else:
                wait = [i for i, ln in enumerate(lines) if ln.startswith(("s_nop 14", "s_nop 12"))]
                assert 1 <= len(wait) <= 2, wait
                windows = [(ends[0] + 2, wait[0])]
            for a, b in windows:
                assert a <= b, (kind, a, b)
                for ln in lines[a:b]:
                    bad = {r for r in _agpr_refs(ln) if lo <= r < hi}
                    assert not bad, (kind, ln)
            checked += 1
    assert checked > 0, f"no {kind} kernel found"
