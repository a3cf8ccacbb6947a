"""CPU: the gfx950 code object of the built library, disassembled, keeps the
explicit wait states around the inline-asm MFMAs of the Gram kernel (NB >= 5,
k > 64: kernels.hip mfma_entry_guard / mfma_exit_guard; an asm statement is
opaque to LLVM's hazard recognizer, cdna_hip_programming.md section 5.7).
A scheduling or compiler change that moved an accumulator read or a VALU
write next to the MFMAs would make wrong normal equations without a fault;
this check fails the build instead.

For every gram_kernel<NB >= 5> instance (and every gram_pair_kernel, whose
accumulators are VGPRs: there the exit check is that each role's last MFMA
run is followed at once by the 20 wait states of mfma_exit_guard_v):
  * every run of consecutive v_mfma instructions (s_nop pads between them
    allowed) is entered >= 3 wait states after the last VALU instruction
    (the guard's `s_nop 4`, or LDS loads / waits of the pair kernel's
    partner operands; VALU writes of P / the zeroed accumulators ->
    SrcA/B/C need <= 2);
  * no v_accvgpr_read / write inside a run (the accumulators stay pinned);
  * between the last v_mfma and the first later instruction touching the
    accumulators (v_accvgpr_read, or an AGPR source), >= 12 wait states on
    the straight-line fall-through path (8-pass XDL result -> reader; an
    issued instruction counts 1, `s_nop n` counts n + 1) before any forward
    branch that could skip them.  The main loop's last half is peeled, so
    the last MFMA in program order is the peeled one and mfma_exit_guard's
    nops (which take every accumulator as an operand, so the compiler's
    accumulator copies cannot move above them) must follow it."""
import os
import re
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "movie_recommender_amd", "lib", "cpp_ls_lib.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _gfx950_objects(so):
    sec = subprocess.run([f"{LLVM}/llvm-readelf", "-S", so], capture_output=True,
                         text=True).stdout
    line = next(l for l in sec.splitlines() if ".hip_fatbin" in l)
    f = line.split("]")[1].split()
    off, size = int(f[3], 16), int(f[4], 16)
    with open(so, "rb") as fh:
        fh.seek(off)
        data = fh.read(size)
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    objs = []
    p = data.find(magic)
    while p >= 0:
        n = struct.unpack_from("<Q", data, p + 24)[0]
        q = p + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", data, q)
            q += 24
            triple = data[q:q + tl].decode()
            q += tl
            if "gfx950" in triple and es:
                objs.append(data[p + eo:p + eo + es])
        p = data.find(magic, p + 1)
    return objs


def _functions(asm):
    out = {}
    for chunk in re.split(r"\n(?=[0-9a-f]{16} <)", asm):
        m = re.match(r"[0-9a-f]{16} <([^>]+)>:", chunk)
        if m:
            out[m.group(1)] = [l.split("//")[0].strip() for l in chunk.splitlines()[1:]]
    return out


def _nop_states(ins):
    m = re.match(r"s_nop\s+(0x[0-9a-f]+|\d+)", ins)
    return int(m.group(1), 0) + 1 if m else 0


def _vregs(ops):
    """Set of VGPR numbers named in an operand string (v7, v[8:11])."""
    out = set()
    for lo, hi, one in re.findall(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", ops):
        if one:
            out.add(int(one))
        else:
            out |= set(range(int(lo), int(hi) + 1))
    return out


def _backward(ins):
    # llvm-objdump prints a branch target as a signed 16-bit word offset
    # (e.g. `s_cbranch_scc0 64781` = -755): >= 0x8000 jumps back
    m = re.search(r"\s(\d+)$", ins)
    return bool(m) and int(m.group(1)) >= 0x8000


@pytest.mark.skipif(not os.path.exists(SO) or not shutil.which(f"{LLVM}/llvm-objdump"),
                    reason="library or llvm-objdump missing")
def test_gram_mfma_wait_state_guards(tmp_path):
    checked = 0
    checked_pair = []
    for j, obj in enumerate(_gfx950_objects(SO)):
        path = tmp_path / f"co{j}.o"
        path.write_bytes(obj)
        asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(path)], capture_output=True,
                             text=True).stdout
        for name, lines in _functions(asm).items():
            pair = "gram_pair_kernel" in name
            m = re.search(r"gram_kernelILi(\d+)E", name)
            if not pair and (not m or int(m.group(1)) < 5):
                continue
            ins = [l.split(None, 1)[1] if re.match(r"^[0-9a-f]+:?\s", l) else l
                   for l in lines if l and not l.endswith(":")]
            ins = [re.sub(r"^([0-9a-f]{8}\s)+", "", i).strip() for i in ins]
            ins = [i for i in ins if i]
            mf = [t for t, i in enumerate(ins) if i.startswith("v_mfma")]
            assert mf, name
            runs = []   # consecutive MFMAs (the compiler may pad asm boundaries with s_nop)
            for t in mf:
                if runs and all(i.startswith("s_nop") for i in ins[runs[-1][1] + 1:t]):
                    runs[-1][1] = t
                else:
                    runs.append([t, t])
            for a, b in runs:
                # >= 3 wait states between the last VALU instruction (a
                # VGPR writer) and the run: the guard's nops, or (the pair
                # kernel's partner operands) LDS loads / waits, which write
                # no VGPR by VALU and count one state each
                states, t = 0, a - 1
                while states < 3 and t >= 0:
                    i = ins[t]
                    if i.startswith("v_") and not i.startswith("v_mfma"):
                        break
                    states += _nop_states(i) or 1
                    t -= 1
                assert states >= 3, (name, ins[a - 4:a + 1])
                assert not any("accvgpr" in i for i in ins[a:b + 1]), name
            if pair:
                # VGPR accumulators (no AGPR reads to find): each role's last
                # MFMA is followed at once by mfma_exit_guard_v's 20 wait
                # states, which take every accumulator as an operand
                exits = [b for a, b in runs
                         if [_nop_states(i) for i in ins[b + 1:b + 4]] == [8, 8, 4]]
                assert len(exits) >= 2, (name, [ins[b + 1:b + 4] for a, b in runs][-4:])
                assert exits[-1] == runs[-1][1], (name, "last MFMA run unguarded")
                # per run: the first later non-MFMA instruction that touches a
                # register the run wrote comes >= 12 wait states after it on
                # the straight-line path (8-pass XDL result -> VALU / VMEM /
                # LDS reader), or a later MFMA run takes over (XDL -> XDL
                # srcC forwarding); a run may not be left by a forward branch
                # before its results are safe (a role's last run is followed
                # by the guard, whichever role's code comes after it)
                for a, b in runs:
                    dst = set()
                    for i in ins[a:b + 1]:
                        if i.startswith("v_mfma"):
                            dst |= _vregs(i.split(None, 1)[1].split(",")[0])
                    states = 0
                    for t in range(b + 1, len(ins)):
                        i = ins[t]
                        if i.startswith("v_mfma"):
                            break
                        if re.match(r"s_(c)?branch", i) and not _backward(i):
                            assert states >= 12, (name, "forward branch", ins[b:t + 1])
                            break
                        if (i.startswith(("v_", "ds_", "global_", "buffer_", "flat_"))
                                and " " in i and _vregs(i.split(None, 1)[1]) & dst):
                            assert states >= 12, (name, ins[b:t + 1])
                            break
                        states += _nop_states(i) or 1
                checked_pair.append(name)
                continue
            last = mf[-1]
            nxt = next(t for t in range(last + 1, len(ins))
                       if "accvgpr" in ins[t] or re.search(r"\ba\d+|\ba\[", ins[t]))
            states = 0      # wait states issued before a reader or a forward branch
            for i in ins[last + 1:nxt]:
                if re.match(r"s_(c)?branch", i) and not _backward(i):
                    break
                states += _nop_states(i) or 1
            assert states >= 12, (name, ins[last + 1:nxt + 1])
            checked += 1
    assert checked >= 16     # NB = 5..8 x user/item x fused/unfused (x buffer forms)
    # the NB = 8 pair kernel: user (rhs on MFMA or VALU) / item x fused /
    # unfused x buffer forms
    assert len(checked_pair) >= 12, checked_pair
