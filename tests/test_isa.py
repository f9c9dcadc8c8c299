"""ISA checks on the built fp64 direct kernel (direct.h's pinned Gram).

The fp64 k = 112 / 128 Gram issues its MFMAs from inline asm so that each accumulator tile
stays in the register class it was pinned to.  The hazard recognizer cannot see those asm
writes, so correctness rests on the register allocator never copying or reading a pinned tile
between the MFMAs of a step, and on the hand-counted wait states.  This test disassembles the
compiled object (no GPU involved) and checks, for every 4-signal step of the Gram loop:
  * the step's MFMAs all accumulate in place (dst == srcC) on distinct tiles;
  * between the step's first and last MFMA nothing but MFMAs and their `s_nop` wait states,
    VMEM/LDS/scalar traffic and VALU work on OTHER registers appears: no v_accvgpr_read/write,
    no scratch access, and no instruction other than an MFMA writes a tile register;
  * each asm MFMA is preceded by its `s_nop 1` (the VALU-write → MFMA-read wait states).
Skipped when the object or the LLVM tools are absent (build() makes them)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "qmf_amd", "_build", "wals_direct_f64.o")
LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLER = os.path.join(LLVM, "clang-offload-bundler")
OBJDUMP = os.path.join(LLVM, "llvm-objdump")

needs = pytest.mark.skipif(not (os.path.exists(OBJ) and os.path.exists(BUNDLER)
                                and os.path.exists(OBJDUMP) and shutil.which("objcopy")),
                           reason="built object or LLVM tools missing")


def _disasm(tmp_path):
    fat, co = str(tmp_path / "fat.bin"), str(tmp_path / "d.co")
    subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fat, OBJ], check=True)
    subprocess.run([BUNDLER, "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    "--input=" + fat, "--output=" + co, "--unbundle"], check=True)
    return subprocess.run([OBJDUMP, "-d", co], check=True, capture_output=True,
                          text=True).stdout.split("\n")


def _regs(tok):
    """'a[8:15]' / 'v[2:3]' / 'v7' -> set of (file, index)."""
    m = re.match(r"([av])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([av])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def _kernel(lines, nt):
    name = "_ZN4qmfx18wals_direct_kernelIdLi%dELb0ELi0EEEvNS_9SolveArgsIT_EE" % nt
    start = next(i for i, l in enumerate(lines) if l.endswith("<%s>:" % name))
    end = next((i for i in range(start + 1, len(lines)) if re.match(r"^[0-9a-f]+ <", lines[i])),
               len(lines))
    return [l.split("//")[0].strip() for l in lines[start + 1:end] if l.strip()]


@needs
@pytest.mark.parametrize("nt", [7, 8])
def test_pinned_gram_steps_touch_no_tile_between_mfmas(tmp_path, nt):
    ins = _kernel(_disasm(tmp_path), nt)
    ntt = nt * (nt + 1) // 2
    mf = [i for i, l in enumerate(ins) if l.startswith("v_mfma_f64_16x16x4_f64")]
    # the Gram steps: runs of ntt MFMAs on ntt distinct in-place accumulators
    steps = []
    i = 0
    while i + ntt <= len(mf):
        grp = mf[i:i + ntt]
        accs = []
        for j in grp:
            ops = [o.strip() for o in ins[j].split(None, 1)[1].split(",")]
            accs.append((ops[0], ops[3]))
        if all(d == c for d, c in accs) and len({d for d, _ in accs}) == ntt:
            steps.append(grp)
            i += ntt
        else:
            i += 1
    assert len(steps) >= 4, "no Gram step of %d pinned MFMAs found" % ntt
    for grp in steps:
        tiles = set()
        for j in grp:
            tiles |= _regs(ins[j].split(None, 1)[1].split(",")[0].strip())
        for j in range(grp[0], grp[-1] + 1):
            l = ins[j]
            op = l.split()[0]
            if op.startswith("v_mfma"):
                assert ins[j - 1] == "s_nop 1", "asm MFMA without its wait states: %s" % l
                continue
            assert not op.startswith(("v_accvgpr_read", "v_accvgpr_write", "v_accvgpr_mov",
                                      "scratch_", "buffer_store", "buffer_load_dword_lds")), l
            # VALU results and load destinations (stores name an address first)
            if (op.startswith(("v_", "global_load", "buffer_load", "ds_read", "flat_load"))
                    and not op.startswith("v_cmpx") and " " in l):
                dst = l.split(None, 1)[1].split(",")[0].strip()
                assert not (_regs(dst) & tiles), "a tile register written between MFMAs: %s" % l
