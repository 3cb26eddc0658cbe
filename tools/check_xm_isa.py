#!/usr/bin/env python3
"""Build-time guard for the X/M kernel's hand-written K loop
(csrc/band.hip: xm_load_asm / xm_wait_slot / xm_drain_slot).

The loop issues its A22 / YT loads as inline-asm ``global_load_dwordx2``
whose destination registers the compiler treats as written at issue; only
the counted ``s_waitcnt vmcnt(N)`` that ties a slot's registers says when the
data is there.  A compiler-inserted copy, spill or extra vector-memory op in
the loop would therefore read stale data silently.  This script disassembles
the gfx950 code object of build/band.o and, for xm_kernel<1> and <2>:

* requires no scratch (private segment 0, no VGPR/SGPR spills) and no
  scratch / store / buffer instruction inside the K loop;
* requires the loop body to hold exactly DA x (loads per step) loads of the
  build's kind (``global_load_dwordx2``; ``dwordx4`` for NBC = 2 with
  TG_XM_PACK) and no other vector-memory instruction, and its waits to be
  the expected ``vmcnt((DA - 1) x loads per step)`` -- the constants are read
  from band.hip's defaults;
* simulates the vector-memory counter in issue order (loads return in order
  for vmcnt) over the prologue's loads, two passes of the loop body and the
  loop exit, and fails on ANY instruction that reads or writes a register
  whose load is still outstanding.

Exit status 0 = safe; non-zero prints the offending instruction.  Run by
``__graft_entry__.build()`` after the library is built.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
HERE = os.path.dirname(os.path.abspath(__file__))
OBJ = os.path.join(HERE, "..", "gptq-svd_amd", "build", "band.o")
SRC = os.path.join(HERE, "..", "gptq-svd_amd", "csrc", "band.hip")


def build_config(src=SRC):
    """The default build's X/M constants (band.hip's #define / constexpr):
    NBC -> (mangled-name fragment, DA, loads per step, vmcnt of a slot wait,
    load mnemonics)"""
    text = open(src).read()

    def define(name):
        return int(re.search(rf"#define {name} (\d+)", text).group(1))
    pack, da2 = define("TG_XM_PACK"), define("TG_XM_DA2")
    pack1, da1 = define("TG_XM_PACK1"), define("TG_XM_DA1")
    lps2, lps1 = (2 if pack else 4), (2 if pack1 else 3)
    return {
        2: ("xm_kernelILi2E", da2, lps2, (da2 - 1) * lps2,
            {"global_load_dwordx4"} if pack else {"global_load_dwordx2"}),
        1: ("xm_kernelILi1E", da1, lps1, (da1 - 1) * lps1,
            {"global_load_dwordx2", "global_load_dwordx4"} if pack1 else {"global_load_dwordx2"}),
    }


KERNELS = build_config()
VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
REG = re.compile(r"^([va])(?:(\d+)|\[(\d+):(\d+)\])$")


def code_object(obj: str, tmp: str) -> str:
    fat = os.path.join(tmp, "fatbin")
    co = os.path.join(tmp, "band.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj,
                    os.path.join(tmp, "host.o")], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}",
                    f"--output={co}"], check=True)
    return co


def kernel_meta(co: str):
    out = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                         capture_output=True, text=True).stdout
    meta, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"\s+\.(name|private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):"
                     r"\s+(\S+)", line)
        if not m:
            continue
        if m.group(1) == "name":
            cur = m.group(2)
            meta[cur] = {}
        elif cur is not None:
            meta[cur][m.group(1)] = int(m.group(2))
    return meta


def disasm(co: str):
    """{kernel symbol: [(address, mnemonic, [operands], branch target or None)]}"""
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is None or not line.startswith("\t"):
            continue
        body, _, comment = line.strip().partition("//")
        parts = body.split(None, 1)
        if not parts:
            continue
        mn = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        am = re.search(r"([0-9A-F]+):", comment)
        if not am:          # objdump's "..." padding marker
            continue
        addr = int(am.group(1), 16)
        tm = re.search(r"<\S+\+0x([0-9a-f]+)>", comment)
        target = int(tm.group(1), 16) if tm and mn.startswith("s_cbranch") or (
            tm and mn == "s_branch") else None
        funcs[cur].append((addr, mn, ops, target))
    return funcs


def regs(op: str):
    m = REG.match(op)
    if not m:
        return set()
    kind = m.group(1)
    if m.group(2) is not None:
        return {(kind, int(m.group(2)))}
    return {(kind, r) for r in range(int(m.group(3)), int(m.group(4)) + 1)}


def check_kernel(name, insns, nbc, da, lps, wait, lmn):
    base = insns[0][0]
    off = [a - base for a, _, _, _ in insns]
    # the K loop: the backward branch whose body holds the slot waits
    loop = None
    for i, (_, mn, _, tgt) in enumerate(insns):
        if tgt is None or tgt >= off[i]:
            continue
        j = off.index(tgt)
        if any(m == "s_waitcnt" and f"vmcnt({wait})" in " ".join(o) for _, m, o, _ in insns[j:i]):
            loop = (j, i)
            break
    if loop is None:
        return [f"{name}: K loop with vmcnt({wait}) waits not found"]
    j, i = loop
    body = insns[j:i + 1]
    errs = []
    loads = [x for x in body if x[1] in lmn]
    other = [x for x in body if VMEM.match(x[1]) and x[1] not in lmn]
    if len(loads) != da * lps:
        errs.append(f"{name}: {len(loads)} loads in the K loop, expected {da * lps}")
    for x in other:
        errs.append(f"{name}: unexpected vector-memory op in the K loop: {x[1]} {', '.join(x[2])}")
    waits = [" ".join(x[2]) for x in body if x[1] == "s_waitcnt" and "vmcnt" in " ".join(x[2])]
    bad_w = [w for w in waits if f"vmcnt({wait})" not in w]
    if bad_w:
        errs.append(f"{name}: unexpected waits in the K loop: {bad_w}")
    # prologue: the DA (NBC + 2) loads before the loop head and what follows
    pro = j
    seen = 0
    while pro > 0 and seen < da * lps:
        pro -= 1
        if insns[pro][1] in lmn:
            seen += 1
    # exit: from the instruction after the back edge to the drain
    k = i + 1
    while k < len(insns) and not (insns[k][1] == "s_waitcnt" and "vmcnt(0)" in " ".join(insns[k][2])):
        k += 1
    trace = insns[pro:j] + body + body + insns[i + 1:k + 1]
    q = []  # outstanding loads: sets of destination registers, oldest first
    for addr, mn, ops, _ in trace:
        if mn == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", " ".join(ops))
            if m:
                while len(q) > int(m.group(1)):
                    q.pop(0)
            continue
        touched = set().union(*[regs(o) for o in ops]) if ops else set()
        pend = set().union(*q) if q else set()
        hit = touched & pend
        if hit and mn not in lmn:
            errs.append(f"{name}: {mn} {', '.join(ops)} at 0x{addr:x} touches "
                        f"{sorted(hit)[:4]} before its load's wait")
            break
        if VMEM.match(mn):
            if mn in lmn and hit:
                errs.append(f"{name}: load at 0x{addr:x} reuses a register with a load in flight")
                break
            q.append(regs(ops[0]) if "load" in mn else set())
    return errs


def main(obj=OBJ) -> int:
    with tempfile.TemporaryDirectory() as tmp:
        co = code_object(obj, tmp)
        meta = kernel_meta(co)
        funcs = disasm(co)
    errs = []
    for nbc, (frag, da, lps, wait, lmn) in KERNELS.items():
        names = [n for n in funcs if frag in n]
        if len(names) != 1:
            errs.append(f"xm_kernel<{nbc}> not found exactly once ({names})")
            continue
        name = names[0]
        md = meta.get(name, {})
        for key in ("private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count"):
            if md.get(key, 0) != 0:
                errs.append(f"{name}: {key} = {md[key]} (the asm K loop requires none)")
        if any(m.startswith("scratch_") for _, m, _, _ in funcs[name]):
            errs.append(f"{name}: scratch instructions present")
        errs += check_kernel(name, funcs[name], nbc, da, lps, wait, lmn)
    if errs:
        print("check_xm_isa: FAILED\n  " + "\n  ".join(errs), file=sys.stderr)
        return 1
    print("check_xm_isa: xm_kernel<1>, <2> K loops safe (no scratch, waits cover every read)")
    return 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
