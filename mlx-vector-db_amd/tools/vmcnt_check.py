#!/usr/bin/env python3
"""vmcnt_check.py -- static check of the vector-memory waits in the built gfx950 code objects.

The candidate passes (vdb_scan2_kernel.h, vdb_scan8_kernel.h) issue their stream loads as inline
asm (`global_load_dwordx4`) and wait for them with explicit `s_waitcnt vmcnt(N)`: the compiler
does not know those registers are still being filled, so nothing but this check stops it from
reading, copying or reusing one of them before its wait (VERDICT r3 "what's weak" #2: a cold first
search returned wrong, certified results).

For every kernel of an object file this script disassembles the device code object and runs a
forward dataflow over its control-flow graph:

  state  = the VGPRs / AGPRs a vector-memory load has not yet filled, each with the number of
           vector-memory operations (loads, stores, atomics: on gfx9 all count in vmcnt and retire
           in issue order) issued after it;
  issue  = every pending count + 1; a load's destination registers become pending with 0;
  wait   = `s_waitcnt vmcnt(N)` retires every entry with count >= N (63 outstanding stall the
           issue, so an entry with 63 younger operations has retired too);
  merge  = union, the smaller count (a register pending on any incoming path is pending);
  call   = s_swappc: the callee starts with vmcnt(0).

Any instruction other than a wait that names a pending register -- as a source, a destination,
or an address -- is a HAZARD: the hardware may still write the register after it was read or
overwritten.  (A younger LOAD into a pending register is not: loads return in issue order.)  The compiler's own loads pass by construction (its wait pass inserts the waits);
the asm streams pass only if every use sits behind a wait that covers it.

Usage: vmcnt_check.py [--filter REGEX] [--verbose] obj.o [obj.o ...]   (exit 1 on a hazard)
       vmcnt_check.py --dis file.dis ...   (an llvm-objdump -d listing)
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

LLVM = os.environ.get("VDB_LLVM_BIN", "/opt/rocm/lib/llvm/bin")
ARCH = os.environ.get("VDB_ARCH", "gfx950")
VM_PREFIX = ("global_", "buffer_", "flat_", "scratch_")
CAP = 63  # vmcnt saturates: the wave cannot issue a 64th outstanding vector-memory operation

_reg_range = re.compile(r"\b([va])\[(\d+):(\d+)\]")
_reg_one = re.compile(r"\b([va])(\d+)\b")
_func_hdr = re.compile(r"^([0-9a-fA-F]+) <([^>]+)>:\s*$")
_inst = re.compile(r"^\s+([a-z][a-z0-9_]*)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
_target = re.compile(r"<([^>+]+)\+0x([0-9a-fA-F]+)>\s*$")


def regs_of(ops):
    """The VGPR / AGPR names an operand string mentions (v[4:7] -> v4 v5 v6 v7)."""
    out = []
    for m in _reg_range.finditer(ops):
        out += [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    rest = _reg_range.sub(" ", ops)
    out += [f"{m.group(1)}{m.group(2)}" for m in _reg_one.finditer(rest)]
    return out


def split_ops(ops):
    depth, cur, out = 0, "", []
    for ch in ops:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def vmcnt_of(mn, ops):
    """The vmcnt an s_waitcnt waits for, or None when it leaves vmcnt alone."""
    if mn != "s_waitcnt":
        return None
    m = re.search(r"vmcnt\((\d+)\)", ops)
    if m:
        return int(m.group(1))
    m = re.match(r"^(0x[0-9a-fA-F]+|\d+)$", ops.strip())
    if m:  # raw gfx9 encoding: vmcnt = bits [3:0] | [15:14] << 4
        v = int(m.group(1), 0)
        return (v & 0xF) | (((v >> 14) & 3) << 4)
    return None


class Inst:
    __slots__ = ("addr", "mn", "ops", "text", "target", "is_vm", "defs", "uses", "vmcnt")

    def __init__(self, addr, mn, ops, text, target):
        self.addr, self.mn, self.ops, self.text, self.target = addr, mn, ops, text, target
        self.is_vm = mn.startswith(VM_PREFIX)
        self.vmcnt = vmcnt_of(mn, ops)
        parts = split_ops(ops)
        loads = self.is_vm and ("_load" in mn and "load_lds" not in mn)
        ret_atomic = self.is_vm and "_atomic" in mn and re.search(r"\b(sc0|glc)\b", ops) is not None
        if (loads or ret_atomic) and parts:
            self.defs = regs_of(parts[0])
            self.uses = regs_of(", ".join(parts[1:]))
        else:
            self.defs = []
            self.uses = regs_of(ops) if not mn.startswith("s_") else regs_of(ops)


def parse_dis(text):
    """{kernel: [Inst]} from an llvm-objdump -d listing."""
    funcs, cur, base = {}, None, 0
    for line in text.splitlines():
        m = _func_hdr.match(line)
        if m:
            cur = m.group(2)
            base = int(m.group(1), 16)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        m = _inst.match(line)
        if not m:
            continue
        mn, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        tgt = None
        if mn.startswith("s_cbranch") or mn == "s_branch":
            t = _target.search(line)
            if t:
                tgt = base + int(t.group(2), 16)
            else:  # simm16 words after the next instruction
                simm = int(ops.split(",")[-1].strip(), 0)
                if simm >= 0x8000:
                    simm -= 0x10000
                tgt = addr + 4 + 4 * simm
        funcs[cur].append(Inst(addr, mn, ops, line.split("//")[0].strip(), tgt))
    return funcs


def check_function(insts):
    """[(inst, reg, origin_addr, younger)] hazards of one kernel."""
    if not insts:
        return []
    index = {ins.addr: i for i, ins in enumerate(insts)}
    leaders = {0}
    for i, ins in enumerate(insts):
        if ins.target is not None:
            if ins.target in index:
                leaders.add(index[ins.target])
            leaders.add(i + 1)
        if ins.mn in ("s_endpgm", "s_setpc_b64", "s_swappc_b64"):
            leaders.add(i + 1)
    leaders = sorted(l for l in leaders if l < len(insts))
    starts = {l: n for n, l in enumerate(leaders)}
    blocks = []
    for n, l in enumerate(leaders):
        end = leaders[n + 1] if n + 1 < len(leaders) else len(insts)
        blocks.append((l, end))
    succ = []
    for (l, end) in blocks:
        last = insts[end - 1]
        s = []
        if last.mn == "s_endpgm":
            pass
        elif last.mn == "s_branch":
            if last.target in index:
                s.append(starts[index[last.target]])
        else:
            if last.target is not None and last.target in index:
                s.append(starts[index[last.target]])
            if end < len(insts):
                s.append(starts[end])
        succ.append(s)

    state_in = [None] * len(blocks)
    state_in[0] = {}
    work = [0]
    hazards = {}
    while work:
        b = work.pop()
        st = dict(state_in[b])
        l, end = blocks[b]
        for i in range(l, end):
            ins = insts[i]
            if ins.vmcnt is not None:
                st = {r: v for r, v in st.items() if v[0] < ins.vmcnt}
                continue
            if ins.mn in ("s_swappc_b64", "s_setpc_b64"):  # a callee starts with vmcnt(0)
                st = {}
                continue
            for r in ins.uses + ([] if ins.is_vm else ins.defs):
                if r in st:
                    hazards[(ins.addr, r)] = (ins, r, st[r][1], st[r][0])
            if ins.is_vm:
                # a second load into a register still being filled is no hazard: loads
                # return in issue order, so the younger one's data lands last
                st = {r: (v[0] + 1, v[1]) for r, v in st.items() if v[0] + 1 < CAP}
                for r in ins.defs:
                    st[r] = (0, ins.addr)
            else:
                for r in ins.defs:
                    st.pop(r, None)
                # a non-memory instruction that writes a register also ends its pending state
                for r in regs_of(split_ops(ins.ops)[0]) if ins.ops and not ins.mn.startswith(("s_", "ds_")) else []:
                    st.pop(r, None)
        for s in succ[b]:
            old = state_in[s]
            if old is None:
                new = dict(st)
            else:
                new = dict(old)
                for r, v in st.items():
                    if r not in new or v[0] < new[r][0]:
                        new[r] = v
            if new != old:
                state_in[s] = new
                work.append(s)
    return sorted(hazards.values(), key=lambda h: h[0].addr)


def disassemble(obj):
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(td, "j.o")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        f"--targets=hipv4-amdgcn-amd-amdhsa--{ARCH}", f"--output={co}"], check=True,
                       capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--mcpu={ARCH}", co], check=True,
                              capture_output=True, text=True).stdout


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("files", nargs="+")
    ap.add_argument("--dis", action="store_true", help="inputs are llvm-objdump listings")
    ap.add_argument("--filter", default=r"scan[0-9]*_kernel|scan_topk", help="kernel-name regex")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    flt = re.compile(a.filter)
    bad, n_k = 0, 0
    for f in a.files:
        text = open(f).read() if a.dis else disassemble(f)
        funcs = parse_dis(text)
        for name, insts in funcs.items():
            if not flt.search(name):
                continue
            n_k += 1
            hz = check_function(insts)
            if hz:
                bad += 1
                print(f"{os.path.basename(f)}: {name}: {len(hz)} hazard(s)")
                for ins, r, org, yc in hz[: (None if a.verbose else 8)]:
                    print(f"    {ins.addr:#x}: {ins.text}    <- {r} loaded at {org:#x}, {yc} younger vm ops")
    print(f"vmcnt_check: {n_k} kernels, {bad} with hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
