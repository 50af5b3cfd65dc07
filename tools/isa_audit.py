"""Static audit of the gfx950 ISA hipcc emits for the hand-written kernels.

hipcc treats an `asm volatile` statement as one opaque instruction (cdna_hip_programming.md §5.7):
a VGPR written by an asm `global_load_*` counts as defined at `;;#ASMEND`, so the compiler may read,
copy or reuse that register while the load is still in flight, and a value the compiler keeps in
M0 is not preserved across an asm statement that writes M0.  This tool checks the emitted assembly
for exactly those two hazards, plus spills:

1. every VGPR/AGPR destination of an asm-issued vector-memory load is untouched (read or written
   by any other instruction) until an `s_waitcnt vmcnt(N)` retires that load.  Vector-memory
   operations (loads, stores, atomics, LDS-DMA) retire in issue order (MI355X_MICROARCH.md, the
   vmcnt paragraph), so a load is retired by vmcnt(N) once at least N younger ones were issued
   after it.  The analysis is a forward dataflow over the basic blocks of each kernel; at a merge
   a pending load keeps the smallest "younger" count of its predecessors (the conservative one);
2. no instruction outside an asm statement reads or writes M0 (the LDS-DMA statements set M0
   without saving it);
3. `.vgpr_spill_count` and `.private_segment_fixed_size` are 0 (a spill into a register an asm
   statement names is silent corruption).

Usage: python tools/isa_audit.py [file.hip ...]   (default: every csrc/*.hip that contains asm)
Exit status 1 on any finding.  tests/test_isa_audit.py runs it on the CPU.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "twotower_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

_REG = re.compile(r"(?<![\w.])([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")
_LABEL = re.compile(r"^(\.LBB\d+_\d+):")
_VMEM_PREFIX = ("global_", "buffer_", "scratch_", "tbuffer_")


def compile_to_asm(src: str, out_dir: str, extra=()) -> str:
    out = os.path.join(out_dir, os.path.basename(src) + ".s")
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
           "-I" + os.path.join(ROOT, "include"), *extra, "--cuda-device-only", "-S", src, "-o", out]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return out


def _regs(text: str):
    out = set()
    for m in _REG.finditer(text):
        f = m.group(1)
        if m.group(4) is not None:
            out.add((f, int(m.group(4))))
        else:
            out.update((f, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


class Inst:
    __slots__ = ("op", "args", "in_asm", "line")

    def __init__(self, op, args, in_asm, line):
        self.op, self.args, self.in_asm, self.line = op, args, in_asm, line


def parse_functions(path: str, text: str | None = None):
    """-> {kernel name: blocks, kernel name + '@meta': {...}}; blocks: list of (label, [Inst])."""
    funcs = {}
    lines = (open(path).read() if text is None else text).splitlines()
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\S+):", lines[i])
        if not m:
            i += 1
            continue
        name = m.group(1)
        blocks = [(name, [])]
        in_asm = False
        j = i + 1
        while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
            raw = lines[j]
            s = raw.strip()
            j += 1
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                continue
            lm = _LABEL.match(s)
            if lm:
                blocks.append((lm.group(1), []))
                continue
            if not s or s.startswith(";") or s.startswith("."):
                continue
            s = s.split(";")[0].strip()
            if not s:
                continue
            parts = s.split(None, 1)
            blocks[-1][1].append(Inst(parts[0], parts[1] if len(parts) > 1 else "", in_asm, j))
            if parts[0].startswith(("s_cbranch", "s_branch")):
                blocks.append((f".anon{j}", []))  # a branch ends its basic block
        meta = {}
        k = j
        while k < len(lines) and k < j + 400:
            mm = re.match(r"^\s*\.(vgpr_spill_count|private_segment_fixed_size|sgpr_spill_count):\s*(\d+)", lines[k])
            if mm and mm.group(1) not in meta:
                meta[mm.group(1)] = int(mm.group(2))
            mm = re.match(r"^\s*\.amdhsa_private_segment_fixed_size\s+(\d+)", lines[k])
            if mm:
                meta.setdefault("private_segment_fixed_size", int(mm.group(1)))
            k += 1
        funcs[name] = blocks
        funcs[name + "@meta"] = meta
        i = j
    return funcs


def _succs(blocks):
    labels = {b[0]: n for n, b in enumerate(blocks)}
    succ = []
    for n, (_, insts) in enumerate(blocks):
        s = []
        last = insts[-1] if insts else None
        fall = True
        if last is not None:
            if last.op == "s_branch":
                s.append(labels[last.args.strip()])
                fall = False
            elif last.op.startswith("s_cbranch"):
                s.append(labels[last.args.strip()])
            elif last.op in ("s_endpgm", "s_setpc_b64"):
                fall = False
        if fall and n + 1 < len(blocks):
            s.append(n + 1)
        succ.append(s)
    return succ


def _is_vmem(op: str) -> bool:
    return op.startswith(_VMEM_PREFIX)


def _transfer(state, inst, findings, kname):
    """state: dict load_key -> (younger count, dest regs).  Mutates findings."""
    op = inst.op
    regs = _regs(inst.args)
    if _is_vmem(op) and "load" in op and "_lds" not in op:
        # two loads into one register retire in issue order (the later one wins): only the
        # address operands of a load count as a use
        regs = _regs(inst.args.split(",", 1)[1]) if "," in inst.args else set()
    # hazard: any other instruction touching an in-flight asm-load destination
    for key, (_, dest) in state.items():
        hit = regs & dest
        if hit:
            findings.append(f"{kname}: line {inst.line}: `{op} {inst.args}` touches "
                            f"{sorted(hit)[:4]} while an asm load into them (line {key[1]}) is in flight")
    if op == "s_waitcnt":
        m = _VMCNT.search(inst.args)
        if m:
            n = int(m.group(1))
            state = {k: v for k, v in state.items() if v[0] < n}
        return state
    if _is_vmem(op):
        state = {k: (c + 1, d) for k, (c, d) in state.items()}
        if inst.in_asm and "load" in op and "_lds" not in op:
            dest = _regs(inst.args.split(",")[0])
            state[("load", inst.line)] = (0, dest)
    return state


def _merge(a, b):
    out = dict(a)
    for k, (c, d) in b.items():
        out[k] = (min(c, out[k][0]), d) if k in out else (c, d)
    return out


def audit_kernel(kname, blocks):
    findings = []
    succ = _succs(blocks)
    n = len(blocks)
    entry_state = [None] * n
    entry_state[0] = {}
    work = [0]
    visits = 0
    while work:
        b = work.pop()
        visits += 1
        if visits > 200 * n + 1000:
            findings.append(f"{kname}: dataflow did not converge")
            break
        st = dict(entry_state[b])
        scratch = []
        for inst in blocks[b][1]:
            st = _transfer(st, inst, scratch, kname)
            st = {k: (min(c, 64), d) for k, (c, d) in st.items()}
        for s in succ[b]:
            new = st if entry_state[s] is None else _merge(entry_state[s], st)
            if entry_state[s] != new:
                entry_state[s] = new
                work.append(s)
    # final pass with converged entry states collects findings once
    for b in range(n):
        if entry_state[b] is None:
            continue
        st = dict(entry_state[b])
        for inst in blocks[b][1]:
            st = _transfer(st, inst, findings, kname)
            if not inst.in_asm and re.search(r"\bm0\b", inst.args):
                findings.append(f"{kname}: line {inst.line}: compiler instruction uses m0: `{inst.op} {inst.args}`")
    return sorted(set(findings))


def audit_file(src: str, only: str | None = None, extra=()):
    with tempfile.TemporaryDirectory() as d:
        s = compile_to_asm(src, d, extra)
        funcs = parse_functions(s)
    return audit_functions(funcs, only)


def audit_asm_text(text: str, only: str | None = None):
    return audit_functions(parse_functions("", text), only)


_MFMA = re.compile(r"^v_mfma")
_OPND = re.compile(r"([va])\[(\d+):(\d+)\]|([va])(\d+)\b")
XDL_VALU_STATES = 12  # 8-pass XDL (v_mfma_f32_32x32x16_bf16) result -> any other access
VALU_XDL_STATES = 2   # VALU write -> MFMA operand read


def _operands(args: str):
    """-> list of register sets, one per comma-separated operand (literals give an empty set)."""
    return [_regs(a) for a in args.split(",")]


def _states(inst) -> int:
    if inst.op == "s_nop":
        try:
            return int(inst.args.strip(), 0) + 1
        except ValueError:
            return 1
    return 1


def _linear(blocks):
    out = []
    for label, insts in blocks:
        for i in insts:
            out.append((label, i))
    return out


def audit_asm_mfma(kname, blocks):
    """Wait states hipcc cannot insert around an MFMA issued from inline asm (cdna_hip_programming.md
    §5.7 item 2): (a) a VALU write of any of its operands in the VALU_XDL_STATES before it; (b) any
    access to its destination in the XDL_VALU_STATES after it, except the next MFMA taking it whole as
    srcC (an accumulation chain).  Scanned in program order and across every branch to a label."""
    findings = []
    lin = _linear(blocks)
    pos = {}
    for n, (label, _) in enumerate(lin):
        pos.setdefault(label, n)
    # predecessors by branch (fall-through is program order)
    branch_in = {}
    for n, (_, i) in enumerate(lin):
        if i.op.startswith(("s_branch", "s_cbranch")):
            branch_in.setdefault(i.args.strip(), []).append(n)

    def back(n, need, seen=None):
        """instructions within `need` wait states before lin[n] (all paths)."""
        seen = seen or set()
        out = []
        k, left = n - 1, need
        label = lin[n][0]
        starts = [n]
        while k >= 0 and left > 0:
            out.append(lin[k][1])
            left -= _states(lin[k][1])
            if lin[k][0] != lin[k + 1][0] and lin[k + 1][0] in branch_in:
                for b in branch_in[lin[k + 1][0]]:
                    if (b, left) not in seen:
                        seen.add((b, left))
                        out += back(b + 1, left, seen)
            k -= 1
        del label, starts
        return out

    def fwd(n, need, seen=None):
        seen = seen or set()
        out = []
        k, left = n + 1, need
        while k < len(lin) and left > 0:
            inst = lin[k][1]
            out.append(inst)
            left -= _states(inst)
            if inst.op.startswith(("s_branch", "s_cbranch")):
                tgt = inst.args.strip()
                if tgt in pos and (tgt, left) not in seen:
                    seen.add((tgt, left))
                    out += fwd(pos[tgt] - 1, left, seen)
                if inst.op == "s_branch":
                    break
            k += 1
        return out

    for n, (_, inst) in enumerate(lin):
        if not (inst.in_asm and _MFMA.match(inst.op)):
            continue
        ops = _operands(inst.args)
        dst, srcs = ops[0], set().union(*ops[1:])
        for prev in back(n, VALU_XDL_STATES):
            if prev.op.startswith("v_") and not _MFMA.match(prev.op) and not prev.op.startswith("v_cmp"):
                w = _operands(prev.args)[0] if prev.args else set()
                if w & srcs:
                    findings.append(f"{kname}: line {inst.line}: asm MFMA reads {sorted(w & srcs)[:2]} written by "
                                    f"`{prev.op}` (line {prev.line}) fewer than {VALU_XDL_STATES} wait states before")
        for nxt in fwd(n, XDL_VALU_STATES):
            touched = _regs(nxt.args)
            if not (touched & dst):
                continue
            if _MFMA.match(nxt.op):
                o = _operands(nxt.args)
                if o[-1] == dst and not (set().union(*o[1:-1]) & dst):
                    continue  # accumulation chain: the next MFMA takes it whole as srcC
            findings.append(f"{kname}: line {nxt.line}: `{nxt.op}` touches {sorted(touched & dst)[:2]} fewer than "
                            f"{XDL_VALU_STATES} wait states after the asm MFMA at line {inst.line}")
    return findings


def audit_functions(funcs, only=None):
    findings = []
    n_asm_loads = 0
    for name, blocks in funcs.items():
        if name.endswith("@meta"):
            continue
        if only and only not in name:
            continue
        meta = funcs[name + "@meta"]
        n_asm_loads += sum(1 for _, insts in blocks for i in insts
                           if i.in_asm and _is_vmem(i.op) and "load" in i.op and "_lds" not in i.op)
        findings += audit_kernel(name, blocks)
        findings += audit_asm_mfma(name, blocks)
        for key in ("vgpr_spill_count", "private_segment_fixed_size"):
            if meta.get(key, 0):
                findings.append(f"{name}: .{key} = {meta[key]}")
    return findings, n_asm_loads


def default_sources():
    out = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".hip") and "asm volatile" in open(os.path.join(CSRC, f)).read():
            out.append(os.path.join(CSRC, f))
    return out


def main(argv):
    srcs = argv or default_sources()
    bad = 0
    for src in srcs:
        findings, nload = audit_file(src)
        print(f"{os.path.basename(src)}: {len(findings)} finding(s); {nload} asm VGPR loads tracked")
        for f in findings:
            print("  " + f)
        bad += len(findings)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
